set -o pipefail
mkdir -p gpurun_out/r6_dw_est
free -g > gpurun_out/r6_dw_est/mem_before.txt
timeout -k 10 300 python benchmarks/bench_deepwalk.py --steps 200 --warmup 10 --eval-nodes 0 > gpurun_out/r6_dw_est/bench_deepwalk.log 2>&1 && \
timeout -k 10 600 python benchmarks/bench_deepwalk_estimator.py --phase train --steps 2000 --log-steps 200 --model-dir /dev/shm/dwck > gpurun_out/r6_dw_est/train.log 2>&1 && \
du -sh /dev/shm/dwck >> gpurun_out/r6_dw_est/train.log && \
timeout -k 10 600 python benchmarks/bench_deepwalk_estimator.py --phase resume --steps 2000 --resume-steps 1000 --log-steps 200 --model-dir /dev/shm/dwck > gpurun_out/r6_dw_est/resume.log 2>&1
rc=$?
rm -rf /dev/shm/dwck
exit $rc
