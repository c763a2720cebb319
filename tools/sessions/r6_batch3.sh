set -o pipefail
O=gpurun_out/r6_b3; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_scalable_trainer.py tests/test_gcn_trainer.py::test_fused_gcn_overflow_regrows tests/test_engine.py -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; echo "tests rc=$?" >> $O/summary.txt
timeout -k 10 400 python benchmarks/bench_gcn.py --model scalable_sage --dataset ppi --common=--fanouts,10 --steps 400 --engine-steps 40 > $O/scalable_sage.log 2>&1; echo "scalable_sage rc=$?" >> $O/summary.txt
timeout -k 10 400 python benchmarks/bench_gcn.py --model scalable_gcn --dataset ppi --steps 200 --engine-steps 20 > $O/scalable_gcn.log 2>&1; echo "scalable_gcn rc=$?" >> $O/summary.txt
timeout -k 10 600 python benchmarks/bench_upload.py --make /tmp/g10m --num-nodes 10000000 > $O/upload_make.log 2>&1 || exit 1
timeout -k 10 500 python benchmarks/bench_upload.py --data /tmp/g10m --ranks 1 > $O/upload_w1.log 2>&1 || exit 1
timeout -k 10 500 python benchmarks/bench_upload.py --data /tmp/g10m --ranks 2 > $O/upload_w2.log 2>&1; echo "upload w2 rc=$?" >> $O/summary.txt
rm -rf /tmp/g10m
cat $O/summary.txt
