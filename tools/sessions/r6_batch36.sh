set -o pipefail
# final: GPU suite, smoke, bench.py (driver protocol), 2-rank shared-GPU rehearsal of bench.py
O=gpurun_out/r6_b36; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; echo "smoke rc=$?" >> $O/summary.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread --maxfail 15 -p no:cacheprovider > $O/gpu_tests.log 2>&1; echo "suite rc=$?" >> $O/summary.txt
tail -2 $O/gpu_tests.log >> $O/summary.txt
grep FAILED $O/gpu_tests.log | head >> $O/summary.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1; echo "bench rc=$?" >> $O/summary.txt
timeout -k 10 400 python bench.py --gpus 2 --shared-gpu --steps 20 --warmup 5 > $O/bench_shared2.log 2>&1; echo "bench shared2 rc=$?" >> $O/summary.txt
grep -h '"metric"' $O/bench_*.log | cut -c1-300 >> $O/summary.txt
cat $O/summary.txt
