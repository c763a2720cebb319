set -o pipefail
# final check of the round's tree: smoke, the full GPU suite, bench.py at the driver protocol
O=gpurun_out/r6_b16; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; echo "smoke rc=$?" >> $O/summary.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread --maxfail 15 -p no:cacheprovider > $O/gpu_tests.log 2>&1; echo "suite rc=$?" >> $O/summary.txt
tail -3 $O/gpu_tests.log >> $O/summary.txt
grep FAILED $O/gpu_tests.log | head >> $O/summary.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1; echo "bench rc=$?" >> $O/summary.txt
grep '"metric"' $O/bench_driver.log | cut -c1-200 >> $O/summary.txt
cat $O/summary.txt
