set -o pipefail
# full GPU suite + bench.py (driver protocol and default) + sharded-graph SAGE kernel table
O=gpurun_out/r6_b10; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread --maxfail 15 -p no:cacheprovider > $O/gpu_tests.log 2>&1; echo "suite rc=$?" >> $O/summary.txt
tail -8 $O/gpu_tests.log
grep FAILED $O/gpu_tests.log | head
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1; echo "bench driver rc=$?" >> $O/summary.txt
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1; echo "bench default rc=$?" >> $O/summary.txt
timeout -k 10 300 python benchmarks/bench_sharded_sage.py --gpus 1 --num-nodes 100000000 --steps 100 --warmup 5 --graph > $O/sharded_sage_graph.log 2>&1; echo "sharded rc=$?" >> $O/summary.txt
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_sh -o sh -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_sharded_sage.py --gpus 1 --num-nodes 100000000 --steps 30 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1); echo "prof rc=$?" >> $O/summary.txt
find /tmp/prof_sh -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_sharded.csv \;
grep -h '"metric"' $O/bench_*.log $O/sharded_sage_graph.log | cut -c1-300 >> $O/summary.txt
cat $O/summary.txt
