set -o pipefail
# full GPU suite after the shared-export fix + the sharded-graph SAGE bench (int32 tree, direct single-rank tables)
O=gpurun_out/r6_b11; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread --maxfail 15 -p no:cacheprovider > $O/gpu_tests.log 2>&1; echo "suite rc=$?" >> $O/summary.txt
tail -4 $O/gpu_tests.log
grep FAILED $O/gpu_tests.log | head
timeout -k 10 300 python benchmarks/bench_sharded_sage.py --gpus 1 --num-nodes 100000000 --steps 200 --warmup 10 --graph > $O/sharded_sage_graph.log 2>&1; echo "sharded rc=$?" >> $O/summary.txt
timeout -k 10 300 python benchmarks/bench_sharded_sage.py --gpus 1 --num-nodes 100000000 --steps 100 --warmup 10 > $O/sharded_sage_eager.log 2>&1; echo "sharded eager rc=$?" >> $O/summary.txt
grep -h '"metric"' $O/sharded_sage_*.log | cut -c1-260 >> $O/summary.txt
cat $O/summary.txt
