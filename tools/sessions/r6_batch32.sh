set -o pipefail
O=gpurun_out/r6_b32; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_mp.py tests/test_sharded_graph.py -m gpu -k "gather_sum or unsup" -v --timeout 100 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; echo "tests rc=$?" >> $O/summary.txt
tail -1 $O/tests.log >> $O/summary.txt
timeout -k 10 300 python benchmarks/bench_sharded_sage.py --model unsup --num-nodes 100000000 --steps 30 --warmup 5 --graph > $O/unsup_graph.log 2>&1; echo "unsup graph rc=$?" >> $O/summary.txt
timeout -k 10 300 python benchmarks/bench_sharded_sage.py --model unsup --num-nodes 100000000 --steps 30 --warmup 5 --force-comm --graph > $O/unsup_fc_graph.log 2>&1; echo "unsup fc graph rc=$?" >> $O/summary.txt
grep -h '"metric"' $O/unsup_*.log | cut -c1-300 >> $O/summary.txt
cat $O/summary.txt
