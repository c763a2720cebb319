set -o pipefail
# sampled-flow sharded trainer captured over RCCL; GPU tests; flow benches
O=gpurun_out/r6_b26; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_sharded_graph.py -m gpu -v --timeout 100 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; echo "tests rc=$?" >> $O/summary.txt
tail -2 $O/tests.log >> $O/summary.txt
for mode in "" "--force-comm"; do
  for gr in "" "--graph"; do
    timeout -k 10 300 python benchmarks/bench_sharded_sage.py --model flow --conv gcn --num-nodes 100000000 --steps 30 --warmup 5 $mode $gr > $O/flow${mode}${gr}.log 2>&1; echo "flow $mode $gr rc=$?" >> $O/summary.txt
  done
done
grep -h '"metric"' $O/flow*.log | cut -c1-330 >> $O/summary.txt
cat $O/summary.txt
