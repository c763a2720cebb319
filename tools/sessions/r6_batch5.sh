set -o pipefail
# deterministic KG + sharded graph GPU tests, KG step kernel stats (atomic vs deterministic)
O=gpurun_out/r6_b5; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_sharded_graph.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; echo "tests rc=$?" >> $O/summary.txt
grep -E "PASSED|FAILED|ERROR|Error|assert" $O/tests.log | head -60
for mode in atomic det; do
  extra=""; [ $mode = det ] && extra="--deterministic"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$mode -o kg -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_kg.py --steps 30 --warmup 5 --eval-after 0 --no-graph $extra > $GRAFT_REPO_ROOT/$O/prof_$mode.log 2>&1); echo "prof $mode rc=$?" >> $O/summary.txt
  find /tmp/prof_$mode -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_$mode.csv \;
done
cat $O/summary.txt
