set -o pipefail
# deterministic KG backward v2 (kernel-written keys, det_occ CSR, block segment sums): tests, timing, kernel stats
O=gpurun_out/r6_b6; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kg_step.py tests/test_graph_memset.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; echo "tests rc=$?" >> $O/summary.txt
grep -E "PASSED|FAILED|ERROR" $O/tests.log | head -40
for i in 1; do
  timeout -k 10 300 python benchmarks/bench_kg.py --steps 400 --warmup 20 --eval-after 0 > $O/kg_atomic$i.log 2>&1; echo "kg atomic rc=$?" >> $O/summary.txt
  timeout -k 10 300 python benchmarks/bench_kg.py --steps 400 --warmup 20 --eval-after 0 --deterministic > $O/kg_det$i.log 2>&1; echo "kg det rc=$?" >> $O/summary.txt
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_det -o kg -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_kg.py --steps 30 --warmup 5 --eval-after 0 --no-graph --deterministic > $GRAFT_REPO_ROOT/$O/prof_det.log 2>&1); echo "prof det rc=$?" >> $O/summary.txt
find /tmp/prof_det -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_det.csv \;
grep -h '"metric"' $O/kg_*.log | python -c "import sys,json; [print(json.loads(l)['ms_per_step'], json.loads(l)['config'].get('deterministic')) for l in sys.stdin]" >> $O/summary.txt
cat $O/summary.txt
