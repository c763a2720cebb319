set -o pipefail
# deterministic KG backward: tests, step time atomic vs deterministic, kernel stats
O=gpurun_out/r6_b4; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kg_step.py tests/test_graph_memset.py tests/test_sharded_graph.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; echo "tests rc=$?" >> $O/summary.txt
timeout -k 10 300 python benchmarks/bench_kg.py --steps 400 --warmup 20 --eval-after 0 > $O/kg_atomic.log 2>&1; echo "kg atomic rc=$?" >> $O/summary.txt
timeout -k 10 300 python benchmarks/bench_kg.py --steps 400 --warmup 20 --eval-after 0 --deterministic > $O/kg_det.log 2>&1; echo "kg det rc=$?" >> $O/summary.txt
timeout -k 10 300 python benchmarks/bench_kg.py --steps 400 --warmup 20 --eval-after 0 > $O/kg_atomic2.log 2>&1; echo "kg atomic2 rc=$?" >> $O/summary.txt
timeout -k 10 300 python benchmarks/bench_kg.py --steps 400 --warmup 20 --eval-after 0 --deterministic > $O/kg_det2.log 2>&1; echo "kg det2 rc=$?" >> $O/summary.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_det -o det -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_kg.py --steps 200 --warmup 10 --eval-after 0 --deterministic > $GRAFT_REPO_ROOT/$O/prof_det.log 2>&1; echo "prof det rc=$?" >> $GRAFT_REPO_ROOT/$O/summary.txt
cd $GRAFT_REPO_ROOT
grep -h '"metric"' $O/kg_*.log | python -c "import sys,json; [print(json.loads(l)['ms_per_step'], json.loads(l)['config'].get('deterministic')) for l in sys.stdin]" >> $O/summary.txt
cat $O/summary.txt
