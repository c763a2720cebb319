export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/r40
mkdir -p $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kg_step.py > $R/pytest.log 2>&1 || { tail -30 $R/pytest.log; exit 10; }
tail -1 $R/pytest.log
for rep in 8 0 16 4; do
  for i in 1 2; do
    EULER_AMD_KG_REL_REP=$rep timeout -k 10 200 python -u benchmarks/bench_kg.py --steps 300 --warmup 20 --eval-after 0 > $R/kg_rep${rep}_$i.log 2>&1 || exit 11
    echo "rep $rep $(tail -1 $R/kg_rep${rep}_$i.log | cut -c1-140)"
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_kg.py --steps 200 --warmup 10 --eval-after 0 > $R/prof.log 2>&1 || exit 12
find $R -name "*kernel_trace.csv" -delete
