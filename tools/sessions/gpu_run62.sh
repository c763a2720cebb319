R=$GRAFT_REPO_ROOT/gpurun_out/r62
mkdir -p $R
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $R/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $R/smoke.log; exit 1; }
tail -1 $R/smoke.log
timeout -k 10 300 python -u bench.py > $R/bench_default.log 2>&1 || { echo "bench failed"; tail -20 $R/bench_default.log; exit 1; }
tail -1 $R/bench_default.log | cut -c1-220
echo done
