R=$GRAFT_REPO_ROOT/gpurun_out/r52
mkdir -p $R
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_dgi_trainer.py tests/test_rgcn_trainer.py > $R/pytest.log 2>&1 || { grep -E "Error|error|assert|FAILED" $R/pytest.log | head -20; tail -5 $R/pytest.log; exit 1; }
grep -E "PASSED|FAILED" $R/pytest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $R/smoke.log 2>&1 || { tail -20 $R/smoke.log; exit 1; }
tail -1 $R/smoke.log
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 > $R/bench.log 2>&1 || { tail -20 $R/bench.log; exit 1; }
tail -1 $R/bench.log | cut -c1-300
