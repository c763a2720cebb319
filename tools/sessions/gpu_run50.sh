R=$GRAFT_REPO_ROOT/gpurun_out/r50
mkdir -p $R
timeout -k 10 1100 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/ > $R/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $R/pytest.log | head -20
tail -2 $R/pytest.log
exit $rc
