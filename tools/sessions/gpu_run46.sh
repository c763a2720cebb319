R=$GRAFT_REPO_ROOT/gpurun_out/r46
mkdir -p $R
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_full_trainer.py -k "gcn_family" > $R/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|Error|assert" $R/pytest.log | tail -25
exit $rc
