R=$GRAFT_REPO_ROOT/gpurun_out/r45
mkdir -p $R
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_dgi_trainer.py tests/test_gae_trainer.py tests/test_deepwalk_estimator.py > $R/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|Error" $R/pytest.log | tail -25
exit $rc
