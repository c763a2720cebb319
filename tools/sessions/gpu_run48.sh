R=$GRAFT_REPO_ROOT/gpurun_out/r48
mkdir -p $R
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_full_trainer.py -k "lgcn or solution" > $R/pytest.log 2>&1 || { grep -E "Error|error|assert" $R/pytest.log | head -20; tail -5 $R/pytest.log; exit 1; }
grep -E "PASSED|FAILED" $R/pytest.log
timeout -k 10 400 python -u benchmarks/bench_gcn.py --model solution --dataset ppi --steps 400 --engine-steps 40 > $R/bench_solution.log 2>&1 || { echo "bench failed"; tail -20 $R/bench_solution.log; exit 1; }
echo "solution $(tail -1 $R/bench_solution.log | cut -c1-400)"
