R=$GRAFT_REPO_ROOT/gpurun_out/r51
mkdir -p $R
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_rgcn_trainer.py tests/test_full_trainer.py -k "rgcn or gcn_family" > $R/pytest.log 2>&1 || { grep -E "Error|error|assert|FAILED" $R/pytest.log | head -20; tail -5 $R/pytest.log; exit 1; }
grep -E "PASSED|FAILED" $R/pytest.log
timeout -k 10 400 python -u benchmarks/bench_gcn.py --model rgcn --dataset wn18 --steps 400 --engine-steps 40 > $R/bench_rgcn.log 2>&1 || { echo "bench failed"; tail -20 $R/bench_rgcn.log; exit 1; }
echo "rgcn $(tail -1 $R/bench_rgcn.log | cut -c1-400)"
