R=$GRAFT_REPO_ROOT/gpurun_out/r47
mkdir -p $R
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_deepwalk_estimator.py > $R/pytest.log 2>&1 || { tail -30 $R/pytest.log; exit 1; }
grep -E "PASSED|FAILED" $R/pytest.log
for spec in "line cora" "dgi cora" "vgae cora" "fastgcn ppi" "adaptivegcn ppi"; do
  set -- $spec
  timeout -k 10 400 python -u benchmarks/bench_gcn.py --model $1 --dataset $2 --steps 400 --engine-steps 40 > $R/bench_$1.log 2>&1 || { echo "bench $1 failed"; tail -20 $R/bench_$1.log; exit 1; }
  echo "$1 $(tail -1 $R/bench_$1.log | cut -c1-400)"
done
