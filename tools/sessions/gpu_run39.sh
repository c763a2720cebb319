R=$GRAFT_REPO_ROOT/gpurun_out/r39
mkdir -p $R
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gnn_kernels.py -k "gather" > $R/pytest.log 2>&1 || { tail -20 $R/pytest.log; exit 10; }
tail -1 $R/pytest.log
for m in "gae cora" "transe fb15k" "deepwalk cora" "graphsage ppi"; do
  set -- $m
  for i in 1 2; do
    timeout -k 10 300 python -u benchmarks/bench_gcn.py --model $1 --dataset $2 --steps 400 --engine-steps 40 > $R/${1}_$i.log 2>&1 || { tail -20 $R/${1}_$i.log; exit 11; }
    tail -1 $R/${1}_$i.log | cut -c1-420
  done
done
