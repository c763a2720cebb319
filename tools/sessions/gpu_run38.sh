R=$GRAFT_REPO_ROOT/gpurun_out/r38
mkdir -p $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gnn_kernels.py tests/test_full_trainer.py tests/test_gae_trainer.py > $R/pytest.log 2>&1 || { tail -40 $R/pytest.log; exit 10; }
tail -1 $R/pytest.log
for i in 1 2 3; do
  timeout -k 10 300 python -u benchmarks/bench_gcn.py --steps 400 --engine-steps 40 > $R/gcn_$i.log 2>&1 || exit 11
  tail -1 $R/gcn_$i.log | cut -c1-400
done
