R=$GRAFT_REPO_ROOT/gpurun_out/r43
mkdir -p $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_graph_trainer.py > $R/pytest.log 2>&1 || { tail -40 $R/pytest.log; exit 10; }
tail -1 $R/pytest.log
for m in gin graphgcn set2set; do
  timeout -k 10 300 python -u benchmarks/bench_gcn.py --model $m --dataset mutag --batch-size 64 --steps 400 --engine-steps 40 > $R/${m}.log 2>&1 || { tail -20 $R/${m}.log; exit 11; }
  tail -1 $R/${m}.log | cut -c1-400
done
