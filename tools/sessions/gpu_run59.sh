R=$GRAFT_REPO_ROOT/gpurun_out/r59
mkdir -p $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_deepwalk_estimator.py tests/test_deepwalk_graph.py tests/test_zoo.py tests/test_parallel.py tests/test_gnn_kernels.py > $R/tests.log 2>&1 || { echo "tests failed"; tail -30 $R/tests.log; exit 1; }
tail -1 $R/tests.log
timeout -k 10 200 python -u benchmarks/bench_gcn.py --model deepwalk --dataset cora --steps 800 > $R/dw_est_1.log 2>&1 || { echo "dw est failed"; tail -20 $R/dw_est_1.log; exit 1; }
tail -1 $R/dw_est_1.log | cut -c1-250
for rep in 1 2; do
timeout -k 10 300 python -u benchmarks/bench_deepwalk.py --eval-nodes 0 --steps 100 --warmup 10 > $R/dw_bench_$rep.log 2>&1 || { echo "dw bench failed"; tail -20 $R/dw_bench_$rep.log; exit 1; }
tail -1 $R/dw_bench_$rep.log | cut -c1-200
done
echo done
