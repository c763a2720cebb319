R=$GRAFT_REPO_ROOT/gpurun_out/r55
mkdir -p $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gnn_kernels.py tests/test_deepwalk_estimator.py tests/test_deepwalk_graph.py tests/test_zoo.py > $R/tests.log 2>&1 || { echo "tests failed"; tail -30 $R/tests.log; exit 1; }
tail -2 $R/tests.log
for rep in 1 2; do
timeout -k 10 200 python -u benchmarks/bench_gcn.py --model deepwalk --dataset cora --steps 800 > $R/dw_est_$rep.log 2>&1 || { echo "dw est failed"; tail -20 $R/dw_est_$rep.log; exit 1; }
tail -1 $R/dw_est_$rep.log | cut -c1-300
done
timeout -k 10 300 python -u benchmarks/bench_deepwalk.py --eval-nodes 0 --steps 100 --warmup 10 > $R/dw_bench.log 2>&1 || { echo "dw bench failed"; tail -20 $R/dw_bench.log; exit 1; }
tail -1 $R/dw_bench.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/prof -o dw -- python $GRAFT_REPO_ROOT/benchmarks/bench_gcn.py --model deepwalk --dataset cora --steps 200 > $R/prof.log 2>&1 || { echo "prof failed"; tail -20 $R/prof.log; exit 1; }
echo done
