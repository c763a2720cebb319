R=$GRAFT_REPO_ROOT/gpurun_out/r61
mkdir -p $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $R/tests.log 2>&1 || { echo "tests failed"; tail -30 $R/tests.log; exit 1; }
tail -1 $R/tests.log
for rep in 1 2; do
timeout -k 10 300 python -u benchmarks/bench_deepwalk.py --eval-nodes 0 --steps 100 --warmup 10 > $R/dw_bench_$rep.log 2>&1 || { echo "dw bench failed"; tail -20 $R/dw_bench_$rep.log; exit 1; }
tail -1 $R/dw_bench_$rep.log | cut -c1-200
done
timeout -k 10 300 python -u benchmarks/bench_deepwalk.py --steps 100 --warmup 10 --eval-nodes 1000000 --eval-steps 3000 > $R/dw_bench_learn.log 2>&1 || { echo "dw learn failed"; tail -20 $R/dw_bench_learn.log; exit 1; }
tail -1 $R/dw_bench_learn.log | grep -o '"heldout_link_prediction": [^}]*}' || true
timeout -k 10 200 python -u benchmarks/bench_gcn.py --model deepwalk --dataset cora --steps 800 > $R/dw_est_1.log 2>&1 || { echo "dw est failed"; tail -20 $R/dw_est_1.log; exit 1; }
tail -1 $R/dw_est_1.log | cut -c1-250
echo done
