set -o pipefail
O=gpurun_out/r6_b19; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gnn_kernels.py tests/test_gat_full.py tests/test_full_trainer.py -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; echo "tests rc=$?" >> $O/summary.txt
tail -2 $O/tests.log >> $O/summary.txt
timeout -k 10 400 python benchmarks/bench_gcn.py --model gat --dataset ppi --steps 300 --paths device > $O/est_gat.log 2>&1; echo "gat rc=$?" >> $O/summary.txt
timeout -k 10 400 python benchmarks/bench_gat.py --epochs 20 --warmup 3 --eval-epochs 0 > $O/gat_full.log 2>&1; echo "gat full rc=$?" >> $O/summary.txt
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_gat -o gat -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_gcn.py --model gat --dataset ppi --steps 200 --paths device > $GRAFT_REPO_ROOT/$O/prof.log 2>&1); echo "prof rc=$?" >> $O/summary.txt
find /tmp/prof_gat -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_gat.csv \;
grep -h '"metric"' $O/est_gat.log $O/gat_full.log | cut -c1-250 >> $O/summary.txt
cat $O/summary.txt
