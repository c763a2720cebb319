set -o pipefail
# kernel table of the estimator's GAT device path (FullFlowTrainer, PPI, batch 512)
O=gpurun_out/r6_b17; mkdir -p $O
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_gat -o gat -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_gcn.py --model gat --dataset ppi --steps 200 --paths device > $GRAFT_REPO_ROOT/$O/prof.log 2>&1); echo "prof rc=$?" >> $O/summary.txt
find /tmp/prof_gat -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_gat.csv \;
cat $O/summary.txt
