set -o pipefail
# GAT full-graph epoch kernel breakdown (ogbn-products shape)
O=gpurun_out/r6_b28; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_gat -o run -- python $GRAFT_REPO_ROOT/benchmarks/bench_gat.py --epochs 5 --warmup 2 --eval-epochs 0 > $GRAFT_REPO_ROOT/$O/prof_gat.log 2>&1; echo "prof rc=$?" >> $GRAFT_REPO_ROOT/$O/summary.txt
cp $(find /tmp/prof_gat -name '*kernel_stats.csv' | head -1) $GRAFT_REPO_ROOT/$O/kernel_stats_gat.csv
cd $GRAFT_REPO_ROOT
cat $O/summary.txt
