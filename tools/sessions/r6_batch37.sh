set -o pipefail
O=gpurun_out/r6_b37; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_gcn -o run -- python $GRAFT_REPO_ROOT/benchmarks/bench_sharded_sage.py --model gcn --num-nodes 20000000 --steps 40 --warmup 3 --force-comm --graph > $GRAFT_REPO_ROOT/$O/prof_gcn.log 2>&1; echo "prof rc=$?" >> $GRAFT_REPO_ROOT/$O/summary.txt
cp $(find /tmp/prof_gcn -name '*kernel_stats.csv' | head -1) $GRAFT_REPO_ROOT/$O/kernel_stats_gcn_fc_graph.csv
cd $GRAFT_REPO_ROOT
cat $O/summary.txt
