set -o pipefail
# the W > 1 exchange path on one GPU (1-rank RCCL group): GCN full flow and SAGE trees
O=gpurun_out/r6_b24; mkdir -p $O
timeout -k 10 300 python benchmarks/bench_sharded_sage.py --model gcn --num-nodes 100000000 --steps 30 --warmup 5 --force-comm > $O/gcn_fc.log 2>&1; echo "gcn fc rc=$?" >> $O/summary.txt
timeout -k 10 300 python benchmarks/bench_sharded_sage.py --num-nodes 100000000 --steps 50 --warmup 5 --force-comm --graph > $O/sage_fc_graph.log 2>&1; echo "sage fc graph rc=$?" >> $O/summary.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_gcn -o run -- python $GRAFT_REPO_ROOT/benchmarks/bench_sharded_sage.py --model gcn --num-nodes 20000000 --steps 20 --warmup 3 --force-comm > $GRAFT_REPO_ROOT/$O/prof_gcn.log 2>&1; echo "prof rc=$?" >> $GRAFT_REPO_ROOT/$O/summary.txt
cp $(find /tmp/prof_gcn -name '*kernel_stats.csv' | head -1) $GRAFT_REPO_ROOT/$O/kernel_stats_gcn_fc.csv
cd $GRAFT_REPO_ROOT
grep -h '"metric"' $O/*.log | cut -c1-420 >> $O/summary.txt
cat $O/summary.txt
