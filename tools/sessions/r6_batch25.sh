set -o pipefail
# sharded full flow after the slot-CSR requester expansion: GPU tests, force-comm GCN bench + profile
O=gpurun_out/r6_b25; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_sharded_graph.py -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; echo "tests rc=$?" >> $O/summary.txt
tail -2 $O/tests.log >> $O/summary.txt
timeout -k 10 300 python benchmarks/bench_sharded_sage.py --model gcn --num-nodes 100000000 --steps 30 --warmup 5 --force-comm > $O/gcn_fc.log 2>&1; echo "gcn fc rc=$?" >> $O/summary.txt
timeout -k 10 300 python benchmarks/bench_sharded_sage.py --model gcn --num-nodes 100000000 --steps 30 --warmup 5 > $O/gcn_w1_eager.log 2>&1; echo "gcn eager rc=$?" >> $O/summary.txt
timeout -k 10 300 python benchmarks/bench_sharded_sage.py --model gcn --num-nodes 100000000 --steps 50 --warmup 5 --graph > $O/gcn_w1_graph.log 2>&1; echo "gcn graph rc=$?" >> $O/summary.txt
timeout -k 10 400 python benchmarks/bench_sharded_sage.py --model gcn --gpus 2 --shared-gpu --num-nodes 20000000 --steps 20 --warmup 3 > $O/gcn_shared2.log 2>&1; echo "gcn shared2 rc=$?" >> $O/summary.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_gcn -o run -- python $GRAFT_REPO_ROOT/benchmarks/bench_sharded_sage.py --model gcn --num-nodes 20000000 --steps 20 --warmup 3 --force-comm > $GRAFT_REPO_ROOT/$O/prof_gcn.log 2>&1; echo "prof rc=$?" >> $GRAFT_REPO_ROOT/$O/summary.txt
cp $(find /tmp/prof_gcn -name '*kernel_stats.csv' | head -1) $GRAFT_REPO_ROOT/$O/kernel_stats_gcn_fc.csv
cd $GRAFT_REPO_ROOT
grep -h '"metric"' $O/gcn_*.log | cut -c1-420 >> $O/summary.txt
cat $O/summary.txt
