set -o pipefail
# kernel table of the sharded-graph SAGE step (W = 1, eager) at 100M nodes
O=gpurun_out/r6_b9; mkdir -p $O
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_sh -o sh -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_sharded_sage.py --gpus 1 --num-nodes 100000000 --steps 30 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1); echo "prof rc=$?" >> $O/summary.txt
find /tmp/prof_sh -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
cat $O/summary.txt
