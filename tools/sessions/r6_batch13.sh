set -o pipefail
# round-6 closing measurements: headline x3, config 2 x3, config 4 (bare) x2, config 5 x2, headline kernel trace + gaps
O=$PWD/gpurun_out/r6_b13; mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; echo "$name rc=$? $(grep '"metric"' $O/$name.log | cut -c1-150)" >> $O/summary.txt; }
for i in 1 2 3; do run headline_$i 300 python -u bench.py --steps 1000 --warmup 50; done
for i in 1 2 3; do run driver_$i 300 python -u bench.py --steps 20 --warmup 5; done
for i in 1 2; do run config2_$i 300 python -u bench.py --steps 1000 --warmup 50 --num-nodes 10000000; done
for i in 1 2; do run kg_$i 300 python -u benchmarks/bench_kg.py --steps 300 --warmup 20 --eval-after 0; done
for i in 1 2; do run dw_$i 300 python -u benchmarks/bench_deepwalk.py --eval-nodes 0 --mode graph --steps 200; done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_h -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 200 --warmup 20 > $O/prof_headline.log 2>&1); echo "prof rc=$?" >> $O/summary.txt
find /tmp/prof_h -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_headline.csv \;
T=$(find /tmp/prof_h -name "*kernel_trace.csv" | head -1)
[ -n "$T" ] && python tools/trace_gaps.py "$T" --last 6 --first-kernel tr_fwd > $O/trace_gaps.txt 2>&1
cat $O/summary.txt
