#!/usr/bin/env bash
# Closing measurements of a round on one MI355X (BASELINE.md protocol: 3 runs each, medians
# reported in README.md), written under gpurun_out/measure/.  Run it through gpurun:
#   gpurun --timeout 1200 -- 'bash tools/measure_round.sh'
# Kernel tables: rocprofv3 --kernel-trace --stats --output-format csv (the per-dispatch
# traces are deleted before the results travel back: gpurun merges at most 64 MiB).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD/gpurun_out/measure
mkdir -p "$R"
run() {  # name timeout command...
  local name=$1 t=$2
  shift 2
  timeout -k 10 "$t" "$@" > "$R/$name.log" 2>&1 || { echo "$name failed: $?"; tail -20 "$R/$name.log"; exit 1; }
  echo "$name $(tail -1 "$R/$name.log" | cut -c1-160)"
}
for i in 1 2 3; do run "headline_$i" 300 python -u bench.py --steps 1000 --warmup 50; done
for i in 1 2 3; do run "config2_$i" 300 python -u bench.py --steps 1000 --warmup 50 --num-nodes 10000000; done
for i in 1 2 3; do run "unsup_$i" 300 python -u benchmarks/bench_unsup_sage.py --steps 2000; done
for i in 1 2 3; do run "kg_$i" 300 python -u benchmarks/bench_kg.py --steps 300 --warmup 20 --eval-after 0; done
for i in 1 2 3; do run "gcn_$i" 400 python -u benchmarks/bench_gcn.py --steps 400 --engine-steps 40; done
for i in 1 2 3; do run "dw_$i" 300 python -u benchmarks/bench_deepwalk.py --eval-nodes 0 --mode graph --steps 200; done
for i in 1 2 3; do run "gat_$i" 400 python -u benchmarks/bench_gat.py --epochs 200 --eval-epochs 0; done
for b in bench.py benchmarks/bench_kg.py; do
  n=$(basename "$b" .py)
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/prof_$n" -o run \
    -- python3 "$OLDPWD/$b" --steps 200 --warmup 20 $([ "$n" = bench_kg ] && echo --eval-after 0) \
    > "$R/prof_$n.log" 2>&1) || { echo "profile $n failed"; exit 1; }
done
find "$R" -name "*kernel_trace.csv" -delete
find "$R" -size +4M -delete
echo done
