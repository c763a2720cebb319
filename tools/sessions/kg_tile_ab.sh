#!/usr/bin/env bash
# GPU box: KG step and rel_gemm kernel time at message-GEMM tile sizes 64 / 128 (EULER_AMD_RG_TILE)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
python -m euler_amd._build > $O/build.log 2>&1 || exit 4
for t in ${TILES:-64 128}; do
  EULER_AMD_RG_TILE=$t timeout -k 10 300 python -u benchmarks/bench_kg.py --steps 50 --warmup 5 --eval-after 0 > $O/kg_t$t.log 2>&1 || exit $?
  echo "tile $t: $(tail -1 $O/kg_t$t.log | cut -c1-200)"
  EULER_AMD_RG_TILE=$t timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kg_prof_t$t -o run --output-format csv -- python3 benchmarks/bench_kg.py --steps 30 --warmup 5 --eval-after 0 > $O/kg_prof_t$t.log 2>&1 || exit $?
done
