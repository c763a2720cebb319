#!/usr/bin/env bash
# Fused-step tuning sweep on a gpurun box: fused-step tests, one rocprofv3 kernel
# profile of the default config, then bench.py for a few (BM0, DW_KPS) variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT"
python -m euler_amd._build >"$OUT/build.log" 2>&1 || { cat "$OUT/build.log"; exit 4; }
timeout -k 10 600 python -m pytest tests/test_sage_step.py -q -p no:cacheprovider -rf >"$OUT/sweep_tests.log" 2>&1
rc=$?; tail -n 5 "$OUT/sweep_tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc"; exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_sweep" -o run --output-format csv -- \
  python3 bench.py --num-nodes 10000000 --steps 50 --warmup 5 >"$OUT/sweep_prof.log" 2>&1 || { tail -5 "$OUT/sweep_prof.log"; exit 5; }
for bm in 32 64; do
  for kps in 16 32 64; do
    EULER_AMD_BM0=$bm EULER_AMD_DW_KPS=$kps timeout -k 10 300 python bench.py --num-nodes 10000000 --steps 100 \
      --warmup 10 >"$OUT/sweep_bm${bm}_kps${kps}.log" 2>&1 || { echo "bench failed bm=$bm kps=$kps"; exit 6; }
    echo "bm=$bm kps=$kps $(grep -o '"ms_per_step": [0-9.]*' "$OUT/sweep_bm${bm}_kps${kps}.log")"
  done
done
echo "=== sweep done"
