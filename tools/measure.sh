#!/usr/bin/env bash
# Measurement session on a gpurun box: build, fused-step GPU tests, the headline bench
# (100M nodes, 1 GPU), a rocprofv3 kernel profile, and the reference-equivalent CPU
# baseline on the same 100M-node config with the box's 16-thread
# CPU share.  Every GPU step has its own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT"
STEPS=${STEPS:-200}
python -m euler_amd._build >"$OUT/build.log" 2>&1 || { tail -20 "$OUT/build.log"; exit 4; }
timeout -k 10 600 python -m pytest tests/test_sage_step.py -q -p no:cacheprovider -rf >"$OUT/m_tests.log" 2>&1
rc=$?; tail -n 3 "$OUT/m_tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc"; exit $rc; fi
timeout -k 10 300 python tools/prof_head.py >"$OUT/m_head.log" 2>&1 || { tail -5 "$OUT/m_head.log"; exit 8; }
cat "$OUT/m_head.log"
timeout -k 10 600 python bench.py --steps "$STEPS" --warmup 20 >"$OUT/m_bench.log" 2>&1 || { tail -5 "$OUT/m_bench.log"; exit 5; }
tail -n 1 "$OUT/m_bench.log"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/m_prof" -o run --output-format csv -- \
  python3 bench.py --num-nodes 10000000 --steps 50 --warmup 5 >"$OUT/m_prof.log" 2>&1 || { tail -5 "$OUT/m_prof.log"; exit 6; }
if [ "${CPU_BASELINE:-1}" = "1" ]; then
  timeout -k 10 900 python -m euler_amd.tools.cpu_baseline --num-nodes 100000000 --threads 16 --steps 50 --warmup 5 \
    --out "$OUT/cpu_baseline.json" >"$OUT/m_cpu.log" 2>&1 || { tail -5 "$OUT/m_cpu.log"; exit 7; }
  cat "$OUT/cpu_baseline.json"
fi
echo "=== measure done"
