#!/usr/bin/env bash
# One GPU session on a gpurun box: GPU tests, a short bench, a rocprofv3 kernel profile.
# Every GPU step has its own time limit; a crash/abort/timeout (exit >= 124 or signal)
# ends the script immediately.  Plain test failures (exit 1) let the bench still run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out
STEPS="${STEPS:-all}"

run() {  # run <name> <timeout> cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "fatal rc=$rc in $name: stopping the session"; exit $rc
  fi
  return $rc
}

python -c "import torch; print(torch.__version__, torch.cuda.get_device_name(0))" || exit 3
python -m euler_amd._build >"$OUT/build.log" 2>&1 || { cat "$OUT/build.log"; exit 4; }

if [[ "$STEPS" == *tests* || "$STEPS" == all ]]; then
  run pytest_gpu 900 python -m pytest tests -m gpu --maxfail=20 -q -p no:cacheprovider -rf
fi
if [[ "$STEPS" == *bench* || "$STEPS" == all ]]; then
  run bench_small 400 python bench.py --num-nodes 2000000 --steps 50 --warmup 10 --log
  run bench_full 900 python bench.py --steps 200 --warmup 20 --log
fi
if [[ "$STEPS" == *prof* || "$STEPS" == all ]]; then
  run rocprof 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
      python3 bench.py --num-nodes 10000000 --steps 50 --warmup 5
fi
echo "=== done"
