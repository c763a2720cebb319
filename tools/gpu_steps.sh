#!/usr/bin/env bash
# Run named GPU steps on a gpurun box, each under its own time limit, output under
# gpurun_out/$OUT_DIR/<name>.log.  Usage (through gpurun):
#   OUT_DIR=r5a bash tools/gpu_steps.sh 'name|timeout|command' 'name|timeout|command' ...
# A plain failure (exit 1: a failing test, a refused config) lets the later steps run; a
# time limit, abort, segfault or GPU fault ends the script at once (nothing more touches
# the GPU after a fault).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD/gpurun_out/${OUT_DIR:-steps}
mkdir -p "$R"
status=0
for spec in "$@"; do
  name=${spec%%|*}
  rest=${spec#*|}
  to=${rest%%|*}
  cmd=${rest#*|}
  echo "=== $name ($(date +%T), limit ${to}s)"
  timeout -k 10 "$to" bash -c "$cmd" > "$R/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc"
  tail -n 12 "$R/$name.log" | cut -c1-400
  if grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR|faulted:" "$R/$name.log"; then
    echo "GPU fault in $name: stopping"; exit 70
  fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "fatal rc=$rc in $name: stopping"; exit $rc
  fi
  [ $rc -ne 0 ] && status=1
done
find "$R" -name "*kernel_trace.csv" -delete 2>/dev/null
find "$R" -size +4M -delete 2>/dev/null
exit $status
