#!/usr/bin/env bash
# PMC counter passes (one counter group per run, as rocprofv3 cannot split passes) over a
# short run of a benchmark; run on the GPU box through gpurun.  Usage:
#   tools/pmc_passes.sh <name> <python script + args...>
# writes gpurun_out/pmc_<name>/<pass>/... (csv)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
NAME=$1; shift
OUT=$REPO/gpurun_out/pmc_$NAME
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
PASSES=${PASSES:-"FETCH_SIZE|WRITE_SIZE|SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE|SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"}
IFS='|' read -ra PL <<< "$PASSES"
for pass in "${PL[@]}"; do
  tag=$(echo "$pass" | tr ' ' '+')
  timeout -s KILL 180 rocprofv3 --pmc $pass --output-format csv -d "$OUT/$tag" -o run -- python3 "$REPO/$1" "${@:2}" \
    > "$OUT/$tag.log" 2>&1 || { echo "pass $pass failed rc=$?"; tail -5 "$OUT/$tag.log"; exit 1; }
  echo "pass $pass ok"
done
