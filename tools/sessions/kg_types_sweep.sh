#!/usr/bin/env bash
# Learning evidence for config 5 (R-GCN + TransE) on the typed KG (dataset/synthetic.py
# typed_kg: the test triples are cold entities' has_type triples; only message passing can
# place a cold entity).  Each run trains KG_STEPS steps (unnormalised TransE rows) and ranks
# the held-out triples; one JSON line per run in gpurun_out/kg_types/.
#   KG_TYPES="layers:bases:rel_wd:lr:margin[:self_drop] ..."   KG_ARGS: extra bench_kg.py arguments
#   KG_TAG: log-name suffix
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/kg_types
for c in ${KG_TYPES:-0:0:0:0.01:10 1:0:0:0.01:4}; do
  IFS=':' read -r l b wd lr mg sd <<< "$c"
  sd=${sd:-0}
  name="types_l${l}_b${b}_wd${wd}_lr${lr}_m${mg}_sd${sd}${KG_TAG:-}"
  timeout -k 10 300 python -u benchmarks/bench_kg.py --task types --layers "$l" --num-bases "$b" --rel-wd "$wd" \
    --lr "$lr" --margin "$mg" --normalize 0 --steps 50 --warmup 5 --eval-after "${KG_STEPS:-3000}" --self-drop "$sd" ${KG_ARGS:-} \
    > "gpurun_out/kg_types/$name.log" 2>&1
  rc=$?
  echo "$name rc=$rc $(tail -1 gpurun_out/kg_types/$name.log | python3 -c 'import json,sys
try:
  d=json.loads(sys.stdin.read()); t=d["config"]["heldout_tail_ranking"]; print(d["ms_per_step"], t["trained"])
except Exception as e: print("no json", e)')"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
