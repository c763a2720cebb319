#!/usr/bin/env bash
# GPU box: segment / relation / KG GPU tests, then the KG step with the wave-per-segment sums
# (EULER_AMD_SEG_WAVE=1) vs the lane-group segment kernel (0), each with a rocprofv3 profile
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
python -m euler_amd._build > $O/build.log 2>&1 || exit 4
timeout -k 10 300 python -u -m pytest tests/test_gnn_kernels.py tests/test_zoo.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $O/seg_tests.log 2>&1; rc=$?; tail -2 $O/seg_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  EULER_AMD_SEG_WAVE=$v timeout -k 10 300 python -u benchmarks/bench_kg.py --steps 50 --warmup 5 --eval-after 0 > $O/kg_seg$v.log 2>&1 || exit $?
  echo "seg_wave $v: $(tail -1 $O/kg_seg$v.log | cut -c1-200)"
  EULER_AMD_SEG_WAVE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kg_prof_seg$v -o run --output-format csv -- python3 benchmarks/bench_kg.py --steps 30 --warmup 5 --eval-after 0 > $O/kg_prof_seg$v.log 2>&1 || exit $?
done
