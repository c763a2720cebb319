#!/usr/bin/env bash
# GPU box: relation-transform GPU tests, then the KG benchmark and a rocprofv3 kernel profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
python -m euler_amd._build > $O/build.log 2>&1 || exit 4
timeout -k 10 300 python -u -m pytest tests/test_gnn_kernels.py tests/test_zoo.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $O/rg_tests.log 2>&1; rc=$?; tail -2 $O/rg_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/bench_kg.py --steps 50 --warmup 5 --eval-after 0 > $O/kg.log 2>&1 || exit $?
tail -1 $O/kg.log | cut -c1-250
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kg_prof -o run --output-format csv -- python3 benchmarks/bench_kg.py --steps 30 --warmup 5 --eval-after 0 > $O/kg_prof.log 2>&1 || exit $?
