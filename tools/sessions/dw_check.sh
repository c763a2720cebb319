#!/usr/bin/env bash
# GPU box: DeepWalk / skip-gram GPU tests, the static-mode DeepWalk step and a rocprofv3 kernel profile
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
python -m euler_amd._build > $O/build.log 2>&1 || exit 4
timeout -k 10 300 python -u -m pytest tests/test_deepwalk_graph.py tests/test_gnn_kernels.py tests/test_parallel.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $O/dw_tests.log 2>&1; rc=$?; tail -2 $O/dw_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u benchmarks/bench_deepwalk.py --eval-nodes 0 --mode static > $O/dw_static.log 2>&1 || exit $?
tail -1 $O/dw_static.log | cut -c1-260
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/dw_prof -o run --output-format csv -- python3 benchmarks/bench_deepwalk.py --eval-nodes 0 --mode static --steps 20 > $O/dw_prof.log 2>&1 || exit $?
