export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/r41
mkdir -p $R
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof_unsup -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_unsup_sage.py --steps 300 > $R/prof_unsup.log 2>&1 || exit 11
find $R -name "*kernel_trace.csv" -delete
cd $GRAFT_REPO_ROOT && timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $R/pytest.log 2>&1 || { tail -30 $R/pytest.log; exit 10; }
tail -1 $R/pytest.log
