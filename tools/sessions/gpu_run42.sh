export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/r42
mkdir -p $R
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof_gat -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_gat.py --epochs 10 --eval-epochs 0 > $R/prof_gat.log 2>&1 || exit 11
find $R -name "*kernel_trace.csv" -delete
