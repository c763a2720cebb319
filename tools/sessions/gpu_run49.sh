R=$GRAFT_REPO_ROOT/gpurun_out/r49
mkdir -p $R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof -o run -- python3 -c "
import sys; sys.path.insert(0, '$GRAFT_REPO_ROOT')
from euler_amd.tools.runner import main
r = main(['--dataset','ppi','--batch_size','512','--total_step','200','--log_steps','100','--device','cuda','--seed','1','--model_dir','/tmp/gp_ck','--device_graph','--data_dir','/tmp/gp_data','--hidden_dim','32'], model='geniepath')
print(r)
" > $R/prof.log 2>&1 || { tail -20 $R/prof.log; exit 1; }
tail -3 $R/prof.log
find $R -name "*kernel_trace.csv" -delete
f=$(find $R -name "*kernel_stats.csv" | head -1); head -25 "$f" | cut -d, -f1-4 | cut -c1-250
