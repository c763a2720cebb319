R=$GRAFT_REPO_ROOT/gpurun_out/r53
mkdir -p $R
for rep in 2 3; do
for spec in "line cora" "dgi cora" "vgae cora" "fastgcn ppi" "adaptivegcn ppi" "geniepath ppi" "lgcn ppi" "solution ppi" "rgcn wn18"; do
  set -- $spec
  timeout -k 10 200 python -u benchmarks/bench_gcn.py --model $1 --dataset $2 --steps 400 --engine-steps 40 > $R/bench_$1_$rep.log 2>&1 || { echo "bench $1 failed"; tail -20 $R/bench_$1_$rep.log; exit 1; }
  echo "$1 $rep $(tail -1 $R/bench_$1_$rep.log | grep -o '"device": {[^}]*}' | grep -o 'samples_per_sec": [0-9.]*') $(tail -1 $R/bench_$1_$rep.log | grep -o '"speedup": [0-9.]*')"
done
done
