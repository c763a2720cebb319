set -o pipefail
# every node-classification zoo model through NodeEstimator: device path vs engine path (PPI, batch 512)
O=gpurun_out/r6_b21; mkdir -p $O
for m in dna gat agnn appnp arma sgcn tagcn geniepath lgcn fastgcn adaptivegcn graphsage gcn; do
  timeout -k 10 240 python benchmarks/bench_gcn.py --model $m --dataset ppi --steps 200 --engine-steps 20 > $O/est_$m.log 2>&1; echo "$m rc=$?" >> $O/summary.txt
done
python - >> $O/summary.txt <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/r6_b21/est_*.log")):
    for l in open(f):
        if l.startswith('{"metric"'):
            d = json.loads(l)
            print(f.split("est_")[1][:-4], round(d["device"]["samples_per_sec"]), round(d["engine"]["samples_per_sec"]), d.get("speedup"))
PY
cat $O/summary.txt
