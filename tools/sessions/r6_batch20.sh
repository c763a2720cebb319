set -o pipefail
O=gpurun_out/r6_b20; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread --maxfail 15 -p no:cacheprovider > $O/gpu_tests.log 2>&1; echo "suite rc=$?" >> $O/summary.txt
tail -2 $O/gpu_tests.log >> $O/summary.txt
grep FAILED $O/gpu_tests.log | head >> $O/summary.txt
for m in gat agnn dna; do
  timeout -k 10 400 python benchmarks/bench_gcn.py --model $m --dataset ppi --steps 300 --engine-steps 30 > $O/est_$m.log 2>&1; echo "$m rc=$?" >> $O/summary.txt
done
timeout -k 10 300 python benchmarks/bench_kg.py --steps 300 --warmup 20 --eval-after 0 --deterministic > $O/kg_det.log 2>&1; echo "kg det rc=$?" >> $O/summary.txt
grep -h '"metric"' $O/est_*.log $O/kg_det.log | cut -c1-330 >> $O/summary.txt
cat $O/summary.txt
