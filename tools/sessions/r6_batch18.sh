set -o pipefail
# SegmentIndex on the bit-limited radix CSR + EdgeCSR reusing cached block CSRs: GPU suite, estimator GAT / GCN / SAGE-flow
O=gpurun_out/r6_b18; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread --maxfail 15 -p no:cacheprovider > $O/gpu_tests.log 2>&1; echo "suite rc=$?" >> $O/summary.txt
tail -3 $O/gpu_tests.log >> $O/summary.txt
grep FAILED $O/gpu_tests.log | head >> $O/summary.txt
timeout -k 10 400 python benchmarks/bench_gcn.py --model gat --dataset ppi --steps 300 --paths device > $O/est_gat.log 2>&1; echo "gat rc=$?" >> $O/summary.txt
timeout -k 10 400 python benchmarks/bench_gcn.py --model agnn --dataset ppi --steps 300 --paths device > $O/est_agnn.log 2>&1; echo "agnn rc=$?" >> $O/summary.txt
timeout -k 10 400 python benchmarks/bench_gcn.py --model gcn --dataset ppi --steps 300 --paths device > $O/est_gcn.log 2>&1; echo "gcn rc=$?" >> $O/summary.txt
grep -h '"metric"' $O/est_*.log | cut -c1-250 >> $O/summary.txt
cat $O/summary.txt
