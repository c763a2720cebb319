set -o pipefail
# config 3 through the product (captured full-graph GAT), estimator GAT row, sharded-graph SAGE at 100M nodes
O=gpurun_out/r6_b7; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gat_full.py -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; echo "tests rc=$?" >> $O/summary.txt
grep -E "PASSED|FAILED|ERROR" $O/tests.log | head
timeout -k 10 400 python benchmarks/bench_gat.py --epochs 20 --warmup 3 --eval-epochs 0 > $O/gat_graph.log 2>&1; echo "gat graph rc=$?" >> $O/summary.txt
timeout -k 10 400 python benchmarks/bench_gat.py --epochs 20 --warmup 3 --eval-epochs 0 --no-graph > $O/gat_eager.log 2>&1; echo "gat eager rc=$?" >> $O/summary.txt
timeout -k 10 500 python benchmarks/bench_gcn.py --model gat --dataset ppi --steps 300 --engine-steps 30 > $O/est_gat.log 2>&1; echo "est gat rc=$?" >> $O/summary.txt
timeout -k 10 500 python benchmarks/bench_sharded_sage.py --gpus 1 --num-nodes 100000000 --steps 50 --warmup 5 > $O/sharded_sage_eager.log 2>&1; echo "sharded sage rc=$?" >> $O/summary.txt
timeout -k 10 500 python benchmarks/bench_sharded_sage.py --gpus 1 --num-nodes 100000000 --steps 100 --warmup 5 --graph > $O/sharded_sage_graph.log 2>&1; echo "sharded sage graph rc=$?" >> $O/summary.txt
grep -h '"metric"' $O/*.log | cut -c1-400 >> $O/summary.txt
cat $O/summary.txt
