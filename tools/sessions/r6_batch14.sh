set -o pipefail
# shared-GPU rehearsals (2 ranks on the box's one GPU, gloo, all-to-alls staged through host memory):
# config 4 DeepWalk with sharded tables, config 5 R-GCN + TransE, GraphSAGE on a row-sharded graph
O=gpurun_out/r6_b14; mkdir -p $O
timeout -k 10 400 python benchmarks/bench_deepwalk.py --gpus 2 --shared-gpu --num-nodes 1000000 --steps 50 --warmup 5 --eval-nodes 0 > $O/dw_shared2.log 2>&1; echo "dw rc=$?" >> $O/summary.txt
timeout -k 10 400 python benchmarks/bench_kg.py --gpus 2 --shared-gpu --steps 50 --warmup 5 --eval-after 0 > $O/kg_shared2.log 2>&1; echo "kg rc=$?" >> $O/summary.txt
timeout -k 10 400 python benchmarks/bench_sharded_sage.py --gpus 2 --shared-gpu --num-nodes 10000000 --steps 30 --warmup 5 > $O/sharded_sage_shared2.log 2>&1; echo "sharded rc=$?" >> $O/summary.txt
grep -h '"metric"' $O/*.log | cut -c1-330 >> $O/summary.txt
cat $O/summary.txt
