set -o pipefail
# sharded unsupervised GraphSAGE: GPU test + benches (100M nodes, B=1024 sources, 5 negatives)
O=gpurun_out/r6_b31; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_sharded_graph.py -m gpu -k unsup -v --timeout 100 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; echo "tests rc=$?" >> $O/summary.txt
timeout -k 10 300 python benchmarks/bench_sharded_sage.py --model unsup --num-nodes 100000000 --steps 30 --warmup 5 --graph > $O/unsup_graph.log 2>&1; echo "unsup graph rc=$?" >> $O/summary.txt
timeout -k 10 300 python benchmarks/bench_sharded_sage.py --model unsup --num-nodes 100000000 --steps 30 --warmup 5 --force-comm --graph > $O/unsup_fc_graph.log 2>&1; echo "unsup fc graph rc=$?" >> $O/summary.txt
timeout -k 10 300 python benchmarks/bench_sharded_sage.py --model unsup --num-nodes 100000000 --steps 20 --warmup 3 --force-comm > $O/unsup_fc_eager.log 2>&1; echo "unsup fc eager rc=$?" >> $O/summary.txt
timeout -k 10 400 python benchmarks/bench_sharded_sage.py --model unsup --gpus 2 --shared-gpu --num-nodes 20000000 --steps 10 --warmup 2 > $O/unsup_shared2.log 2>&1; echo "unsup shared2 rc=$?" >> $O/summary.txt
timeout -k 10 300 python benchmarks/bench_unsup_sage.py --fanouts 25,10 --dims 256,256,64 --batch-size 1024 --num-negs 5 --steps 300 --eval-pairs 2000 > $O/whole_fused.log 2>&1; echo "whole fused rc=$?" >> $O/summary.txt
grep -h "\"metric\"" $O/unsup_*.log $O/whole_fused.log | cut -c1-330 >> $O/summary.txt
cat $O/summary.txt
