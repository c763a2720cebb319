set -o pipefail
O=gpurun_out/r6_b35; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_sharded_graph.py -m gpu -v --timeout 100 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; echo "tests rc=$?" >> $O/summary.txt
tail -1 $O/tests.log >> $O/summary.txt
grep FAILED $O/tests.log | head >> $O/summary.txt
timeout -k 10 300 python benchmarks/bench_sharded_sage.py --model gcn --num-nodes 100000000 --steps 50 --warmup 5 --force-comm --graph > $O/gcn_fc_graph.log 2>&1; echo "gcn fc graph rc=$?" >> $O/summary.txt
timeout -k 10 300 python benchmarks/bench_sharded_sage.py --model gcn --num-nodes 100000000 --steps 30 --warmup 5 --force-comm > $O/gcn_fc_eager.log 2>&1; echo "gcn fc eager rc=$?" >> $O/summary.txt
timeout -k 10 300 python benchmarks/bench_sharded_sage.py --model gcn --num-nodes 100000000 --steps 50 --warmup 5 --graph > $O/gcn_w1_graph.log 2>&1; echo "gcn w1 graph rc=$?" >> $O/summary.txt
timeout -k 10 400 python benchmarks/bench_sharded_sage.py --model gcn --gpus 2 --shared-gpu --num-nodes 20000000 --steps 20 --warmup 3 > $O/gcn_shared2.log 2>&1; echo "gcn shared2 rc=$?" >> $O/summary.txt
grep -h '"metric"' $O/gcn_*.log | cut -c1-330 >> $O/summary.txt
cat $O/summary.txt
