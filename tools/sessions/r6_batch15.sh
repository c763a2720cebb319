set -o pipefail
# 10M-node graph: per-rank engine shards (W = 2, 4; gloo on the one GPU) vs the whole-graph engine per rank
O=gpurun_out/r6_b15; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_sharded_graph.py -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; echo "tests rc=$?" >> $O/summary.txt
timeout -k 10 600 python benchmarks/bench_upload.py --make /tmp/g10m --num-nodes 10000000 > $O/make.log 2>&1 && \
timeout -k 10 400 python benchmarks/bench_upload.py --data /tmp/g10m --ranks 2 --engine-shards > $O/shards_w2.log 2>&1; echo "w2 rc=$?" >> $O/summary.txt
timeout -k 10 400 python benchmarks/bench_upload.py --data /tmp/g10m --ranks 4 --engine-shards > $O/shards_w4.log 2>&1; echo "w4 rc=$?" >> $O/summary.txt
rm -rf /tmp/g10m
grep -h phase $O/*.log | cut -c1-400 >> $O/summary.txt
cat $O/summary.txt
