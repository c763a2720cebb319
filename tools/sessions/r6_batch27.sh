set -o pipefail
O=gpurun_out/r6_b27; mkdir -p $O
timeout -k 10 150 python -u -m pytest tests/test_sharded_graph.py -m gpu -k captures_over_rccl -v -o faulthandler_timeout=50 -p no:cacheprovider > $O/alone.log 2>&1; echo "alone rc=$?" >> $O/summary.txt
cat $O/summary.txt
