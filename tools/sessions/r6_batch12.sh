set -o pipefail
O=gpurun_out/r6_b12; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sharded_graph.py tests/test_deepwalk_graph.py tests/test_kg_trainer.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; echo "tests rc=$?" >> $O/summary.txt
grep -E "PASSED|FAILED|ERROR" $O/tests.log | head -30
cat $O/summary.txt
