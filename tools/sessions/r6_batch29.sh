set -o pipefail
O=gpurun_out/r6_b29; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_sharded_graph.py tests/test_device_infer.py tests/test_unsup_sage.py -m gpu -v --timeout 100 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; echo "tests rc=$?" >> $O/summary.txt
tail -2 $O/tests.log >> $O/summary.txt
grep -E "FAILED|Error" $O/tests.log | head -5 >> $O/summary.txt
cat $O/summary.txt
