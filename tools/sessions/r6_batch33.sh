set -o pipefail
O=gpurun_out/r6_b33; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sage_trainer.py tests/test_unsup_sage.py tests/test_device_infer.py tests/test_sharded_graph.py -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; echo "tests rc=$?" >> $O/summary.txt
tail -1 $O/tests.log >> $O/summary.txt
grep FAILED $O/tests.log | head >> $O/summary.txt
cat $O/summary.txt
