set -o pipefail
O=gpurun_out/r6_b2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gcn_trainer.py::test_fused_gcn_overflow_regrows "tests/test_full_trainer.py::test_estimator_device_graph_gcn_family_gpu" -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/fixed_tests.log 2>&1; echo "fixed tests rc=$?" >> $O/summary.txt
timeout -k 10 300 python tools/oracle_margins.py > $O/oracle_margins.json 2> $O/oracle_margins.err || exit 1
timeout -k 10 300 python benchmarks/bench_gcn.py --model transe --dataset fb15k --paths device --steps 400 > $O/transe_dense.log 2>&1 || exit 1
timeout -k 10 300 python benchmarks/bench_gcn.py --model transe --dataset fb15k --paths device --steps 400 --extra=--row_sparse_tables,on > $O/transe_rowsparse.log 2>&1 || exit 1
timeout -k 10 120 python benchmarks/bench_deepwalk.py --gpus 2 --num-nodes 1000000 --steps 5 --eval-nodes 0 > $O/dw_gpus2.log 2>&1; echo "bench_deepwalk --gpus 2 rc=$?" >> $O/summary.txt
timeout -k 10 120 python benchmarks/bench_kg.py --gpus 2 --steps 5 > $O/kg_gpus2.log 2>&1; echo "bench_kg --gpus 2 rc=$?" >> $O/summary.txt
cat $O/summary.txt
