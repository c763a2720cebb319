OUT_DIR=r5pz2 bash tools/gpu_steps.sh \
 "dw|300|python benchmarks/bench_gcn.py --model deepwalk --dataset cora --paths device --steps 800" \
 "prof_dw|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5pz2/prof -o dw -- python benchmarks/bench_gcn.py --model deepwalk --dataset cora --paths device --steps 200" \
 "line|300|python benchmarks/bench_gcn.py --model line --dataset cora --paths device --steps 800" \
 "prof_line|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5pz2/prof -o line -- python benchmarks/bench_gcn.py --model line --dataset cora --paths device --steps 200"
