OUT_DIR=r5pz bash tools/gpu_steps.sh \
 "prof_genie|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5pz/prof -o genie -- python benchmarks/bench_gcn.py --model geniepath --dataset ppi --paths device --steps 100" \
 "prof_rgcn|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5pz/prof -o rgcn -- python benchmarks/bench_gcn.py --model rgcn --dataset wn18 --paths device --steps 100"
