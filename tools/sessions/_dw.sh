OUT_DIR=r5dw2 bash tools/gpu_steps.sh \
 "dw_default|400|python benchmarks/bench_deepwalk.py --eval-nodes 0" \
 "dw_static|400|python benchmarks/bench_deepwalk.py --eval-nodes 0 --mode static --steps 100 --warmup 10"
