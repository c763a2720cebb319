set -o pipefail
# batch6 (deterministic KG v3: radix-sort CSR) + batch7 (captured GAT, estimator GAT, sharded SAGE at 100M)
# + the 10M-node engine load after the loader fixes
bash tools/sessions/r6_batch6.sh
bash tools/sessions/r6_batch7.sh
O=gpurun_out/r6_b8; mkdir -p $O
timeout -k 10 600 python benchmarks/bench_upload.py --make /tmp/g10m --num-nodes 10000000 > $O/upload_make.log 2>&1 && \
EULER_LOG_LEVEL=info timeout -k 10 500 python benchmarks/bench_upload.py --data /tmp/g10m --ranks 1 > $O/upload_w1.log 2>&1; echo "upload rc=$?" >> $O/summary.txt
rm -rf /tmp/g10m
grep -h "phase\|graph load" $O/upload_w1.log | tail -12
