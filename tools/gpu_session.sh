#!/usr/bin/env bash
# One GPU session on a gpurun box.  STEPS selects comma-separated steps:
#   tests=<pytest args>   (default tests: the whole -m gpu suite)
#   bench_small, bench_full, bench_fp32, prof, sweep_batch
# Every GPU step has its own time limit; a crash/abort/timeout (exit >= 124 or a signal)
# ends the script immediately.  Plain test failures (exit 1) let later steps still run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out
STEPS="${STEPS:-tests,bench_small,bench_full,prof}"
TESTS="${TESTS:-tests -m gpu}"

run() {  # run <name> <timeout> cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 30 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "fatal rc=$rc in $name: stopping the session"; exit $rc
  fi
  if grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR|faulted:" "$OUT/$name.log"; then
    echo "GPU fault in $name: stopping the session"; exit 70
  fi
  return $rc
}

python -m euler_amd._build >"$OUT/build.log" 2>&1 || { cat "$OUT/build.log"; exit 4; }

IFS=',' read -ra S <<< "$STEPS"
for st in "${S[@]}"; do
  case "$st" in
    debug)
      EULER_AMD_TREE_SYNC=1 run tree_debug 300 python -u tools/tree_debug.py 0 1 2 3 4 5 6 7 8 9 || exit 71 ;;
    tests)
      run pytest_gpu 900 python -u -m pytest $TESTS -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -rf ;;
    kernels)
      run tree_kernels 300 python -u tools/tree_kernels.py ;;
    sweep_dw)
      for wg in 256 512 768; do
        EULER_AMD_DW_ROUTE_WG=$wg run "tree_kernels_rwg$wg" 300 python -u tools/tree_kernels.py
      done
      EULER_AMD_TREE_FORK=0 run tree_kernels_nofork 300 python -u tools/tree_kernels.py ;;
    sweep_sample)
      EULER_AMD_SAMPLE_IN=opt run tree_kernels_sample_opt 300 python -u tools/tree_kernels.py ;;
    sweep_pipe)
      # pipelined step: gather tiles first / last in the optimizer grid, parameter tiles per block
      for cfg in "1:4" "1:1" "0:4" "0:8" "1:8"; do
        IFS=':' read -r gf tpb <<< "$cfg"
        EULER_AMD_GATHER_FIRST=$gf EULER_AMD_OPT_TPB=$tpb run "tree_kernels_pipe_gf${gf}_tpb${tpb}" 300 \
          python -u tools/tree_kernels.py || exit $?
      done
      EULER_AMD_PIPELINE=0 run tree_kernels_nopipe 300 python -u tools/tree_kernels.py ;;
    gemm_bench)
      run gemm_bench 300 python -u tools/gemm_bench.py ;;
    sweep_fwd)
      for bm in 32 64 128; do
        EULER_AMD_FWD_BM=$bm run "tree_kernels_fbm$bm" 300 python -u tools/tree_kernels.py
      done ;;
    trace)
      run trace 300 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- \
          python3 -u tools/tree_kernels.py --reps 20 && \
      python tools/trace_gaps.py "$OUT/trace/run_kernel_trace.csv" --last 3 > "$OUT/trace_gaps.txt" 2>&1; \
      cat "$OUT/trace_gaps.txt" ;;
    pmc)
      PASSES="FETCH_SIZE|TCC_HIT_sum TCC_MISS_sum|SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD|SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE|SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS" \
        run pmc 600 bash tools/pmc_passes.sh tree "$PWD/tools/tree_kernels.py" --reps 10 ;;
    pmc_calib)
      PASSES="FETCH_SIZE|WRITE_SIZE|TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" \
        run pmc_calib 300 bash tools/pmc_passes.sh calib "$PWD/tools/pmc_calibrate.py" ;;
    pmc_fwd)
      run pmc_fwd_plain 300 python -u tools/pmc_fwd_check.py || exit $?
      PASSES="FETCH_SIZE|TCC_HIT_sum TCC_MISS_sum" run pmc_fwd 300 bash tools/pmc_passes.sh fwd "$PWD/tools/pmc_fwd_check.py" ;;
    ppi_device)
      run ppi_device 600 python -u examples/run_graphsage.py --dataset ppi --device_graph --device cuda \
          --batch_size 512 --total_step 3000 --log_steps 500 --model_dir /tmp/ppi_dev --fanouts 10 10 \
          --learning_rate 0.01 ;;
    ppi_device_b32)
      run ppi_device_b32 600 python -u examples/run_graphsage.py --dataset ppi --device_graph --device cuda \
          --batch_size 32 --total_step 3000 --log_steps 500 --model_dir /tmp/ppi_dev32 --fanouts 10 10 \
          --learning_rate 0.01 ;;
    engine_sage)
      run engine_sage 900 python -u benchmarks/bench_engine_sage.py --steps 300 --warmup 20 \
        --native_workers ${ENGINE_WORKERS:-4 8 16} ;;
    engine_remote)
      # native pipeline over 2 same-host shard servers: input alone, then with the model step
      run engine_remote_pipeline 600 python -u benchmarks/bench_engine_sage.py --mode remote --pipeline_only \
        --native_workers 4 8 16 --steps 200 || exit $?
      run engine_remote 900 python -u benchmarks/bench_engine_sage.py --mode remote --native_workers 8 16 \
        --only native_8workers,native_16workers --steps 200 ;;
    engine_prof)
      run engine_sage_cprofile 600 python -u benchmarks/bench_engine_sage.py --steps 200 --warmup 20 \
        --only native_8workers --cprofile gpurun_out/engine_sage_cprofile.txt ;;
    engine_rocprof)
      run engine_rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/engine_prof" -o run --output-format csv -- \
          python3 benchmarks/bench_engine_sage.py --steps 300 --warmup 20 --native_workers 16 --only native_16workers ;;
    cpu_baseline)
      run cpu_baseline 900 python -u -m euler_amd.tools.cpu_baseline --num-nodes 100000000 --threads 16 \
        --sweep 4,8,16 --out "$OUT/cpu_baseline.json" ;;
    learn_kg)
      run bench_kg 600 python -u benchmarks/bench_kg.py ;;
    learn_gat)
      run bench_gat 900 python -u benchmarks/bench_gat.py ;;
    shard_prof)
      RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29552 \
        run shard_prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/shard_prof" -o run --output-format csv -- \
          python3 bench.py --force-dist --shard-features --steps 50 --warmup 5 ;;
    shard_bench)
      # bench.py with the feature table row-sharded: one rank through the all-to-all path
      run bench_shard 600 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29541 bench.py --force-dist --shard-features --steps 200 \
        --warmup 20 || exit $?
      run bench_force_dist 600 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29542 bench.py --force-dist --steps 200 --warmup 20 ;;
    community_f1)
      run community_f1 900 python -u benchmarks/bench_community_f1.py --steps "${F1_STEPS:-1000}" ;;
    gat_compare)
      # same task, same seed, same epochs: fused gat.hip vs the composed autograd reference
      for impl in fused composed; do
        # 1M nodes: the composed variant's fp32 per-edge messages of the full 124M-edge
        # graph do not fit next to its autograd buffers
        run "bench_gat_$impl" 900 python -u benchmarks/bench_gat.py --impl $impl \
          --num-nodes "${GAT_NODES:-1000000}" --eval-epochs "${GAT_EPOCHS:-400}" || exit $?
      done ;;
    gat_ab)
      run gat_ab 600 python -u tools/gat_ab.py --num-nodes "${GAT_AB_NODES:-1000000}" ;;
    gat_variants)
      # GAT_VARIANTS="-DGAT_FWD_U=4|-DGAT_FWD_U=8": rebuild gat.hip per flag set, time the edge kernels
      IFS='|' read -ra VL <<< "${GAT_VARIANTS:-}"
      i=0
      for v in "${VL[@]}"; do
        i=$((i+1))
        touch euler_amd/csrc/hip/gat.hip
        EULER_AMD_HIP_FLAGS="$v" python -m euler_amd._build > "$OUT/build_gat_variant$i.log" 2>&1 || exit 4
        EULER_AMD_HIP_FLAGS="$v" run "gat_kernels_variant$i" 300 python -u tools/gat_kernels.py || exit $?
      done ;;
    kg_tasks)
      # learning evidence: unnormalised TransE alone vs R-GCN + TransE on the lattice and on
      # the cold-entity task (KG_STEPS untimed training steps before the ranking)
      for t in lattice cold; do
        for l in 0 2; do
          run "kg_${t}_l$l" 600 python -u benchmarks/bench_kg.py --task $t --layers $l --normalize 0 \
            --eval-after "${KG_STEPS:-3000}" || exit $?
        done
      done ;;
    kg_sweep)
      # KG_SWEEP="task:layers:lr:margin ..." (3000 training steps each, unnormalised TransE)
      for c in ${KG_SWEEP:-lattice:0:0.01:10}; do
        IFS=':' read -r t l lr mg <<< "$c"
        run "kgs_${t}_l${l}_lr${lr}_m${mg}" 600 python -u benchmarks/bench_kg.py --task $t --layers $l --normalize 0 \
          --lr $lr --margin $mg --eval-after "${KG_STEPS:-3000}" || exit $?
      done ;;
    final_benches)
      # BASELINE.md protocol for the secondary configs: 3 runs of >= 200 timed steps each
      # (tools/median_summary.py takes the medians)
      for r in 1 2 3; do
        run "fb_unsup_$r" 300 python -u benchmarks/bench_unsup_sage.py --steps 1000 || exit $?
        run "fb_kg_$r" 300 python -u benchmarks/bench_kg.py --steps 200 --warmup 10 --eval-after 0 || exit $?
        run "fb_dw_$r" 300 python -u benchmarks/bench_deepwalk.py --eval-nodes 0 --mode graph --steps 200 || exit $?
        run "fb_dw_dist_$r" 300 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 1 \
          --master-addr 127.0.0.1 --master-port 2956$r benchmarks/bench_deepwalk.py --eval-nodes 0 --mode graph \
          --steps 200 --force-dist || exit $?
        run "fb_gat_$r" 600 python -u benchmarks/bench_gat.py --epochs 200 --eval-epochs 0 || exit $?
        run "fb_headline_$r" 300 python -u bench.py --steps 1000 --warmup 20 || exit $?
      done ;;
    final_benches_hd)
      # the 3-run protocol for the benchmarks this session changed: headline, DeepWalk local
      # and its one-rank all-to-all path
      for r in 1 2 3; do
        run "fb_dw_$r" 300 python -u benchmarks/bench_deepwalk.py --eval-nodes 0 --mode graph --steps 200 || exit $?
        run "fb_dw_dist_$r" 300 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 1 \
          --master-addr 127.0.0.1 --master-port 2956$r benchmarks/bench_deepwalk.py --eval-nodes 0 --mode graph \
          --steps 200 --force-dist || exit $?
        run "fb_headline_$r" 300 python -u bench.py --steps 1000 --warmup 20 || exit $?
      done ;;
    final_benches_other)
      # the 3-run protocol for unsupervised GraphSAGE, R-GCN + TransE and GAT
      for r in 1 2 3; do
        run "fb_unsup_$r" 300 python -u benchmarks/bench_unsup_sage.py --steps 1000 || exit $?
        run "fb_kg_$r" 300 python -u benchmarks/bench_kg.py --steps 200 --warmup 10 --eval-after 0 || exit $?
        run "fb_gat_$r" 600 python -u benchmarks/bench_gat.py --epochs 200 --eval-epochs 0 || exit $?
      done ;;
    kg_dw_sweep)
      # KG_DW="chunk:slab ..." (rel_gemm_dw edges per chunk, slab width)
      for c in ${KG_DW:-512:128 256:128 1024:128 512:64 256:64}; do
        EULER_AMD_RG_CH=${c%%:*} EULER_AMD_RG_DW_T=${c##*:} run "kg_dw_${c%%:*}_${c##*:}" 300 \
          python -u benchmarks/bench_kg.py --steps 100 --warmup 10 --eval-after 0 || exit $?
      done ;;
    kg_prof)
      run kg_prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/kg_prof" -o run --output-format csv -- \
          python3 benchmarks/bench_kg.py --steps 50 --warmup 5 --eval-after 0 ;;
    gat_time)
      run bench_gat_time 600 python -u benchmarks/bench_gat.py --eval-epochs 0 ;;
    gat_prof)
      run gat_prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/gat_prof" -o run --output-format csv -- \
          python3 benchmarks/bench_gat.py --epochs 5 --warmup 2 --eval-epochs 0 ;;
    learn_deepwalk_dist)
      # learning evidence through the sharded exchange (bf16 rows/grads on the wire)
      run bench_deepwalk_dist 900 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29535 benchmarks/bench_deepwalk.py --mode static --force-dist ;;
    learn_deepwalk)
      run bench_deepwalk 900 python -u benchmarks/bench_deepwalk.py ;;
    deepwalk_modes)
      for m in dynamic static graph; do
        run "deepwalk_$m" 600 python -u benchmarks/bench_deepwalk.py --eval-nodes 0 --mode $m || exit $?
        run "deepwalk_${m}_dist" 600 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 1 \
          --master-addr 127.0.0.1 --master-port 29531 benchmarks/bench_deepwalk.py --eval-nodes 0 --mode $m \
          --force-dist || exit $?
      done ;;
    dw_probe)
      RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 \
        run dw_probe_eager 120 python -u -X faulthandler tools/dw_overlap_probe.py eager || exit $?
      RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29562 \
        run dw_probe_graph 120 python -u -X faulthandler tools/dw_overlap_probe.py graph ;;
    deepwalk_overlap)
      # graph mode: no-comm step vs one-rank all-to-all path with 1 and 2 micro-batches
      run deepwalk_graph 600 python -u benchmarks/bench_deepwalk.py --eval-nodes 0 --mode graph || exit $?
      for mb in 1 2; do
        run "deepwalk_graph_dist_mb$mb" 600 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 1 \
          --master-addr 127.0.0.1 --master-port 2953$mb benchmarks/bench_deepwalk.py --eval-nodes 0 --mode graph \
          --force-dist --micro-batches $mb || exit $?
      done ;;
    deepwalk_prof)
      run deepwalk_prof_local 600 rocprofv3 --kernel-trace --stats -d "$OUT/dw_prof_local" -o run --output-format csv -- \
          python3 benchmarks/bench_deepwalk.py --eval-nodes 0 --mode static --steps 20 || exit $?
      RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 \
        run deepwalk_prof_dist 600 rocprofv3 --kernel-trace --stats -d "$OUT/dw_prof_dist" -o run --output-format csv -- \
          python3 benchmarks/bench_deepwalk.py --eval-nodes 0 --mode static --steps 20 --force-dist ;;
    rkb_sweep)
      for v in ${RKB_VALUES:-6 4}; do
        touch euler_amd/csrc/hip/sage_tree.hip
        EULER_AMD_HIP_FLAGS="-DTR_RKB=$v" python -m euler_amd._build > "$OUT/build_rkb$v.log" 2>&1 || exit 4
        run "tree_kernels_rkb$v" 300 python -u tools/tree_kernels.py || exit $?
      done ;;
    bpf_sweep)
      for v in ${BPF_VALUES:-2 4}; do
        touch euler_amd/csrc/hip/sage_tree.hip
        EULER_AMD_HIP_FLAGS="-DTR_FWD_BPF=$v" python -m euler_amd._build > "$OUT/build_bpf$v.log" 2>&1 || exit 4
        run "tree_kernels_bpf$v" 300 python -u tools/tree_kernels.py || exit $?
      done ;;
    variants)
      # VARIANTS="-DA=1|-DB=2": rebuild the HIP extension with each flag set, time the
      # step launches, and (VARIANT_TESTS=1) run the tree-step oracle tests on that build
      IFS='|' read -ra VL <<< "${VARIANTS:-}"
      i=0
      for v in "${VL[@]}"; do
        i=$((i+1))
        touch euler_amd/csrc/hip/sage_tree.hip
        EULER_AMD_HIP_FLAGS="$v" python -m euler_amd._build > "$OUT/build_variant$i.log" 2>&1 || exit 4
        echo "variant $i: $v" > "$OUT/variant$i.txt"
        if [ "${VARIANT_TESTS:-0}" = 1 ]; then
          run "variant${i}_tests" 300 python -u -m pytest tests/test_sage_trainer.py -m gpu -x -q --timeout 120 \
            --timeout-method thread -p no:cacheprovider -k "oracle or replay or trajectory" || exit $?
        fi
        run "tree_kernels_variant$i" 300 python -u tools/tree_kernels.py || exit $?
      done ;;
    kernels_full)
      run tree_kernels_full 300 python -u tools/tree_kernels.py --num-nodes 100000000 ;;
    kernels_sizes)
      for nn in 2000000 100000000; do
        run "tree_kernels_n$nn" 300 python -u tools/tree_kernels.py --num-nodes $nn
      done ;;
    xgmi)
      # two-shot xGMI all-reduce: 2 ranks sharing the box's GPU (protocol + capture), the
      # headline step through it on 2 ranks (rehearsal), and its one-rank cost next to RCCL's
      run xgmi_test 300 python -u -m pytest tests/test_xgmi.py -x -v --timeout 120 --timeout-method thread \
        -p no:cacheprovider || exit $?
      run bench_shared_gpu_2r 600 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29571 bench.py --shared-gpu --num-nodes 2000000 --steps 100 \
        --warmup 10 || exit $?
      for gs in xgmi rccl; do
        run "bench_force_dist_$gs" 600 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 1 \
          --master-addr 127.0.0.1 --master-port 29572 bench.py --force-dist --grad-sync $gs --steps 200 \
          --warmup 20 || exit $?
      done ;;
    xgmi_bench)
      run xgmi_test 300 python -u -m pytest tests/test_xgmi.py -x -v --timeout 120 --timeout-method thread \
        -p no:cacheprovider || exit $?
      for nb in "" 4 16 32 64; do
        EULER_AMD_XAR_BLOCKS=$nb RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=2958${#nb} \
          run "xgmi_bench_1r_b${nb:-auto}" 120 python -u tools/xgmi_bench.py --numel 278784 1048576 || exit $?
      done
      run xgmi_bench_2r_shared 120 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29589 tools/xgmi_bench.py --shared-gpu || exit $?
      for gs in xgmi tune; do
        run "bench_force_dist_$gs" 600 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 1 \
          --master-addr 127.0.0.1 --master-port 29572 bench.py --force-dist --grad-sync $gs --steps 200 \
          --warmup 20 || exit $?
      done
      run bench_shared_gpu_2r 600 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29571 bench.py --shared-gpu --num-nodes 2000000 --steps 100 \
        --warmup 10 ;;
    xgmi_variants)
      # XAR_VARIANTS="|-DXAR_FENCE_ALL=1|-DXAR_UNCACHED_DATA=1": rebuild xgmi_ar.hip per flag set,
      # one-rank call times + the 2-ranks-on-one-GPU test
      IFS='|' read -ra VL <<< "${XAR_VARIANTS:-}"
      i=0
      for v in "${VL[@]}"; do
        i=$((i+1))
        touch euler_amd/csrc/hip/xgmi_ar.hip
        EULER_AMD_HIP_FLAGS="$v" python -m euler_amd._build > "$OUT/build_xar_variant$i.log" 2>&1 || exit 4
        echo "variant $i: $v" > "$OUT/xar_variant$i.txt"
        RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=2959$i \
          run "xgmi_bench_1r_variant$i" 120 python -u tools/xgmi_bench.py --numel 278784 1048576 || exit $?
        run "xgmi_test_variant$i" 300 python -u -m pytest tests/test_xgmi.py -x -q --timeout 120 \
          --timeout-method thread -p no:cacheprovider || exit $?
      done
      touch euler_amd/csrc/hip/xgmi_ar.hip
      python -m euler_amd._build > "$OUT/build_xar_default.log" 2>&1 || exit 4 ;;
    spg_sweep)
      # complete steps per hipGraph replay (bench.py --steps-per-graph)
      for k in ${SPG_VALUES:-4 8 16}; do
        run "bench_spg$k" 300 python -u bench.py --steps 1000 --warmup 20 --steps-per-graph $k || exit $?
      done ;;
    xgmi_prof)
      # kernel table of the xGMI all-reduce (one rank: the launch, staging, both barriers,
      # reduce) and of RCCL's one-rank all_reduce, hipGraph-replayed
      RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29597 \
        run xgmi_prof 300 rocprofv3 --kernel-trace --stats -d "$OUT/xgmi_prof" -o run --output-format csv -- \
          python3 tools/xgmi_bench.py --numel 278784 --calls 100 --reps 3 ;;
    bench_default)
      # exactly the driver's 1-GPU bench command shape (bench.py defaults)
      run bench_default 600 python -u bench.py --gpus 1 --steps 200 --warmup 20 ;;
    smoke)
      run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench_small)
      run bench_small 300 python bench.py --num-nodes 2000000 --steps 100 --warmup 10 --log ;;
    bench_full)
      run bench_full 600 python bench.py --steps 200 --warmup 20 --log ;;
    dist_bench)
      # the multi-GPU code path (process group, bucketed all-reduce captured in the step) on one rank
      for cfg in ${DIST_CFGS:-fp32:1 fp32:2}; do
        dt=${cfg%%:*}; nb=${cfg##*:}
        run "bench_dist_${dt}_b$nb" 600 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 1 \
          --master-addr 127.0.0.1 --master-port 29541 bench.py --force-dist --grad-reduce-dtype $dt \
          --grad-buckets $nb --steps 200 --warmup 20 || exit $?
      done ;;
    trace_bench)
      # whole-step timeline of the bench (dp1, then the one-rank process-group path)
      run trace_bench 300 rocprofv3 --kernel-trace -d "$OUT/trace_bench" -o run --output-format csv -- \
          python3 bench.py --num-nodes 10000000 --steps 30 --warmup 5 && \
      python tools/trace_gaps.py "$OUT/trace_bench/run_kernel_trace.csv" --last 2 > "$OUT/trace_bench_gaps.txt" 2>&1
      RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 \
        run trace_dist 300 rocprofv3 --kernel-trace -d "$OUT/trace_dist" -o run --output-format csv -- \
          python3 bench.py --num-nodes 10000000 --steps 30 --warmup 5 --force-dist && \
      python tools/trace_gaps.py "$OUT/trace_dist/run_kernel_trace.csv" --last 2 > "$OUT/trace_dist_gaps.txt" 2>&1
      cat "$OUT/trace_bench_gaps.txt" "$OUT/trace_dist_gaps.txt" ;;
    unsup)
      run bench_unsup 900 python -u benchmarks/bench_unsup_sage.py ${UNSUP_ARGS:-} ;;
    unsup_ab)
      for m in mixed torch gemm; do
        EULER_AMD_TOWER_GEMM=$m run "bench_unsup_$m" 600 python -u benchmarks/bench_unsup_sage.py --steps 1000 || exit $?
      done ;;
    unsup_prof)
      run unsup_prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/unsup_prof" -o run --output-format csv -- \
          python3 benchmarks/bench_unsup_sage.py --steps 100 --eval-pairs 2000 ;;
    pmc_lds)
      PASSES="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE" \
        run pmc_lds 300 bash tools/pmc_passes.sh lds "$PWD/tools/tree_kernels.py" --reps 10 ;;
    bench_fp32)
      run bench_fp32 600 python bench.py --steps 200 --warmup 20 --feature-dtype fp32 ;;
    sweep_batch)
      for b in 1024 2048 4096 8192 16384; do
        run "bench_b$b" 600 python bench.py --steps 100 --warmup 10 --batch-size "$b"
      done ;;
    prof)
      run rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
          python3 bench.py --num-nodes 10000000 --steps 100 --warmup 5 ;;
    prof_full)
      run rocprof_full 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof_full" -o run --output-format csv -- \
          python3 bench.py --steps 100 --warmup 5 ;;
    *)
      echo "unknown step $st"; exit 2 ;;
  esac
done
echo "=== done"
