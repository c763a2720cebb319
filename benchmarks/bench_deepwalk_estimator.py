#!/usr/bin/env python3
"""BASELINE config 4 through the PRODUCT: ``NodeEstimator(device_graph=True)`` trains a
``DeepWalk(..., sharded=True)`` model (128-d target + context tables) on a 100M-node
synthetic graph, checkpoints it as per-rank shard files and resumes from them.

This is the estimator path, not the bare trainer of ``bench_deepwalk.py``: the model's
two ``ShardedEmbedding`` tables become views of the DeepWalk trainer's row-sharded table
(models/deepwalk_step.py DeepWalkEstimatorTrainer), so the 102 GB of tables exist once;
every log line carries samples/s (walks/s), peak HBM and peak host RSS; the checkpoint is
this rank's rows + sparse-optimizer slots in ``.npy`` files next to
``model.ckpt-<step>[-rank<r>].pt`` (parallel/shard_io.py) — no whole-table assembly on
save or restore, at any world size.

Phases (one process each, so the resume really starts from the files):
  --phase train   : build graph + model, train ``--steps`` steps, save the checkpoint
  --phase resume  : build graph + model, restore, train ``--resume-steps`` more steps
                    (no final save: a second 100M-node checkpoint would not fit the box)

The graph comes from ``params["device_graph_factory"]`` (``DeviceGraph.synthetic``,
generated in HBM; there is no engine behind it).  Usage:
    python benchmarks/bench_deepwalk_estimator.py --phase train --model-dir /dev/shm/dw
    python benchmarks/bench_deepwalk_estimator.py --phase resume --model-dir /dev/shm/dw
    python benchmarks/bench_deepwalk_estimator.py --gpus 2 ...   (one rank per GPU)
"""
from __future__ import annotations

import os

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL (before torch)

import argparse  # noqa: E402
import json  # noqa: E402
import logging  # noqa: E402
import sys  # noqa: E402
import time  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def parse(argv=None):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--phase", choices=["train", "resume"], default="train")
    p.add_argument("--gpus", type=int, default=1, help="ranks (self-spawned, one per GPU) when not under torchrun")
    p.add_argument("--num-nodes", type=int, default=100_000_000)
    p.add_argument("--avg-degree", type=float, default=10.0)
    p.add_argument("--max-degree", type=int, default=1024)
    p.add_argument("--dim", type=int, default=128)
    p.add_argument("--batch", type=int, default=16384, help="walks per rank per step")
    p.add_argument("--steps", type=int, default=1000)
    p.add_argument("--resume-steps", type=int, default=200)
    p.add_argument("--log-steps", type=int, default=100)
    p.add_argument("--steps-per-graph", type=int, default=8)
    p.add_argument("--optimizer", choices=["auto", "adam", "adagrad", "sgd"], default="auto")
    p.add_argument("--lr", type=float, default=0.01)
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--model-dir", default="/dev/shm/euler_dw_ckpt")
    p.add_argument("--device", default="cuda")
    p.add_argument("--no-save", action="store_true", help="train phase: skip the checkpoint")
    return p.parse_args(argv)


def main(argv=None):
    args = parse(argv)
    from euler_amd.parallel.launch import LAUNCHED_ENV, spawn_local

    if args.gpus > 1 and "RANK" not in os.environ and LAUNCHED_ENV not in os.environ:
        # one child process per GPU (parallel/launch.py); this parent never touches the GPU
        raise SystemExit(spawn_local(args.gpus, sys.argv[1:], script=os.path.abspath(__file__)))
    import torch

    from euler_amd import models as Z
    from euler_amd.estimator import NodeEstimator
    from euler_amd.graph.device_graph import DeviceGraph
    from euler_amd.parallel import dp
    from euler_amd.parallel.sparse_table import ShardedTable

    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(message)s")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device(args.device, local) if args.device == "cuda" else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    dp.init_distributed(backend="nccl" if dev.type == "cuda" else "gloo", device=dev)
    rank = dp.rank()
    if args.optimizer == "auto":
        # Adam keeps 2 slots per row: 2 x 100M x 128 fp32 tables + slots = 286 GiB, more
        # than one GPU holds; Adagrad's single slot fits (bench_deepwalk.py's rule)
        rows = (args.num_nodes + 1 + world - 1) // world
        need = 2 * rows * ShardedTable.bytes_per_row(args.dim, "adam")
        free = torch.cuda.mem_get_info(dev)[0] if dev.type == "cuda" else need * 2
        args.optimizer = "adam" if need < 0.75 * free else "adagrad"

    def factory(r, device):
        return DeviceGraph.synthetic(args.num_nodes, args.avg_degree, args.max_degree, seed=args.seed, device=device)

    t0 = time.time()
    torch.manual_seed(args.seed)
    # the tables are allocated and initialised straight in HBM (a 100M x 128 table pair is
    # 102 GB: no host copy), then adopted by the trainer as views
    with torch.device(dev):
        model = Z.DeepWalk(-1, -1, args.num_nodes - 1, args.dim, walk_len=3, num_negs=5, sharded=True)
    total = args.steps + (args.resume_steps if args.phase == "resume" else 0)
    params = {"model_dir": args.model_dir, "batch_size": args.batch, "total_step": total,
              "optimizer": args.optimizer, "learning_rate": args.lr, "log_steps": args.log_steps,
              "device": str(dev), "device_graph": True, "device_graph_factory": factory, "seed": args.seed,
              "steps_per_graph": args.steps_per_graph, "keep_checkpoint_max": 1,
              "save_final_checkpoint": args.phase == "train" and not args.no_save}
    est = NodeEstimator(model, params)
    setup = time.time() - t0
    t1 = time.time()
    last = est.train()
    wall = time.time() - t1
    tr = est.device_trainer
    pairs_per_walk = tr.inner.pairs_per_walk
    ck = [f for f in os.listdir(args.model_dir)] if os.path.isdir(args.model_dir) else []
    ck_bytes = sum(os.path.getsize(os.path.join(args.model_dir, f)) for f in ck)
    out = {
        "metric": "DeepWalk 128-d through NodeEstimator(device_graph=True), 100M-node synthetic graph",
        "phase": args.phase, "n_gpus": world, "num_nodes": args.num_nodes, "dim": args.dim,
        "optimizer": args.optimizer, "walks_per_rank_step": args.batch, "pairs_per_walk": pairs_per_walk,
        "steps_total": est.global_step, "restored_from_step": args.steps if args.phase == "resume" else 0,
        "last_log": last, "pairs_per_sec_last_interval": round(last.get("samples_per_sec", 0.0) * pairs_per_walk, 1),
        "setup_s": round(setup, 1), "train_wall_s_incl_capture_and_ckpt": round(wall, 1),
        "model_tables_are_trainer_views": bool(tr._bound),
        "checkpoint_files": len(ck), "checkpoint_gib": round(ck_bytes / 2 ** 30, 2),
        "tables_plus_slots_gib_per_rank": round(tr.inner.table.nbytes() / 2 ** 30, 1),
        "data": "synthetic power-law graph (DeviceGraph.synthetic), random-init tables",
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    dp.barrier()


if __name__ == "__main__":
    main()
