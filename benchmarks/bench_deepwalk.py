#!/usr/bin/env python3
"""BASELINE config 4: DeepWalk 128-d embeddings on a 100M-node graph, data parallel over
N GPUs with the embedding tables row-sharded across the ranks (RCCL all-to-all over
xGMI for ids, rows and row gradients).

Per rank and step: ``--batch`` random walks (walk_len 3, p = q = 1) on the GPU-resident
graph, skip-gram pairs with window 1/1 (6 per walk), 5 negatives per pair, fused
sigmoid-CE forward/backward, row-sparse Adam on the owners' shards (reference
examples/deepwalk: walk_len 3, window 1/1, 5 negatives, Adam; embedding_dim 128 per
BASELINE config 4).  Nothing is skipped inside the timed region.

Learning evidence (after the timed run, untimed, tables of the timed run freed): the same
trainer on a 1M-node planted-community graph (dataset/synthetic.py community_graph: 90 %
of a node's edges stay in its community) with 100K edges held out; link-prediction AUC
of held-out edges vs random pairs (cosine of target embeddings) at init and during
training goes into the JSON.

Usage:  python benchmarks/bench_deepwalk.py [--steps K] [--warmup W] [--gpus N]
        torchrun --nproc-per-node N benchmarks/bench_deepwalk.py   (one rank per GPU)
``--gpus N`` without torchrun starts N ranks itself (parallel/launch.py maybe_spawn).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# dmabuf IPC (the only mode the host driver supports): RCCL fails without it; set before
# torch loads HIP, here as in bench.py and parallel/launch.py's children
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def link_prediction_eval(args, dev):
    """DeepWalk on a planted-community graph; AUC of held-out edges vs random pairs."""
    import numpy as np

    from euler_amd.dataset.synthetic import auc, community_graph
    from euler_amd.graph.device_graph import DeviceGraph
    from euler_amd.models.deepwalk_step import DeepWalkTrainer

    N = args.eval_nodes
    src, dst, _ = community_graph(N, max(2, N // 1000), args.avg_degree, 0.9, seed=args.seed)
    gen = torch.Generator().manual_seed(args.seed + 5)
    perm = torch.randperm(src.numel(), generator=gen)
    n_hold = min(100_000, src.numel() // 10)
    hold, keep = perm[:n_hold], perm[n_hold:]
    s, d = src[keep], dst[keep]
    o = torch.argsort(s, stable=True)
    s, d = s[o], d[o]
    indptr = torch.zeros(N + 1, dtype=torch.int64)
    indptr[1:] = torch.cumsum(torch.bincount(s, minlength=N), 0)
    g = DeviceGraph.from_csr(indptr.numpy(), d.int().numpy(), np.ones(d.numel(), np.float32), seed=args.seed,
                             device=dev)
    # same exchange path as the timed run (--force-dist / --mode / --wire-dtype)
    tr = DeepWalkTrainer(g, N, args.dim, args.walk_len, 1, 1, args.num_negs, args.batch, args.eval_lr, "adam",
                         seed=args.seed, force_comm=args.force_dist, static=args.mode != "dynamic",
                         wire_dtype=args.wire_dtype, micro_batches=args.micro_batches)
    pu, pv = src[hold].to(dev), dst[hold].to(dev)
    nu = torch.randint(0, N, (n_hold,), generator=gen).to(dev)
    nv = torch.randint(0, N, (n_hold,), generator=gen).to(dev)

    def score():
        e = torch.nn.functional.normalize(tr.embedding(torch.arange(N, device=dev)), dim=-1)
        return round(auc((e[pu] * e[pv]).sum(-1).cpu(), (e[nu] * e[nv]).sum(-1).cpu()), 4)

    curve = {0: score()}
    for i in range(1, args.eval_steps + 1):
        tr.step()
        if i % max(1, args.eval_steps // 4) == 0 or i == args.eval_steps:
            curve[i] = score()
    return {"nodes": N, "edges_train": int(keep.numel()), "heldout_edges": n_hold, "lr": args.eval_lr,
            "optimizer": "adam", "auc_by_step": curve, "chance_auc": 0.5, "final_loss": round(float(tr.loss), 4)}


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--gpus", type=int, default=None, help="ranks, one per GPU (default: WORLD_SIZE or 1)")
    p.add_argument("--shared-gpu", action="store_true",
                   help="rehearsal: every rank on GPU 0 over gloo (the all-to-alls staged through host memory, "
                        "eager steps); RCCL needs one GPU per rank")
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--num-nodes", type=int, default=100_000_000)
    p.add_argument("--avg-degree", type=float, default=10.0)
    p.add_argument("--max-degree", type=int, default=1024)
    p.add_argument("--dim", type=int, default=128)
    p.add_argument("--batch", type=int, default=16384, help="walks per GPU per step")
    p.add_argument("--walk-len", type=int, default=3)
    p.add_argument("--num-negs", type=int, default=5)
    p.add_argument("--optimizer", choices=["auto", "adam", "adagrad", "sgd"], default="auto")
    p.add_argument("--lr", type=float, default=0.01)
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--force-dist", action="store_true",
                   help="process group + all-to-all path even with one rank (validates the N>1 path)")
    p.add_argument("--wire-dtype", choices=["bf16", "fp32"], default="bf16",
                   help="dtype of the row / gradient all-to-alls (the table and its update stay fp32)")
    p.add_argument("--micro-batches", type=int, choices=[1, 2], default=1,
                   help="static/graph modes with collectives: 2 = two micro-batches per step, each one's "
                        "all-to-alls on a comm stream under the other's compute")
    p.add_argument("--mode", choices=["graph", "static", "dynamic"], default="graph",
                   help="graph: fixed-capacity step captured in one hipGraph and replayed; static: the same "
                        "step eager; dynamic: exact-size step (host-read unique counts / all-to-all splits)")
    p.add_argument("--eval-nodes", type=int, default=1_000_000, help="0: skip the learning-evidence run")
    p.add_argument("--eval-steps", type=int, default=3000)
    p.add_argument("--eval-lr", type=float, default=0.05)
    args = p.parse_args(argv)
    from euler_amd.parallel.launch import maybe_spawn, require_gpu

    rc = maybe_spawn(args.gpus, sys.argv[1:] if argv is None else argv, __file__)
    if rc is not None:
        return rc
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.shared_gpu:
        dev = torch.device("cuda", 0)
        if args.mode == "graph":
            args.mode = "static"  # gloo collectives are not capturable: the same static step, eager
    else:
        require_gpu(local_rank, world, "bench_deepwalk.py (or --shared-gpu)")
        dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    dist_on = world > 1 or args.force_dist
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.shared_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    from euler_amd.graph.device_graph import DeviceGraph
    from euler_amd.models.deepwalk_step import DeepWalkTrainer
    from euler_amd.parallel.sparse_table import ShardedTable

    if args.optimizer == "auto":
        # Adam keeps 2 slots per row: two 100M x 128 fp32 tables + slots need 286 GiB, more
        # than one GPU holds next to the graph; there (world 1) Adagrad's single slot fits
        rows_per_rank = (args.num_nodes + 1 + world - 1) // world
        need = 2 * rows_per_rank * ShardedTable.bytes_per_row(args.dim, "adam")
        free = torch.cuda.mem_get_info(dev)[0]
        args.optimizer = "adam" if need < 0.8 * free else "adagrad"
    t0 = time.time()
    g = DeviceGraph.synthetic(args.num_nodes, args.avg_degree, args.max_degree, seed=args.seed, device=dev)
    g.manual_seed(args.seed * 7919 + rank)
    tr = DeepWalkTrainer(g, args.num_nodes, args.dim, args.walk_len, 1, 1, args.num_negs, args.batch, args.lr,
                         args.optimizer, seed=args.seed, force_comm=args.force_dist, static=args.mode != "dynamic",
                         wire_dtype=args.wire_dtype, micro_batches=args.micro_batches)
    torch.cuda.synchronize()
    if rank == 0:
        gib = tr.table.nbytes() / 2 ** 30
        print(f"[bench_deepwalk] {args.num_nodes} nodes, {g.num_edges} edges, tables+slots {gib:.1f} GiB/rank, "
              f"setup {time.time() - t0:.1f}s", file=sys.stderr, flush=True)

    if args.mode == "graph":
        tr.capture(warm=max(1, args.warmup))  # warm-up steps run inside, then one step is captured
    else:
        for _ in range(args.warmup):
            tr.step()
    torch.cuda.synchronize()
    first = float(tr.warm_loss if args.mode == "graph" else tr.loss)
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        tr.step()
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    el = time.perf_counter() - t1
    elt = torch.tensor([el], dtype=torch.float64, device=dev)
    if dist_on:
        dist.all_reduce(elt, op=dist.ReduceOp.MAX)
    el = float(elt.item())
    pairs = tr.pairs_per_step() * world * args.steps
    tr.table.check_overflow()
    pairs_per_step, table_comm, loss_last = tr.pairs_per_step(), bool(tr.table.comm), float(tr.loss)
    peak = torch.cuda.max_memory_allocated() / 2 ** 30
    tr.release()
    del tr, g
    torch.cuda.empty_cache()
    heldout = link_prediction_eval(args, dev) if args.eval_nodes > 0 else None
    if rank == 0:
        print(json.dumps({
            "metric": "train pairs/sec (whole node), DeepWalk 128-d skip-gram on 100M-node synthetic graph",
            "value": round(pairs / el, 1),
            "unit": "pairs/s",
            "n_gpus": 1 if args.shared_gpu else world,
            "ranks": world,
            "shared_gpu_rehearsal": bool(args.shared_gpu) or None,
            "parallelism": f"dp{world}+sharded-emb",
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el * 1e3 / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (power-law random graph, random-init tables)",
            "config": {"model": f"DeepWalk (walk_len 3, window 1/1, 5 negs, row-sparse {args.optimizer})",
                       "exchange_dtype": args.wire_dtype,
                       "num_nodes": args.num_nodes, "dim": args.dim, "walks_per_gpu": args.batch,
                       "pairs_per_gpu_step": pairs_per_step, "parallelism": f"dp{world}+sharded-emb",
                       "all_to_all": table_comm, "step_mode": args.mode, "micro_batches": args.micro_batches,
                       "optimizer_schedule": ("one sparse update per step" if args.micro_batches == 1 else
                                              "two half-batch sparse updates per step (each micro-batch applies its "
                                              "own update; not the same optimizer step as one full batch)"),
                       "loss_first_last": [round(first, 4), round(loss_last, 4)],
                       "peak_mem_gib": round(peak, 1), "heldout_link_prediction": heldout},
        }), flush=True)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    raise SystemExit(main())
