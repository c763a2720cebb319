#!/usr/bin/env python3
"""Headline benchmark: GraphSAGE 2-hop training throughput (samples/sec, whole node).

BASELINE.json metric: "train samples/sec (whole node), GraphSAGE 2-hop on 100M-node
synthetic graph".  Config (defaults): 100M-node power-law synthetic graph (avg degree
10, ~1B weighted edges), 128-d bf16 node features, 64 classes, supervised GraphSAGE
(reference examples/graphsage: SAGEConv x2 + fc + out_fc, sigmoid CE, Adam), fanouts
[25, 10], 1024 roots per GPU per step (weak scaling), hidden 256.

One process per GPU (torchrun); every rank holds the whole graph + feature table
resident in its own HBM and samples on the GPU; dense gradients are synchronised
with one flat RCCL all-reduce per step.  One "step" = sample roots + 2 hops of
neighbor sampling + forward + backward + all-reduce + optimizer update; nothing is
skipped inside the timed region.  On one GPU the whole step is a single hipGraph
replay; with N>1 the forward/backward and the optimizer are two graphs around an
eager all-reduce.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [...]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--num-nodes", type=int, default=100_000_000)
    p.add_argument("--avg-degree", type=float, default=10.0)
    p.add_argument("--max-degree", type=int, default=1024)
    p.add_argument("--batch-size", type=int, default=1024, help="roots per GPU per step")
    p.add_argument("--fanouts", type=str, default="25,10")
    p.add_argument("--feature-dim", type=int, default=128)
    p.add_argument("--hidden-dim", type=int, default=256)
    p.add_argument("--label-dim", type=int, default=64)
    p.add_argument("--lr", type=float, default=0.01)
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--no-graph", action="store_true", help="eager steps instead of hipGraph replay")
    p.add_argument("--impl", choices=["fused", "autograd"], default="fused",
                   help="fused = the 10-kernel gfx950 training step (models/sage_step.py); "
                        "autograd = fused SAGE layers under torch autograd (models/fused_sage.py)")
    p.add_argument("--log", action="store_true")
    p.add_argument("--force-dist", action="store_true",
                   help="take the multi-GPU code path (process group, graph segments around the gradient "
                        "all-reduce) even with one rank: validates that path on a single GPU")
    p.add_argument("--grad-sync", choices=["graph", "single", "overlap"], default="graph",
                   help="N>1: graph = the RCCL all-reduce is captured into the step's hipGraph (one replay per "
                        "step, no host launches in between); single = eager all-reduce between two graph "
                        "segments; overlap = fused impl, all-reduce W1/fc/out grads while dW0 is computed")
    return p.parse_args(argv)


def _cpu_baseline():
    """BASELINE.md publishes no reference number; its prescribed comparison point is the
    reference-equivalent CPU path measured on the MI355X host (euler_amd/tools/cpu_baseline.py,
    result committed in profiles/cpu_baseline.json)."""
    path = os.path.join(ROOT, "profiles", "cpu_baseline.json")
    try:
        with open(path) as f:
            b = json.loads(f.readline())
        note = (f"profiles/cpu_baseline.json: reference-equivalent CPU path, {b['value']} samples/s "
                f"({b.get('threads')} host threads, {b['config']['num_nodes']} nodes)")
        return float(b["value"]), note
    except (OSError, ValueError, KeyError):
        return None, None


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def main(argv=None):
    args = parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist_on = world > 1 or args.force_dist
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU (run through gpurun on an MI355X)")
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)

    from euler_amd.graph.device_graph import DeviceGraph
    from euler_amd.models.fused_sage import FusedSupervisedGraphSage, synthetic_features, synthetic_labels
    from euler_amd.parallel.flat import FlatOptimizer, FlatParams

    fanouts = [int(x) for x in args.fanouts.split(",")]
    B = args.batch_size
    t0 = time.time()
    graph = DeviceGraph.synthetic(args.num_nodes, args.avg_degree, args.max_degree, seed=args.seed, device=dev)
    graph.manual_seed(args.seed * 7919 + rank)  # different root/neighbor draws per rank
    feats = synthetic_features(args.num_nodes, args.feature_dim, args.seed + 1, dev)
    labels = synthetic_labels(feats, args.label_dim)
    torch.cuda.synchronize()
    if rank == 0:
        log(f"graph: {graph.num_rows} nodes, {graph.num_edges} edges, csr {graph.nbytes()/2**30:.2f} GiB, "
            f"features {feats.numel()*2/2**30:.2f} GiB, build {time.time()-t0:.1f}s")

    torch.manual_seed(args.seed)
    model = FusedSupervisedGraphSage(args.feature_dim, args.hidden_dim, args.label_dim, fanouts).to(dev)
    grad_scale = 1.0 / world
    if args.impl == "fused":
        from euler_amd.models.sage_step import FusedSageTrainer

        trainer = FusedSageTrainer(graph, feats, labels, B, fanouts, args.hidden_dim, args.label_dim, lr=args.lr,
                                   init_model=model)
        if dist_on:
            dist.broadcast(trainer.flat, 0)
            trainer.refresh_shadows()
        loss_buf = trainer.loss_out
        grad_buf = trainer.grad

        def fwd_bwd():
            trainer.forward_backward()

        def opt_step():
            trainer.optimizer_step(grad_scale=grad_scale)
    else:
        flat = FlatParams(model.parameters(), dev)
        if dist_on:
            dist.broadcast(flat.flat, 0)
        opt = FlatOptimizer(flat, "adam", args.lr)
        loss_buf = torch.zeros((), device=dev)
        grad_buf = flat.grad

        def fwd_bwd():
            graph.advance()
            roots = graph.sample_node(B, stream_id=1)
            levels, nbrs = model.sample(graph, roots)
            logits = model(feats, levels, nbrs)
            loss = model.loss(logits, labels[roots.long()])
            flat.zero_grad()
            loss.backward()
            loss_buf.copy_(loss.detach())

        def opt_step():
            opt.step(grad_scale=grad_scale)

    def allreduce():
        if dist_on:
            dist.all_reduce(grad_buf)

    # fused impl, N > 1: all-reduce the W1/fc/out_fc gradients (77 % of the bytes) on RCCL's
    # stream while the outer layer's dW0 is still being computed, then W0's
    overlap = (args.impl == "fused" and dist_on and args.grad_sync == "overlap" and not trainer.pipelined)

    def synced_step(head, outer, opt):
        head()
        w1 = dist.all_reduce(trainer.grad_bucket_head, async_op=True)
        outer()
        w2 = dist.all_reduce(trainer.grad_bucket_outer, async_op=True)
        w1.wait()  # stream-ordered: the optimizer kernels wait for both reductions
        w2.wait()
        opt()

    def eager_step():
        if overlap:
            synced_step(lambda: trainer.forward_backward("head"), lambda: trainer.forward_backward("outer"), opt_step)
        else:
            fwd_bwd()
            allreduce()
            opt_step()

    use_graph = not args.no_graph
    if use_graph:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                eager_step()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        if args.impl == "autograd":
            flat.rebind_grads()
        # the fused trainer double-buffers its samples (next step's roots/hops are drawn on a
        # side stream during this step): one captured graph per sample-set parity
        pipelined = args.impl == "fused" and trainer.pipelined
        parities = (0, 1) if pipelined else (0,)

        def parity():
            return trainer.parity if pipelined else 0

        def next_parity():
            if pipelined:
                trainer.advance_parity()

        captured = False
        if not dist_on or args.grad_sync == "graph":
            # one graph per step; with N > 1 the flat-gradient all-reduce is captured too
            # (RCCL kernels inside the hipGraph)
            try:
                g_all = {}
                for _ in parities:
                    p_ = parity()
                    g_all[p_] = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g_all[p_]):
                        fwd_bwd()
                        allreduce()
                        opt_step()
                # capture toggled the parity once per graph: back where the eager warmup left it
                captured = True
            except Exception as e:  # pragma: no cover - RCCL capture unsupported: graph segments
                if not dist_on:
                    raise
                log(f"all-reduce capture failed ({e!r}); falling back to --grad-sync single")
                args.grad_sync = "single"
                torch.cuda.synchronize()
                if pipelined:  # the failed capture toggled the parity
                    trainer.advance_parity()

        if captured:
            def step():
                g_all[parity()].replay()
                next_parity()
        elif overlap:
            g_head, g_outer, g_opt = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_head):
                trainer.forward_backward("head")
            with torch.cuda.graph(g_outer):
                trainer.forward_backward("outer")
            with torch.cuda.graph(g_opt):
                opt_step()

            def step():
                synced_step(g_head.replay, g_outer.replay, g_opt.replay)
        else:
            g_fb = {}
            for _ in parities:
                p_ = parity()
                g_fb[p_] = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g_fb[p_]):
                    fwd_bwd()
            g_opt = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_opt):
                opt_step()

            def step():
                g_fb[parity()].replay()
                next_parity()
                allreduce()
                g_opt.replay()
    else:
        step = eager_step

    for i in range(args.warmup):
        step()
    torch.cuda.synchronize()
    first_loss = float(loss_buf.item())

    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for i in range(args.steps):
        step()
        if args.log and rank == 0 and (i + 1) % 50 == 0:
            torch.cuda.synchronize()
            log(f"step {i+1} loss {float(loss_buf.item()):.4f}")
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if dist_on:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    last_loss = float(loss_buf.item())
    ms = elapsed * 1000.0 / max(args.steps, 1)
    value = world * B * args.steps / elapsed
    base_value, base_note = _cpu_baseline()
    if rank == 0:
        log(f"loss after warmup {first_loss:.4f} -> after timed steps {last_loss:.4f}")
        out = {
            "metric": "train samples/sec (whole node), GraphSAGE 2-hop on 100M-node synthetic graph",
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / base_value, 2) if base_value else None,
            "dtype": "bf16",
            "data": "synthetic (power-law random graph + random-normal features, random-init weights)",
            "config": {
                "model": "GraphSAGE supervised (2x SAGEConv mean + fc + out_fc, sigmoid CE, Adam)",
                "global_batch": B * world,
                "seq_len": None,
                "parallelism": f"dp{world}",
                "num_nodes": args.num_nodes,
                "num_edges": graph.num_edges,
                "fanouts": fanouts,
                "feature_dim": args.feature_dim,
                "hidden_dim": args.hidden_dim,
                "label_dim": args.label_dim,
                "hipgraph": use_graph,
                "grad_sync": ("overlap" if overlap else args.grad_sync) if dist_on else None,
                "impl": args.impl,
                "loss_first_last": [round(first_loss, 4), round(last_loss, 4)],
                "baseline": base_note,
            },
        }
        print(json.dumps(out), flush=True)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
