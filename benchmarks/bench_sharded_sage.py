#!/usr/bin/env python3
"""GraphSAGE on a graph row-sharded over the ranks (graph/sharded_graph.py,
models/sharded_sage.py): every GPU holds 1/W of the CSR, the features and the labels; each
step's tree is drawn across the ranks (owner-side neighbour draws over all-to-all), the
input features and the roots' labels come from their owners, then the fused tree step
(forward, head, backward, split-K dW, gradient all-reduce, Adam) runs as on a whole graph.

The headline shape by default (B = 1024 roots per GPU, fanouts 25 x 10, 128-d bf16
features, hidden 256, 64 classes, Adam) on a synthetic power-law graph generated in HBM.

    python benchmarks/bench_sharded_sage.py --gpus 1 --num-nodes 100000000
    python benchmarks/bench_sharded_sage.py --gpus 8 ...        (one rank per GPU, self-spawned)
    python benchmarks/bench_sharded_sage.py --model gcn ...     (2-layer GCN on full-neighbourhood
        blocks expanded by the rows' owners: ShardedDeviceGraph.full_neighbors + DeviceFullFlow)

Prints one JSON line (rank 0): whole-job samples/s, ms per step, per-GPU graph bytes.
Reference: tf_euler/python/dataflow/sage_dataflow.py:35-50 over remote_op.cc:60-146.
"""
from __future__ import annotations

import os

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL (before torch)

import argparse  # noqa: E402
import json  # noqa: E402
import sys  # noqa: E402
import time  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--num-nodes", type=int, default=100_000_000)
    p.add_argument("--avg-degree", type=float, default=10.0)
    p.add_argument("--batch", type=int, default=1024)
    p.add_argument("--fanouts", type=int, nargs="+", default=[25, 10])
    p.add_argument("--hidden", type=int, default=256)
    p.add_argument("--feature-dim", type=int, default=128)
    p.add_argument("--classes", type=int, default=64)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--model", choices=["sage", "gcn", "flow", "unsup"], default="sage",
                   help="sage: the fused tree step; gcn: GCNConv on full-neighbourhood blocks; flow: --conv on "
                        "the sampled flow's blocks (ShardedFlowTrainer); unsup: unsupervised GraphSAGE "
                        "(ShardedUnsupSageTrainer, --negs negatives per source)")
    p.add_argument("--negs", type=int, default=5)
    p.add_argument("--conv", default="gcn", help="the convolution of --model flow")
    p.add_argument("--graph", action="store_true", help="capture the step (sampling exchanges included) in a hipGraph")
    p.add_argument("--force-comm", action="store_true",
                   help="one rank: run every exchange through a 1-rank RCCL group (the W > 1 code path)")
    p.add_argument("--shared-gpu", action="store_true",
                   help="rehearsal: every rank on GPU 0 over gloo (exchanges and gradients through host memory, "
                        "eager steps); RCCL needs one GPU per rank")
    args = p.parse_args(argv)
    from euler_amd.parallel.launch import LAUNCHED_ENV, require_gpu, spawn_local

    if args.gpus > 1 and "RANK" not in os.environ and LAUNCHED_ENV not in os.environ:
        return spawn_local(args.gpus, sys.argv[1:], script=os.path.abspath(__file__))
    import torch
    import torch.distributed as dist

    from euler_amd.graph.sharded_graph import ShardedDeviceGraph
    from euler_amd.models.sharded_sage import ShardedSageTrainer
    from euler_amd.parallel import dp

    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.shared_gpu:
        dev = torch.device("cuda", 0)
        args.graph = False
    else:
        require_gpu(local, world, "bench_sharded_sage (or --shared-gpu)")
        dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    dp.init_distributed(backend="gloo" if args.shared_gpu else "nccl", device=dev)
    if args.force_comm and world == 1:
        import socket

        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    rank = dp.rank()
    t0 = time.time()
    gcn = args.model == "gcn"
    generic = args.model in ("gcn", "flow")  # ShardedFlowTrainer (multi-label sigmoid loss)
    unsup = args.model == "unsup"
    g = ShardedDeviceGraph.synthetic(args.num_nodes, args.avg_degree, feature_dim=args.feature_dim,
                                     num_classes=args.classes, multi_label=generic, seed=3, device=dev,
                                     force_comm=args.force_comm)
    dims = [args.hidden] * len(args.fanouts) + [args.hidden]
    if args.model == "unsup":
        from euler_amd.models.sharded_unsup import ShardedUnsupSageTrainer

        if len(args.fanouts) != 2:
            raise SystemExit("--model unsup trains 2-hop towers")
        tr = ShardedUnsupSageTrainer(g, args.batch, args.fanouts, [args.hidden, args.hidden, args.classes],
                                     num_negs=args.negs, learning_rate=0.01, init_seed=0)
    elif args.model == "flow":
        from euler_amd import models as Z
        from euler_amd.dataflow.device_flow import DeviceSageFlow
        from euler_amd.models.full_trainer import ShardedFlowTrainer

        torch.manual_seed(0)
        L = len(args.fanouts)
        m = Z.SupervisedGNN(args.conv, "sage", [args.hidden] * L + [args.classes], args.fanouts, [[0]] * L, "f",
                            args.feature_dim, "l", args.classes, max_id=args.num_nodes).to(dev)
        flow = DeviceSageFlow(g, [None] * L, args.fanouts, args.batch, True)
        tr = ShardedFlowTrainer(m, g, args.batch, flow, learning_rate=0.01)
    elif gcn:
        # the reference's SupervisedGCN shape: GCNConv layers on GCNDataFlow (full
        # neighbourhoods, self loops), sigmoid cross-entropy; one layer per --fanouts entry
        from euler_amd import models as Z
        from euler_amd.dataflow.device_flow import DeviceFullFlow
        from euler_amd.models.full_trainer import ShardedFlowTrainer

        torch.manual_seed(0)
        L = len(args.fanouts)
        m = Z.SupervisedGNN("gcn", "full", [args.hidden] * L + [args.classes], [1] * L, [[0]] * L, "f",
                            args.feature_dim, "l", args.classes, max_id=args.num_nodes).to(dev)
        flow = DeviceFullFlow(g, [1] * L, args.batch, True, "bounded")
        tr = ShardedFlowTrainer(m, g, args.batch, flow, learning_rate=0.01)
    else:
        tr = ShardedSageTrainer(g, args.batch, args.fanouts, dims, args.classes, learning_rate=0.01, init_seed=0)
    sync = None
    if world > 1:
        def sync(buf):
            if args.shared_gpu:  # gloo: through host memory
                host = buf.cpu()
                dist.all_reduce(host)
                buf.copy_(host)
            else:
                dist.all_reduce(buf)
            return 1.0 / world
    torch.cuda.synchronize()
    build_s = time.time() - t0
    if args.graph and (args.model == "sage" or tr.capturable()):  # gloo rehearsals run eagerly
        tr.capture(sync, warmup=args.warmup, steps=1)
        run = tr.replay_steps
    else:
        for _ in range(args.warmup):
            tr.step(sync)

        def run(n):
            for _ in range(n):
                tr.step(sync)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    el = float(el.item())
    g.check_overflow()
    if gcn:
        tr.flow.check()
    if rank == 0:
        print(json.dumps({
            "metric": {"gcn": "GCN", "sage": "GraphSAGE", "flow": f"{args.conv} (sampled flow)",
                       "unsup": "unsupervised GraphSAGE (sources; 1 + negs contexts each)"}[args.model] + " train samples/s on a row-sharded graph (whole job)",
            "value": round(args.batch * world * args.steps / el, 1), "unit": "samples/s",
            "n_gpus": 1 if args.shared_gpu else world, "ranks": world,
            "shared_gpu_rehearsal": bool(args.shared_gpu) or None, "exchanges": bool(g.comm),
            "ms_per_step": round(el * 1e3 / args.steps, 3), "steps": args.steps, "warmup": args.warmup,
            "loss": float(tr.loss.item()), "hipgraph": bool(tr._graphs) if args.model != "sage" else bool(args.graph),
            "build_s": round(build_s, 1), "flow_caps": tr.flow.caps if gcn else None,
            "graph_gib_per_gpu": round((g.nbytes() + g.features.shard.numel() * 2) / 2 ** 30, 2),
            "config": {"model": args.model, "num_nodes": args.num_nodes, "batch_per_gpu": args.batch,
                       "fanouts": None if gcn else args.fanouts, "conv": args.conv if args.model == "flow" else None,
                       "negs": args.negs if unsup else None, "layers": len(args.fanouts),
                       "hidden": args.hidden, "feature_dim": args.feature_dim, "classes": args.classes},
            "data": "synthetic power-law graph generated in HBM, random features / labels"}), flush=True)
    if world > 1:
        tr.release_graphs()
        dist.barrier()
    elif dist.is_initialized():
        tr.release_graphs()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
