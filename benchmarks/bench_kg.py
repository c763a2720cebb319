#!/usr/bin/env python3
"""BASELINE config 5: R-GCN encoder + TransE decoder on an FB15k-shaped knowledge graph
(relation-typed SpMM), data parallel over N GPUs.

Graph (FB15k shape, synthetic): 14,951 entities, 1,345 relations, 483,142 training
triples; relation ids drawn from a power law (a few relations dominate, like FB15k).
The triples follow a planted TransE structure (dataset/synthetic.py lattice_kg: entities
on a 3-D lattice, each relation a lattice translation), and 5,000 held-out triples are
ranked against all entities after training (raw tail ranking: MRR, hit@1/3/10, also at
initialisation) — the JSON carries learning evidence, not only throughput.

Model (reference examples/rgcn/rgcn.py:30-105 RelationConv + examples/TransX/transE.py):
  h = entity embedding [Ne, 128]
  2 x  h = act(RelationConv(h))     mean over in-edges of W_{rel(e)} h_src + self loop
                                    (rgcn.hip: relation-grouped MFMA GEMM, gather fused)
  TransE margin loss on a batch of training triples, 8 corruptions (front + tail), l2
  score on l2-normalised rows (embed.hip kg_fwd / kg_bwd), Adam.
Full-graph encoder every step (the graph is small; the relation transform over all
483K edges is the hot op).  DP: bucketed RCCL all-reduce of the dense gradients
overlapped with the backward (parallel/dp.py GradSync).

Usage: python benchmarks/bench_kg.py [--steps K] [--warmup W] [--gpus N];  or torchrun for N GPUs
(``--gpus N`` without torchrun starts N ranks itself: parallel/launch.py maybe_spawn).
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

from euler_amd.models.rgcn_kg_step import RgcnTransE, RgcnTransEStep  # noqa: E402
from euler_amd.ops import gnn_ops  # noqa: E402


def synthetic_kg(num_ent, num_rel, num_triples, seed, device, num_test=5000):
    from euler_amd.dataset.synthetic import lattice_kg

    train, test = lattice_kg(num_ent, num_rel, num_triples, num_test, seed=seed)
    return tuple(t.to(device) for t in train), tuple(t.to(device) for t in test)


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--gpus", type=int, default=None, help="ranks, one per GPU (default: WORLD_SIZE or 1)")
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--num-ent", type=int, default=14951)
    p.add_argument("--num-rel", type=int, default=1345)
    p.add_argument("--num-triples", type=int, default=483142)
    p.add_argument("--dim", type=int, default=128)
    p.add_argument("--batch", type=int, default=4096, help="training triples per GPU per step")
    p.add_argument("--num-negs", type=int, default=8)
    p.add_argument("--lr", type=float, default=1e-3)
    p.add_argument("--margin", type=float, default=1.0, help="TransE margin (reference run_transX --margin)")
    p.add_argument("--seed", type=int, default=3)
    p.add_argument("--layers", type=int, default=1,
                   help="R-GCN layers before the TransE decoder (0: TransE alone; the reference "
                        "examples/rgcn/run_rgcn.py:35 runs 1)")
    p.add_argument("--num-bases", type=int, default=0,
                   help="basis decomposition of the relation matrices (0: one full matrix per relation, as the "
                        "reference)")
    p.add_argument("--rel-wd", type=float, default=0.0,
                   help="weight decay on the relation matrices / bases only (a flat-optimizer decay range)")
    p.add_argument("--normalize", type=int, default=1,
                   help="1: l2-normalised rows in the score (reference transX.py:63-66); 0: raw rows")
    p.add_argument("--task", choices=["lattice", "cold", "types"], default="lattice",
                   help="cold: a fraction of the entities never appears in a loss triple (their edges stay in "
                        "the encoder graph); held-out triples with a cold head are ranked.  types: "
                        "dataset/synthetic.py typed_kg — rank the type hub of cold entities, whose type only "
                        "their neighbourhood carries")
    p.add_argument("--cold-frac", type=float, default=0.1)
    p.add_argument("--num-types", type=int, default=50, help="types task: type hubs (entities 0 .. n - 1)")
    p.add_argument("--type-negs", type=int, default=0,
                   help="types task: corrupt has_type triples with other type hubs (type-constrained negatives)")
    p.add_argument("--self-drop", type=float, default=0.0,
                   help="R-GCN self-loop dropout while training; cold entities (never in a loss triple) are then "
                        "placed by their neighbours alone at evaluation (inductive)")
    p.add_argument("--deterministic", action="store_true",
                   help="atomic-free, bit-reproducible fused step (occurrence rows + fixed-order sums)")
    p.add_argument("--no-graph", action="store_true", help="eager steps (default: one hipGraph per step)")
    p.add_argument("--fused", type=int, default=1,
                   help="1: the fused step (models/rgcn_kg_step.py: hand-written launches only, Philox draws in the "
                        "scoring kernel) where it applies; 0: the autograd step (torch.randint draws)")
    p.add_argument("--device", default="cuda", help="cpu: torch reference ops (exploration only, eager)")
    p.add_argument("--shared-gpu", action="store_true",
                   help="rehearsal: every rank on GPU 0 over gloo (gradients through host memory, eager steps); "
                        "RCCL needs one GPU per rank")
    p.add_argument("--eval-after", type=int, default=2000,
                   help="keep training (untimed) to this many steps, then rank the held-out triples")
    args = p.parse_args(argv)
    from euler_amd.parallel.launch import maybe_spawn, require_gpu

    rc = maybe_spawn(args.gpus, sys.argv[1:] if argv is None else argv, __file__)
    if rc is not None:
        return rc
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.device == "cpu":
        dev = torch.device("cpu")
        args.no_graph = True
    elif args.shared_gpu:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        args.no_graph = True  # gloo collectives are not capturable
    else:
        require_gpu(local_rank, world, "bench_kg.py (or --device cpu, or --shared-gpu)")
        dev = torch.device("cuda", local_rank)
        torch.cuda.set_device(dev)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if dev.type == "cuda" and not args.shared_gpu:
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    from euler_amd.parallel.flat import FlatOptimizer, FlatParams

    norm = bool(args.normalize)
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    if args.task == "types":
        from euler_amd.dataset.synthetic import typed_kg

        tr_, gr_, te_ = typed_kg(args.num_ent, args.num_rel, args.num_triples, num_types=args.num_types,
                                 cold_frac=args.cold_frac,
                                 seed=args.seed)
        (src, rel, dst), (gsrc, grel, gdst), (te_src, te_rel, te_dst) = (tuple(x.to(dev) for x in t)
                                                                         for t in (tr_, gr_, te_))
        # encoder graph: every link triple (cold ones too) + the warm type triples; the loss
        # samples the training triples only
        edge_index, edge_rel = torch.stack([gdst, gsrc]), grel
    else:
        (src, rel, dst), (te_src, te_rel, te_dst) = synthetic_kg(args.num_ent, args.num_rel, args.num_triples,
                                                                 args.seed, dev)
        # message direction src -> dst (row 0 = destination, row 1 = source); every training
        # triple is an encoder edge, also in the cold task
        edge_index, edge_rel = torch.stack([dst, src]), rel
    pool = torch.arange(src.numel(), device=dev)
    if args.task == "cold":
        g = torch.Generator().manual_seed(args.seed + 5)
        cold = torch.zeros(args.num_ent, dtype=torch.bool)
        cold[torch.randperm(args.num_ent, generator=g)[: int(args.cold_frac * args.num_ent)]] = True
        cold = cold.to(dev)
        pool = pool[~(cold[src] | cold[dst])]            # loss triples: warm head and tail
        keep = cold[te_src] & ~cold[te_dst]               # test: cold head, warm tail
        te_src, te_rel, te_dst = te_src[keep], te_rel[keep], te_dst[keep]
    torch.manual_seed(args.seed * 101 + rank)
    model = RgcnTransE(args.num_ent, args.num_rel, args.dim, layers=args.layers, margin=args.margin,
                       num_bases=args.num_bases).to(dev)
    model.norm = norm
    model.self_drop = float(args.self_drop)

    def batch():
        idx = pool[torch.randint(0, pool.numel(), (args.batch,), device=dev)]
        negs = torch.randint(0, args.num_ent, (args.batch, args.num_negs), device=dev)
        if args.type_negs and args.task == "types":
            # type-constrained corruption of has_type triples (relation 0): half the negatives
            # are other type hubs (entities 0 .. num_types - 1), so training separates the hubs;
            # half of them: uniform corruptions still teach that a non-hub is no type
            hub = torch.randint(0, args.num_types, (args.batch, args.num_negs), device=dev)
            half = (torch.arange(args.num_negs, device=dev) % 2 == 0).view(1, -1)
            negs = torch.where((rel[idx] == 0).view(-1, 1) & half, hub, negs)
        return src[idx], rel[idx], dst[idx], negs

    model(edge_index, edge_rel, *batch()).backward()  # materialise lazy layers before the optimizer
    if world > 1:
        from euler_amd.parallel.dp import broadcast_module

        broadcast_module(model)
    # every parameter (entity / relation tables, relation weights, self-loop fc) in ONE flat
    # fp32 buffer: one flat Adam launch (optim.hip), one all-reduce with data parallelism
    flat = FlatParams(model.parameters(), dev)
    for conv in model.convs:
        if conv.num_bases == 0:
            # the relation dW accumulates straight into its flat-grad view (no [R, D, D] temporary
            # + AccumulateGrad pass per layer; the flat grad is all-reduced as one buffer)
            gnn_ops.enable_grad_sink(conv.matrix, zeroed=True)  # opt.zero_grad() runs before every backward
    opt = FlatOptimizer(flat, "adam", args.lr)
    if args.rel_wd > 0 and model.convs:
        # decay on the relation transforms only: they are contiguous in the flat buffer
        rel_params = {id(p) for c in model.convs for p in ([c.matrix] if c.num_bases == 0 else [c.bases, c.coef])}
        spans = [(o, o + n) for p, (o, n) in zip(flat.params, flat.offsets) if id(p) in rel_params]
        lo, hi = min(a for a, _ in spans), max(b for _, b in spans)
        if hi - lo != sum(b - a for a, b in spans):
            raise SystemExit("relation parameters are not contiguous in the flat buffer")
        opt.set_decay_range(lo, hi, args.rel_wd)
    loss_buf = torch.zeros((), device=dev)

    def evaluate():
        from euler_amd.dataset.synthetic import rank_metrics, tail_ranks

        model.eval()
        if args.self_drop > 0 and args.task in ("types", "cold"):
            # inductive: the test heads' own embeddings never saw a loss triple
            keep = torch.ones(args.num_ent, dtype=torch.bool, device=dev)
            keep[te_src] = False
            model.self_keep = keep
        with torch.no_grad():
            h = model.encode(edge_index, edge_rel).float()
            if not bool(torch.isfinite(h).all()):
                bad = [n for n, p in model.named_parameters() if not bool(torch.isfinite(p).all())]
                print(f"[bench_kg] non-finite encoder output; non-finite parameters: {bad}", file=sys.stderr,
                      flush=True)
        model.self_keep = None
        model.train()
        m = rank_metrics(tail_ranks(h, model.rel, te_src, te_rel, te_dst, normalize=norm))
        out = {k: round(v, 4) for k, v in m.items()}
        if args.task == "types":
            # type prediction proper: the true hub ranked among the num_types hubs
            hubs = torch.arange(args.num_types, device=dev)
            mt = rank_metrics(tail_ranks(h, model.rel, te_src, te_rel, te_dst, normalize=norm, cands=hubs))
            out.update({"type_" + k: round(v, 4) for k, v in mt.items()})
        return out

    eval_init = evaluate()

    grad_sync, sync_name, sync_info = None, None, {}
    if world > 1:
        # xGMI two-shot peer-memory all-reduce or RCCL, whichever times faster on this node
        from euler_amd.parallel.xgmi import make_grad_sync

        grad_sync, sync_name, sync_info = make_grad_sync(flat.grad)
        sync_info.pop("xar", None)

    fused = None
    if args.fused and dev.type == "cuda" and not (args.type_negs and args.task == "types") and args.dim % 8 == 0:
        fused = RgcnTransEStep(model, flat, opt, edge_index, edge_rel, (src, rel, dst), pool, args.batch,
                               args.num_negs, seed=args.seed * 7919 + rank, grad_sync=grad_sync,
                               deterministic=args.deterministic)
        loss_buf = fused.loss

    def step_body():
        if fused is not None:
            fused.step()
            return
        opt.zero_grad()
        loss = model(edge_index, edge_rel, *batch())
        loss.backward()
        scale = 1.0
        if grad_sync is not None:
            scale = grad_sync(flat.grad)
        opt.step(scale)
        loss_buf.copy_(loss.detach())

    graph = None
    if not args.no_graph:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                step_body()
        torch.cuda.current_stream().wait_stream(s)
        sync()
        flat.rebind_grads()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            step_body()

    def step():
        if graph is not None:
            graph.replay()
        else:
            step_body()
        return loss_buf

    for _ in range(args.warmup):
        step()
    sync()
    first = float(loss_buf.reshape(-1)[0])
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync()
    last = float(loss_buf.reshape(-1)[0])
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    elt = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elt, op=dist.ReduceOp.MAX)
    el = float(elt.item())
    done = args.warmup + args.steps + (0 if args.no_graph else 2)
    probe = os.environ.get("EULER_AMD_KG_NAN_PROBE", "0") == "1"  # debugging: stop at the first non-finite step
    while done < args.eval_after:  # untimed: learning evidence only
        snap = (flat.flat.clone(), opt.m.clone(), opt.v.clone(), opt.step_count.clone()) if probe else None
        step()
        done += 1
        if probe and not bool(torch.isfinite(flat.flat).all()):
            print(f"[bench_kg] non-finite parameters after step {done}", file=sys.stderr, flush=True)
            if fused is not None:
                flat.flat.copy_(snap[0])
                opt.m.copy_(snap[1])
                opt.v.copy_(snap[2])
                opt.step_count.copy_(snap[3])
                RgcnTransEStep._check = True
                try:
                    fused.forward_backward()
                    print("[bench_kg] eager re-run of that step: finite", file=sys.stderr, flush=True)
                except FloatingPointError as e:
                    print(f"[bench_kg] eager re-run: {e}", file=sys.stderr, flush=True)
            break
    eval_final = evaluate()
    if rank == 0:
        print(json.dumps({
            "metric": f"train triples/sec (whole node), R-GCN ({args.layers} layer(s)) + TransE on FB15k-shaped KG",
            "value": round(args.batch * world * args.steps / el, 1),
            "unit": "triples/s",
            "n_gpus": 1 if args.shared_gpu else world,
            "ranks": world,
            "shared_gpu_rehearsal": bool(args.shared_gpu) or None,
            "parallelism": f"dp{world}",
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el * 1e3 / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16 relation GEMMs (fp32 accumulate), fp32 scores",
            "data": "synthetic (FB15k-shaped lattice KG, power-law relations)",
            "config": {"model": f"R-GCN {args.layers}x RelationConv(mean, self-loop"
                                f"{', %d bases' % args.num_bases if args.num_bases else ''}) + TransE-l2 margin, "
                                f"flat Adam{', relation weight decay %g' % args.rel_wd if args.rel_wd else ''}",
                       "num_ent": args.num_ent, "num_rel": args.num_rel, "num_triples": args.num_triples,
                       "dim": args.dim, "batch_per_gpu": args.batch, "num_negs": args.num_negs,
                       "normalize": norm, "task": args.task, "hipgraph": graph is not None,
                       "lr": args.lr, "margin": args.margin, "num_bases": args.num_bases, "rel_wd": args.rel_wd,
                       "self_drop": args.self_drop, "type_negs": bool(args.type_negs),
                       "step": "fused (hand-written launches, Philox draws)" if fused is not None else "autograd",
                       "deterministic": bool(fused is not None and fused.deterministic),
                       "parallelism": f"dp{world}", "loss_first_last": [round(first, 4), round(last, 4)],
                       "grad_sync": sync_name, "grad_sync_choice": sync_info or None,
                       "heldout_tail_ranking": {"triples": int(te_src.numel()), "entities": args.num_ent,
                                                "after_steps": done, "init": eval_init, "trained": eval_final,
                                                "chance_mrr": round(sum(1.0 / k for k in range(1, args.num_ent + 1))
                                                                    / args.num_ent, 5)}},
        }), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    raise SystemExit(main())
