#!/usr/bin/env python3
"""Unsupervised GraphSAGE on the device path (euler_amd.models.sage_tower.UnsupSageTrainer):
training throughput and held-out link-prediction AUC.

Reference model: examples/graphsage/graphsage.py:70-98 (UnsupervisedGraphSage, source +
context towers, 1 sampled positive neighbour, num_negs sample_node negatives, sigmoid CE,
MRR).  Data: a planted-community graph (dataset/synthetic.py community_graph) whose node
features carry a weak community cue (community_features: one node's row is a noisy hint,
its neighbourhood's mean a strong one); 5 % of the edges are held out.  AUC = P(score of a
held-out edge > score of a random pair), score(u, v) = <src_emb(u), ctx_emb(v)> (the
trained objective), before and after training.  Prints one JSON line.

    python benchmarks/bench_unsup_sage.py [--num-nodes 1000000] [--steps 2000] [--batch-size 1024]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def build(num_nodes, num_comm, avg_degree, feat_dim, signal, seed, device, holdout=0.05):
    from euler_amd.dataset.synthetic import community_features, community_graph
    from euler_amd.graph.device_graph import DeviceGraph

    src, dst, comm = community_graph(num_nodes, num_comm, avg_degree, p_in=0.9, seed=seed)
    g = torch.Generator().manual_seed(seed + 11)
    test = torch.rand(src.numel(), generator=g) < holdout
    ts, td = src[test], dst[test]
    src, dst = src[~test], dst[~test]
    order = torch.argsort(src * num_nodes + dst)
    src, dst = src[order], dst[order]
    indptr = np.zeros(num_nodes + 1, np.int64)
    np.add.at(indptr, src.numpy() + 1, 1)
    indptr = np.cumsum(indptr)
    graph = DeviceGraph.from_csr(indptr, dst.numpy().astype(np.int32), np.ones(dst.numel(), np.float32), seed=seed,
                                 device=device)
    x = community_features(comm, feat_dim, signal=signal, seed=seed).to(device)
    if device.type == "cuda":
        x = x.to(torch.bfloat16)
    return graph, x, (ts, td)


@torch.no_grad()
def link_auc(tr, test_edges, num_nodes, n_eval, seed):
    from euler_amd.dataset.synthetic import auc

    ts, td = test_edges
    g = torch.Generator().manual_seed(seed + 13)
    k = torch.randperm(ts.numel(), generator=g)[:n_eval]
    u, v = ts[k], td[k]
    nu = torch.randint(0, num_nodes, (n_eval,), generator=g)
    nv = torch.randint(0, num_nodes, (n_eval,), generator=g)
    es = tr.embed(torch.cat([u, nu]), "gnn")
    ec = tr.embed(torch.cat([v, nv]), "context_gnn")
    s = (es * ec).sum(1).float().cpu()
    return auc(s[:n_eval], s[n_eval:])


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--num-nodes", type=int, default=1_000_000)
    ap.add_argument("--num-comm", type=int, default=1000)
    ap.add_argument("--avg-degree", type=float, default=10.0)
    ap.add_argument("--feature-dim", type=int, default=128)
    ap.add_argument("--signal", type=float, default=0.5)
    ap.add_argument("--batch-size", type=int, default=1024)
    ap.add_argument("--fanouts", default="10,5")
    ap.add_argument("--dims", default="128,128,128")
    ap.add_argument("--num-negs", type=int, default=5)
    ap.add_argument("--lr", type=float, default=0.003)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--eval-pairs", type=int, default=20000)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--steps-per-graph", type=int, default=16)
    ap.add_argument("--per-op", action="store_true", help="the per-op autograd step instead of the fused PairPlan")
    args = ap.parse_args(argv)
    from euler_amd.models.sage_tower import UnsupSageTrainer

    dev = torch.device(args.device)
    t0 = time.time()
    graph, x, test = build(args.num_nodes, args.num_comm, args.avg_degree, args.feature_dim, args.signal, args.seed,
                           dev)
    tr = UnsupSageTrainer(graph, args.batch_size, [int(f) for f in args.fanouts.split(",")],
                          [int(d) for d in args.dims.split(",")], features=x, num_negs=args.num_negs,
                          learning_rate=args.lr, init_seed=args.seed, fused=not args.per_op)
    print(f"[unsup] graph {args.num_nodes} nodes, {graph.num_edges} train edges, build {time.time() - t0:.1f}s",
          file=sys.stderr, flush=True)
    auc0 = link_auc(tr, test, args.num_nodes, args.eval_pairs, args.seed)
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    graphed = dev.type == "cuda" and not args.no_graph
    chunk = max(args.steps // 5, 1)
    if graphed:
        # several complete steps per hipGraph replay (the timed loop still runs exactly
        # --steps steps)
        spg = max(1, args.steps_per_graph)
        tr.capture(warmup=min(2, args.warmup), steps=spg, extra_sizes=(chunk % spg, args.warmup % spg,
                                                                        args.steps % chunk % spg))
        run = tr.replay_steps
    else:
        def run(n):
            for _ in range(n):
                tr.step()
    run(args.warmup)
    sync()
    first = float(tr.loss)
    tr.reset_metric()
    t1 = time.perf_counter()
    done = 0
    while done < args.steps:
        n = min(chunk, args.steps - done)
        run(n)
        done += n
        sync()
        print(f"[unsup] step {done} loss {float(tr.loss):.4f} mrr {tr.metric():.4f}", file=sys.stderr, flush=True)
    sync()
    el = time.perf_counter() - t1
    mrr = tr.metric()
    auc1 = link_auc(tr, test, args.num_nodes, args.eval_pairs, args.seed)
    out = {"metric": "unsupervised GraphSAGE train samples/sec (1 device)", "value": round(args.batch_size * args.steps
                                                                                     / el, 1),
           "unit": "samples/s", "ms_per_step": round(el * 1000 / args.steps, 4), "steps": args.steps,
           "device": str(dev), "hipgraph": dev.type == "cuda" and not args.no_graph,
           "loss_first_last": [round(first, 4), round(float(tr.loss), 4)], "train_mrr_last": round(mrr, 4),
           "heldout_link_auc_init": round(auc0, 4), "heldout_link_auc": round(auc1, 4),
           "config": {k: getattr(args, k) for k in ("num_nodes", "num_comm", "avg_degree", "feature_dim", "signal",
                                                     "batch_size", "fanouts", "dims", "num_negs", "lr")},
           "impl": ("euler_amd.models.sage_tower.UnsupSageTrainer: " + (
               "fused 7-launch step (PairPlan: tower samplers drawing the roots, layer-0 forwards, pair head, "
               "one dW launch, one optimizer launch)" if tr.pair is not None else
               "per-op step (layer-0 tower kernels, GEMM autograd heads, pair-loss kernels)")),
           "data": "synthetic planted communities, features = weak community cue + noise"}
    print(json.dumps(out), flush=True)
    return out


if __name__ == "__main__":
    main()
