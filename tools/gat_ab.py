#!/usr/bin/env python3
"""Fused vs composed GAT (benchmarks/bench_gat.py) on one synthetic graph from the same
initial weights: loss and every parameter gradient of one step, with and without bf16
autocast, then a few Adam steps of each.  Prints one JSON line per comparison.

Usage: python tools/gat_ab.py [--num-nodes N] [--steps S]"""
import argparse
import copy
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))


def main():
    from bench_gat import GATNet, add_self_loops, planted_labels
    from euler_amd.graph.device_graph import DeviceGraph
    from euler_amd.ops import gnn_ops

    p = argparse.ArgumentParser()
    p.add_argument("--num-nodes", type=int, default=200_000)
    p.add_argument("--avg-degree", type=float, default=50.5)
    p.add_argument("--steps", type=int, default=30)
    args = p.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(7)
    g = DeviceGraph.synthetic(args.num_nodes, args.avg_degree, 4096, seed=7, device=dev)
    indptr, col = add_self_loops(g.indptr, g.nbr)
    csr = gnn_ops.EdgeCSR.from_csr(indptr, col, args.num_nodes)
    N = args.num_nodes
    x = torch.randn(N, 100, device=dev).to(torch.bfloat16)
    y = planted_labels(indptr, col, x, 47, hops=2)
    rows = torch.randperm(N, device=dev)[: N // 10]
    base = GATNet(100, 8, 16, 47, 2, "fused").to(dev)
    models = {}
    for impl in ("fused", "composed"):
        m = copy.deepcopy(base)
        m.impl = impl
        models[impl] = m

    def grads(m, amp):
        m.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            logits = m(x if amp else x.float(), csr, rows)
        loss = gnn_ops.xent(logits.float(), y[rows])
        loss.backward()
        return float(loss), {k: v.grad.detach().float().clone() for k, v in m.named_parameters()}

    for amp in (False, True):
        lf, gf = grads(models["fused"], amp)
        lc, gc = grads(models["composed"], amp)
        out = {"amp": amp, "loss_fused": round(lf, 6), "loss_composed": round(lc, 6)}
        for k in gf:
            a, b = gf[k].reshape(-1), gc[k].reshape(-1)
            out[k] = {"cos": round(float(torch.nn.functional.cosine_similarity(a, b, dim=0)), 5),
                      "rel": round(float((a - b).norm() / b.norm().clamp(min=1e-12)), 5)}
        print(json.dumps(out), flush=True)
    # a few Adam steps each (bf16 autocast, like the benchmark)
    for impl, m in models.items():
        opt = torch.optim.Adam(m.parameters(), lr=5e-3)
        losses = []
        for _ in range(args.steps):
            opt.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                logits = m(x, csr, rows)
            loss = gnn_ops.xent(logits.float(), y[rows])
            loss.backward()
            opt.step()
            losses.append(round(float(loss), 4))
        print(json.dumps({"impl": impl, "losses": losses[::5] + losses[-1:]}), flush=True)


if __name__ == "__main__":
    main()
