#!/usr/bin/env python3
"""Time the GAT edge kernels (gat.hip) on the ogbn-products-shaped graph of
benchmarks/bench_gat.py: forward, backward destination+source passes, each with al
gathered per edge and with al recomputed from the gathered row (a_src passed)."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))

from bench_gat import add_self_loops  # noqa: E402
from euler_amd.graph.device_graph import DeviceGraph  # noqa: E402
from euler_amd.ops import gnn_ops  # noqa: E402
from euler_amd.ops._native import hip  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--num-nodes", type=int, default=2_449_029)
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--tag", default=os.environ.get("EULER_AMD_HIP_FLAGS", "default"))
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    g = DeviceGraph.synthetic(a.num_nodes, 50.5, 4096, seed=7, device=dev)
    indptr, col = add_self_loops(g.indptr, g.nbr)
    del g
    csr = gnn_ops.EdgeCSR.from_csr(indptr, col, a.num_nodes)
    H, C, N = 8, 16, a.num_nodes
    z = torch.randn(N, H * C, device=dev).to(torch.bfloat16)
    a_s, a_d = torch.randn(H, C, device=dev) * 0.3, torch.randn(H, C, device=dev) * 0.3
    al, ar = hip().gat_att_fwd(z, a_s, a_d, H, C)
    ip, cl = csr.csr()
    ci, cr = csr.csc()
    o, lse = hip().gat_fwd(ip, cl, csr.csr_order(), z, al, ar, H, C, 0.2)
    dout = torch.randn_like(o)
    res = {"tag": a.tag}
    for name, asrc in (("gather_al", None), ("recompute_al", a_s)):
        res[name] = {
            "fwd_ms": round(timed(lambda: hip().gat_fwd(ip, cl, csr.csr_order(), z, al, ar, H, C, 0.2, asrc), a.reps), 3),
            "bwd_ms": round(timed(lambda: hip().gat_bwd(ip, cl, csr.csr_order(), ci, cr, csr.csc_order(), z, al, ar, H, C,
                                                        0.2, o, dout, lse, asrc), a.reps), 3),
        }
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
