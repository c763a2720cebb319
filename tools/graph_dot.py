#!/usr/bin/env python3
"""Dump the captured R-GCN + TransE step's hipGraph with the gradient zeroing done by
hipMemsetAsync (EULER_AMD_ZERO_MEMSET=1) and by the zero kernel: hipGraphDebugDotPrint
(.dot) and a node / edge summary (hip().graph_summary on the graph torch keeps with
CUDAGraph(keep_graph=True)), and check the structure every replay relies on — one linear
chain: each node has at most one predecessor and one successor, and every memset node
sits between two kernels.  Usage (GPU box): python tools/graph_dot.py <out_dir>"""
import collections
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def capture_kg(mode):
    from tests.test_kg_step import _setup

    old = os.environ.get("EULER_AMD_ZERO_MEMSET")
    os.environ["EULER_AMD_ZERO_MEMSET"] = mode
    try:
        m, flat, opt, step, ei, erel = _setup("cuda", 1)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                step.step()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph(keep_graph=True)
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            step.step()
    finally:  # the zeroing mode is read per call: never leak it into the caller's process
        if old is None:
            os.environ.pop("EULER_AMD_ZERO_MEMSET", None)
        else:
            os.environ["EULER_AMD_ZERO_MEMSET"] = old
    return g, (m, flat, opt, step)


def analyse(summary):
    nodes, edges = summary["nodes"], summary["edges"]
    preds, succs = collections.defaultdict(list), collections.defaultdict(list)
    for a, b in edges:
        succs[a].append(b)
        preds[b].append(a)
    chain = all(len(preds[i]) <= 1 and len(succs[i]) <= 1 for i, _, _ in nodes) and len(edges) == len(nodes) - 1
    roots = [i for i, _, _ in nodes if not preds[i]]
    mem = []
    for i, kind, detail in nodes:
        if kind == "memset":
            mem.append({"node": i, "detail": detail, "preds": [nodes[p][1:] for p in preds[i]],
                        "succs": [nodes[q][1:] for q in succs[i]]})
    return {"nodes": len(nodes), "edges": len(edges), "kinds": dict(collections.Counter(k for _, k, _ in nodes)),
            "linear_chain": chain, "roots": roots, "memset_nodes": mem}


def main(out):
    from euler_amd.ops._native import hip

    os.makedirs(out, exist_ok=True)
    res = {}
    for mode in ("1", "0"):
        g, _ = capture_kg(mode)
        path = os.path.join(out, f"kg_step_memset{mode}.dot")
        summ = hip().graph_summary(g.raw_cuda_graph(), path)
        res[mode] = analyse(summ)
        with open(os.path.join(out, f"kg_step_memset{mode}_nodes.json"), "w") as f:
            json.dump({"nodes": [list(x) for x in summ["nodes"]], "edges": [list(x) for x in summ["edges"]]}, f,
                      indent=1)
        print(f"EULER_AMD_ZERO_MEMSET={mode}: {json.dumps(res[mode])}", flush=True)
        g.reset()
    return res


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/graph_dot")
