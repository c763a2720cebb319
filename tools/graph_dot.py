#!/usr/bin/env python3
"""Dump the captured R-GCN + TransE step's hipGraph (hipGraphDebugDotPrint through
torch.cuda.CUDAGraph.debug_dump) with the gradient zeroing done by hipMemsetAsync
(EULER_AMD_ZERO_MEMSET=1) and by the zero kernel, and print each graph's node kinds and
its edge count.  Usage (GPU box): python tools/graph_dot.py <out_dir>"""
import collections
import os
import re
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(out):
    from tests.test_kg_step import _setup

    os.makedirs(out, exist_ok=True)
    for mode in ("1", "0"):
        os.environ["EULER_AMD_ZERO_MEMSET"] = mode
        m, flat, opt, step, ei, erel = _setup("cuda", 1)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                step.step()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        g.enable_debug_mode()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            step.step()
        path = os.path.join(out, f"kg_step_memset{mode}.dot")
        g.debug_dump(path)
        txt = open(path).read()
        kinds = collections.Counter(re.findall(r'\\<B\\>(\w+)', txt) or re.findall(r'label="\{?(\w+)', txt))
        edges = len(re.findall(r"->", txt))
        print(f"memset={mode}: {path} nodes by kind {dict(kinds)}, edges {edges}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/graph_dot")
