#!/usr/bin/env python3
"""Loss trajectories of the fused GCN step: eager twice, hipGraph replay twice (bf16
features, batch 64) — separates nondeterminism from a replay-only difference."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gcn_trainer import _graph, _materialize, _setup  # noqa: E402


def run(captured, fdt=torch.bfloat16, steps=8):
    from euler_amd.models.gcn_trainer import GcnTrainer

    m = _setup("cuda").to("cuda")
    g = _graph(m, "cuda", fdt)
    _materialize(m, g, 64)
    tr = GcnTrainer.from_model(m, g, 64, caps="exact")
    out = []
    if captured:
        tr.capture(warmup=2, steps=4)
        for _ in range(steps - 2):
            tr.replay(1)
            out.append(round(float(tr.loss.item()), 5))
    else:
        for _ in range(steps):
            tr.step()
            out.append(round(float(tr.loss.item()), 5))
        out = out[2:]
    return out, int(tr.flow.overflow.item())


if __name__ == "__main__":
    for fdt in (torch.bfloat16, torch.float32):
        for cap in (False, False, True, True):
            print(fdt, "graph" if cap else "eager", run(cap, fdt), flush=True)
