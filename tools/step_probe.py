#!/usr/bin/env python3
"""A short, fixed run of the headline training step for rocprofv3 counter passes: the
bench-shaped SageTrainer (B 1024, fanouts [25, 10], 128-d bf16 features, hidden 256, 64
classes) on a synthetic graph, 4 warm steps, then ``--reps`` replays of a 4-step hipGraph
(the kernels exactly as bench.py runs them).  ``--dw-only``: the routed dW problem alone,
``--reps`` launches.  Usage: rocprofv3 --pmc ... -- python3 tools/step_probe.py"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--num-nodes", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--dw-only", action="store_true")
    a = ap.parse_args()
    from euler_amd.dataset.synthetic import synthetic_features, synthetic_labels
    from euler_amd.graph.device_graph import DeviceGraph
    from euler_amd.models.sage_trainer import SageTrainer

    dev = torch.device("cuda", 0)
    g = DeviceGraph.synthetic(a.num_nodes, 10.0, 1024, seed=1234, device=dev)
    x = synthetic_features(a.num_nodes, 128, 1235, dev)
    y = synthetic_labels(x, 64)
    tr = SageTrainer(g, 1024, [25, 10], [256, 256, 256], 64, features=x, labels=y, keep_samples=False)
    for _ in range(4):
        tr.step()
    torch.cuda.synchronize()
    if a.dw_only:
        for _ in range(a.reps):
            tr.plan.dw([0])
    else:
        tr.capture(steps=4)
        for _ in range(a.reps):
            tr.replay_steps(4)
    torch.cuda.synchronize()
    print("probe done", float(tr.loss.item()))


if __name__ == "__main__":
    main()
