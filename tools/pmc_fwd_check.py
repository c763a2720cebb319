#!/usr/bin/env python3
"""Reconcile the memory counters of the tree forward: run tr_fwd once and a plain
gather_rows of exactly the rows it reads (every leaf row + every layer-0 self row), each
after a 1 GiB copy that evicts L2 and the MALL, so both see the same cold rows.  Under
`rocprofv3 --pmc FETCH_SIZE` the two FETCH values should agree if the counter sees the
forward's row traffic."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from euler_amd.graph.device_graph import DeviceGraph
    from euler_amd.dataset.synthetic import synthetic_features, synthetic_labels
    from euler_amd.models.sage_trainer import SageTrainer
    from euler_amd.ops._native import hip

    dev = torch.device("cuda", 0)
    n = 10_000_000
    g = DeviceGraph.synthetic(n, 9.5, 256, seed=1234, device=dev)
    x = synthetic_features(n, 128, 1235, dev)
    y = synthetic_labels(x, 64)
    tr = SageTrainer(g, 1024, [25, 10], [256] * 3, 64, features=x, labels=y, learning_rate=0.01, init_seed=1)
    big = torch.empty(256 << 20, device=dev)
    big2 = torch.empty_like(big)
    p = tr.plan
    p.sample()
    torch.cuda.synchronize()
    nodes = tr.nodes.long()
    leaf = tr.leaf.long()
    rows = torch.cat([nodes[nodes >= 0], leaf[leaf >= 0]])
    print(f"rows read by tr_fwd: {rows.numel()} ({rows.numel() * 256 / 2**20:.1f} MiB of bf16 rows), "
          f"unique {torch.unique(rows).numel()}", flush=True)
    for _ in range(3):
        big2.copy_(big)      # evict
        p.fwd()
        big2.copy_(big)      # evict
        hip().gather_rows(x, rows)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
