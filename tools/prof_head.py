#!/usr/bin/env python3
"""Phase timing of the fused head kernel (st_head) from in-kernel wall-clock stamps.

Builds the bench-shaped FusedSageTrainer on a small synthetic graph, runs a few steps,
then launches st_head with a ``prof`` buffer: every block records the 100 MHz wall clock
at the start, after each __syncthreads and at the end.  Prints per-phase microseconds
(median over blocks) next to the event-timed kernel duration.
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from euler_amd.graph.device_graph import DeviceGraph  # noqa: E402
from euler_amd.models.fused_sage import synthetic_features, synthetic_labels  # noqa: E402
from euler_amd.models.sage_step import FusedSageTrainer  # noqa: E402
from euler_amd.ops._native import hip  # noqa: E402

PHASES = ["load A1", "S0 h1", "S2 emb", "S3 logits", "S4 demb", "S5 g1", "S6 dA1"]


def main():
    dev = torch.device("cuda", 0)
    n = 1_000_000
    g = DeviceGraph.synthetic(n, 10.0, 1024, seed=1, device=dev)
    feats = synthetic_features(n, 128, 2, dev)
    labels = synthetic_labels(feats, 64)
    B = int(os.environ.get("B", "1024"))
    tr = FusedSageTrainer(g, feats, labels, B, [25, 10], 256, 64)
    for _ in range(3):
        tr.step()
    torch.cuda.synchronize()
    h = hip()
    rows = h.st_head_rows
    prof = torch.zeros((B // rows) * 8, dtype=torch.int64, device=dev)

    def head(p=None):
        h.st_head(tr.A1, tr.W1b, tr.Wfcb, tr.WfcT, tr.bfc, tr.Woutb, tr.WoutT, tr.W1T, tr.label_idx, tr.A1_kt,
                  tr.h1_kt, tr.emb_kt, tr.dlog_kt, tr.demb_kt, tr.g1_kt, tr.dA1, tr.gbfc, tr.loss_acc, p)

    for _ in range(5):
        head()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        head()
    e1.record()
    torch.cuda.synchronize()
    print(f"st_head event time: {e0.elapsed_time(e1) * 1000 / 50:.1f} us/launch (B={B}, {B // rows} blocks)")
    head(prof)
    torch.cuda.synchronize()
    t = prof.view(-1, 8).cpu().double() / 100.0  # 100 MHz -> us
    span = float(t[:, 7].max() - t[:, 0].min())
    print(f"stamped span (first start -> last end): {span:.1f} us; start skew {float(t[:, 0].max() - t[:, 0].min()):.1f} us")
    for k, name in enumerate(PHASES):
        d = (t[:, k + 1] - t[:, k]).tolist()
        print(f"  {name:10s} median {statistics.median(d):6.2f} us  max {max(d):6.2f} us")


if __name__ == "__main__":
    main()
