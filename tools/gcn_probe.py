#!/usr/bin/env python3
"""Per-phase timing of the fused GCN head launch (csrc/hip/gcn.hip, wall-clock stamps) at the
bench_gcn shape (PPI schema, batch 512, hidden 32, 2 layers).  Usage (GPU box):
    python tools/gcn_probe.py [--batch-size 512] [--scale 1.0]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch-size", type=int, default=512)
    ap.add_argument("--scale", type=float, default=1.0)
    a = ap.parse_args()
    import tempfile

    from euler_amd.graph.device_graph import DeviceGraph
    from euler_amd.models.full_trainer import FullFlowTrainer
    from euler_amd.models.gcn_trainer import GcnTrainer
    from euler_amd.tools import runner

    args = runner.parse_args(["--dataset", "ppi", "--scale", str(a.scale), "--batch_size", str(a.batch_size),
                              "--device", "cuda", "--seed", "1", "--data_dir", tempfile.mkdtemp()], model="gcn")
    torch.manual_seed(0)
    m, _ = runner.build(args)
    m.to("cuda")
    g = DeviceGraph.from_engine(features=m.gnn.feature_idx, feature_dims=m.gnn.feature_dim, label=m.label_idx,
                                label_dim=m.label_dim, feature_dtype=torch.bfloat16, seed=5, device="cuda")
    FullFlowTrainer.from_model(m, g, a.batch_size, caps="exact")  # materialise the lazy layers
    tr = GcnTrainer.from_model(m, g, a.batch_size, caps="bounded")
    for _ in range(5):
        tr.step()
    torch.cuda.synchronize()
    print("caps", tr.flow.caps, "counts", tr.plan.flow()["cnt"].tolist())
    names = ["copy+zero", "labels+aggregate", "z", "emb", "logits+loss", "d emb", "d z", "w-grad partials",
             "d agg", "d agg rows out"]
    ks = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 15]
    acc = None
    for _ in range(5):
        p = tr.plan.head_profile()
        torch.cuda.synchronize()
        t = p.double().cpu() / 100.0  # wall_clock64: 100 MHz
        d = torch.stack([t[:, ks[i + 1]] - t[:, ks[i]] for i in range(len(ks) - 1)], 1)
        acc = d if acc is None else acc + d
    d = acc / 5
    print("head blocks", d.shape[0], "span us", round(float((t[:, 15].max() - t[:, 0].min())), 2),
          "start skew", round(float(t[:, 0].max() - t[:, 0].min()), 2))
    for i, n in enumerate(names):
        print(f"  {n:18s} mean {float(d[:, i].mean()):6.2f} us  max {float(d[:, i].max()):6.2f}")


if __name__ == "__main__":
    main()
