#!/usr/bin/env python3
"""Is the headline head launch slower inside the step graph (20.6 us) than alone (16.4 us)
because of cold caches?  Times tr_head (+ sampler blocks) alone back to back, after a
256 MiB streaming kernel (L2 and much of MALL flushed), after fwd (as in the step), and
after the flush followed by a read of the head's weight shadows (W1, W1^T, Wfc, Wout).
Usage (GPU box): python tools/head_cache_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from euler_amd.dataset.synthetic import synthetic_features, synthetic_labels
    from euler_amd.graph.device_graph import DeviceGraph
    from euler_amd.models.sage_trainer import SageTrainer

    dev = torch.device("cuda", 0)
    g = DeviceGraph.synthetic(10_000_000, 9.5, 256, seed=1234, device=dev)
    x = synthetic_features(10_000_000, 128, 1235, dev)
    y = synthetic_labels(x, 64)
    tr = SageTrainer(g, 1024, [25, 10], [256, 256, 256], 64, features=x, labels=y, learning_rate=0.01,
                     init_seed=1234, keep_samples=False)
    p = tr.plan
    for _ in range(3):
        tr.step()
    torch.cuda.synchronize()
    junk = torch.empty(64 << 20, dtype=torch.float32, device=dev)
    d = tr._buf
    weights = [d[k] for k in ("W1_sh", "W1_shT", "Wfc_sh", "Wfc_shT", "Wout_sh", "Wout_shT") if k in d]
    sink = torch.zeros(1, device=dev)

    def run(prep, reps=40):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        tot = 0.0
        for _ in range(reps):
            prep()
            s.record()
            p.head(None, True)
            e.record()
            torch.cuda.synchronize()
            tot += s.elapsed_time(e) * 1000.0
        return round(tot / reps, 2)

    def flush():
        junk.add_(1.0)

    def flush_warm():
        junk.add_(1.0)
        for w in weights:
            sink.add_(w.float().sum() * 0)

    print("head+sample us: warm", run(lambda: None), "| after flush", run(flush), "| after fwd", run(tr._fwd),
          "| after flush + weight read", run(flush_warm), flush=True)


if __name__ == "__main__":
    main()
