"""Fixed cost of a timed region made of one hipGraph replay (bench.py's protocol at
--steps 20): wall time of replay_steps(n) + synchronize for a graph replayed for the first
time vs. again, with and without hipGraphUpload after capture, against the per-step time
of a long run.  SageTrainer on a 10M-node synthetic graph.

    python tools/replay_overhead_probe.py [--nodes 10000000] [--upload 0|1]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=10_000_000)
    ap.add_argument("--upload", type=int, default=0)
    a = ap.parse_args()
    import torch

    from euler_amd.dataset.synthetic import synthetic_features, synthetic_labels
    from euler_amd.graph.device_graph import DeviceGraph
    from euler_amd.models.sage_trainer import SageTrainer
    from euler_amd.ops._native import hip

    dev = torch.device("cuda", 0)
    g = DeviceGraph.synthetic(a.nodes, 10.0, 1024, seed=1, device=dev)
    f = synthetic_features(a.nodes, 128, 2, dev, dtype=torch.bfloat16)
    tr = SageTrainer(g, 1024, [25, 10], [256, 256, 256], 64, features=f, labels=synthetic_labels(f, 64),
                     keep_samples=False)
    tr.capture(None, steps=32, extra_sizes=(2, 4, 5, 10, 20))
    if a.upload:
        for gr in tr._graphs.values():
            hip().graph_upload(gr.raw_cuda_graph_exec())
        torch.cuda.synchronize()
    out = {"upload": a.upload}

    def timed(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.replay_steps(n)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e6

    tr.replay_steps(5)
    torch.cuda.synchronize()
    out["first_20_us"] = round(timed(20), 1)
    out["second_20_us"] = round(timed(20), 1)
    out["third_20_us"] = round(timed(20), 1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    tr.replay_steps(20)
    e1.record()
    torch.cuda.synchronize()
    out["events_20_us"] = round(e0.elapsed_time(e1) * 1e3, 1)
    out["long_1024_us_per_step"] = round(timed(1024) / 1024, 2)

    def chunks(k, n=20):  # n steps as n / k replays of the k-step graph
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n // k):
            tr._graphs[k].replay()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e6

    for k in (1, 2, 4, 10, 20):
        out[f"20_as_{20 // k}x{k}_us"] = round(min(chunks(k) for _ in range(3)), 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
