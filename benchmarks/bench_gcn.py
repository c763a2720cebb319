#!/usr/bin/env python3
"""GCN-family training throughput through NodeEstimator: the engine path (CPU graph engine
builds every GCNDataFlow batch, the GPU runs the model) next to the device path
(``--device_graph``: dataflow/device_flow.py + models/full_trainer.py, sampling, blocks,
model, backward and optimizer captured in hipGraphs on an HBM copy of the graph).  Same
model, dataset, flags and seed; samples/s is the estimator's own rate over the last log
interval.  Prints one JSON line.

Reference: examples/gcn/run_gcn.py (GNN('gcn', 'full', ...), examples/gcn/gcn.py:52-58).

    python benchmarks/bench_gcn.py [--model gcn] [--dataset ppi] [--batch-size 512] [--steps 300]
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def run(path, args, work):
    from euler_amd.tools.runner import main

    steps = args.steps if path == "device" else args.engine_steps
    argv = ["--dataset", args.dataset, "--batch_size", str(args.batch_size), "--total_step", str(steps),
            "--log_steps", str(max(steps // 4, 1)), "--model_dir", os.path.join(work, path), "--learning_rate",
            str(args.lr), "--device", args.device, "--seed", str(args.seed), "--hidden_dim", str(args.hidden_dim)]
    if args.scale != 1.0:
        argv += ["--scale", str(args.scale)]
    if path == "device":
        argv.append("--device_graph")
    t0 = time.time()
    res = main(argv, model=args.model)
    return {k: round(float(v), 4) for k, v in res.items()} | {"wall_s": round(time.time() - t0, 1)}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--model", default="gcn")
    ap.add_argument("--dataset", default="ppi")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--batch-size", dest="batch_size", type=int, default=512)
    ap.add_argument("--hidden-dim", dest="hidden_dim", type=int, default=32)
    ap.add_argument("--steps", type=int, default=400, help="device-path steps")
    ap.add_argument("--engine-steps", type=int, default=40, help="engine-path steps (slower)")
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--paths", default="engine,device")
    args = ap.parse_args(argv)
    work = tempfile.mkdtemp(prefix="bench_gcn_")
    out = {"metric": f"{args.model} train samples/s (NodeEstimator, 1 device)", "dataset": args.dataset,
           "batch_size": args.batch_size, "hidden_dim": args.hidden_dim, "device": args.device}
    for path in args.paths.split(","):
        out[path] = run(path, args, work)
        print(f"[bench_gcn] {path}: {out[path]}", file=sys.stderr, flush=True)
    if "engine" in out and "device" in out:
        out["speedup"] = round(out["device"]["samples_per_sec"] / max(out["engine"]["samples_per_sec"], 1e-9), 2)
    print(json.dumps(out), flush=True)
    return out


if __name__ == "__main__":
    main()
