#!/usr/bin/env python3
"""Held-out F1 of supervised GraphSAGE through NodeEstimator: the engine path (GQL
sampling + torch layers) next to the device path (``--device_graph``: fused gfx950
SageTrainer on an HBM copy of the graph), same dataset, flags and seed.

Dataset ``community`` (dataset/base.py Community): planted communities, labels =
community mod 16 with 10 % flipped, features a weak community cue — learnable only by
aggregating neighbours.  Training nodes: the first 80 %; F1 (micro, the reference's
utils/metrics.py f1) on the held-out 20 % after training.  Prints one JSON line.

    python benchmarks/bench_community_f1.py [--steps 1000] [--device cuda]
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

    argv = ["--dataset", "community", "--batch_size", str(args.batch_size), "--total_step", str(args.steps),
            "--log_steps", str(max(args.steps // 5, 1)), "--model_dir", os.path.join(work, path), "--fanouts",
            "10", "10", "--learning_rate", str(args.lr), "--run_mode", "train_and_evaluate", "--device", args.device,
            "--seed", str(args.seed)]
    if path == "device":
        argv.append("--device_graph")
    t0 = time.time()
    if args.model != "graphsage":
        argv = [a for a in argv]
        i = argv.index("--fanouts")
        del argv[i:i + 3]  # full-neighbourhood models take no fanouts
    res, ev = main(argv, model=args.model)
    return {"train_last": {k: round(float(v), 4) for k, v in res.items()}, "heldout": {k: round(float(v), 4)
                                                                                       for k, v in ev.items()},
            "wall_s": round(time.time() - t0, 1)}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--batch-size", dest="batch_size", type=int, default=256)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--model", default="graphsage", help="graphsage, or a full-neighbourhood model (gcn, appnp, "
                                                          "sgcn, tagcn)")
    args = ap.parse_args(argv)
    work = tempfile.mkdtemp(prefix="community_f1_")
    os.environ.setdefault("EULER_AMD_DATA", os.path.join(work, "data"))
    out = {"metric": f"held-out micro-F1, supervised {args.model} (NodeEstimator)", "dataset": "community (synthetic "
           "planted communities, 20000 nodes, 16 classes, 10% label noise)", "steps": args.steps,
           "batch_size": args.batch_size, "fanouts": [10, 10] if args.model == "graphsage" else None,
           "device": args.device}
    for path in ("engine", "device"):
        out[path] = run(path, args, work)
        print(f"[community_f1] {path}: {out[path]}", file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)
    return out


if __name__ == "__main__":
    main()
