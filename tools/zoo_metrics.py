#!/usr/bin/env python3
"""Held-out metrics of the GCN-family device paths on the learnable community graph
(dataset ``community``: planted communities, weak feature cue, labels from the community)
and of the GCN engine path, for calibrating tests/test_full_trainer.py and the fused-GCN
F1 parity check.  Usage (GPU box): python tools/zoo_metrics.py [--steps 200] [models...]"""
import argparse
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(model, steps, device_graph, extra=()):
    from euler_amd.tools import runner

    tmp = tempfile.mkdtemp()
    argv = ["--dataset", "community", "--scale", "0.5", "--batch_size", "64", "--log_steps", str(steps),
            "--device", "cuda", "--seed", "1", "--model_dir", os.path.join(tmp, "ckpt"), "--total_step", str(steps),
            "--learning_rate", "0.01", "--run_mode", "train_and_evaluate", "--data_dir", os.path.join(tmp, "d")]
    argv += list(extra) + (["--device_graph"] if device_graph else [])
    res, ev = runner.main(argv, model=model)
    return {"train": res, "eval": ev}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--engine", nargs="*", default=["gcn"], help="models also run on the engine path")
    ap.add_argument("models", nargs="*", default=["gcn", "appnp", "sgcn", "tagcn", "agnn", "gat", "arma", "dna",
                                                  "fastgcn", "adaptivegcn", "geniepath", "lgcn", "solution"])
    a = ap.parse_args()
    out = {}
    for m in a.models:
        out[m] = run(m, a.steps, True)
        print(m, json.dumps(out[m]["eval"]), flush=True)
    for m in a.engine:
        out[m + "_engine"] = run(m, a.steps, False)
        print(m + "_engine", json.dumps(out[m + "_engine"]["eval"]), flush=True)


if __name__ == "__main__":
    main()
