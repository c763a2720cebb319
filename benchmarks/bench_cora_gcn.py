#!/usr/bin/env python3
"""BASELINE config 1: 2-layer GCN on Cora through the CPU graph engine and CPU message
passing (plumbing check: no GPU involved).

The full reference stack on the CPU: Cora-schema graph (2,708 nodes, 1,433-d features,
7 classes; synthetic same-schema data, no download possible) converted to the reference
on-disk format, loaded by the C++ engine, NodeEstimator training of SupervisedGCN
(GCNConv + full-neighbour dataflow, hidden 32, batch 32, Adam lr 0.01: reference
examples/gcn/run_gcn.py defaults).  Prints one JSON line with train samples/sec.

Usage: python benchmarks/bench_cora_gcn.py [--steps K] [--warmup W] [--threads T]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--batch", type=int, default=32)
    p.add_argument("--threads", type=int, default=8)
    args = p.parse_args(argv)
    torch.set_num_threads(args.threads)

    import euler_amd as ea
    from euler_amd import models as Z
    from euler_amd.dataset import get_dataset
    from euler_amd.estimator import NodeEstimator

    ds = get_dataset("cora", data_dir=tempfile.mkdtemp(prefix="euler_amd_cora_"))
    ds.load_graph()
    ea.set_seed(1)
    torch.manual_seed(1)
    model = Z.SupervisedGCN([32, 32, ds.label_dim], [["train"], ["train"]], "feature", 1433, "label", ds.label_dim)
    tnt = ds.train_node_type[0] if isinstance(ds.train_node_type, list) else ds.train_node_type

    def params(total):
        return {"model_dir": tempfile.mkdtemp(prefix="euler_amd_ckpt_"), "batch_size": args.batch,
                "total_step": total, "optimizer": "adam", "learning_rate": 0.01, "log_steps": max(total, 1),
                "train_node_type": tnt, "device": "cpu", "prefetch": 0}

    est = NodeEstimator(model, params(args.warmup))
    first = est.train()
    est2 = NodeEstimator(model, params(args.steps))
    est2.optimizer = None
    t0 = time.perf_counter()
    last = est2.train()
    el = time.perf_counter() - t0
    print(json.dumps({
        "metric": "train samples/sec, 2-layer GCN on Cora via the CPU graph engine + CPU message passing",
        "value": round(args.batch * args.steps / el, 1),
        "unit": "samples/s",
        "n_gpus": 0,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el * 1e3 / args.steps, 3),
        "higher_is_better": True,
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic Cora-schema graph (2,708 nodes, 1,433-d features, 7 classes)",
        "config": {"model": "SupervisedGCN [32, 32, 7], full-neighbour dataflow, Adam", "batch": args.batch,
                   "threads": args.threads, "loss_first_last": [round(first.get("loss", float("nan")), 4),
                                                                round(last.get("loss", float("nan")), 4)]},
    }), flush=True)


if __name__ == "__main__":
    main()
