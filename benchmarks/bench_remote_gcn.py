#!/usr/bin/env python3
"""GCN (PPI schema) through NodeEstimator against a 2-shard REMOTE graph cluster: the engine
per-op path (every hop a remote GQL query, features over RPC) vs the device path
(``device_graph=True``: DeviceGraph assembled from the shards' API_EXPORT_SHARD exports
once, then the fused GCN step on the GPU).  Prints one JSON line with both rates and the
time the HBM assembly took.  Usage (GPU box): python benchmarks/bench_remote_gcn.py"""
import argparse
import json
import os
import sys
import tempfile
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=0.3)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--engine-steps", type=int, default=10)
    ap.add_argument("--device-steps", type=int, default=400)
    a = ap.parse_args()
    import euler_amd as ea
    from bench_engine_sage import start_cluster
    from euler_amd import models as Z
    from euler_amd.dataset import get_dataset
    from euler_amd.estimator import NodeEstimator
    from euler_amd.graph.device_graph import DeviceGraph

    tmp = tempfile.mkdtemp()
    ds = get_dataset("ppi", data_dir=os.path.join(tmp, "ppi"), scale=a.scale)
    ds.partition_num = 2
    d = ds.load_graph()
    tnt = ds.train_node_type[0] if isinstance(ds.train_node_type, list) else ds.train_node_type
    reg, procs = start_cluster(d, 2, 6)
    out = {"metric": "gcn train samples/s over a 2-shard remote cluster", "dataset": "ppi", "scale": a.scale,
           "batch_size": a.batch}
    try:
        ea.initialize_shared_graph(reg, shard_num=2)
        t = time.time()
        DeviceGraph.from_engine(features="feature", feature_dims=ds.feature_dim, label="label",
                                label_dim=ds.label_dim, device="cuda")
        out["hbm_assembly_s"] = round(time.time() - t, 3)
        for name, dev_graph, steps in (("engine_remote", False, a.engine_steps), ("device_remote", True,
                                                                                   a.device_steps)):
            ea.set_seed(3)
            torch.manual_seed(0)
            m = Z.SupervisedGCN([32, 32, ds.label_dim], [["train"], ["train"]], "feature", ds.feature_dim, "label",
                                ds.label_dim)
            p = {"model_dir": os.path.join(tmp, name), "batch_size": a.batch, "total_step": steps,
                 "learning_rate": 0.01, "log_steps": steps, "train_node_type": tnt, "device": "cuda", "seed": 4,
                 "device_graph": dev_graph}
            res = NodeEstimator(m, p).train()
            out[name] = {"samples_per_sec": round(float(res["samples_per_sec"]), 1), "loss": round(res["loss"], 4),
                         "steps": steps}
            print(name, out[name], flush=True)
    finally:
        for pr in procs:
            pr.terminate()
            pr.wait(timeout=30)
    out["speedup"] = round(out["device_remote"]["samples_per_sec"] / max(out["engine_remote"]["samples_per_sec"],
                                                                          1e-9), 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
