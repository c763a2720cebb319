#!/usr/bin/env python3
"""GraphSAGE through the C++ graph engine (the reference's architecture: CPU-side graph
store + sampler, tensors streamed to the GPU) with the estimator loop, with and without
the asynchronous input pipelines: the Python prefetcher (utils/prefetch.py) and the
native C++ batch pipeline (dataflow/native_loader.py: worker threads write complete
batches — every hop, features, labels — into reused pinned slots; 3 H2D copies per
batch on a side stream).  The per-step
subgraph (sampling, per-hop unique, edge index) is one GIL-free engine call
(``_engine.sage_flow``), so the worker thread overlaps the model step.

Data: PPI-schema synthetic graph (``get_dataset("ppi")``: 56,944 nodes, 50-d features,
121 multi-hot labels; reference examples/graphsage default dataset family), converted
to the reference on-disk format and loaded by the engine.  Model: SupervisedGraphSage
[128, 128, 121], fanouts [10, 10], sigmoid CE, Adam.

Usage: python benchmarks/bench_engine_sage.py [--steps K] [--scale S] [--batch B]
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


def start_cluster(data_dir, shards, threads=8):
    """``shards`` same-host shard servers over the reference-format ``data_dir``, found
    through a file registry; returns (registry, processes)."""
    import subprocess

    reg = tempfile.mkdtemp(prefix="euler_amd_bench_reg_")
    env = dict(os.environ, PYTHONPATH=ROOT)
    procs = [subprocess.Popen([sys.executable, "-m", "euler_amd.tools.service", "--data_path", data_dir,
                               "--shard_idx", str(s), "--shard_num", str(shards), "--registry", reg,
                               "--threads", str(threads)], env=env, stdout=subprocess.DEVNULL,
                              stderr=subprocess.STDOUT) for s in range(shards)]
    deadline = time.time() + 120
    while time.time() < deadline and len([f for f in os.listdir(reg) if "#" in f]) < shards:
        time.sleep(0.2)
    if len([f for f in os.listdir(reg) if "#" in f]) < shards:
        raise RuntimeError("shard servers did not register")
    return reg, procs


def run(ds, args, prefetch, device, workers=2, native=False, graph="auto"):
    import euler_amd as ea
    from euler_amd import models as Z
    from euler_amd.estimator import NodeEstimator

    ea.set_seed(1)
    torch.manual_seed(1)
    model = Z.SupervisedGraphSage([128, 128, ds.label_dim], [10, 10], [["train"], ["train"]], "feature",
                                  ds.feature_dim, "label", ds.label_dim, max_id=ds.max_node_id)
    tnt = ds.train_node_type[0] if isinstance(ds.train_node_type, list) else ds.train_node_type

    def params(total):
        return {"model_dir": tempfile.mkdtemp(prefix="euler_amd_ckpt_"), "batch_size": args.batch,
                "total_step": total, "optimizer": "adam", "learning_rate": 0.01, "log_steps": 10 ** 9,
                "train_node_type": tnt, "device": device, "prefetch": prefetch,
                "prefetch_workers": workers, "native_pipeline": native, "pipeline_workers": workers,
                "cuda_graph": graph}

    NodeEstimator(model, params(args.warmup)).train()
    est = NodeEstimator(model, params(args.steps))
    if device == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = est.train()
    if device == "cuda":
        torch.cuda.synchronize()
    return time.perf_counter() - t0, res


def run_pipeline(ds, args, device, workers):
    """input pipeline alone: batches/s of the native C++ pipeline (sampling, unique, feature
    and label fetch — local engine or per-shard RPCs — into pinned slots, + H2D on a GPU),
    drained without a model step"""
    import euler_amd as ea
    from euler_amd import models as Z
    from euler_amd.dataflow.native_loader import NativeSageLoader, native_spec

    ea.set_seed(1)
    model = Z.SupervisedGraphSage([128, 128, ds.label_dim], [10, 10], [["train"], ["train"]], "feature",
                                  ds.feature_dim, "label", ds.label_dim, max_id=ds.max_node_id)
    tnt = ds.train_node_type[0] if isinstance(ds.train_node_type, list) else ds.train_node_type
    flow, names, dims, label, label_dim, node_type = native_spec(model, {"train_node_type": tnt})
    ld = NativeSageLoader(flow, names, dims, label, label_dim, args.batch, node_type, torch.device(device),
                          workers=workers, seed=1)
    sync = torch.cuda.synchronize if device == "cuda" else (lambda: None)
    for _ in range(args.warmup):
        ld.get()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ld.get()
    sync()
    el = time.perf_counter() - t0
    ld.close()
    return el


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--steps", type=int, default=60)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=512)
    p.add_argument("--scale", type=float, default=1.0)
    p.add_argument("--native_workers", type=int, nargs="+", default=[4, 8, 16])
    p.add_argument("--only", default="", help="comma list of variant names to run (default: all)")
    p.add_argument("--cprofile", default="", help="write the consumer's cProfile top-40 (cumulative) here")
    p.add_argument("--mode", choices=["local", "remote"], default="local",
                   help="remote: the graph on --shards same-host shard servers (initialize_shared_graph)")
    p.add_argument("--shards", type=int, default=2)
    p.add_argument("--server_threads", type=int, default=8)
    p.add_argument("--device", default=None)
    p.add_argument("--pipeline_only", action="store_true",
                   help="time the native pipeline alone (no model step) for each --native_workers count")
    args = p.parse_args(argv)
    from euler_amd.dataset import get_dataset

    dev = args.device or ("cuda" if torch.cuda.is_available() else "cpu")
    t0 = time.time()
    ds = get_dataset("ppi", data_dir=tempfile.mkdtemp(prefix="euler_amd_ppi_"), scale=args.scale)
    if args.mode == "remote":
        ds.partition_num = args.shards  # partition p is served by shard p % shards
    data_dir = ds.load_graph()
    procs = []
    if args.mode == "remote":
        import euler_amd as ea

        reg, procs = start_cluster(data_dir, args.shards, args.server_threads)
        ea.initialize_shared_graph(reg, shard_num=args.shards)
    print(f"[bench_engine_sage] ppi-schema graph scale {args.scale} ready in {time.time() - t0:.1f}s "
          f"({args.mode})", file=sys.stderr, flush=True)
    out = {}
    if args.pipeline_only:
        for w in args.native_workers:
            el = run_pipeline(ds, args, dev, w)
            out[f"pipeline_{w}workers"] = {"samples_per_s": round(args.batch * args.steps / el, 1),
                                           "ms_per_batch": round(el * 1e3 / args.steps, 2)}
            print(f"[bench_engine_sage] pipeline {w} workers: {out[f'pipeline_{w}workers']}", file=sys.stderr,
                  flush=True)
        for pr in procs:
            pr.terminate()
            pr.wait(timeout=30)
        best = max(out, key=lambda k: out[k]["samples_per_s"])
        print(json.dumps({"metric": "native input pipeline samples/sec (no model step)" + (
            ", graph on %d shard servers" % args.shards if args.mode == "remote" else ""),
            "value": out[best]["samples_per_s"], "unit": "samples/s", "steps": args.steps,
            "config": {"batch": args.batch, "fanouts": [10, 10], "mode": args.mode, "device": dev,
                       "shards": args.shards if args.mode == "remote" else 0, **out}}), flush=True)
        return
    variants = [("serial", 0, 1, False, False), ("py_prefetch_1worker", 2, 1, False, False)]
    variants += [("native_%dworkers_eager" % w, 0, w, True, False) for w in args.native_workers[:1]]
    # native pipeline + graph-captured step (the estimator default on a GPU)
    variants += [("native_%dworkers" % w, 0, w, True, "auto") for w in args.native_workers]
    if args.only:
        keep = set(args.only.split(","))
        variants = [v for v in variants if v[0] in keep]
    for name, pf, wk, nat, gr in variants:
        if args.cprofile:
            import cProfile
            import io
            import pstats

            pr = cProfile.Profile()
            pr.enable()
            el, res = run(ds, args, pf, dev, wk, nat, gr)
            pr.disable()
            buf = io.StringIO()
            pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(40)
            with open(args.cprofile, "a") as f:
                f.write(f"==== {name}\n{buf.getvalue()}\n")
        else:
            el, res = run(ds, args, pf, dev, wk, nat, gr)
        out[name] = {"samples_per_s": round(args.batch * args.steps / el, 1), "ms_per_step": round(el * 1e3 / args.steps, 2),
                     "loss": round(float(res.get("loss", float("nan"))), 4)}
        print(f"[bench_engine_sage] {name}: {out[name]}", file=sys.stderr, flush=True)
    for pr in procs:
        pr.terminate()
        pr.wait(timeout=30)
    best = max((k for k in out if k.startswith("native") and not k.endswith("eager")) or out, key=lambda k: out[k]["samples_per_s"])
    print(json.dumps({
        "metric": "train samples/sec, GraphSAGE via the C++ graph engine + estimator (reference architecture)"
                  + (", graph on %d shard servers" % args.shards if args.mode == "remote" else ""),
        "value": out[best]["samples_per_s"],   # the estimator default on a GPU: the native pipeline
        "unit": "samples/s",
        "n_gpus": 1 if dev == "cuda" else 0,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": out[best]["ms_per_step"],
        "higher_is_better": True,
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic PPI-schema graph (56,944 nodes, 50-d features, 121 labels)",
        "config": {"model": "SupervisedGraphSage [128, 128, 121], fanouts [10, 10], Adam", "batch": args.batch,
                   "scale": args.scale, "mode": args.mode, "shards": args.shards if args.mode == "remote" else 0,
                   **out},
    }), flush=True)


if __name__ == "__main__":
    main()
