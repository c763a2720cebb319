#!/usr/bin/env python3
"""Engine -> HBM at scale: a graph in the Euler on-disk format loaded by the C++ engine and
uploaded to the GPU by ``DeviceGraph.from_engine`` — seconds, host memory and HBM, with one
rank and with data-parallel ranks sharing a node (the export then happens once: local rank
0 writes it to /dev/shm and every rank maps it, ``graph/device_graph.py shared_export``).

    python benchmarks/bench_upload.py --make /tmp/g10m --num-nodes 10000000      # write the data
    python benchmarks/bench_upload.py --data /tmp/g10m --ranks 1                  # W = 1
    python benchmarks/bench_upload.py --data /tmp/g10m --ranks 2                  # W = 2 (gloo, one GPU)

Each rank prints one JSON line: engine load seconds, upload seconds, the rank's private
(anonymous) host memory growth during the upload (sampled every 20 ms), its mapped shared
memory, and the HBM the graph takes.  Reference loader: euler/core/graph/graph.cc:72-120,
graph_builder.cc:57-158.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _status():
    out = {}
    with open("/proc/self/status") as f:
        for line in f:
            k, _, v = line.partition(":")
            if k in ("VmRSS", "RssAnon", "RssShmem", "RssFile", "VmHWM"):
                out[k] = int(v.split()[0]) / 2 ** 20  # GiB
    return out


class _Peak:
    """the peak of RssAnon / RssShmem while running (20 ms samples)"""

    def __init__(self):
        self.peak = _status()
        self._stop = False
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()

    def _run(self):
        while not self._stop:
            s = _status()
            for k, v in s.items():
                self.peak[k] = max(self.peak.get(k, 0.0), v)
            time.sleep(0.02)

    def stop(self):
        self._stop = True
        self._t.join()
        return self.peak


def make(args):
    import euler_amd as ea

    t0 = time.time()
    e = ea.synthetic_graph(args.num_nodes, args.avg_degree, args.max_degree, node_types=1, edge_types=1,
                           feature_dim=args.feature_dim, label_dim=args.label_dim, seed=7, make_current=False)
    t1 = time.time()
    e.save(args.make, partitions=args.partitions, threads=args.threads)
    t2 = time.time()
    size = sum(os.path.getsize(os.path.join(dp, f)) for dp, _, fs in os.walk(args.make) for f in fs)
    print(json.dumps({"phase": "make", "num_nodes": args.num_nodes, "build_s": round(t1 - t0, 1),
                      "save_s": round(t2 - t1, 1), "on_disk_gib": round(size / 2 ** 30, 2),
                      "partitions": args.partitions}), flush=True)


def upload(args):
    import torch

    import euler_amd as ea
    from euler_amd.graph.device_graph import DeviceGraph
    from euler_amd.parallel import dp

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    dp.init_distributed(backend="gloo", device=dev)  # shared-GPU rehearsal: every rank on cuda:0
    before_load = _status()
    t0 = time.time()
    if args.engine_shards:  # this rank's partitions only (p % W == rank)
        from euler_amd.ops.base import initialize_graph

        initialize_graph({"mode": "local", "data_path": args.data, "shard_idx": rank, "shard_num": world})
    else:
        ea.initialize_embedded_graph(args.data)
    load_s = time.time() - t0
    after_load = _status()
    if world > 1:
        dp.barrier()
    if dev.type == "cuda":
        torch.cuda.reset_peak_memory_stats(dev)
        base_hbm = torch.cuda.memory_allocated(dev)
    pk = _Peak()
    t1 = time.time()
    kw = dict(features=["feature"], feature_dims=[args.feature_dim], label="label", label_dim=args.label_dim,
              feature_dtype=torch.bfloat16, seed=1, device=dev)
    if args.engine_shards:
        from euler_amd.graph.sharded_graph import ShardedDeviceGraph

        sg = ShardedDeviceGraph.from_engine_shard(**kw)
        g = sg.local
    else:
        g = DeviceGraph.from_engine(share=world > 1, **kw)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    up_s = time.time() - t1
    peak = pk.stop()
    hbm = (torch.cuda.max_memory_allocated(dev) - base_hbm) / 2 ** 30 if dev.type == "cuda" else 0.0
    print(json.dumps({
        "phase": "upload", "rank": rank, "world": world, "num_nodes": g.num_rows, "num_edges": g.num_edges,
        "engine_load_s": round(load_s, 1), "engine_rss_gib": round(after_load["VmRSS"] - before_load["VmRSS"], 2),
        "upload_s": round(up_s, 1),
        "upload_private_peak_gib": round(peak["RssAnon"] - after_load["RssAnon"], 2),
        "upload_shared_mapped_peak_gib": round(peak.get("RssShmem", 0.0) - after_load.get("RssShmem", 0.0), 2),
        "hbm_peak_gib": round(hbm, 2), "graph_hbm_gib": round((g.nbytes() + g.features.numel() * 2) / 2 ** 30, 2),
        "shared_export": world > 1 and not args.engine_shards, "engine_shards": bool(args.engine_shards)}),
        flush=True)
    dp.barrier()


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--make", default=None, help="write a synthetic graph in the on-disk format to this dir")
    p.add_argument("--data", default=None, help="upload the graph in this dir")
    p.add_argument("--ranks", type=int, default=1)
    p.add_argument("--engine-shards", action="store_true",
                   help="every rank's engine loads only its partitions and uploads its rows of the row-sharded "
                        "graph (graph/sharded_graph.py from_engine_shard): host memory per rank 1/W")
    p.add_argument("--num-nodes", type=int, default=10_000_000)
    p.add_argument("--avg-degree", type=float, default=10.0)
    p.add_argument("--max-degree", type=int, default=1024)
    p.add_argument("--feature-dim", type=int, default=64)
    p.add_argument("--label-dim", type=int, default=16)
    p.add_argument("--partitions", type=int, default=8)
    p.add_argument("--threads", type=int, default=16)
    args = p.parse_args(argv)
    if args.make:
        return make(args)
    from euler_amd.parallel.launch import LAUNCHED_ENV, spawn_local

    if args.ranks > 1 and "RANK" not in os.environ and LAUNCHED_ENV not in os.environ:
        return spawn_local(args.ranks, sys.argv[1:], script=os.path.abspath(__file__))
    return upload(args)


if __name__ == "__main__":
    raise SystemExit(main())
