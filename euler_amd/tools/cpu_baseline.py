"""Reference-equivalent CPU training path: the in-house baseline of BASELINE.md.

The reference publishes no throughput numbers, so BASELINE.md ("How the baseline will be
established", step 1) prescribes measuring the *reference's algorithm* on the MI355X
host CPUs: the same supervised GraphSAGE as ``bench.py`` run the way Euler-2.0 + TF run
it -- everything on the CPU:

* roots: global weighted node sampling in the C++ engine
  (reference ``tf_euler/python/euler_ops/sample_ops.py`` ``sample_node`` ->
  ``euler/core/graph/graph.cc:333-403``);
* 2 hops of weighted with-replacement neighbour sampling in the engine, ragged
  idx + flat result (reference ``sample_ops.py`` ``sample_fanout``,
  ``euler/core/kernels/sample_neighbor_op.cc``);
* dense feature lookup of every sampled node in the engine (reference
  ``feature_ops.py`` ``get_dense_feature``);
* CPU gather / segment-mean and dense linears in fp32 (reference
  ``tf_euler/python/mp_utils/base_graph.py`` + ``convolution/sage_conv.py``), sigmoid
  cross-entropy, Adam -- here torch CPU (oneDNN/MKL GEMMs), which is at least as fast as
  the TF-1.x CPU kernels the reference runs.

Identical synthetic graph config: same power-law degree law (avg 10, max 1024) with the
same number of nodes, 128-d N(0,1) features, labels = argmax of the first ``label_dim``
feature columns, fanouts [25, 10], 1024 roots per step, hidden 256, 64 classes.

``python -m euler_amd.tools.cpu_baseline --num-nodes 100000000 --threads 16`` prints one
JSON line; ``--out profiles/cpu_baseline.json`` stores it for ``bench.py``'s
``vs_baseline``.

Whole-node figure: a GPU box grants one GPU's share of the host (16 threads), so the run
measures that share and ``--sweep 4,8,16`` records how the path scales with threads.  The
reference would fill a whole node with independent data-parallel CPU workers, so
``value_node_linear`` = value x node_cores / threads (perfect linear scaling to every core
of the node — an upper bound for the CPU) is the denominator ``bench.py`` uses: the
reported ``vs_baseline`` is conservative.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--num-nodes", type=int, default=10_000_000)
    p.add_argument("--avg-degree", type=float, default=10.0)
    p.add_argument("--max-degree", type=int, default=1024)
    p.add_argument("--batch-size", type=int, default=1024)
    p.add_argument("--fanouts", type=str, default="25,10")
    p.add_argument("--feature-dim", type=int, default=128)
    p.add_argument("--hidden-dim", type=int, default=256)
    p.add_argument("--label-dim", type=int, default=64)
    p.add_argument("--lr", type=float, default=0.01)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--threads", type=int, default=16, help="CPU threads for the engine and torch")
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--out", type=str, default="", help="also write the JSON result to this file")
    p.add_argument("--node-cores", type=int, default=0, help="cores of the whole node (default os.cpu_count())")
    p.add_argument("--sweep", type=str, default="", help="also time these thread counts, e.g. 4,8,16")
    return p.parse_args(argv)


def build_model(feature_dim, hidden_dim, label_dim):
    import torch
    from torch import nn

    class SageMean(nn.Module):
        """SAGEConv(mean): relu(W [x_self | mean_k x_nbr_k])"""

        def __init__(self, din, dout):
            super().__init__()
            self.lin = nn.Linear(2 * din, dout, bias=False)

        def forward(self, x_self, x_nbr):  # [n, d], [n, k, d]
            return torch.relu(self.lin(torch.cat([x_self, x_nbr.mean(1)], 1)))

    class Model(nn.Module):
        def __init__(self):
            super().__init__()
            self.conv0 = SageMean(feature_dim, hidden_dim)
            self.conv1 = SageMean(hidden_dim, hidden_dim)
            self.fc = nn.Linear(hidden_dim, hidden_dim)
            self.out = nn.Linear(hidden_dim, label_dim, bias=False)

        def forward(self, x0, x1, x2, B, F1, F2):
            # hop 0 over (roots + level-1) targets, hop 1 over the roots
            d = x0.shape[1]
            h0 = self.conv0(x0, x1.view(B, F1, d))
            h1 = self.conv0(x1, x2.view(B * F1, F2, d))
            h = self.conv1(h0, h1.view(B, F1, -1))
            return self.out(self.fc(h))

    return Model()


def run(args) -> dict:
    import numpy as np
    import torch

    os.environ.setdefault("EULER_NUM_THREADS", str(args.threads))
    torch.set_num_threads(args.threads)
    from euler_amd.ops import base

    fanouts = [int(x) for x in args.fanouts.split(",")]
    F1, F2 = fanouts
    B = args.batch_size
    t0 = time.time()
    eng = base.synthetic_graph(args.num_nodes, args.avg_degree, args.max_degree, 1, 1, args.feature_dim,
                               args.label_dim, args.seed, make_current=False, out_only=True)
    build_s = time.time() - t0
    torch.manual_seed(args.seed)
    model = build_model(args.feature_dim, args.hidden_dim, args.label_dim)
    opt = torch.optim.Adam(model.parameters(), lr=args.lr)
    D, C = args.feature_dim, args.label_dim
    loss_val = [0.0]
    stage = {"sample": 0.0, "feature": 0.0, "compute": 0.0}

    def step():
        ta = time.perf_counter()
        roots = eng.sample_node(-1, B)
        nb1, _, _ = eng.sample_neighbor(roots, [], F1, np.uint64(args.num_nodes))
        nb2, _, _ = eng.sample_neighbor(nb1.reshape(-1), [], F2, np.uint64(args.num_nodes))
        tb = time.perf_counter()
        ids = np.concatenate([roots, nb1.reshape(-1), nb2.reshape(-1)])
        feats = torch.from_numpy(eng.dense_feature(ids, "dense_feature", D))
        labels = torch.from_numpy(eng.dense_feature(roots, "dense_label", C))
        tc = time.perf_counter()
        x0, x1, x2 = feats[:B], feats[B:B + B * F1], feats[B + B * F1:]
        logits = model(x0, x1, x2, B, F1, F2)
        loss = torch.nn.functional.binary_cross_entropy_with_logits(logits, labels)
        opt.zero_grad(set_to_none=False)
        loss.backward()
        opt.step()
        loss_val[0] = loss.item()
        td = time.perf_counter()
        stage["sample"] += tb - ta
        stage["feature"] += tc - tb
        stage["compute"] += td - tc

    for _ in range(args.warmup):
        step()
    first = loss_val[0]
    for k in stage:
        stage[k] = 0.0
    t1 = time.perf_counter()
    for _ in range(args.steps):
        step()
    el = time.perf_counter() - t1
    return {
        "metric": "train samples/sec (whole node), GraphSAGE 2-hop, reference-equivalent CPU path",
        "value": round(B * args.steps / el, 1),
        "unit": "samples/s",
        "ms_per_step": round(el * 1000 / args.steps, 3),
        "steps": args.steps,
        "warmup": args.warmup,
        "threads": args.threads,
        "dtype": "fp32",
        "data": "synthetic (engine power-law graph, N(0,1) features, argmax labels)",
        "config": {"num_nodes": args.num_nodes, "avg_degree": args.avg_degree, "max_degree": args.max_degree,
                   "batch_size": B, "fanouts": fanouts, "feature_dim": D, "hidden_dim": args.hidden_dim,
                   "label_dim": C, "graph_build_s": round(build_s, 1),
                   "stage_ms_per_step": {k: round(v * 1000 / args.steps, 3) for k, v in stage.items()},
                   "loss_first_last": [round(first, 4), round(loss_val[0], 4)]},
    }


def main(argv=None):
    args = parse_args(argv)
    sweep = {}
    if args.sweep:
        import subprocess

        given = sys.argv[1:] if argv is None else list(argv)
        keep, skip = [], False
        for x in given:  # the child gets every flag but --sweep / --out / --threads
            if skip:
                skip = False
                continue
            name = x.split("=", 1)[0]
            if name in ("--sweep", "--out", "--threads"):
                skip = "=" not in x
                continue
            keep.append(x)
        for t in [int(x) for x in args.sweep.split(",") if x]:
            if t == args.threads:
                continue
            # a fresh process per thread count (torch's intra-op pool is fixed at first use)
            a = keep
            out = subprocess.run([sys.executable, "-m", "euler_amd.tools.cpu_baseline", *a, "--threads", str(t)],
                                 capture_output=True, text=True, check=True).stdout.strip().splitlines()[-1]
            sweep[t] = json.loads(out)["value"]
    res = run(args)
    sweep[args.threads] = res["value"]
    cores = int(args.node_cores or os.cpu_count() or args.threads)
    res["node_cores"] = cores
    res["value_node_linear"] = round(res["value"] * cores / args.threads, 1)
    res["thread_sweep"] = {str(k): sweep[k] for k in sorted(sweep)}
    line = json.dumps(res)
    print(line, flush=True)
    if args.out:
        d = os.path.dirname(args.out)
        if d:
            os.makedirs(d, exist_ok=True)
        with open(args.out, "w") as f:
            f.write(line + "\n")
    return res


if __name__ == "__main__":
    sys.exit(0 if main() else 1)
