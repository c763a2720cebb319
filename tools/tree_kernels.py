#!/usr/bin/env python3
"""Per-kernel timing of the SageTrainer step (csrc/hip/sage_tree.hip) at the bench shape.

Times every launch of the step on its own (CUDA events over ``--reps`` back-to-back
launches) and the whole captured step, and prints the head kernel's per-phase
wall-clock stamps.  Usage (GPU box):
    python tools/tree_kernels.py [--num-nodes 10000000] [--batch-size 1024] [--reps 50]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / reps  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--num-nodes", type=int, default=10_000_000)
    ap.add_argument("--batch-size", type=int, default=1024)
    ap.add_argument("--fanouts", default="25,10")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--feature-dtype", default="bf16")
    args = ap.parse_args()
    from euler_amd.graph.device_graph import DeviceGraph
    from euler_amd.dataset.synthetic import synthetic_features, synthetic_labels
    from euler_amd.models.sage_trainer import SageTrainer

    dev = torch.device("cuda", 0)
    fan = [int(x) for x in args.fanouts.split(",")]
    g = DeviceGraph.synthetic(args.num_nodes, 9.5, 256, seed=1234, device=dev)
    fdt = torch.bfloat16 if args.feature_dtype == "bf16" else torch.float32
    x = synthetic_features(args.num_nodes, 128, 1235, dev, dtype=fdt)
    y = synthetic_labels(x, 64)
    tr = SageTrainer(g, args.batch_size, fan, [256] * (len(fan) + 1), 64, features=x, labels=y,
                     learning_rate=0.01, init_seed=1234, keep_samples=False)
    p = tr.plan
    for _ in range(3):
        tr.step()
    torch.cuda.synchronize()
    res = {}
    for name, fn in tr.plan_launches():
        res[name] = round(timeit(fn, args.reps), 2)
    res["sum"] = round(sum(v for k, v in res.items() if k not in ("sample", "head")), 2)
    for i in range(p.num_problems()):
        res[f"dw[{i}]"] = round(timeit(lambda: p.dw([i]), args.reps), 2)
    res["dw_splits"] = p.splits()
    res["route_profile"] = route_profile(tr)
    tr.capture(steps=4)
    res["graph_step"] = round(timeit(lambda: tr.replay(1), args.reps), 2)
    res["graph_step_x4"] = round(timeit(lambda: tr.replay_steps(4), args.reps) / 4, 2)  # per step
    print(json.dumps(res))
    if hasattr(p, "head"):
        rows = torch.ops  # noqa: F841
        hr = __import__("euler_amd.ops._native", fromlist=["hip"]).hip().tree_head_rows
        prof = torch.zeros((args.batch_size // hr) * 8, dtype=torch.int64, device=dev)
        p.head(prof)
        torch.cuda.synchronize()
        t = prof.view(-1, 8).cpu().double() / 100.0
        t0 = t[:, 0].min()
        ph = [(t[:, k] - t[:, k - 1]).mean().item() for k in range(1, 8)]
        nb = p.fwd_blocks()
        fprof = torch.zeros(nb * 8, dtype=torch.int64, device=dev)
        p.fwd(fprof)
        torch.cuda.synchronize()
        f = fprof.view(-1, 8).cpu().double() / 100.0
        raw = fprof.view(-1, 8).cpu()
        live = raw[:, 0] > 0
        f = f[live]  # blocks of the launched kernel (64-row tiles: half the 32-row count)
        cu = raw[live, 6]
        last = 5  # stamps 0..5: ids / gather / kt / gemm / epilogue (slot 6: the CU id)
        st = (f[:, 0] - f[:, 0].min())
        uniq, cnt = torch.unique(cu, return_counts=True)
        print("fwd blocks", int(live.sum()), "distinct CUs", int(uniq.numel()), "max blocks per CU", int(cnt.max()),
              "start-time percentiles (us) 50/90/99/max",
              [round(float(torch.quantile(st, q)), 2) for q in (0.5, 0.9, 0.99)], round(float(st.max()), 2),
              "end-time spread (us)", round(float((f[:, last] - f[:, last].min()).max()), 2))
        f0 = f[:, 0].min()
        names = "ids, gather, kt, gemm, epilogue"
        fph = [(f[:, k] - f[:, k - 1]).mean().item() for k in range(1, last + 1)]
        print(f"fwd phases (us, mean over blocks: {names}):", [round(v, 2) for v in fph],
              "span", round(float(f[:, last].max() - f0), 2), "start skew", round(float(f[:, 0].max() - f0), 2),
              "block time", round(float((f[:, last] - f[:, 0]).mean()), 2))
        print("head phases (us, mean over blocks):", [round(v, 2) for v in ph],
              "span", round(float(t[:, 7].max() - t0), 2), "start skew", round(float(t[:, 0].max() - t0), 2))


def route_profile(tr, reps=3):
    """wall-clock stamps of the routed dW blocks (problem 0): start, progress points, end"""
    p = tr.plan
    nb = p.route_blocks(0)
    if nb == 0:
        return None
    prof = torch.zeros(nb * 8, dtype=torch.int64, device=tr.device)
    for _ in range(reps):
        prof.zero_()
        p.dw([0], prof)
    torch.cuda.synchronize()
    t = prof.view(-1, 8).cpu().double() / 100.0  # wall_clock64 = 100 MHz
    t0 = t[:, 0].min()
    out = {"blocks": nb, "start_skew_us": round(float(t[:, 0].max() - t0), 2),
           "span_us": round(float(t[:, 7].max() - t0), 2),
           "block_time_mean_us": round(float((t[:, 7] - t[:, 0]).mean()), 2),
           "block_time_max_us": round(float((t[:, 7] - t[:, 0]).max()), 2)}
    prog = []
    prev = t[:, 0]
    for k in range(1, 7):
        col = t[:, k]
        ok = col > 0
        if not bool(ok.any()):
            break
        prog.append(round(float((col[ok] - prev[ok]).mean()), 2))
        prev = torch.where(ok, col, prev)
    out["progress_deltas_us"] = prog
    out["tail_us"] = round(float((t[:, 7] - prev).mean()), 2)
    return out


if __name__ == "__main__":
    main()
