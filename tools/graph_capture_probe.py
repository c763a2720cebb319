#!/usr/bin/env python3
"""Capture one piece of the engine-path training step into a hipGraph and replay it.

Usage: python tools/graph_capture_probe.py --stage {adam,fwd,bwd,full}
  adam  fused capturable Adam over random grads
  fwd   model forward + loss over the static native-pipeline inputs
  bwd   forward + backward
  full  forward + backward + Adam (the estimator's captured step)
  est   NodeEstimator.train with the graph-captured step (as tests/test_native_pipeline.py)
  est2  an eager estimator run, then the graph-captured one, in one process
Run the stages as separate processes, least to most complete, chained with &&.
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stage", required=True, choices=["adam", "fwd", "bwd", "full", "est", "est2", "est3"])
    args = ap.parse_args()
    dev = torch.device("cuda")
    if args.stage == "adam":
        ps = [torch.nn.Parameter(torch.randn(64, 64, device=dev)) for _ in range(3)]
        opt = torch.optim.Adam(ps, lr=1e-2, fused=True, capturable=True)
        for p in ps:
            p.grad = torch.randn_like(p)
        opt.step()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            opt.step()
        g.replay()
        torch.cuda.synchronize()
        print("adam ok", flush=True)
        return
    import euler_amd as ea
    from euler_amd import models as Z
    from euler_amd.dataflow.native_loader import NativeSageLoader

    N, FD, LD = 5000, 50, 16
    ea.synthetic_graph(N, 8.0, 64, 1, 1, FD, LD, seed=3)
    if args.stage.startswith("est"):
        import logging
        import tempfile

        from euler_amd.estimator import NodeEstimator

        logging.basicConfig(level=logging.INFO)
        modes = {"est": [True], "est2": [False, True], "est3": [False, False, True, True]}[args.stage]
        finals = []
        for graph in modes:
            ea.set_seed(2)
            torch.manual_seed(0)
            m = Z.SupervisedGraphSage([32, 32, LD], [6, 4], [["0"], ["0"]], "feature", FD, "label", LD,
                                      max_id=N - 1)
            params = {"model_dir": tempfile.mkdtemp(), "batch_size": 64, "total_step": int(os.environ.get("PROBE_STEPS", "20")), "optimizer": "adam",
                      "learning_rate": 0.01, "log_steps": 1, "train_node_type": -1, "device": "cuda", "seed": 4,
                      "native_pipeline": True, "pipeline_workers": 2, "cuda_graph": graph}
            print("graph", graph, NodeEstimator(m, params).train(), flush=True)
            finals.append((graph, {k: v.detach().float().clone() for k, v in m.state_dict().items()}))
        cos = torch.nn.functional.cosine_similarity
        for i in range(1, len(finals)):
            print("run0 vs run%d (graph=%s):" % (i, finals[i][0]), {
                k: round(float(cos(v.reshape(-1), finals[i][1][k].reshape(-1), dim=0)), 5)
                for k, v in finals[0][1].items() if v.numel() > 1}, flush=True)
        return
    torch.manual_seed(0)
    m = Z.SupervisedGraphSage([32, 32, LD], [6, 4], [["0"], ["0"]], "feature", FD, "label", LD, max_id=N - 1)
    ld = NativeSageLoader(m.gnn.sampler, ["feature"], [FD], "label", LD, 64, -1, dev, workers=2, seed=5, static=True)
    src = ld.get()
    m.to(dev)
    with torch.no_grad():
        m(torch.arange(64))  # materialise the lazy layers (generic path, raw roots)
    m.to(dev)
    opt = torch.optim.Adam(m.parameters(), lr=1e-2, fused=True, capturable=True)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            _, loss, _, _ = m(src)
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    print("eager warm ok", flush=True)
    opt.zero_grad(set_to_none=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        _, loss, _, _ = m(src)
        if args.stage in ("bwd", "full"):
            loss.backward()
        if args.stage == "full":
            opt.step()
    print("captured", flush=True)
    for _ in range(3):
        ld.get()
        g.replay()
    torch.cuda.synchronize()
    print(args.stage, "ok loss", float(loss), flush=True)
    ld.close()


if __name__ == "__main__":
    main()
