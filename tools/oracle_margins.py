#!/usr/bin/env python3
"""Worst relative errors of the fused kernels against their bf16-aware fp32 oracles
(SageTrainer.reference_loss_and_grads_bf16 over the 15 tree cases of
tests/test_sage_trainer.py, GcnTrainer.reference_loss_and_grads_bf16 for L = 1, 2 with and
without self loops), and against the plain fp32 model for comparison.  GPU box only."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def rel(a, b):
    a, b = a.float().reshape(-1).cpu(), b.float().reshape(-1).cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-12))


def sage():
    from test_sage_trainer import CASES, _trainer

    out = []
    for i, cfg in enumerate(CASES):
        tr = _trainer("cuda", **cfg)
        tr.forward_backward()
        torch.cuda.synchronize()
        lk, gk = float(tr.loss_acc.item()), tr.gradients()
        lb, gb = tr.reference_loss_and_grads_bf16()
        lr_, gr = tr.reference_loss_and_grads()
        out.append({"case": i, "loss_rel_bf16": abs(lk - lb) / abs(lb), "grad_rel_bf16": max(rel(gk[k], gb[k]) for k in gb),
                    "loss_rel_fp32": abs(lk - lr_) / abs(lr_), "grad_rel_fp32": max(rel(gk[k], gr[k]) for k in gr)})
    return out


def gcn():
    from test_gcn_trainer import _graph, _materialize, _setup
    from euler_amd.models.gcn_trainer import GcnTrainer

    out = []
    for layers, sl in ((2, False), (2, True), (1, False), (1, True)):
        m = _setup("cuda", layers, sl, 64).to("cuda")
        g = _graph(m, "cuda")
        _materialize(m, g, 64)
        tr = GcnTrainer.from_model(m, g, 64, caps="exact")
        lk = float(tr.forward_backward_only())
        torch.cuda.synchronize()
        gk = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
        lb, gb = tr.reference_loss_and_grads_bf16()
        out.append({"layers": layers, "self_loops": sl, "loss_rel_bf16": abs(lk - lb) / abs(lb),
                    "grad_rel_bf16": {n: rel(gk[n], r) for n, r in gb.items()}})
    return out


if __name__ == "__main__":
    print(json.dumps({"sage_tree": sage(), "gcn": gcn()}, indent=1))
