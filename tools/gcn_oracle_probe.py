#!/usr/bin/env python3
"""Where the fused GCN step's gradient error against fp32 autograd comes from: the same
comparison as tests/test_gcn_trainer.py, plus a reference whose operands (features,
weights) are rounded to bf16 first.  Usage (GPU box): python tools/gcn_oracle_probe.py"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gcn_trainer import _graph, _materialize, _setup  # noqa: E402


def main():
    from euler_amd.models.full_trainer import FullFlowTrainer
    from euler_amd.models.gcn_trainer import GcnTrainer

    for layers, loops in ((1, False), (1, True), (2, False)):
        B = 64
        m = _setup("cuda", layers, loops, B).to("cuda")
        g = _graph(m, "cuda")
        _materialize(m, g, B)
        tr = GcnTrainer.from_model(m, g, B, caps="exact")
        rng = g.rng.clone()
        agg_k = tr.plan.head_aggregates()  # one step with the aggregates written out
        g.rng.copy_(rng)  # the same roots again (the epoch stamp moves on: fresh node tables)
        for p in m.parameters():
            if p.grad is not None:
                p.grad.zero_()
        tr.forward_backward_only()  # the same draw again: the gradients compared below
        torch.cuda.synchronize()
        gk = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
        roots = tr.plan.flow()["roots"].long().clone()
        for mode in ("fp32", "bf16 operands"):
            ref = FullFlowTrainer.from_model(m, g, B, caps="exact")
            saved = None
            if mode != "fp32":
                saved = [p.detach().clone() for p in m.parameters()]
                with torch.no_grad():
                    for p in m.parameters():
                        p.copy_(p.bfloat16().float())
                    ref.features = ref.features.bfloat16().float()
            for p in m.parameters():
                p.grad = None
            cap = {}
            fc0 = m.gnn.convs[-1].fc  # the conv the head computes (its dW is the head's)
            h1 = fc0.register_forward_hook(lambda mod, i, o: cap.__setitem__("inp", i[0].detach()))
            h2 = fc0.register_full_backward_hook(lambda mod, gi, go: cap.__setitem__("go", go[0].detach()))
            logits, _ = ref._forward(roots)
            F.binary_cross_entropy_with_logits(logits, g.labels[roots].float()).backward()
            h1.remove()
            h2.remove()
            if "inp" in cap and layers == 1:
                xr = cap["inp"].float()
                xk = agg_k[:, : xr.shape[1]]
                rowerr = (xk - xr).norm(dim=1) / xr.norm(dim=1).clamp(min=1e-9)
                bad = torch.nonzero(rowerr > 1e-3).reshape(-1).tolist()
                fl = tr.plan.flow()
                deg = (fl["hops"][0]["off"][1:B + 1] - fl["hops"][0]["off"][:B]).tolist()
                print(f"  aggregates: max row error {float(rowerr.max()):.4g}; rows off {bad[:12]} "
                      f"(their in-block degree {[deg[i] for i in bad[:12]]}, roots "
                      f"{[int(roots[i]) for i in bad[:12]]}, repeated roots "
                      f"{int(roots.numel() - roots.unique().numel())})", flush=True)
            if "inp" in cap and "go" in cap:
                x, d = cap["inp"].float(), cap["go"].float()
                x = x.reshape(-1, x.shape[-1])
                d = d.reshape(-1, d.shape[-1])
                dw = d.t() @ x
                dwb = d.bfloat16().float().t() @ x.bfloat16().float()
                cancel = float((d.abs().t() @ x.abs()).norm() / dw.norm().clamp(min=1e-12))
                print(f"  last conv dW: bf16(dz)^T bf16(agg) vs fp32 {float((dwb - dw).norm() / dw.norm()):.5f}, "
                      f"cancellation |dz|^T|agg| / |dW| = {cancel:.1f}", flush=True)
            errs = {n: round(float((gk[n] - p.grad).norm() / p.grad.norm().clamp(min=1e-12)), 5)
                    for n, p in m.named_parameters()}
            wn = f"gnn.convs.{layers - 1}.fc.weight"
            ref_w = dict(m.named_parameters())[wn].grad
            dd = (gk[wn] - ref_w)
            rows = (dd.norm(dim=1) / ref_w.norm(dim=1).clamp(min=1e-12))
            cols = (dd.norm(dim=0) / ref_w.norm(dim=0).clamp(min=1e-12))
            print(f"  {wn} error by output row (top 6): {[(int(i), round(float(rows[i]), 4)) for i in rows.argsort(descending=True)[:6]]}"
                  f"; by input column (top 6): {[(int(i), round(float(cols[i]), 4)) for i in cols.argsort(descending=True)[:6]]}",
                  flush=True)
            print(f"layers={layers} self_loops={loops} reference={mode}: {errs}", flush=True)
            if saved is not None:
                with torch.no_grad():
                    for p, s in zip(m.parameters(), saved):
                        p.copy_(s)


if __name__ == "__main__":
    main()
