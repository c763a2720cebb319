"""Fused autograd pieces of the unsupervised GraphSAGE device step (models/sage_tower.py).

``tower_head``: layer 0 of a tower (TowerPlan: sample + gather + MFMA GEMM + tree mean)
followed by the last SAGE conv and the fc layer, as ONE autograd node on the tiled MFMA
GEMM (csrc/hip/gemm.hip: ReLU, bias and the ReLU-mask product fused as epilogues; the
[R]-row weight-gradient products split-K — hipBLASLt ran them on a handful of 256 x 128
tiles, 20-38 us per call in ``profiles/r3_unsup/``), whose backward writes every parameter
gradient straight into its flat-gradient view (``out=``), dA1 into the plan's buffer and
the routed layer-0 dW through the plan.  Nothing is accumulated, so the trainer never
zeroes the flat gradient (each step overwrites all of it).

``pair_loss``: the source / context dot products of the B positives and B*K negatives,
sigmoid cross-entropy (mean over the B + B*K logits, the reference's
``mp_utils/base.py:80-91``) and its gradient, one node with batched GEMMs.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


class _TowerHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, W0, W1, Wfc, bfc, tower):
        from euler_amd.ops.gnn_ops import gemm

        p = tower.plan
        p.shadow()
        p.sample()
        p.fwd()
        A1 = tower.A1.view(tower.R, 2 * tower.H0)  # bf16 rows [self | mean] from layer 0
        h1 = gemm(A1, W1, trans_b=True, relu=True)
        e = gemm(h1, Wfc, trans_b=True, bias=bfc)
        ctx.tower = tower
        ctx.params = (W1, Wfc, bfc)
        ctx.save_for_backward(A1, h1)
        return e

    @staticmethod
    def backward(ctx, de):
        from euler_amd.ops.gnn_ops import _gemm_splits, gemm

        A1, h1 = ctx.saved_tensors
        W1, Wfc, bfc = ctx.params
        t = ctx.tower
        de = de.contiguous()
        R = de.shape[0]
        # weight gradients: split-K over the R rows, written into the flat-gradient views
        gemm(de, h1, out=Wfc.grad, trans_a=True, splits=_gemm_splits(R, _tiles(Wfc)))
        torch.sum(de, 0, out=bfc.grad)
        dh1 = gemm(de, Wfc, rmask=h1)  # (de Wfc) * relu'(h1)
        gemm(dh1, A1, out=W1.grad, trans_a=True, splits=_gemm_splits(R, _tiles(W1)))
        gemm(dh1, W1, out=t.dA1.view(R, 2 * t.H0))
        t.plan.bwd()  # routed layer-0 dW, reduced into the W0 gradient view
        return None, None, None, None, None


def _tiles(w):
    return -(-w.shape[0] // 64) * -(-w.shape[1] // 64)


def tower_head(W0, W1, Wfc, bfc, tower):
    """fc output rows [R, E] of a tower (see module docstring); every parameter's gradient
    view (``.grad`` of W1 / Wfc / bfc, the plan's W0 gradient buffer) is overwritten by the
    backward."""
    return _TowerHead.apply(W0, W1, Wfc, bfc, tower)


class _PairLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, es, ec, B, K):
        # context rows: the B positives, then the B x K negatives (source-major)
        ecv = torch.cat([ec[:B].unsqueeze(1), ec[B:].view(B, K, -1)], 1)  # [B, 1 + K, E]
        logits = torch.bmm(ecv, es.unsqueeze(2)).squeeze(2)               # [B, 1 + K]
        n = logits.numel()
        # sigmoid CE: softplus(x) - x * y, y = 1 for the positive column
        loss = (F.softplus(logits).sum() - logits[:, 0].sum()) / n
        ctx.save_for_backward(es, ecv, logits)
        ctx.B, ctx.K, ctx.n = B, K, n
        out = logits.detach()
        ctx.mark_non_differentiable(out)
        return loss, out

    @staticmethod
    def backward(ctx, dloss, _dlogits):
        es, ecv, logits = ctx.saved_tensors
        B, K, n = ctx.B, ctx.K, ctx.n
        g = torch.sigmoid(logits)
        g[:, 0] -= 1.0
        g.mul_(dloss / n)                                                  # dloss/dlogit [B, 1 + K]
        des = torch.bmm(g.unsqueeze(1), ecv).squeeze(1)                   # [B, E]
        decv = g.unsqueeze(2) * es.unsqueeze(1)                           # [B, 1 + K, E]
        dec = torch.cat([decv[:, 0], decv[:, 1:].reshape(B * K, -1)], 0)  # context row order
        return des, dec, None, None


def pair_loss(es, ec, B, K):
    """(loss, logits [B, 1 + K] with the positive first) of the unsupervised objective"""
    return _PairLoss.apply(es, ec, B, K)
