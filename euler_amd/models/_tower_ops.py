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

import os

import torch
import torch.nn.functional as F


# products of the tower heads: "gemm" = the tiled MFMA kernel (gemm.hip), "torch" = torch
# matmuls (hipBLASLt; fp32 A1); "mixed" = the kernel for the row-parallel products, torch
# for the [R]-row weight-gradient reductions
_HEAD_GEMM = os.environ.get("EULER_AMD_TOWER_GEMM", "gemm")


def _mm(a, b, out=None, trans_a=False, trans_b=False, relu=False, bias=None, rmask=None, wgrad=False):
    from euler_amd.ops.gnn_ops import _gemm_splits, gemm

    use = _HEAD_GEMM == "gemm" or (_HEAD_GEMM == "mixed" and not wgrad)
    if use:
        splits = 1
        if wgrad:
            M, N = (a.shape[1] if trans_a else a.shape[0]), (b.shape[0] if trans_b else b.shape[1])
            splits = _gemm_splits(a.shape[0], -(-M // 64) * -(-N // 64))
        return gemm(a, b, out=out, trans_a=trans_a, trans_b=trans_b, relu=relu, bias=bias, rmask=rmask,
                    splits=splits)
    A = (a.t() if trans_a else a).float()
    B = (b.t() if trans_b else b).float()
    y = torch.addmm(bias, A, B) if bias is not None else A @ B
    if relu:
        y = torch.relu_(y)
    if rmask is not None:
        y = torch.ops.aten.threshold_backward(y, rmask, 0.0)
    if out is None:
        return y
    out.copy_(y)
    return out


class _TowerHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, W0, W1, Wfc, bfc, tower):
        p = tower.plan
        p.shadow()
        p.sample()
        p.fwd()
        A1 = tower.A1.view(tower.R, 2 * tower.H0)  # bf16 rows [self | mean] from layer 0
        h1 = _mm(A1, W1, trans_b=True, relu=True)
        e = _mm(h1, Wfc, trans_b=True, bias=bfc)
        ctx.tower = tower
        ctx.params = (W1, Wfc, bfc)
        ctx.save_for_backward(A1, h1)
        return e

    @staticmethod
    def backward(ctx, de):
        A1, h1 = ctx.saved_tensors
        W1, Wfc, bfc = ctx.params
        t = ctx.tower
        de = de.contiguous()
        R = de.shape[0]
        # weight gradients (reductions over the R rows) written into the flat-gradient views
        _mm(de, h1, out=Wfc.grad, trans_a=True, wgrad=True)
        torch.sum(de, 0, out=bfc.grad)
        dh1 = _mm(de, Wfc, rmask=h1)  # (de Wfc) * relu'(h1)
        _mm(dh1, A1, out=W1.grad, trans_a=True, wgrad=True)
        _mm(dh1, W1, out=t.dA1.view(R, 2 * t.H0))
        t.plan.bwd()  # routed layer-0 dW, reduced into the W0 gradient view
        return None, None, None, None, None


def tower_head(W0, W1, Wfc, bfc, tower):
    """fc output rows [R, E] of a tower (see module docstring); every parameter's gradient
    view (``.grad`` of W1 / Wfc / bfc, the plan's W0 gradient buffer) is overwritten by the
    backward."""
    return _TowerHead.apply(W0, W1, Wfc, bfc, tower)


class _PairLossFused(torch.autograd.Function):
    """csrc/hip/pair.hip: logits + softplus CE + reciprocal ranks in one launch, the
    closed-form gradient in another (the torch composition below is ~20 launches)"""

    @staticmethod
    def forward(ctx, es, ec, B, K, mrr):
        from euler_amd.ops._native import hip

        es, ec = es.contiguous(), ec.contiguous()
        logits, loss = hip().pair_fwd(es, ec, B, K, mrr)
        ctx.save_for_backward(es, ec, logits)
        ctx.B, ctx.K = B, K
        ctx.mark_non_differentiable(logits)
        return loss, logits

    @staticmethod
    def backward(ctx, dloss, _dlogits):
        from euler_amd.ops._native import hip

        es, ec, logits = ctx.saved_tensors
        des, dec = torch.empty_like(es), torch.empty_like(ec)
        hip().pair_bwd(es, ec, ctx.B, ctx.K, logits, dloss.float().reshape(1).contiguous(), des, dec)
        return des, dec, None, None, None


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


def pair_loss(es, ec, B, K, mrr_out=None):
    """(loss, logits [B, 1 + K] with the positive first) of the unsupervised objective.
    ``mrr_out`` (fp32 [1]): the fused kernel adds the batch's reciprocal ranks of the
    positives to it; returns ``(loss, logits, True)`` when it did (else False)."""
    D = es.shape[1]
    if (_PAIR_FUSED and es.is_cuda and es.dtype == torch.float32 and ec.dtype == torch.float32 and D % 4 == 0
            and D <= 256 and 0 <= K <= 15):
        loss, logits = _PairLossFused.apply(es, ec, B, K, mrr_out)
        return loss, logits, mrr_out is not None
    loss, logits = _PairLoss.apply(es, ec, B, K)
    return loss, logits, False


_PAIR_FUSED = os.environ.get("EULER_AMD_PAIR_FUSED", "1") == "1"
