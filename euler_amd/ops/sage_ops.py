"""Fused fixed-fanout aggregate + linear (GraphSAGE/GCN hot path).

``sage_layer(x, self_idx, nbr_idx, weight, bias, include_self, relu)`` computes

    A   = [ x[self_idx] | mean_k( x[nbr_idx[:, k]] (+ x[self_idx]) ) ]    # [M, 2D]
    out = act(A @ weight.T + bias)                                       # [M, H]

i.e. ``SAGEConv.apply_node(scatter_mean(gather(x)))`` of the reference
(``tf_euler/python/convolution/sage_conv.py:33-44``) with ``weight = [W_self | W_neigh]``.
Padding neighbors are ``-1`` (zero rows, still counted — like the reference's
zero-feature ``default_node``).

GPU: one gfx950 kernel for the forward (LDS-staged gather + MFMA GEMM,
``csrc/hip/sage.hip``); backward = ReLU mask kernel + two hipBLASLt GEMMs +
an index-routing kernel (``disjoint=True`` when every input row is used at most
once — tree-layout blocks — gives plain stores, no atomics).
CPU: the same math in eager torch (the numerics oracle).
"""
from __future__ import annotations

import torch

from euler_amd.ops._native import hip, use_hip

__all__ = ["sage_layer", "sage_layer_reference"]


def sage_layer_reference(x, self_idx, nbr_idx, weight, bias=None, include_self=False, relu=True):
    """Eager-torch definition (fp32 accumulation)."""
    xf = x.float()
    zero = torch.zeros(1, x.shape[1], dtype=xf.dtype, device=x.device)
    xz = torch.cat([xf, zero], 0)  # row -1 -> zero row
    n = x.shape[0]
    si = self_idx.long().clone()
    si[si < 0] = n
    ni = nbr_idx.long().clone()
    ni[ni < 0] = n
    xs = xz[si]
    agg = xz[ni].sum(1)
    cnt = nbr_idx.shape[1]
    if include_self:
        agg = agg + xs
        cnt += 1
    agg = agg / float(max(cnt, 1))
    a = torch.cat([xs, agg], 1)
    out = a @ weight.float().t()
    if bias is not None:
        out = out + bias.float()
    if relu:
        out = torch.relu(out)
    return out


class _SageFused(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, self_idx, nbr_idx, include_self, relu, disjoint):
        wb = weight.to(torch.bfloat16).contiguous()
        out, a = hip().sage_fwd(x.contiguous(), self_idx, nbr_idx, wb,
                                None if bias is None else bias.float().contiguous(),
                                bool(include_self), bool(relu), True)
        ctx.include_self, ctx.relu, ctx.disjoint = include_self, relu, disjoint
        ctx.n_in, ctx.has_bias = x.shape[0], bias is not None
        ctx.wdtype = weight.dtype
        ctx.save_for_backward(a, out, wb, self_idx, nbr_idx)
        return out

    @staticmethod
    def backward(ctx, g):
        a, out, wb, self_idx, nbr_idx = ctx.saved_tensors
        g = g.to(torch.bfloat16).contiguous()
        if ctx.relu:
            g = g.clone()
            hip().relu_bwd_(g, out)
        from euler_amd.ops.gnn_ops import splitk_mm_t

        dw = splitk_mm_t(g, a).to(ctx.wdtype)  # split-K: M rows over many workgroups
        db = g.float().sum(0) if ctx.has_bias else None
        dx = None
        if ctx.needs_input_grad[0]:
            da = torch.mm(g, wb)  # [M, 2D] bf16
            D = a.shape[1] // 2
            dxf = torch.zeros((ctx.n_in, D), dtype=torch.float32, device=g.device)
            hip().sage_bwd_scatter(da, self_idx, nbr_idx, bool(ctx.include_self), bool(ctx.disjoint), dxf)
            dx = dxf.to(torch.bfloat16)
        return dx, dw, db, None, None, None, None, None


def sage_layer(x, self_idx, nbr_idx, weight, bias=None, include_self=False, relu=True, disjoint=False):
    """Fused SAGE layer.  ``x`` bf16 [N, D] (GPU) or any float (CPU)."""
    if use_hip(x, weight) and x.dtype == torch.bfloat16 and x.shape[1] % 16 == 0 and x.shape[1] <= 512:
        si = self_idx if self_idx.dtype == torch.int32 else self_idx.int()
        ni = nbr_idx if nbr_idx.dtype == torch.int32 else nbr_idx.int()
        return _SageFused.apply(x, weight, bias, si.contiguous(), ni.contiguous(), include_self, relu, disjoint)
    out = sage_layer_reference(x, self_idx, nbr_idx, weight, bias, include_self, relu)
    return out.to(x.dtype) if x.is_floating_point() else out
