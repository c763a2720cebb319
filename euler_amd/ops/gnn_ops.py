"""Fused GNN / embedding ops on the gfx950 kernels.

=====================  ==========================================  =================================
op                     replaces (reference)                        kernel
=====================  ==========================================  =================================
``gat_aggregate``      GATConv logits + scatter_softmax + gather   ``gat.hip`` (online softmax, one
                       + scatter_add (gat_conv.py:41-78,            pass per destination; backward:
                       mp_ops.py:76-79), one conv per head          destination + source passes)
``relation_transform`` RelationConv per-edge [dim, fea] matmul      ``rgcn.hip`` (relation-grouped
                       (relation_conv.py:63-70)                     MFMA GEMM, gather in prologue)
``sgns_loss``          matmul + 2x sigmoid-CE + concat + mean       ``embed.hip`` sgns_fwd / sgns_bwd
                       (mp_utils/base.py:80-91)
``kg_score``           4 lookups + 4 l2-normalise + TransE/         ``embed.hip`` kg_fwd / kg_bwd
                       DistMult score (transX.py:72-145)
``unique_first``       tf.unique (first-occurrence order)           ``unique.hip`` (hash table)
=====================  ==========================================  =================================

GPU tensors always take the kernel path (``use_hip``); CPU tensors take a plain torch
composition of the same math, which is also the numerics oracle in the tests.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from euler_amd.ops._native import engine, hip, use_hip
from euler_amd.ops.mp_ops import SegmentIndex

__all__ = ["EdgeCSR", "gat_aggregate", "gat_aggregate_reference", "RelationTiles", "relation_transform",
           "relation_transform_reference", "sgns_loss", "sgns_loss_reference", "kg_score", "kg_score_reference",
           "unique_first", "unique_first_padded", "KG_KINDS", "KG_CORRUPT", "sgns_fwd_idx", "occ_csr", "sgns_grad", "tall_linear", "xent",
           "splitk_mm_t", "splitk_linear"]


# ----------------------------------------------------------------------------- edge structures
class EdgeCSR:
    """Destination CSR + source CSC of an ``edge_index`` ([2, E]: row 0 = destination,
    row 1 = source), with int32 neighbour columns, built once and reused by forward and
    backward.  Edges with a negative endpoint (padding) are dropped."""

    def __init__(self, edge_index: torch.Tensor, size):
        self.edge_index = edge_index
        self.n_dst, self.n_src = int(size[0]), int(size[1])
        self._csr = None
        self._csc = None

    @classmethod
    def from_csr(cls, indptr: torch.Tensor, col: torch.Tensor, n_src: int) -> "EdgeCSR":
        """From an existing destination CSR (e.g. a resident full graph): no sort for the
        forward; the source CSC is built on first backward."""
        n_dst = indptr.numel() - 1
        dst = torch.repeat_interleave(torch.arange(n_dst, device=indptr.device, dtype=torch.int32),
                                      torch.diff(indptr))
        obj = cls(torch.stack([dst, col.to(torch.int32)]), (n_dst, n_src))
        obj._csr = (indptr.to(torch.int64).contiguous(), col.to(torch.int32).contiguous())
        return obj

    def csr(self):
        if self._csr is None:
            # the block's destination CSR when its producer cached one (dataflow/device_flow.py)
            seg = _cached_segment(self.edge_index, 0, self.n_dst)
            col = self.edge_index[1].long()[seg.perm].to(torch.int32)
            self._csr = (seg.indptr, col.contiguous())
        return self._csr

    def csc(self):
        if self._csc is None:
            seg = _cached_segment(self.edge_index, 1, self.n_src)
            row = self.edge_index[0].long()[seg.perm].to(torch.int32)
            self._csc = (seg.indptr, row.contiguous())
        return self._csc

    def _by_degree(self, indptr):
        # longest rows first: the rows sharing a wave have similar lengths and the
        # heaviest work starts first (cdna_hip_programming.md App. B, skewed gathers)
        if os.environ.get("EULER_AMD_GAT_ORDER", "1") == "0":
            return None
        # (a bit-limited radix sort of E - degree measured slower here: its count and scan
        # run over E + 1 key values, more than the rows an argsort orders)
        return torch.argsort(torch.diff(indptr), descending=True).to(torch.int32).contiguous()

    def csr_order(self):
        if getattr(self, "_csr_order", None) is None:
            self._csr_order = self._by_degree(self.csr()[0])
        return self._csr_order

    def csc_order(self):
        if getattr(self, "_csc_order", None) is None:
            self._csc_order = self._by_degree(self.csc()[0])
        return self._csc_order


def _cached_segment(edge_index, i, size):
    from euler_amd.ops.mp_ops import cached_segment

    return cached_segment(edge_index, i, size)


def _cached(edge_index, key, build):
    cache = getattr(edge_index, "_euler_cache", None)
    if cache is None:
        cache = {}
        try:
            edge_index._euler_cache = cache
        except AttributeError:
            return build()
    if key not in cache:
        cache[key] = build()
    return cache[key]


def edge_csr(edge_index, size) -> EdgeCSR:
    return _cached(edge_index, "_euler_csr_%d_%d" % (int(size[0]), int(size[1])), lambda: EdgeCSR(edge_index, size))


# ----------------------------------------------------------------------------- K5 GAT
def gat_aggregate_reference(h, al, ar, edge_index, size, slope=0.2):
    """Plain torch: per-head softmax over each destination's in-edges, weighted sum of
    the source rows.  h [N_src, H, C], al [N_src, H], ar [N_dst, H] -> [N_dst, H, C]."""
    dst, src = edge_index[0].long(), edge_index[1].long()
    keep = (dst >= 0) & (src >= 0)
    dst, src = dst[keep], src[keep]
    S, H = int(size[0]), al.shape[1]
    z = F.leaky_relu(al.float()[src] + ar.float()[dst], slope)  # [E, H]
    mx = torch.full((S, H), float("-inf"), device=z.device).scatter_reduce(
        0, dst.view(-1, 1).expand_as(z), z, reduce="amax", include_self=True)
    p = torch.exp(z - mx[dst])
    den = torch.zeros(S, H, device=z.device).index_add(0, dst, p)
    p = p / den[dst]
    msg = h.float()[src] * p.unsqueeze(-1)
    return torch.zeros((S,) + tuple(h.shape[1:]), device=z.device).index_add(0, dst, msg)


class _GatAggregate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h2, al, ar, csr, H, C, slope):
        indptr, col = csr.csr()
        out, lse = hip().gat_fwd(indptr, col, csr.csr_order(), h2, al, ar, H, C, slope)
        ctx.csr, ctx.H, ctx.C, ctx.slope = csr, H, C, slope
        ctx.save_for_backward(h2, al, ar, out, lse)
        return out

    @staticmethod
    def backward(ctx, dout):
        h2, al, ar, out, lse = ctx.saved_tensors
        indptr, col = ctx.csr.csr()
        cindptr, crow = ctx.csr.csc()
        dout = dout.to(h2.dtype).contiguous()
        dh, dal, dar = hip().gat_bwd(indptr, col, ctx.csr.csr_order(), cindptr, crow, ctx.csr.csc_order(), h2, al,
                                     ar, ctx.H, ctx.C, ctx.slope, out, dout, lse)
        return dh, dal, dar, None, None, None, None


def gat_aggregate(h, al, ar, edge_index, size, slope=0.2, csr=None):
    """Fused multi-head GAT aggregation.

    h [N_src, H, C] (bf16 or fp32) projected source features, al [N_src, H] and
    ar [N_dst, H] the per-node attention terms; returns [N_dst, H, C] with
    ``out[i, h] = sum_j softmax_j(leaky_relu(al[j, h] + ar[i, h])) * h[j, h]``.
    Differentiable in h, al and ar.  ``csr`` (an :class:`EdgeCSR`) may be passed
    instead of ``edge_index`` for a resident graph.
    """
    N, H, C = h.shape
    if csr is not None:
        edge_index, size = csr.edge_index, (csr.n_dst, csr.n_src)
    if use_hip(h, al, ar) and h.dtype in (torch.bfloat16, torch.float32) and \
            hip().gat_supported(H, C, h.dtype == torch.bfloat16):
        csr = csr if csr is not None else edge_csr(edge_index, size)
        out = _GatAggregate.apply(h.reshape(N, H * C).contiguous(), al.float().contiguous(),
                                  ar.float().contiguous(), csr, H, C, float(slope))
        return out.view(-1, H, C)
    return gat_aggregate_reference(h, al, ar, edge_index, size, slope).to(h.dtype)


def gat_conv_reference(z, a_src, a_dst, edge_index, size, slope=0.2):
    al = (z.float() * a_src.float()).sum(-1)
    ar = (z.float() * a_dst.float()).sum(-1)
    return gat_aggregate_reference(z, al, ar, edge_index, size, slope)


class _GatConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z2, a_src, a_dst, csr, H, C, slope):
        al, ar = hip().gat_att_fwd(z2, a_src, a_dst, H, C)
        indptr, col = csr.csr()
        # al is recomputed from each gathered z row inside the edge kernels (a_src passed):
        # one row fetch per edge instead of a row plus an al line
        out, lse = hip().gat_fwd(indptr, col, csr.csr_order(), z2, al, ar, H, C, slope, a_src)
        ctx.csr, ctx.H, ctx.C, ctx.slope = csr, H, C, slope
        ctx.save_for_backward(z2, a_src, a_dst, al, ar, out, lse)
        return out

    @staticmethod
    def backward(ctx, dout):
        z2, a_src, a_dst, al, ar, out, lse = ctx.saved_tensors
        csr = ctx.csr
        indptr, col = csr.csr()
        cindptr, crow = csr.csc()
        dout = dout.to(z2.dtype).contiguous()
        dz, dal, dar = hip().gat_bwd(indptr, col, csr.csr_order(), cindptr, crow, csr.csc_order(), z2, al, ar,
                                     ctx.H, ctx.C, ctx.slope, out, dout, lse, a_src)
        # dz += dal (x) a_src + dar (x) a_dst in place; attention-vector grads in the same pass
        da_src, da_dst = hip().gat_att_bwd_(z2, a_src, a_dst, ctx.H, ctx.C, dal, dar, dz)
        return dz, da_src, da_dst, None, None, None, None


def gat_conv(z, a_src, a_dst, csr: EdgeCSR, slope=0.2):
    """Whole GAT convolution over ONE node set (full-graph training: sources and
    destinations are the same N nodes): attention terms, per-head edge softmax and the
    weighted aggregation, forward and backward, in 2 + 3 kernels.  z [N, H, C] projected
    features, a_src / a_dst [H, C] attention vectors; returns [N, H, C]."""
    N, H, C = z.shape
    assert csr.n_dst == csr.n_src == N, "gat_conv needs one node set (use gat_aggregate for blocks)"
    if use_hip(z, a_src, a_dst) and z.dtype in (torch.bfloat16, torch.float32) and \
            hip().gat_supported(H, C, z.dtype == torch.bfloat16):
        out = _GatConv.apply(z.reshape(N, H * C).contiguous(), a_src.float().contiguous(),
                             a_dst.float().contiguous(), csr, H, C, float(slope))
        return out.view(N, H, C)
    return gat_conv_reference(z, a_src, a_dst, csr.edge_index, (N, N), slope).to(z.dtype)


def gemm(a, b, out=None, trans_a=False, trans_b=False, bias=None, relu=False, rmask=None, splits=1, alpha=1.0,
         out_dtype=torch.float32, addend=None, row_scale=None):
    """``out = row_scale * alpha * op(a) @ op(b) (+ bias) (+ addend) (relu) (* (rmask > 0))`` with op(x) = x^T when
    trans_x (BLAS convention).  GPU: the tiled MFMA kernel of csrc/hip/gemm.hip (bf16
    operands, fp32 accumulation; ``splits`` > 1 splits the reduction dimension into
    deterministic partial slabs + one reduce, for [R]-row weight-gradient products) —
    hipBLASLt runs these skinny shapes on a few large tiles.  CPU: the torch composition."""
    A = a.t() if trans_a else a
    Bm = b.t() if trans_b else b
    M, N = A.shape[0], Bm.shape[1]
    if use_hip(a, b):
        if out is None:
            out = torch.empty(M, N, device=a.device, dtype=out_dtype)
        aa = a if a.stride(-1) == 1 else a.contiguous()
        bb = b if b.stride(-1) == 1 else b.contiguous()
        hip().gemm(aa, bb, out, bool(trans_a), bool(trans_b), bias, rmask, bool(relu), int(splits), float(alpha),
                   addend, row_scale)
        return out
    y = (A.float() @ Bm.float()) * alpha
    if row_scale is not None:
        y = y * row_scale.float().view(-1, 1)
    if bias is not None:
        y = y + bias.float()
    if addend is not None:
        y = y + addend[: y.shape[0], : y.shape[1]].float()
    if relu:
        y = torch.relu(y)
    if rmask is not None:
        y = y * (rmask > 0).to(y.dtype)
    if out is None:
        return y.to(out_dtype)
    out.copy_(y)
    return out


def _gemm_splits(k_rows, tiles):
    """split-K count for a weight-gradient product over k_rows rows with `tiles` 64x64
    output tiles: about 512 workgroups (two per CU: the k loop is a dependent load chain),
    at least 128 rows (2 k-stages) per split, at most 64 slabs for the reduce"""
    return int(max(1, min(64, k_rows // 128, -(-512 // max(tiles, 1)))))


class _Linear(torch.autograd.Function):
    """``x @ w^T`` on the tiled MFMA GEMM (forward, dx, split-K dW)"""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return gemm(x, w, trans_b=True, out_dtype=x.dtype if x.dtype in (torch.float32, torch.bfloat16)
                    else torch.float32)

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = gemm(g, w, out_dtype=x.dtype)
        if ctx.needs_input_grad[1]:
            tiles = -(-w.shape[0] // 64) * -(-w.shape[1] // 64)
            dw = gemm(g, x, trans_a=True, splits=_gemm_splits(x.shape[0], tiles), out_dtype=w.dtype)
        return dx, dw


def linear(x, w):
    """``x @ w^T`` (no bias) for 2-D x: the tiled MFMA GEMM on the GPU (self-loop transforms
    of full-graph layers), torch elsewhere"""
    if use_hip(x, w) and x.dim() == 2 and w.dtype == torch.float32:
        return _Linear.apply(x, w)
    return x @ w.t().to(x.dtype)


class _TallLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, chunk):
        ctx.save_for_backward(x, w)
        ctx.chunk = chunk
        ctx.has_bias = b is not None
        y = x @ w.t().to(x.dtype)
        return y if b is None else y + b.to(y.dtype)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.to(x.dtype)
        dx = dy @ w.to(x.dtype)
        n = x.shape[0]
        p = max(1, n // ctx.chunk)
        n0 = (n // p) * p
        # dW = dy^T x split over row chunks: P batched GEMMs fill the chip where a single
        # [M x N] x [N x K] reduction GEMM over millions of rows runs on a few workgroups
        dyv = dy[:n0].view(p, n0 // p, -1)
        dw = torch.bmm(dyv.transpose(1, 2), x[:n0].view(p, n0 // p, -1)).float().sum(0)
        if n0 < n:
            dw += (dy[n0:].t() @ x[n0:]).float()
        db = None
        if ctx.has_bias:
            # column sums as the same split-K GEMM (ones^T dy): a plain dim-0 reduction of a
            # [millions, C] tensor with a few dozen columns runs on a few workgroups
            ones = torch.ones(p, 1, n0 // p, device=dy.device, dtype=dy.dtype)
            db = torch.bmm(ones, dyv).float().sum((0, 1))
            if n0 < n:
                db += dy[n0:].float().sum(0)
        return dx, dw.to(w.dtype), db, None


def splitk_mm_t(a, b, parts=None):
    """``a^T @ b`` (fp32 result) for tall a [M, P], b [M, Q] as ``parts`` batched row chunks +
    a sum: dW-shaped products with few output tiles otherwise run on one or two workgroups
    (hipBLASLt picks one 128x128 tile over all M rows)."""
    M = a.shape[0]
    p = parts or max(1, min(32, M // 128))
    if not (a.is_cuda and p > 1):
        return torch.mm(a.t().float(), b.float()) if not a.is_cuda else torch.mm(a.t(), b, out_dtype=torch.float32)
    n0 = (M // p) * p
    av, bv = a[:n0].reshape(p, n0 // p, -1), b[:n0].reshape(p, n0 // p, -1)
    if a.dtype == torch.float32:
        out = torch.bmm(av.transpose(1, 2), bv).sum(0)
    else:
        try:
            out = torch.bmm(av.transpose(1, 2), bv, out_dtype=torch.float32).sum(0)
        except (RuntimeError, TypeError, NotImplementedError):
            out = torch.bmm(av.transpose(1, 2).float(), bv.float()).sum(0)
    if n0 < M:
        out = out + (torch.mm(a[n0:].t(), b[n0:], out_dtype=torch.float32) if a.dtype != torch.float32
                     else a[n0:].t() @ b[n0:])
    return out


class _SplitKLinear(torch.autograd.Function):
    """``x @ w^T + b`` whose weight / bias gradients use :func:`splitk_mm_t` (GPU)."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        return torch.nn.functional.linear(x, w, b)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        dx = dy @ w if ctx.needs_input_grad[0] else None
        dw = splitk_mm_t(dy, x).to(w.dtype) if ctx.needs_input_grad[1] else None
        db = dy.float().sum(0).to(w.dtype) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return dx, dw, db


def splitk_linear(x, weight, bias=None):
    """Linear layer for GPU batches of >= 512 rows with split-K weight gradients."""
    if x.is_cuda and x.dim() == 2 and x.shape[0] >= 512 and x.dtype == weight.dtype:
        return _SplitKLinear.apply(x, weight, bias)
    return torch.nn.functional.linear(x, weight, bias)


def tall_linear(x, weight, bias=None, chunk=8192):
    """``x @ weight^T (+ bias)`` for x with millions of rows (full-graph layers): the
    weight (and bias) gradients are computed as split-K batched GEMMs instead of one
    skinny reduction."""
    if x.is_cuda and x.dim() == 2 and x.shape[0] >= 4 * chunk:
        return _TallLinear.apply(x, weight, bias, chunk)
    y = x @ weight.t().to(x.dtype)
    return y if bias is None else y + bias.to(y.dtype)


def xent(logits, labels):
    """Mean softmax cross-entropy with row-parallel kernels (logsumexp + gather + mean):
    on ROCm the mean-reduced ``F.cross_entropy`` runs its NLL reduction on one
    workgroup (~0.5 ms fwd + bwd at 200K rows)."""
    logits = logits.float()
    lse = torch.logsumexp(logits, dim=1)
    return (lse - logits.gather(1, labels.long().view(-1, 1)).squeeze(1)).mean()


# ----------------------------------------------------------------------------- K6 relation transform
_TILE = 64


def _round_up(x, m):
    return (x + m - 1) // m * m


class RelationTiles:
    """Edges grouped by relation, for the relation-grouped MFMA GEMM (rgcn.hip).

    Arrays are over the relation-sorted order of the valid edges: ``src``/``dst``
    (int32), ``scale`` (1 / in-degree for mean aggregation, else 1), ``eid`` (arange),
    ``slot_dst`` / ``slot_src`` (the message row of each edge in the forward / backward
    GEMM: its position in the destination / source CSR), tiles ``(rel, start, len)`` of <= 64 edges of one
    relation for the message GEMMs, chunks ``(rel, start, len)`` of <= 1024 edges of one
    relation for the weight gradient, and the destination / source CSRs over the
    messages (``SegmentIndex``) for the deterministic per-node sums.  Built once per
    (edge_index, relation ids)."""

    def __init__(self, edge_index, rel, size, num_rel, aggr="mean", tile=_TILE):
        dst, src = edge_index[0].long(), edge_index[1].long()
        rel = rel.reshape(-1).long()
        valid = (dst >= 0) & (src >= 0) & (rel >= 0) & (rel < num_rel)
        idx = valid.nonzero(as_tuple=True)[0]
        order = idx[torch.argsort(rel[idx], stable=True)]
        r_sorted = rel[order]
        dev = edge_index.device
        n_dst, n_src = int(size[0]), int(size[1])
        self.aggr = aggr
        self.num_edges = int(order.numel())
        self.src = src[order].to(torch.int32).contiguous()
        self.dst = dst[order].to(torch.int32).contiguous()
        self.eid = torch.arange(self.num_edges, device=dev, dtype=torch.int32)
        if aggr == "mean":
            deg = torch.bincount(dst[idx], minlength=n_dst)[:n_dst].clamp(min=1).float()
            self.scale = (1.0 / deg)[self.dst.long()].contiguous()
        else:
            self.scale = torch.ones(order.numel(), device=dev)
        counts = torch.bincount(r_sorted, minlength=num_rel)[:num_rel]
        self.tile = int(tile)
        self.tile_rel, self.tile_start, self.tile_len, self.num_tiles = self._cut(counts, tile, dev)
        chunk = hip().rel_gemm_dw_chunk if dev.type == "cuda" else 1024
        chunk = int(os.environ.get("EULER_AMD_RG_CH", chunk))  # tuning knob (tools/gpu_session.sh kg_dw_sweep)
        self.chunk_rel, self.chunk_start, self.chunk_len, self.num_chunks = self._cut(counts, chunk, dev)
        # a relation's only chunk stores its dW slab instead of adding atomically
        self.chunk_solo = (counts[self.chunk_rel.long()] <= chunk).to(torch.int32).contiguous()
        self.dst_seg = SegmentIndex(self.dst.long(), n_dst)
        self.src_seg = SegmentIndex(self.src.long(), n_src)
        # message rows in destination-CSR order (forward) / source-CSR order (backward):
        # the GEMM epilogue scatters each 16-byte-vector message row to its edge's slot, so
        # the per-node sums stream the messages sequentially (no perm indirection, no
        # random row reads)
        self.slot_dst = self._slots(self.dst_seg.perm, dev)
        self.slot_src = self._slots(self.src_seg.perm, dev)

    @staticmethod
    def _slots(perm, dev):
        slot = torch.empty(perm.numel(), dtype=torch.int32, device=dev)
        slot[perm] = torch.arange(perm.numel(), dtype=torch.int32, device=dev)
        return slot

    @staticmethod
    def _cut(counts, size, dev):
        R = counts.numel()
        n = (counts + size - 1) // size
        T = int(n.sum().item())
        t_rel = torch.repeat_interleave(torch.arange(R, device=dev), n)
        first = torch.cumsum(n, 0) - n
        k = torch.arange(T, device=dev) - first[t_rel]
        start = torch.cumsum(counts, 0) - counts
        return (t_rel.to(torch.int32).contiguous(), (start[t_rel] + size * k).to(torch.int32).contiguous(),
                torch.clamp(counts[t_rel] - size * k, max=size).to(torch.int32).contiguous(), T)

    def tiles(self):
        return self.tile_rel, self.tile_start, self.tile_len

    def chunks(self):
        return self.chunk_rel, self.chunk_start, self.chunk_len

    def det_slots(self):
        """the deterministic weight-gradient layout (``rel_gemm_dw(slot=, part=, mrel=, mrp=)``):
        (chunk -> partial slot, -1 for a relation's only chunk; the relations with several
        chunks; their slot ranges as a CSR; the number of slots).  Chunks are in relation
        order, so each relation's slots are consecutive and summed in chunk order."""
        if getattr(self, "_det", None) is None:
            solo = self.chunk_solo.long()
            multi = 1 - solo
            slot = torch.where(multi.bool(), torch.cumsum(multi, 0) - 1, torch.full_like(multi, -1))
            rel = self.chunk_rel.long()[multi.bool()]
            mrel, cnt = torch.unique_consecutive(rel, return_counts=True)
            mrp = torch.zeros(mrel.numel() + 1, dtype=torch.long, device=rel.device)
            mrp[1:] = torch.cumsum(cnt, 0)
            self._det = (slot.to(torch.int32).contiguous(), mrel.to(torch.int32).contiguous(),
                         mrp.to(torch.int32).contiguous(), int(multi.sum()))
        return self._det


def relation_transform_reference(x, rel, weight, edge_index, size, aggr="mean"):
    """out[i] = aggr_{e: dst(e) = i} weight[rel(e)] @ x[src(e)]  (weight [R, N, K])."""
    dst, src = edge_index[0].long(), edge_index[1].long()
    rel = rel.reshape(-1).long()
    valid = (dst >= 0) & (src >= 0) & (rel >= 0) & (rel < weight.shape[0])
    dst, src, rel = dst[valid], src[valid], rel[valid]
    msg = torch.einsum("enk,ek->en", weight.float()[rel], x.float()[src])
    S = int(size[0])
    out = torch.zeros(S, weight.shape[1], device=x.device).index_add(0, dst, msg)
    if aggr == "mean":
        cnt = torch.bincount(dst, minlength=S)[:S].clamp(min=1).float()
        out = out / cnt.unsqueeze(1)
    return out


def _pad_bf16(t, pad):
    """bf16, contiguous, zero-padded copy — one conversion kernel and no pad copy when the
    shape is already aligned"""
    t = t.to(torch.bfloat16)
    if any(pad):
        t = F.pad(t, pad)
    return t.contiguous()


def _seg_sum(msg, indptr, op):
    """per-node sum (op 0) / mean (1) of CSR-ordered message rows: one wave per node
    (relation graphs have power-law in-degrees) when the row width allows it"""
    lp = msg.shape[1] // (8 if msg.dtype == torch.bfloat16 else 4)
    if _SEG_WAVE and 0 < lp <= 64 and lp & (lp - 1) == 0:
        return hip().segment_reduce_wave(msg, indptr, None, op)
    return hip().segment_reduce(msg, indptr, None, op, 0.0)[0]


_SEG_WAVE = os.environ.get("EULER_AMD_SEG_WAVE", "1") == "1"


class _RelationTransform(torch.autograd.Function):
    """Messages W_rel x_src are stored once per edge (bf16, 16-byte rows) by the grouped
    GEMM and summed per destination by the segment kernel: plain stores + one
    deterministic read-back instead of fp32 atomics into the destination rows."""

    @staticmethod
    def forward(ctx, x, weight, tiles, n_dst):
        R, N, K = weight.shape
        Kp, Np = _round_up(K, 64), _round_up(N, 64)
        xb = _pad_bf16(x, (0, Kp - K))
        wt = None
        if Kp == K and Np == N and weight.dtype == torch.float32:
            # both bf16 operands (forward W, backward W^T) from one pass over the fp32 weights
            wb, wt = hip().rel_weight_bf16(weight.contiguous())
        else:
            wb = _pad_bf16(weight, (0, Kp - K, 0, Np - N))
        msg = torch.empty(tiles.num_edges, Np, device=x.device, dtype=torch.bfloat16)
        tr, ts, tl = tiles.tiles()
        hip().rel_gemm(xb, tiles.src, tr, ts, tl, wb, None, tiles.slot_dst, 0, tiles.tile, msg)
        op = 1 if tiles.aggr == "mean" else 0
        out = _seg_sum(msg, tiles.dst_seg.indptr, op)
        ctx.tiles, ctx.dims = tiles, (R, N, K, Kp, Np, x.shape[0])
        ctx.x_dtype, ctx.w_dtype = x.dtype, weight.dtype
        ctx.weight = weight
        ctx.wt = wt
        ctx.save_for_backward(xb, wb)
        return out[:, :N].to(x.dtype)

    @staticmethod
    def backward(ctx, dout):
        xb, wb = ctx.saved_tensors
        R, N, K, Kp, Np, n_src = ctx.dims
        tiles = ctx.tiles
        gb = _pad_bf16(dout, (0, Np - N))
        dx = dw = None
        if ctx.needs_input_grad[0]:
            wt = ctx.wt if ctx.wt is not None else wb.transpose(1, 2).contiguous()  # [R, Kp, Np]
            msgx = torch.empty(tiles.num_edges, Kp, device=dout.device, dtype=torch.bfloat16)
            tr, ts, tl = tiles.tiles()
            hip().rel_gemm(gb, tiles.dst, tr, ts, tl, wt, tiles.scale, tiles.slot_src, 0, tiles.tile, msgx)
            dxp = _seg_sum(msgx, tiles.src_seg.indptr, 0)
            dx = dxp[:, :K].to(ctx.x_dtype)
        if ctx.needs_input_grad[1]:
            cr, cs, cl = tiles.chunks()
            sink = ctx.weight.grad if getattr(ctx.weight, "_grad_sink", False) else None
            if (sink is not None and sink.dtype == torch.float32 and sink.is_contiguous()
                    and tuple(sink.shape) == (R, Np, Kp)):
                # grad sink (enable_grad_sink): dW accumulates straight into the weight's
                # persistent .grad buffer (e.g. a FlatParams view the optimizer zeroes) — no
                # zero-filled [R, N, K] temporary and no AccumulateGrad add pass over it
                hip().rel_gemm_dw(gb, tiles.dst, xb, tiles.src, tiles.scale, cr, cs, cl, tiles.chunk_solo, sink,
                                  accumulate=ctx.weight._grad_sink != "zeroed")
            else:
                dwp = torch.zeros(R, Np, Kp, device=dout.device, dtype=torch.float32)
                hip().rel_gemm_dw(gb, tiles.dst, xb, tiles.src, tiles.scale, cr, cs, cl, tiles.chunk_solo, dwp)
                dw = dwp[:, :N, :K].to(ctx.w_dtype)
        return dx, dw, None, None


def enable_grad_sink(weight, on: bool = True, zeroed: bool = False):
    """Let :func:`relation_transform`'s backward write dW straight into ``weight.grad``
    (which must then exist and persist, as FlatParams grads do).  ``zeroed``: the owner
    zeroes the gradient before every backward (FlatOptimizer.zero_grad), so relations with
    a single edge chunk store their slab instead of read-modify-writing it; otherwise dW is
    accumulated.  Autograd never sees that gradient: gradient hooks on the weight (e.g.
    dp.GradSync buckets) do not fire for it — sync the owner's flat grad."""
    weight._grad_sink = ("zeroed" if zeroed else "accumulate") if on else False
    return weight


def relation_transform(x, rel, weight, edge_index, size, aggr="mean", tiles=None):
    """R-GCN message + aggregation: ``out[i] = aggr_e weight[rel_e] @ x[src_e]`` over the
    in-edges of ``i`` (aggr ``mean`` or ``add``).  x [N_src, K], weight [R, N, K]."""
    R, N, K = weight.shape
    if use_hip(x, weight) and _rel_lds_row(N, K) * 16 <= 158 * 1024:
        if tiles is None:
            tiles = relation_tiles(edge_index, rel, size, R, N, K, aggr)
        return _RelationTransform.apply(x, weight, tiles, int(size[0]))
    return relation_transform_reference(x, rel, weight, edge_index, size, aggr).to(x.dtype)


def _rel_lds_row(N, K):
    return (_round_up(N, 64) + _round_up(K, 64) + 16) * 2  # bytes per tile row (A + output)


def relation_tiles(edge_index, rel, size, R, N, K, aggr="mean") -> RelationTiles:
    """the (cached) :class:`RelationTiles` of ``edge_index`` for [R, N, K] relation weights:
    the largest tile (edges of one relation per W_rel read) whose LDS rows fit"""
    lds_row = _rel_lds_row(N, K)
    tm = min(hip().rel_gemm_tile, int(os.environ.get("EULER_AMD_RG_TILE", "64")))
    while tm > 16 and lds_row * tm > 158 * 1024:
        tm //= 2
    key = "_euler_reltiles_%d_%d_%s_%d" % (int(size[0]), R, aggr, tm)
    return _cached(edge_index, key, lambda: RelationTiles(edge_index, rel, size, R, aggr, tile=tm))


# ----------------------------------------------------------------------------- multi-label loss + F1
class _BceF1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, rows, counts):
        x = logits.float().contiguous()
        ctx.save_for_backward(x, labels, rows)
        return hip().bce_f1_fwd(x, labels, rows, counts)

    @staticmethod
    def backward(ctx, g):
        x, labels, rows = ctx.saved_tensors
        return hip().bce_bwd(x, labels, rows, g.float().reshape(1).contiguous()), None, None, None


def bce_f1_loss(logits, labels, rows, counts):
    """``F.binary_cross_entropy_with_logits(logits, labels[rows])`` (mean) and the F1 counts
    (tp, fp, fn of ``logits >= 0`` against ``labels > 0.5``) added into ``counts`` [3] —
    two launches forward, one backward on the GPU (the torch composition is ~18 kernels)."""
    rows = rows.reshape(-1).long()
    if use_hip(logits, labels) and labels.dtype == torch.float32 and counts.dtype == torch.int64 \
            and labels.is_contiguous():
        return _BceF1.apply(logits, labels, rows.contiguous(), counts)
    y = labels[rows]
    loss = F.binary_cross_entropy_with_logits(logits.float(), y)
    with torch.no_grad():
        pred, pos = logits >= 0, y > 0.5
        counts += torch.stack([(pred & pos).sum(), (pred & ~pos).sum(), (~pred & pos).sum()])
    return loss


# ----------------------------------------------------------------------------- K11 skip-gram loss
def sgns_loss_reference(emb, pos, neg):
    emb = emb.reshape(emb.shape[0], -1).float()
    lp = torch.einsum("bd,bpd->bp", emb, pos.float())
    ln = torch.einsum("bd,bkd->bk", emb, neg.float())
    lt = F.binary_cross_entropy_with_logits(lp, torch.ones_like(lp), reduction="none")
    lf = F.binary_cross_entropy_with_logits(ln, torch.zeros_like(ln), reduction="none")
    return torch.cat([lt.reshape(-1), lf.reshape(-1)]).mean(), lp, ln


class _Sgns(torch.autograd.Function):
    @staticmethod
    def forward(ctx, emb, pos, neg):
        logits, loss_rows = hip().sgns_fwd(emb, pos, neg)
        count = emb.shape[0] * (pos.shape[1] + neg.shape[1])
        ctx.save_for_backward(emb, pos, neg, logits)
        ctx.count = count
        ctx.mark_non_differentiable(logits)
        return loss_rows.sum() / max(count, 1), logits

    @staticmethod
    def backward(ctx, g, _g_logits):
        emb, pos, neg, logits = ctx.saved_tensors
        demb, dpos, dneg = hip().sgns_bwd(emb, pos, neg, logits, 1.0 / max(ctx.count, 1))
        g = g.to(demb.dtype)
        return demb * g, dpos * g, dneg * g


def sgns_loss(emb, pos, neg):
    """Mean sigmoid cross-entropy of ``<emb, pos>`` (label 1) and ``<emb, neg>`` (label 0).

    emb [B, D] or [B, 1, D]; pos [B, P, D]; neg [B, K, D].  Returns
    ``(loss, pos_logits [B, P], neg_logits [B, K])`` (logits detached)."""
    B = emb.shape[0]
    e2 = emb.reshape(B, -1)
    D = e2.shape[1]
    V = 8 if e2.dtype == torch.bfloat16 else 4
    if use_hip(e2, pos, neg) and e2.dtype in (torch.bfloat16, torch.float32) and pos.dtype == e2.dtype and \
            neg.dtype == e2.dtype and D % V == 0 and D // V <= 64:
        loss, logits = _Sgns.apply(e2.contiguous(), pos.contiguous(), neg.contiguous())
        P = pos.shape[1]
        return loss, logits[:, :P], logits[:, P:]
    loss, lp, ln = sgns_loss_reference(e2, pos, neg)
    return loss, lp.detach(), ln.detach()


# ----------------------------------------------------------------------------- K11b index-driven SGNS
# One skip-gram step over de-duplicated ids without per-pair gradient rows (DeepWalk /
# LINE; embed.hip sgns_fwd_idx / sgns_update).  P pairs, each one positive and K
# negatives; ``tinv`` [P] / ``cinv`` [P*(1+K)] (positives then negatives) index the unique
# target / context ids, ``tmap`` / ``cmap`` map unique ids to table rows (None: identity).

def _rows(table, map_, inv):
    idx = inv if map_ is None else map_[inv]
    return table[idx]


def sgns_fwd_idx(T, tmap, tinv, C, cmap, cinv, K, gscale):
    """``(coef [P, 1+K], loss_rows [P])``: coef = (sigmoid(logit) - label) * gscale, the
    loss gradient of each logit; loss_rows the per-pair sigmoid-CE sums."""
    if use_hip(T, tinv, C, cinv):
        return tuple(hip().sgns_fwd_idx(T.contiguous(), tmap, tinv.contiguous(), C.contiguous(), cmap,
                                        cinv.contiguous(), int(K), float(gscale)))
    P = tinv.numel()
    e = _rows(T, tmap, tinv).float()
    c = _rows(C, cmap, cinv).float()
    ctx = torch.cat([c[:P].view(P, 1, -1), c[P:].view(P, K, -1)], 1)
    x = torch.einsum("pd,psd->ps", e, ctx)
    y = torch.zeros_like(x)
    y[:, 0] = 1.0
    loss = F.binary_cross_entropy_with_logits(x, y, reduction="none").sum(1)
    return (torch.sigmoid(x) - y) * gscale, loss


def unique_first_padded(x: torch.Tensor, fill: int = -1, offset: int = 0):
    """Fixed-capacity :func:`unique_first` for graph-captured steps: ``(uniq [n], inverse
    [n], count [1])`` with the distinct non-negative values in first-occurrence order
    (plus ``offset``) followed by ``fill``; negative values are padding ("no id": not
    counted, inverse -1); the count stays on the device (GPU: no host sync)."""
    x = x.reshape(-1)
    if use_hip(x):
        return tuple(hip().unique_first_padded(x.long().contiguous(), int(fill), int(offset)))
    valid = x >= 0
    u, inv_v = unique_first(x[valid])
    inv = torch.full((x.numel(),), -1, dtype=torch.long, device=x.device)
    inv[valid] = inv_v.long()
    out = torch.full((x.numel(),), int(fill), dtype=torch.long, device=x.device)
    out[: u.numel()] = u + int(offset)
    return out, inv, torch.tensor([u.numel()], dtype=torch.long, device=x.device)


def route_by_owner(ids, W: int, C: int, overflow, self_rank: int = -1):
    """Slots of the fixed-capacity all-to-all exchange (csrc/hip/route.hip): id k (>= 0)
    goes to owner ``ids[k] % W`` at slot ``block(owner) * C + r``, r = its stable rank among
    the ids of that owner; ids < 0 or past an owner's C slots get ``W * C`` (the latter set
    ``overflow[0] = 1``).  ``block(o) = o`` for ``self_rank < 0``; otherwise the caller's own
    block is last and the peers keep rank order (o < self: o, o > self: o - 1), so the
    peers' slots form one prefix.  Returns ``(pos [n] int64, send [W*C + 1] int64)``: the
    slot of every id and the id in every slot (-1 = empty)."""
    ids = ids.reshape(-1).long()
    if use_hip(ids):
        return tuple(hip().route_by_owner(ids.contiguous(), int(W), int(C), overflow, int(self_rank)))
    n = ids.numel()
    trash = W * C
    owner = torch.where(ids >= 0, torch.remainder(ids, W), torch.full_like(ids, W))
    order = torch.sort(owner, stable=True)[1]
    cnt = torch.zeros(W + 1, dtype=torch.long, device=ids.device).index_add_(0, owner, torch.ones_like(owner))
    start = torch.cumsum(cnt, 0) - cnt
    so = owner[order]
    slot = torch.arange(n, device=ids.device) - start[so]
    real = so < W
    fits = real & (slot < C)
    torch.maximum(overflow, (real & ~fits).any().int().view(1), out=overflow)
    blk = so
    if self_rank >= 0:
        blk = torch.where(so < self_rank, so, torch.where(so > self_rank, so - 1, torch.full_like(so, W - 1)))
    dest = torch.where(fits, blk * C + slot, torch.full_like(slot, trash))
    send = torch.full((trash + 1,), -1, dtype=torch.long, device=ids.device)
    send.scatter_(0, dest, torch.where(fits, ids[order], torch.full_like(slot, -1)))
    send[trash] = -1
    pos = torch.empty_like(dest)
    pos[order] = dest
    return pos, send


def occ_csr(inv, n_u):
    """occurrence lists of ``inv`` (values in [0, n_u)): ``(ptr [n_u+1] int64, list int32)``."""
    inv = inv.reshape(-1).long()
    if use_hip(inv):
        return tuple(hip().occ_csr(inv.contiguous(), int(n_u)))
    cnt = torch.zeros(n_u, dtype=torch.long, device=inv.device).index_add_(0, inv, torch.ones_like(inv))
    ptr = torch.zeros(n_u + 1, dtype=torch.long, device=inv.device)
    ptr[1:] = torch.cumsum(cnt, 0)
    return ptr, torch.argsort(inv, stable=True).int()


def _ctx_occ_pairs(P, K, device):
    """(pair, slot) of every context occurrence, in cinv order."""
    pos = torch.arange(P, device=device)
    q = torch.arange(P * K, device=device)
    return torch.cat([pos, q // max(K, 1)]), torch.cat([torch.zeros_like(pos), 1 + q % max(K, 1)])


def sgns_grad_reference(side, coef, K, src, smap, sinv, n_u, inv_self):
    P = coef.shape[0]
    D = src.shape[1]
    if side == 0:   # target u: sum over its pairs of sum_s coef[p, s] * C[ctx(p, s)]
        c = _rows(src, smap, sinv).float()
        ctx = torch.cat([c[:P].view(P, 1, D), c[P:].view(P, K, D)], 1)
        per = torch.einsum("ps,psd->pd", coef, ctx)
    else:           # context occurrence (p, s): coef[p, s] * E[tgt(p)]
        e = _rows(src, smap, sinv).float()
        pp, ss = _ctx_occ_pairs(P, K, coef.device)
        per = coef[pp, ss].unsqueeze(1) * e[pp]
    return torch.zeros(n_u, D, dtype=torch.float32, device=src.device).index_add_(0, inv_self.reshape(-1), per)


def sgns_grad(side, ptr, lst, coef, K, src, smap, sinv, inv_self=None, out=None):
    """per-unique-row gradient ``[n_u, D]`` of one table (side 0 target, 1 context),
    rebuilt from the occurrence lists (no per-pair rows, no atomics).  ``inv_self`` (this
    side's inverse) is only read by the CPU composition.  With ``out`` the rows that have
    occurrences on this side are written into it and the others left untouched, so the
    two sides can fill one buffer."""
    n_u = ptr.numel() - 1
    if use_hip(coef, src):
        return hip().sgns_grad(int(side), ptr, lst, coef.contiguous(), int(K), src.contiguous(), smap,
                               sinv.contiguous(), out)
    g = sgns_grad_reference(side, coef, K, src, smap, sinv, n_u, inv_self)
    if out is None:
        return g
    has = ptr[1:] > ptr[:-1]
    out[has] = g[has].to(out.dtype)
    return out


# ----------------------------------------------------------------------------- K10 KG scores
KG_KINDS = {"l1": 0, "l2": 1, "distmult": 2}
KG_CORRUPT = {"front": 0, "tail": 1, "both": 2}


def kg_score_reference(ent, rel, src, dst, ridx, neg, kind="l1", corrupt="both", normalize=True):
    def row(t, i):
        x = t[i.long()]
        return F.normalize(x, dim=-1) if normalize else x

    h, t, r = row(ent, src.reshape(-1)), row(ent, dst.reshape(-1)), row(rel, ridx.reshape(-1))
    n = row(ent, neg.reshape(src.numel(), -1))

    def score(a, b, c):
        if kind == "distmult":
            return (a * b * c).sum(-1)
        d = a + b - c
        return -(d.abs().sum(-1) if kind == "l1" else d.norm(dim=-1))

    pos = score(h, r, t)
    r1, h1, t1 = r.unsqueeze(1), h.unsqueeze(1), t.unsqueeze(1)
    if corrupt == "front":
        ns = score(n, r1, t1)
    elif corrupt == "tail":
        ns = score(h1, r1, n)
    else:
        ns = torch.cat([score(n, r1, t1), score(h1, r1, n)], -1)
    return pos, ns


class _KgScore(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ent, rel, src, dst, ridx, neg, kind, corrupt, normalize):
        pos_s, neg_s = hip().kg_fwd(ent, rel, src, dst, ridx, neg, kind, corrupt, normalize)
        ctx.save_for_backward(ent, rel, src, dst, ridx, neg)
        ctx.args = (kind, corrupt, normalize)
        return pos_s, neg_s

    @staticmethod
    def backward(ctx, gpos, gneg):
        ent, rel, src, dst, ridx, neg = ctx.saved_tensors
        B = src.numel()
        K = neg.numel() // max(B, 1)
        nneg = (2 if ctx.args[1] == 2 else 1) * K
        gpos = torch.zeros(B, device=ent.device) if gpos is None else gpos.float().contiguous()
        gneg = torch.zeros(B, nneg, device=ent.device) if gneg is None else gneg.float().contiguous()
        D = ent.shape[1]
        if _KG_OCC and (D // 4) & (D // 4 - 1) == 0:
            # per-occurrence gradient rows, then one segment sum per table row (occurrence
            # CSR): hot entities / relations (power-law KGs) no longer serialise fp32 atomics
            # on the same addresses (kg_bwd: 139 us of atomics, profiles/r3_kg/)
            occ_e = torch.empty(B * (2 + K), D, device=ent.device)
            occ_r = torch.empty(B, D, device=ent.device)
            hip().kg_bwd(ent, rel, src, dst, ridx, neg, *ctx.args, gpos, gneg, occ_e, occ_r, True)
            keys = torch.cat([src.view(B, 1), dst.view(B, 1), neg.view(B, K)], 1).view(-1)
            ptr_e, lst_e = occ_csr(keys, ent.shape[0])
            ptr_r, lst_r = occ_csr(ridx, rel.shape[0])
            dent = hip().segment_reduce_wave(occ_e, ptr_e, lst_e.long(), 0)
            drel = hip().segment_reduce_wave(occ_r, ptr_r, lst_r.long(), 0)
            return dent, drel, None, None, None, None, None, None, None
        dent = torch.zeros_like(ent)
        drel = torch.zeros_like(rel)
        hip().kg_bwd(ent, rel, src, dst, ridx, neg, *ctx.args, gpos, gneg, dent, drel)
        return dent, drel, None, None, None, None, None, None, None


_KG_OCC = os.environ.get("EULER_AMD_KG_OCC", "0") == "1"  # measured: +25 us/step vs atomics (profiles/r3_kg/s21/)


def kg_score(ent, rel, src, dst, ridx, neg, kind="l1", corrupt="both", normalize=True):
    """Scores of the positive triples ``(src, ridx, dst)`` [B] and of the corrupted ones
    [B, K] (front or tail) or [B, 2K] (both: front scores first), with rows gathered from
    the entity / relation tables and optionally l2-normalised.  ``kind``: ``l1`` /
    ``l2`` (TransE, score = -|h + r - t|) or ``distmult`` (score = sum h r t).
    Differentiable in both tables."""
    B = src.numel()
    D = ent.shape[1]
    if use_hip(ent, rel) and ent.dtype == torch.float32 and rel.dtype == torch.float32 and D % 4 == 0 and D <= 256:
        def ids(t, n_rows):
            return t.reshape(-1).long().clamp(0, n_rows - 1).contiguous()

        return _KgScore.apply(ent, rel, ids(src, ent.shape[0]), ids(dst, ent.shape[0]), ids(ridx, rel.shape[0]),
                              ids(neg, ent.shape[0]).view(B, -1), KG_KINDS[kind], KG_CORRUPT[corrupt],
                              bool(normalize))
    return kg_score_reference(ent, rel, src, dst, ridx, neg, kind, corrupt, normalize)


# ----------------------------------------------------------------------------- K8 unique
def unique_first(x: torch.Tensor):
    """``(unique values, inverse)`` of a 1-D id tensor in first-occurrence order — the
    semantics of ``tf.unique`` (reference dataflows rely on the previous hop's nodes
    keeping their leading positions).  GPU: hash-table kernel; CPU: the engine's O(n)
    hash pass (``_engine.unique_first``)."""
    x = x.reshape(-1)
    if use_hip(x):
        return tuple(hip().unique_first(x.long().contiguous()))
    if x.device.type == "cpu" and x.numel() > 0:
        # O(n) hash pass in the C++ engine (GIL released) — the CPU dataflows call this per hop
        u, inv = engine().unique_first(x.long().contiguous().numpy())
        return torch.from_numpy(u), torch.from_numpy(inv)
    u, inv = torch.unique(x, sorted=True, return_inverse=True)
    if u.numel() == 0:
        return u, inv
    first = torch.full((u.numel(),), x.numel(), dtype=torch.long, device=x.device)
    first = first.scatter_reduce(0, inv, torch.arange(x.numel(), device=x.device), reduce="amin")
    order = torch.argsort(first)
    rank = torch.empty_like(order)
    rank[order] = torch.arange(order.numel(), device=x.device)
    return u[order], rank[inv]
