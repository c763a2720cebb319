"""Message-passing ops: ``gather`` and ``scatter_{add,mean,max,softmax}``.

Same names and semantics as the reference's ``tf_euler.python.euler_ops.mp_ops``
(``/root/reference/tf_euler/python/euler_ops/mp_ops.py:27-79``):

* ``gather(params, indices)``                 -> ``params[indices]``
* ``scatter_add(updates, indices, size)``     -> segment sum into ``size`` rows
* ``scatter_mean``                            -> segment mean (empty rows = 0)
* ``scatter_max``                             -> segment max (empty rows = 0; reference
  initialises with -1e9 and the TF op keeps that for empty rows, we clamp to 0 to
  match ``scatter_`` usage in convs)
* ``scatter_softmax(logits, indices, size)``  -> per-destination softmax

On GPU tensors every op runs a hand-written gfx950 kernel (``csrc/hip/mp.hip``):
destinations are turned into a CSR once (``SegmentIndex``, cached on the dataflow
block) and reduced deterministically without atomics; gradients are exact
(argmax routing for max, p*(g - <p,g>) for softmax).  CPU tensors use the
pure-torch reference path, which is also the numerics oracle in tests.
"""
from __future__ import annotations

import os

import torch

from euler_amd.ops._native import hip, use_hip

__all__ = ["SegmentIndex", "gather", "gather_sum", "scatter_add", "scatter_mean", "scatter_max", "scatter_softmax",
           "scatter_", "segment_index", "embedding_bag", "weighted_aggregate"]


class SegmentIndex:
    """Destination CSR for a fixed ``(indices, size)`` pair.

    ``perm`` orders edges by destination (stable), ``indptr[s]:indptr[s+1]``
    delimits the edges of destination ``s``.  Built lazily on first use and
    reused by every scatter over the same edges (forward and backward).
    """

    __slots__ = ("indices", "size", "_perm", "_indptr", "_counts")

    def __init__(self, indices: torch.Tensor, size: int):
        self.indices = indices.reshape(-1).long()
        self.size = int(size)
        self._perm = None
        self._indptr = None
        self._counts = None

    @classmethod
    def from_csr(cls, indices, size, perm, indptr):
        """a SegmentIndex whose stable destination order is already known"""
        s = cls(indices, size)
        s._perm, s._indptr = perm, indptr
        s._counts = indptr[1:] - indptr[:-1]
        return s

    def _build(self):
        if use_hip(self.indices) and 0 < self.size < (1 << 30) and self.indices.numel() < (1 << 31):
            # counts + scan for the bounds, a stable radix sort over the key's bits only for
            # the order (csrc/hip/embed.hip det_occ: 2-4 passes instead of a 64-bit argsort's
            # 8); padding (< 0) sorts last, past indptr[size] — the same perm as below
            ptr, perm = hip().det_occ(self.indices.contiguous(), self.size)
            self._perm = perm.long()
            self._indptr = ptr
            self._counts = ptr[1:] - ptr[:-1]
            return
        # padding destinations (< 0) go to a sentinel segment past the end; the segment
        # bounds come from a binary search of the sorted destinations (no bincount: its
        # output size depends on the data, a host sync that a captured step cannot have)
        idx = torch.where(self.indices < 0, torch.full_like(self.indices, self.size), self.indices)
        self._perm = torch.argsort(idx, stable=True)
        bounds = torch.arange(self.size + 1, dtype=torch.long, device=idx.device)
        self._indptr = torch.searchsorted(idx[self._perm].contiguous(), bounds)
        self._counts = self._indptr[1:] - self._indptr[:-1]

    @property
    def perm(self):
        if self._perm is None:
            self._build()
        return self._perm

    @property
    def indptr(self):
        if self._indptr is None:
            self._build()
        return self._indptr

    @property
    def counts(self):
        if self._counts is None:
            if self._perm is None:
                # a histogram (fixed size: capturable) instead of the sort when only the
                # segment sizes are asked for (the GCN degree of the source side)
                if use_hip(self.indices):
                    # one atomic per real entry; torch's int64 index_add_ took 6 ms per call
                    # on the padding bin of a capacity-padded block (profiles/r4_gcn/)
                    self._counts = hip().seg_count(self.indices.contiguous(), self.size)
                else:
                    idx = torch.where(self.indices < 0, torch.full_like(self.indices, self.size), self.indices)
                    c = torch.zeros(self.size + 1, dtype=torch.long, device=idx.device)
                    c.index_add_(0, idx, torch.ones_like(idx))
                    self._counts = c[: self.size]
            else:
                self._build()
        return self._counts


def cached_segment(edge_index, i, size) -> SegmentIndex:
    """The CSR of ``edge_index[i]`` (``size`` segments), built once per edge_index tensor and
    shared by every op over it (degree normalisations, scatters, the SpMM and its
    backward); a producer that already knows the CSR (dataflow/device_flow.py) stores it
    here under the same key."""
    key = "_euler_seg%d_%d" % (i, int(size))
    cache = getattr(edge_index, "_euler_cache", None)
    if cache is None:
        cache = {}
        try:
            edge_index._euler_cache = cache
        except AttributeError:
            return SegmentIndex(edge_index[i], int(size))
    if key not in cache:
        cache[key] = SegmentIndex(edge_index[i], int(size))
    return cache[key]


def segment_index(indices, size) -> SegmentIndex:
    if isinstance(indices, SegmentIndex):
        return indices
    return SegmentIndex(indices, size)


def _deterministic() -> bool:
    return os.environ.get("EULER_AMD_DETERMINISTIC", "0") == "1" or torch.are_deterministic_algorithms_enabled()


# ----------------------------------------------------------------------------- gather
class _Gather(torch.autograd.Function):
    @staticmethod
    def forward(ctx, params, indices):
        ctx.n = params.shape[0]
        ctx.save_for_backward(indices)
        return hip().gather_rows(params.contiguous(), indices.contiguous())

    @staticmethod
    def backward(ctx, g):
        (indices,) = ctx.saved_tensors
        g = g.contiguous()
        g2 = g.reshape(g.shape[0], -1)
        idx = indices.reshape(-1).long()
        if _deterministic():
            seg = SegmentIndex(idx, ctx.n)
            out = hip().segment_reduce(g2, seg.indptr, seg.perm, 0, 0.0)[0]
        else:
            acc = torch.zeros((ctx.n, g2.shape[1]), dtype=torch.float32, device=g.device)
            hip().index_add_rows_(acc, idx, g2)
            out = acc.to(g.dtype)
        return out.reshape((ctx.n,) + tuple(g.shape[1:])), None


def gather(params: torch.Tensor, indices: torch.Tensor) -> torch.Tensor:
    """``params[indices]`` along dim 0 (reference ``mp_ops.gather``)."""
    if use_hip(params, indices) and params.dim() >= 1 and params.is_floating_point():
        idx = indices.reshape(-1)
        if idx.dtype not in (torch.int32, torch.int64):
            idx = idx.long()
        out = _Gather.apply(params, idx)
        return out.reshape(tuple(indices.shape) + tuple(params.shape[1:]))
    idx = indices.long()
    neg = idx < 0
    if not bool(neg.any()):
        return params[idx]
    # a -1 (padding) index reads a zero row, as the HIP gather does
    out = params[idx.clamp(min=0)]
    return torch.where(neg.reshape(tuple(idx.shape) + (1,) * (params.dim() - 1)), torch.zeros((), dtype=out.dtype),
                       out)


def gather_sum(table: torch.Tensor, indices: torch.Tensor) -> torch.Tensor:
    """``sum_f table[indices[:, f]]`` in fp32 [n, D] (``-1`` entries add nothing), no
    gradient: the neighbour-sum of sampled rows without materialising the [n, F, D]
    gather (``mp.hip gather_sum``: fp32 accumulation in f order, as a gather + sum)."""
    idx = indices.reshape(indices.shape[0], -1)
    if (use_hip(table, idx) and table.dim() == 2 and table.dtype in (torch.float32, torch.bfloat16)
            and (table.shape[1] * table.element_size()) % 16 == 0):
        return hip().gather_sum(table.contiguous(), idx.long().contiguous())
    return gather(table, idx.long()).float().sum(1)


# ----------------------------------------------------------------------------- scatter
class _SegmentReduce(torch.autograd.Function):
    @staticmethod
    def forward(ctx, src, seg, op):
        shape = src.shape
        s2 = src.contiguous().reshape(shape[0], -1)
        res = hip().segment_reduce(s2, seg.indptr, seg.perm, op, 0.0)
        ctx.op, ctx.seg, ctx.shape = op, seg, shape
        if op == 2:
            ctx.save_for_backward(res[1])
        return res[0].reshape((seg.size,) + tuple(shape[1:]))

    @staticmethod
    def backward(ctx, g):
        seg, op, shape = ctx.seg, ctx.op, ctx.shape
        g2 = g.contiguous().reshape(seg.size, -1)
        if op == 2:
            (am,) = ctx.saved_tensors
            gs = hip().max_bwd(g2, am, shape[0])
        else:
            if op == 1:
                cnt = seg.counts.clamp(min=1).to(g2.dtype).unsqueeze(1)
                g2 = g2 / cnt
            # gather_rows yields zero rows for negative (padding) destinations
            gs = hip().gather_rows(g2.contiguous(), seg.indices)
        return gs.reshape(shape), None, None


def _cpu_scatter(src, idx, size, reduce):
    idx = idx.reshape(-1).long()
    if idx.numel() and bool((idx < 0).any()):  # padding destinations are dropped
        keep = idx >= 0
        idx, src = idx[keep], src[keep]
    out_shape = (size,) + tuple(src.shape[1:])
    if reduce == "max":
        out = torch.full(out_shape, float("-inf"), dtype=src.dtype, device=src.device)
        ex = idx.view(-1, *([1] * (src.dim() - 1))).expand_as(src)
        out = out.scatter_reduce(0, ex, src, reduce="amax", include_self=True)
        return torch.where(torch.isinf(out), torch.zeros_like(out), out)
    out = torch.zeros(out_shape, dtype=src.dtype, device=src.device)
    out = out.index_add(0, idx, src)
    if reduce == "mean":
        cnt = torch.bincount(idx, minlength=size)[:size].clamp(min=1).to(src.dtype)
        out = out / cnt.view(-1, *([1] * (src.dim() - 1)))
    return out


def _scatter(src, indices, size, reduce):
    if size is None:
        size = int(indices.max().item()) + 1 if indices.numel() else 0
    if isinstance(size, torch.Tensor):
        size = int(size.item())
    if use_hip(src) and src.is_floating_point() and src.dtype in (torch.float32, torch.bfloat16):
        seg = segment_index(indices, size)
        op = {"add": 0, "sum": 0, "mean": 1, "max": 2}[reduce]
        return _SegmentReduce.apply(src, seg, op)
    idx = indices.indices if isinstance(indices, SegmentIndex) else indices
    return _cpu_scatter(src, idx, size, reduce)


def scatter_add(updates, indices, size=None):
    return _scatter(updates, indices, size, "add")


def scatter_mean(updates, indices, size=None):
    return _scatter(updates, indices, size, "mean")


def scatter_max(updates, indices, size=None):
    return _scatter(updates, indices, size, "max")


def scatter_(op, updates, indices, size=None):
    """Dispatch by name, like the reference's ``mp_ops.scatter_`` (``add|mean|max``)."""
    assert op in ("add", "mean", "max")
    return _scatter(updates, indices, size, op)


class _EdgeSoftmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, seg):
        shape = logits.shape
        l2 = logits.contiguous().reshape(shape[0], -1)
        p = hip().edge_softmax(l2, seg.indptr, seg.perm)
        ctx.seg, ctx.shape = seg, shape
        ctx.save_for_backward(p)
        return p.reshape(shape)

    @staticmethod
    def backward(ctx, g):
        (p,) = ctx.saved_tensors
        g2 = g.contiguous().reshape(p.shape).to(p.dtype)
        gin = hip().edge_softmax_bwd(p, g2, ctx.seg.indptr, ctx.seg.perm)
        return gin.reshape(ctx.shape), None


class _SpmmIndex:
    """Destination CSR and source CSC of one ``edge_index`` for weighted aggregation.  The
    CSC (a sort of the sources) is built on first use: only a backward into ``x`` needs it,
    and a first layer over constant features has none."""

    def __init__(self, edge_index, size):
        self.edge_index = edge_index
        self.dst = cached_segment(edge_index, 0, size[0])
        self.src = cached_segment(edge_index, 1, size[1])
        self.col = edge_index[1].reshape(-1).long()[self.dst.perm].contiguous()   # sources, CSR order
        self._row = None

    @property
    def row(self):
        """destinations in CSC order"""
        if self._row is None:
            self._row = self.edge_index[0].reshape(-1).long()[self.src.perm].contiguous()
        return self._row


def _spmm_index(edge_index, size):
    # keyed on the tensor's version counter too: an in-place write to a caller's
    # edge_index (copy_, index_put_) invalidates the cached CSR / CSC
    key = "_euler_spmm_%d_%d_v%d" % (int(size[0]), int(size[1]), int(edge_index._version))
    cache = getattr(edge_index, "_euler_cache", None)
    if cache is None:
        cache = {}
        try:
            edge_index._euler_cache = cache
        except AttributeError:
            return _SpmmIndex(edge_index, size)
    if key not in cache:
        cache[key] = _SpmmIndex(edge_index, size)
    return cache[key]


class _WeightedAggregate(torch.autograd.Function):
    """K4: out = A x with A[dst, src] = w_e (CSR SpMM); backward dx = A^T dout over the
    CSC, both one launch of ``spmm_csr`` with fp32 accumulation."""

    @staticmethod
    def forward(ctx, x, w, idx):
        wd = None if w is None else w[idx.dst.perm].contiguous()
        ctx.idx, ctx.w, ctx.dtype = idx, w, x.dtype
        return hip().spmm_csr(idx.dst.indptr, idx.col, wd, x.contiguous())

    @staticmethod
    def backward(ctx, g):
        idx, w = ctx.idx, ctx.w
        ws = None if w is None else w[idx.src.perm].contiguous()
        dx = hip().spmm_csr(idx.src.indptr, idx.row, ws, g.to(ctx.dtype).contiguous())
        return dx, None, None


def weighted_aggregate(x, edge_index, size, weight=None):
    """``out[i] = sum_{e: dst(e) = i} weight_e * x[src(e)]`` (``edge_index`` row 0 =
    destination, row 1 = source) — the GCN-family normalised aggregation
    (gcn_conv.py:42-54: gather, gather, gather, multiply, scatter_add) as one SpMM.
    ``weight`` (per edge) is treated as a constant (no gradient)."""
    size = (int(size[0]), int(size[1]))
    w = None if weight is None else weight.reshape(-1).float().detach()
    if use_hip(x) and x.dim() == 2 and x.dtype in (torch.float32, torch.bfloat16):
        return _WeightedAggregate.apply(x, w, _spmm_index(edge_index, size))
    dst, src = edge_index[0].reshape(-1).long(), edge_index[1].reshape(-1).long()
    keep = (dst >= 0) & (src >= 0)
    vals = x[src[keep]]
    if w is not None:
        vals = vals * w[keep].to(x.dtype).view(-1, *([1] * (x.dim() - 1)))
    return torch.zeros((size[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device).index_add(0, dst[keep], vals)


class _EmbeddingBag(torch.autograd.Function):
    """K9: out[b] = sum_{j in bag b} w_j table[ids_j] as ONE CSR SpMM launch (no [nnz, D]
    intermediate); backward = per-id rows w_j dout[bag(j)] added into the table grad."""

    @staticmethod
    def forward(ctx, table, indptr, ids, w, bag_of):
        ctx.save_for_backward(ids, w, bag_of)
        ctx.n = table.shape[0]
        return hip().spmm_csr(indptr, ids, w, table.contiguous())

    @staticmethod
    def backward(ctx, g):
        ids, w, bag_of = ctx.saved_tensors
        rows = hip().gather_rows(g.contiguous(), bag_of) * w.unsqueeze(1).to(g.dtype)
        acc = torch.zeros((ctx.n, g.shape[1]), dtype=torch.float32, device=g.device)
        hip().index_add_rows_(acc, ids, rows.contiguous())
        return acc.to(g.dtype), None, None, None, None


def embedding_bag(table, ids, bag_of, num_bags, combiner="sum", weights=None):
    """Embedding-bag (``tf.nn.embedding_lookup_sparse``, reference layers.py:152-169):
    ``out[b] = combine_{j: bag_of[j] == b} weights_j * table[ids_j]`` with combiner
    ``sum`` or ``mean``; ``bag_of`` must be sorted (SparseTensor row order)."""
    ids = ids.reshape(-1).long()
    bag_of = bag_of.reshape(-1).long()
    num_bags = int(num_bags)
    w = torch.ones(ids.numel(), dtype=torch.float32, device=ids.device) if weights is None else \
        weights.reshape(-1).float()
    cnt = torch.bincount(bag_of, minlength=num_bags)[:num_bags]
    if combiner == "mean":
        w = w / cnt.clamp(min=1).to(w.dtype)[bag_of]
    if use_hip(table, ids) and table.dtype in (torch.float32, torch.bfloat16) and table.dim() == 2:
        indptr = torch.zeros(num_bags + 1, dtype=torch.long, device=ids.device)
        torch.cumsum(cnt, 0, out=indptr[1:])
        return _EmbeddingBag.apply(table, indptr, ids.contiguous(), w.contiguous(), bag_of.contiguous())
    vals = table[ids] * w.unsqueeze(1).to(table.dtype)
    return torch.zeros((num_bags, table.shape[1]), dtype=table.dtype, device=table.device).index_add(0, bag_of, vals)


def scatter_softmax(logits, indices, size=None):
    """Softmax of ``logits`` grouped by destination ``indices`` (reference mp_ops.py:76-79)."""
    if size is None:
        size = int(indices.max().item()) + 1 if indices.numel() else 0
    if use_hip(logits) and logits.dtype in (torch.float32, torch.bfloat16):
        return _EdgeSoftmax.apply(logits, segment_index(indices, size))
    idx = indices.indices if isinstance(indices, SegmentIndex) else indices.reshape(-1).long()
    # padding entries (index -1) get 0, as on the GPU, and stay out of every sum (an
    # out-of-range read here would divide by an empty segment's 0 and poison the gradients)
    valid = (idx >= 0).view(-1, *([1] * (logits.dim() - 1)))
    safe = idx.clamp(min=0)
    mx = _cpu_scatter(logits.detach(), idx, size, "max")
    z = torch.exp(logits - mx[safe]) * valid.to(logits.dtype)
    den = _cpu_scatter(z, idx, size, "add")
    return z / den[safe].clamp_min(1e-30)
