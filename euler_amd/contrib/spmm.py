"""``spmm_add`` / ``spmm_mean`` (reference ``contrib/spmm.py:23-41``).

The reference builds an unweighted sparse adjacency ``A[edge_index[0], edge_index[1]] = 1``
of shape ``size`` and returns ``A @ src`` (``spmm_add``) or ``(A @ src) / (A @ 1)``
(``spmm_mean``; rows with no edges divide by zero there — here they yield 0).  Row 0 of
``edge_index`` is the output row, row 1 the ``src`` row, matching the reference.  On a GPU
both are one CSR SpMM launch (``spmm_csr`` in ``csrc/hip/mp.hip``) via
:func:`euler_amd.ops.mp_ops.weighted_aggregate`; the mean folds ``1/deg`` into the
per-edge weight instead of a second SpMM for the counts.
"""
from __future__ import annotations

import torch

from euler_amd.ops import mp_ops


def _size(src, edge_index, size):
    """Output / source row counts, with every index checked against them on the host
    (the reference's SparseTensor raises on out-of-range or negative indices; the GPU
    kernel does not bound-check its source rows, so this is the only guard)."""
    if edge_index.dim() != 2 or edge_index.shape[0] != 2:
        raise ValueError("edge_index must have shape [2, E]")
    n_src = int(src.shape[0])
    if size is None:
        n_out = int(edge_index[0].max().item()) + 1 if edge_index.numel() else 0
        size = (n_out, n_src)
    size = (int(size[0]), int(size[1]))
    if size[1] != n_src:
        raise ValueError(f"size[1] = {size[1]} does not match src rows {n_src}")
    if edge_index.numel():
        lo = edge_index.min(dim=1).values.tolist()
        hi = edge_index.max(dim=1).values.tolist()
        if min(lo) < 0:
            raise ValueError("edge_index holds negative indices")
        if hi[0] >= size[0] or hi[1] >= size[1]:
            raise ValueError(f"edge_index out of range for size {size}: max rows {hi[0]}, {hi[1]}")
    return size


def spmm_add(src, edge_index, size=None, flow="target_to_source"):
    """``out[i] = sum_{e: edge_index[0,e] = i} src[edge_index[1,e]]``."""
    del flow  # the reference accepts and ignores it as well
    return mp_ops.weighted_aggregate(src, edge_index, _size(src, edge_index, size))


def spmm_mean(src, edge_index, size=None, flow="target_to_source"):
    """``spmm_add`` divided by each output row's edge count (0 for empty rows)."""
    del flow
    size = _size(src, edge_index, size)
    dst = edge_index[0].reshape(-1).long()  # indices validated non-negative by _size
    deg = torch.bincount(dst, minlength=size[0])[: size[0]].clamp(min=1).float()
    return mp_ops.weighted_aggregate(src, edge_index, size, weight=1.0 / deg[dst])


def spmm_(op, src, edge_index, size=None, flow="target_to_source"):
    """Dispatch by name: ``op`` in {``add``, ``mean``} (reference ``spmm.py:40-41``)."""
    fn = {"add": spmm_add, "mean": spmm_mean}.get(op)
    if fn is None:
        raise ValueError("spmm_: unknown op %r (expected 'add' or 'mean')" % (op,))
    return fn(src, edge_index, size, flow)
