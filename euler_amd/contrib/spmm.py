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
    if size is None:
        n_out = int(edge_index[0].max().item()) + 1 if edge_index.numel() else 0
        return n_out, int(src.shape[0])
    return int(size[0]), int(size[1])


def spmm_add(src, edge_index, size=None, flow="target_to_source"):
    """``out[i] = sum_{e: edge_index[0,e] = i} src[edge_index[1,e]]``."""
    del flow  # the reference accepts and ignores it as well
    return mp_ops.weighted_aggregate(src, edge_index, _size(src, edge_index, size))


def spmm_mean(src, edge_index, size=None, flow="target_to_source"):
    """``spmm_add`` divided by each output row's edge count (0 for empty rows)."""
    del flow
    size = _size(src, edge_index, size)
    dst = edge_index[0].reshape(-1).long()
    deg = torch.bincount(dst[dst >= 0], minlength=size[0])[: size[0]].clamp(min=1).float()
    w = torch.where(dst >= 0, 1.0 / deg[dst.clamp(min=0)], torch.zeros_like(deg[:1]))
    return mp_ops.weighted_aggregate(src, edge_index, size, weight=w)


def spmm_(op, src, edge_index, size=None, flow="target_to_source"):
    """Dispatch by name: ``op`` in {``add``, ``mean``} (reference ``spmm.py:40-41``)."""
    fn = {"add": spmm_add, "mean": spmm_mean}.get(op)
    if fn is None:
        raise ValueError("spmm_: unknown op %r (expected 'add' or 'mean')" % (op,))
    return fn(src, edge_index, size, flow)
