"""Scatter ops with a ``fill_value`` (reference ``contrib/py_scatter.py:25-58``).

The reference ran these as numpy ``py_func`` loops (one host round trip per call, gradient
``gather(grad, indices)`` registered by hand).  Here they are the HIP segment reductions of
:mod:`euler_amd.ops.mp_ops` with autograd; ``fill_value`` is added to every output row for
``scatter_add`` (the reference initialises the accumulator with it) and used for rows that
receive no update for ``scatter_max`` / ``scatter_mean``.
"""
from __future__ import annotations

import torch

from euler_amd.ops import mp_ops


def _size(indices, size):
    if size is None:
        return int(indices.max().item()) + 1 if indices.numel() else 0
    return int(size)


def _empty_rows(indices, size):
    idx = indices.reshape(-1).long()
    cnt = torch.bincount(idx[idx >= 0], minlength=size)[:size]
    return cnt == 0


def scatter_add(src, indices, size=None, fill_value=0):
    size = _size(indices, size)
    out = mp_ops.scatter_add(src, indices, size)
    return out + fill_value if fill_value != 0 else out


def scatter_mean(src, indices, size=None, fill_value=0):
    size = _size(indices, size)
    out = mp_ops.scatter_mean(src, indices, size)
    if fill_value != 0:
        empty = _empty_rows(indices, size).view(-1, *([1] * (out.dim() - 1)))
        out = torch.where(empty, torch.full_like(out, fill_value), out)
    return out


def scatter_max(src, indices, size=None, fill_value=0):
    size = _size(indices, size)
    out = mp_ops.scatter_max(src, indices, size)
    empty = _empty_rows(indices, size).view(-1, *([1] * (out.dim() - 1)))
    return torch.where(empty, torch.full_like(out, fill_value), out)


def scatter_(op, src, indices, size=None, fill_value=0):
    fn = {"add": scatter_add, "mean": scatter_mean, "max": scatter_max}.get(op)
    if fn is None:
        raise ValueError("scatter_: unknown op %r" % (op,))
    return fn(src, indices, size, fill_value)
