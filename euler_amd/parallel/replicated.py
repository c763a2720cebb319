"""Replicated row stores kept consistent across data-parallel ranks (SURVEY §2.7 C3:
the Scalable* encoders' historical-embedding and gradient stores, "the same row-sharded
store over all-to-all, or replicated when small").

The reference keeps these stores as PS variables that every worker reads and
``scatter_update`` / ``scatter_add``s (``tf_euler/python/utils/encoders.py:373-408``,
657-748), so each worker sees the others' writes.  Here every rank holds a full replica
in HBM (a store is ``(max_id + 2) x dim``: 288 GB per GPU holds billions of rows) and
the per-step row writes are exchanged with one variable-length all-gather per tensor;
every rank then applies all ranks' writes in rank order, so the replicas stay
bitwise identical.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

__all__ = ["sync_group", "all_gather_varlen", "apply_replicated"]


def sync_group(group=None):
    """``group`` when torch.distributed is initialised with more than one rank, else None."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        return group if group is not None else dist.group.WORLD
    return None


def all_gather_varlen(t: torch.Tensor, group=None) -> torch.Tensor:
    """Concatenation over ranks (rank order) of tensors whose first dims differ."""
    W = dist.get_world_size(group)
    n = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
    ns = [torch.empty_like(n) for _ in range(W)]
    dist.all_gather(ns, n, group=group)
    counts = [int(c.item()) for c in ns]
    m = max(counts)
    pad = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[:t.shape[0]] = t
    outs = [torch.empty_like(pad) for _ in range(W)]
    dist.all_gather(outs, pad.contiguous(), group=group)
    return torch.cat([o[:c] for o, c in zip(outs, counts)], 0)


@torch.no_grad()
def apply_replicated(store: torch.Tensor, rows: torch.Tensor, values, op: str, group=None):
    """Apply one step's row writes of every rank to this rank's replica.

    op: ``"copy"`` (store[rows] = values; later ranks win on shared rows), ``"add"``
    (store[rows] += values) or ``"zero"`` (store[rows] = 0; ``values`` ignored).
    Without a multi-rank group it is the local write."""
    g = sync_group(group)
    rows = rows.reshape(-1).long()
    if g is not None:
        rows = all_gather_varlen(rows, g)
        if op != "zero":
            values = all_gather_varlen(values.reshape(-1, store.shape[1]).to(store.dtype).contiguous(), g)
    if op == "copy":
        store.index_copy_(0, rows, values.reshape(-1, store.shape[1]).to(store.dtype))
    elif op == "add":
        store.index_add_(0, rows, values.reshape(-1, store.shape[1]).to(store.dtype))
    elif op == "zero":
        store.index_fill_(0, rows, 0.0)
    else:
        raise ValueError("op must be copy | add | zero")
