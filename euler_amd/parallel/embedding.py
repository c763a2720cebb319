"""Row-sharded embedding tables with all-to-all lookup — the replacement for the
reference's PS ``mod``-partitioned variables (``tf_euler/python/utils/embedding.py:24-58``,
``layers.py:135-140``; SURVEY §2.8 "Embedding / model parallelism").

Row ``r`` of a table of ``num`` rows lives on rank ``r % world`` at local index
``r // world``.  A lookup routes ids to their owners with one ``all_to_all_single``,
gathers the rows locally and routes them back with a second; backward routes the
row gradients to the owners and accumulates them into the local shard.  With 288 GB
of HBM per MI355X a table of billions of rows fits across one node, and the
all-to-all over xGMI moves only the touched rows.

Sharded parameters carry ``_euler_sharded = True`` so the data-parallel gradient
all-reduce (:class:`~euler_amd.parallel.dp.GradSync`) skips them.
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist
import torch.nn as nn

from euler_amd.ops import mp_ops
from euler_amd.parallel import comm

__all__ = ["ShardedEmbedding", "sharded_lookup", "is_sharded", "sharded_param_names", "reshard_rows"]


def is_sharded(p) -> bool:
    return bool(getattr(p, "_euler_sharded", False))


class _ShardedLookup(torch.autograd.Function):
    @staticmethod
    def forward(ctx, weight, ids, group):
        W = dist.get_world_size(group)
        owner = torch.remainder(ids, W)
        order = torch.argsort(owner, stable=True)
        sorted_ids = ids[order]
        send_counts = torch.bincount(owner, minlength=W)
        recv_counts = torch.empty_like(send_counts)
        comm.all_to_all_single(recv_counts, send_counts, group=group)
        send_l, recv_l = send_counts.tolist(), recv_counts.tolist()
        recv_ids = torch.empty(sum(recv_l), dtype=ids.dtype, device=ids.device)
        comm.all_to_all_single(recv_ids, sorted_ids, recv_l, send_l, group=group)
        local = torch.div(recv_ids, W, rounding_mode="floor")
        rows = mp_ops.gather(weight, local) if weight.is_cuda else weight[local]
        out_sorted = torch.empty(ids.numel(), weight.shape[1], dtype=weight.dtype, device=weight.device)
        comm.all_to_all_single(out_sorted, rows.contiguous(), send_l, recv_l, group=group)
        out = torch.empty_like(out_sorted)
        out[order] = out_sorted
        ctx.save_for_backward(order, local)
        ctx.splits = (send_l, recv_l)
        ctx.group = group
        ctx.shape = weight.shape
        return out

    @staticmethod
    def backward(ctx, g):
        order, local = ctx.saved_tensors
        send_l, recv_l = ctx.splits
        g_sorted = g[order].contiguous()
        recv_g = torch.empty(sum(recv_l), g.shape[1], dtype=g.dtype, device=g.device)
        comm.all_to_all_single(recv_g, g_sorted, recv_l, send_l, group=ctx.group)
        gw = torch.zeros(ctx.shape, dtype=g.dtype, device=g.device)
        gw.index_add_(0, local, recv_g)
        return gw, None, None


def sharded_lookup(weight, ids, group=None):
    return _ShardedLookup.apply(weight, ids.reshape(-1).long(), group)


class ShardedEmbedding(nn.Module):
    """``max_id + 1`` rows sharded ``mod world`` across the process group.

    Falls back to a plain local table when not running distributed, so the same model
    code runs on one GPU and on eight.
    """

    def __init__(self, max_id, dim, group=None, initializer=None):
        super().__init__()
        self.num = int(max_id) + 1
        self.dim = int(dim)
        self.group = group
        distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
        self.world = dist.get_world_size(group) if distributed else 1
        self.rank = dist.get_rank(group) if distributed else 0
        local_rows = max(0, math.ceil((self.num - self.rank) / self.world))
        self.weight = nn.Parameter(torch.empty(local_rows, self.dim))
        if initializer is None:
            nn.init.trunc_normal_(self.weight, std=0.1, a=-0.2, b=0.2)
        else:
            initializer(self.weight)
        self.weight._euler_sharded = self.world > 1

    def forward(self, ids):
        ids = torch.as_tensor(ids, device=self.weight.device).long()
        shape = ids.shape
        ids = torch.where((ids < 0) | (ids >= self.num), torch.full_like(ids, self.num - 1), ids).reshape(-1)
        if self.world == 1:
            out = mp_ops.gather(self.weight, ids)
        else:
            out = sharded_lookup(self.weight, ids, self.group)
        return out.reshape(*shape, self.dim)

    def global_ids(self):
        """ids of the rows this rank owns, in local order."""
        return torch.arange(self.weight.shape[0], device=self.weight.device) * self.world + self.rank


def sharded_param_names(model: nn.Module):
    """state_dict names of every ShardedEmbedding table of ``model`` (sharded or not in
    the current run: a one-process run holds the whole table)."""
    return {(name + "." if name else "") + "weight" for name, m in model.named_modules()
            if isinstance(m, ShardedEmbedding)}


def reshard_rows(parts, new_rank: int, new_world: int) -> torch.Tensor:
    """Re-shard a ``mod``-sharded table saved by ``len(parts)`` ranks (part r holds global
    rows r, r + W, r + 2W, ...) for rank ``new_rank`` of ``new_world``: the checkpoint
    restores with a different world size."""
    W = len(parts)
    n = sum(int(p.shape[0]) for p in parts)
    full = torch.empty((n,) + tuple(parts[0].shape[1:]), dtype=parts[0].dtype)
    for r, part in enumerate(parts):
        full[r::W] = part.to(full.device)
    return full[new_rank::new_world].clone()
