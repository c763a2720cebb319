"""Row-sharded historical stores ("the same row-sharded store over
all-to-all, or replicated when small"; the replicated form is parallel/replicated.py).

The Scalable* encoders keep per-layer stale embeddings and gradient stores of every node
(reference ``tf_euler/python/utils/encoders.py:313-408, 657-748``: PS variables read with
``gather`` and written with ``scatter_update`` / ``scatter_add`` by every worker).  When a
store is too large to replicate on every rank, :class:`ShardedRowStore` keeps row ``r`` on
rank ``r % world`` (local row ``r // world``): a read routes the ids to their owners and
the rows back (two ``all_to_all_single``), a write routes ``(id, value)`` pairs to the
owners, which apply them in source-rank order — the same per-row outcome as the
replicated store, with 1/world of the memory and only the touched rows on the wire.
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist

from euler_amd.parallel import comm

__all__ = ["ShardedRowStore"]


class ShardedRowStore:
    def __init__(self, num_rows, dim, device, group=None, init=None, dtype=torch.float32):
        self.num_rows, self.dim = int(num_rows), int(dim)
        self.group = group
        on = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
        self.world = dist.get_world_size(group) if on else 1
        self.rank = dist.get_rank(group) if on else 0
        local = max(0, math.ceil((self.num_rows - self.rank) / self.world))
        self.local = torch.zeros(local, self.dim, dtype=dtype, device=device)
        if init is not None:  # init(global_ids) -> [n, D]: the rows this rank owns
            self.local.copy_(init(self.global_ids()).to(self.local))

    @property
    def device(self):
        return self.local.device

    def global_ids(self):
        return torch.arange(self.local.shape[0], device=self.device) * self.world + self.rank

    def _route(self, ids):
        """(order, send counts, recv counts, received ids) of an owner-routed exchange"""
        W = self.world
        owner = torch.remainder(ids, W)
        order = torch.sort(owner, stable=True)[1]
        send = torch.bincount(owner, minlength=W)
        recv = torch.empty_like(send)
        comm.all_to_all_single(recv, send, group=self.group)
        counts = torch.stack([send, recv]).cpu()
        s, r = counts[0].tolist(), counts[1].tolist()
        rid = torch.empty(sum(r), dtype=ids.dtype, device=ids.device)
        comm.all_to_all_single(rid, ids[order].contiguous(), r, s, group=self.group)
        return order, s, r, rid

    @torch.no_grad()
    def read(self, ids: torch.Tensor) -> torch.Tensor:
        """rows [n, D] of global ids (any order, repeats allowed)"""
        ids = ids.reshape(-1).long().to(self.device)
        if self.world == 1:
            return self.local[ids]
        order, s, r, rid = self._route(ids)
        rows = self.local[torch.div(rid, self.world, rounding_mode="floor")]
        back = torch.empty(ids.numel(), self.dim, dtype=rows.dtype, device=rows.device)
        comm.all_to_all_single(back, rows.contiguous(), s, r, group=self.group)
        out = torch.empty_like(back)
        out[order] = back
        return out

    @torch.no_grad()
    def write(self, ids: torch.Tensor, values, op: str):
        """op ``copy`` (later source ranks win on shared rows), ``add`` or ``zero``"""
        if op not in ("copy", "add", "zero"):
            raise ValueError("op must be copy | add | zero")
        ids = ids.reshape(-1).long().to(self.device)
        if op != "zero":
            values = values.reshape(-1, self.dim).to(self.local.dtype).to(self.device)
        if self.world == 1:
            rows, vals = ids, values
        else:
            order, s, r, rid = self._route(ids)
            rows = torch.div(rid, self.world, rounding_mode="floor")
            vals = None
            if op != "zero":
                vals = torch.empty(sum(r), self.dim, dtype=self.local.dtype, device=self.device)
                comm.all_to_all_single(vals, values[order].contiguous(), r, s, group=self.group)
        if op == "copy":
            self.local.index_copy_(0, rows, vals)
        elif op == "add":
            self.local.index_add_(0, rows, vals)
        else:
            self.local.index_fill_(0, rows, 0.0)

    def nbytes(self):
        return self.local.numel() * self.local.element_size()
