"""Row-sharded node-feature table for the device trainers (GPU-sharded DeviceGraph,
design note docs/DESIGN.md §5 "Sharded features").

The reference scales a graph past one machine by partitioning it (``(id % P) % S``
shards, euler/core/graph/graph.cc:90-98); every worker fetches the features of its
sampled nodes from the owning shard server.  Here the node's GPUs are the shards: row
``r`` of the feature table lives on rank ``r % world`` at local row ``r // world``, so a
node holds ``world x 288 GB`` of features instead of one GPU's worth.

One exchange per step, between the sampler and the fused forward (all of it
hipGraph-capturable: fixed shapes, no host-read sizes):

  ids [n]           every sampled tree row and leaf of this rank's batch (-1 = none)
  unique            ``unique_first_padded`` (hash kernel): each distinct id once
  route             owner = id % W, stable rank per owner (route.hip), C slots per peer
                    (fixed capacity, the ShardedTable.lookup_static scheme); an id that does
                    not fit raises the device ``overflow`` flag and reads the zero trash row
  all-to-all ids    W*C int64 per rank
  gather + all-to-all rows   the owners gather their local rows (bf16) and send them back
                    straight into the trainer's fixed feature-cache buffer
  positions         pos[k] = cache row of ids[k] (-1 stays -1): the fused forward
                    gathers from the cache exactly as it gathers from a whole table

Bytes per step and rank: 8 W C (ids) + 2 D W C (bf16 rows), ~(W-1)/W of it over xGMI.
At the headline shape (B = 1024, fanouts 25 x 10: n = 32768 tree rows + 327680 leaves)
that is ~92 MB of rows for D = 128 (cost model in docs/DESIGN.md §5).
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist

from euler_amd.ops import mp_ops
from euler_amd.ops._native import use_hip
from euler_amd.ops.gnn_ops import route_by_owner, unique_first_padded
from euler_amd.parallel import comm

__all__ = ["ShardedFeatures"]


class ShardedFeatures:
    def __init__(self, shard: torch.Tensor, num_rows: int, group=None, force_comm: bool = False,
                 dedup: bool = True):
        self.group = group
        init = dist.is_available() and dist.is_initialized()
        on = init and dist.get_world_size(group) > 1
        self.world = dist.get_world_size(group) if on else 1
        self.rank = dist.get_rank(group) if on else 0
        self.comm = on or (init and force_comm)
        self.num_rows = int(num_rows)
        want = max(0, math.ceil((self.num_rows - self.rank) / self.world))
        if shard.dim() != 2 or shard.shape[0] != want:
            raise ValueError(f"rank {self.rank} must hold rows r % {self.world} == {self.rank}: {want} rows, "
                             f"got {tuple(shard.shape)}")
        self.shard = shard.contiguous()
        self.dim = int(shard.shape[1])
        self.dedup = bool(dedup)
        self.device = shard.device
        self.overflow = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.cap_override = None
        self.cache = None

    @classmethod
    def from_full(cls, x: torch.Tensor, group=None, force_comm: bool = False, **kw):
        """this rank's shard of a full [N, D] table (tests / small graphs)"""
        init = dist.is_available() and dist.is_initialized()
        on = init and dist.get_world_size(group) > 1
        w, r = (dist.get_world_size(group), dist.get_rank(group)) if on else (1, 0)
        return cls(x[r::w].contiguous(), x.shape[0], group, force_comm, **kw)

    def capacity(self, n: int) -> int:
        """slots per peer for n ids per rank (mean + 6 sigma + 64, rounded to 64)"""
        if self.cap_override is not None:
            return int(self.cap_override)
        if self.world == 1:
            return int(n)
        mean = n / self.world
        return min(int(n), int(math.ceil((mean + 6.0 * math.sqrt(mean) + 64) / 64.0)) * 64)

    def cache_rows(self, n: int) -> int:
        """rows of the feature cache for n ids: W*C exchange slots + the zero trash row"""
        return self.world * self.capacity(n) + 1

    def alloc_cache(self, n: int) -> torch.Tensor:
        self.cache = torch.zeros(self.cache_rows(n), self.dim, dtype=self.shard.dtype, device=self.device)
        return self.cache

    def check_overflow(self):
        if int(self.overflow.item()):
            raise RuntimeError("ShardedFeatures: a fixed-capacity exchange overflowed its per-peer slots "
                               "(those rows read zeros); raise the capacity")

    def _gather(self, local):
        if use_hip(self.shard, local):
            return mp_ops.gather(self.shard, local)
        return self.shard[local.clamp(min=0)]

    def exchange(self, ids: torch.Tensor, pos_out: torch.Tensor = None) -> torch.Tensor:
        """Fill :attr:`cache` with the rows of ``ids`` and return their cache positions
        (int32, -1 where ids < 0); ``pos_out`` receives them in place if given."""
        ids = ids.reshape(-1)
        n = ids.numel()
        if self.cache is None or self.cache.shape[0] != self.cache_rows(n):
            self.alloc_cache(n)
        W, C = self.world, self.capacity(n)
        trash = W * C
        i64 = ids.long()
        if self.dedup:
            u, inv, _ = unique_first_padded(i64)
        else:
            u, inv = i64, None
        if not self.comm:
            # one rank without collectives: the cache is a plain gather
            local = torch.where(u >= 0, u, torch.full_like(u, -1))
            self.cache[:n].copy_(self._gather(local))
            pu = torch.arange(n, device=ids.device)
        else:
            # slot layout: the peers' C-slot blocks in rank order, then this rank's own block;
            # only the peers' prefix goes through the (uneven-split) all-to-alls, the own
            # block's rows are gathered straight into the cache (no RCCL self-copy; with one
            # rank no collective at all)
            pu, send = route_by_owner(u, W, C, self.overflow, self.rank)
            P = trash - C
            if P:
                sp = [0 if r == self.rank else C for r in range(W)]
                recv = torch.empty(P, dtype=torch.long, device=ids.device)
                comm.all_to_all_single(recv, send[:P], sp, sp, group=self.group)
                local = torch.where(recv >= 0, torch.div(recv, W, rounding_mode="floor"), torch.full_like(recv, -1))
                rows = self._gather(local).to(self.cache.dtype).contiguous()
                comm.all_to_all_single(self.cache[:P], rows, sp, sp, group=self.group)
            own = send[P:trash]
            local = torch.where(own >= 0, torch.div(own, W, rounding_mode="floor"), torch.full_like(own, -1))
            self.cache[P:trash].copy_(self._gather(local))
        pos = pu if inv is None else pu[inv]
        pos = torch.where(i64 >= 0, pos, torch.full_like(pos, -1)).int()
        if pos_out is not None:
            pos_out.copy_(pos)
            return pos_out
        return pos
