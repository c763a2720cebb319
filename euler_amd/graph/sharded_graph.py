"""A graph larger than one GPU's HBM: the CSR, the feature table and the labels row-sharded
over the data-parallel ranks, with cross-GPU neighbour sampling.

The reference scales a graph past one machine by partitioning its nodes over shard servers
(``(id % partitions) % shards``, ``euler/core/graph/graph.cc:90-98``); a query's
``API_SAMPLE_NEIGHBOR`` / ``API_GET_P`` is split by owner (``euler/core/kernels/
id_split_op.cc:46-49``), sent to every owning shard (``remote_op.cc:60-146``) and merged
back in the caller's order (``id_unique_op`` / ``merge`` kernels).  Here the node's GPUs are
the shards and RCCL's all-to-all over xGMI is the transport:

* row ``r`` (engine rows: node ids sorted) lives on rank ``r % W`` at local row ``r // W``:
  its out-edges (neighbour values stay GLOBAL rows), its prefix-sum weights, its feature
  row and its label row — each GPU holds ~1/W of the graph;
* ``sample_neighbor(rows, F)``: ``route_by_owner`` gives every requested row a slot in a
  fixed-capacity ``[W, C]`` exchange (``csrc/hip/route.hip``; a row past its owner's C
  slots raises the ``overflow`` flag and draws ``default``), one all-to-all sends the rows
  to their owners, each owner draws F neighbours per received row from its local CSR with
  its Philox stream (the ordinary ``sample_neighbor`` kernel), and one all-to-all returns
  the ``[W, C, F]`` draws (and weights / types) to the requesters' slots — every
  occurrence draws independently, as with the whole graph;
* ``sample_node(B)``: exact global weighted root draws (reference ``sample_node`` over a
  sharded graph: the shards' node-weight sums pick the shard, ``graph.cc:333-403``): each
  root picks its owner from the alias table of the W shard sums, the per-owner tickets go
  through the same exchange, the owner draws that many local roots from its own alias table;
* features and labels: :class:`~euler_amd.graph.sharded_features.ShardedFeatures` exchanges
  (dedup, fixed capacity, zero row for ``-1``).

Every exchange has fixed shapes (no host-read sizes).  With one rank the object is the
ordinary local graph behind the same interface (no collective).

:class:`~euler_amd.models.full_trainer.ShardedFlowTrainer` trains the reference's sampled
``SageDataFlow`` models (any convolution) on it under ``NodeEstimator(device_graph=True,
device_graph_sharded=True)``.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.distributed as dist

from euler_amd.graph.device_graph import DeviceGraph, _upload, build_alias_table, shared_export
from euler_amd.graph.sharded_features import ShardedFeatures
from euler_amd.ops import mp_ops
from euler_amd.ops._native import hip, use_hip
from euler_amd.ops.gnn_ops import route_by_owner
from euler_amd.parallel import comm

__all__ = ["ShardedDeviceGraph", "shard_csr"]


def shard_csr(indptr, nbr, w, T: int, world: int, rank: int):
    """the rows ``r % world == rank`` of a host CSR (``indptr [N*T+1]``, raw edge weights):
    ``(indptr, nbr, w)`` of the local rows (neighbour values unchanged: global rows)"""
    indptr = np.asarray(indptr, np.int64)
    N = (indptr.shape[0] - 1) // T
    rows = np.arange(rank, N, world, dtype=np.int64)
    seg = (rows[:, None] * T + np.arange(T)[None, :]).reshape(-1)
    starts, lens = indptr[seg], indptr[seg + 1] - indptr[seg]
    lip = np.zeros(seg.shape[0] + 1, np.int64)
    np.cumsum(lens, out=lip[1:])
    take = np.repeat(starts - lip[:-1], lens) + np.arange(int(lip[-1]), dtype=np.int64)
    return lip, np.asarray(nbr)[take], np.asarray(w)[take]


class ShardedDeviceGraph:
    """``local``: the :class:`DeviceGraph` of this rank's rows (local row i = global row
    ``i * W + rank``; neighbour values are global rows), its root sampler over the local
    rows with ``root_weight`` their total root weight; ``num_rows`` the global row count;
    ``ids`` the sorted raw node ids of all rows (or None: rows are ids)."""

    def __init__(self, local: DeviceGraph, num_rows: int, root_weight: float = None, ids=None, group=None,
                 force_comm: bool = False, capacity_sigmas: float = 6.0):
        self.local = local
        self.group = group
        on = dist.is_available() and dist.is_initialized()
        multi = on and dist.get_world_size(group) > 1
        self.world = dist.get_world_size(group) if multi else 1
        self.rank = dist.get_rank(group) if multi else 0
        self.comm = multi or (on and force_comm)
        self.num_rows = int(num_rows)
        want = max(0, math.ceil((self.num_rows - self.rank) / self.world))
        if local.num_rows != want:
            raise ValueError(f"rank {self.rank} must hold the {want} rows r % {self.world} == {self.rank}, "
                             f"its local graph has {local.num_rows}")
        self.num_types = local.num_types
        self.device = local.device
        self.rng = local.rng
        self.ids = ids
        self.sigmas = float(capacity_sigmas)
        self.overflow = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.features = ShardedFeatures(local.features, self.num_rows, group, force_comm) \
            if local.features is not None else None
        # labels are fetched for a batch's roots only (few repeats): no dedup pass
        self.labels = ShardedFeatures(local.labels.float(), self.num_rows, group, force_comm, dedup=False) \
            if local.labels is not None else None
        self.set_root_weight(root_weight)

    # ------------------------------------------------------------------ construction
    @classmethod
    def from_full(cls, g: DeviceGraph, group=None, force_comm: bool = False, **kw):
        """this rank's shard of a whole :class:`DeviceGraph` (tests / small graphs): same
        rows, same edges, same root weights (the local alias tables are rebuilt from the
        whole graph's node weights when ``node_weights`` is given)"""
        on = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
        W, r = (dist.get_world_size(group), dist.get_rank(group)) if on else (1, 0)
        T = g.num_types
        indptr = g.indptr.cpu().numpy()
        cumw = g.cumw.cpu().numpy().astype(np.float64)
        # raw weights back from the per-segment prefix sums
        seg_start = np.repeat(indptr[:-1], np.diff(indptr))
        prev = np.where(np.arange(cumw.shape[0]) > seg_start, np.concatenate([[0.0], cumw[:-1]]), 0.0)
        w = cumw - prev
        lip, nbr, lw = shard_csr(indptr, g.nbr.cpu().numpy(), w, T, W, r)
        nw = kw.pop("node_weights", None)
        if nw is None:
            nw = _alias_weights(g)
        nw = np.asarray(nw, np.float64)
        local = DeviceGraph.from_csr(lip, nbr, lw, T, node_weights=nw[r::W] if nw[r::W].size else None,
                                     seed=int(g.rng[0]) + 7919 * r, device=g.device)
        if g.features is not None:
            local.features = g.features[r::W].contiguous()
        if g.labels is not None:
            local.labels = g.labels[r::W].contiguous()
        return cls(local, g.num_rows, float(nw[r::W].sum()), ids=g.ids, group=group, force_comm=force_comm, **kw)

    @classmethod
    def synthetic(cls, num_nodes: int, avg_degree: float = 10.0, max_degree: int = 1024, feature_dim: int = 128,
                  num_classes: int = 64, multi_label: bool = False, seed: int = 0, device="cuda", group=None,
                  force_comm: bool = False):
        """this rank's rows of a synthetic power-law graph generated straight in HBM (no
        host copy): the local CSR from the device generator with its neighbour values spread
        over every rank's rows, bf16 features and class (or multi-label) labels"""
        on = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
        W, r = (dist.get_world_size(group), dist.get_rank(group)) if on else (1, 0)
        n_local = max(0, math.ceil((int(num_nodes) - r) / W))
        loc = DeviceGraph.synthetic(n_local, avg_degree, max_degree, seed=seed * 7919 + r, device=device)
        if W > 1:
            v = loc.nbr.long()
            g = v * W + (v * 40503 + 17 * r) % W  # spread over the owners
            loc.nbr = torch.where(g < num_nodes, g, g - W).to(torch.int32)
        gen = torch.Generator(device=loc.device).manual_seed(seed * 31 + r)
        loc.features = torch.randn(n_local, feature_dim, generator=gen, device=loc.device).to(torch.bfloat16)
        if multi_label:
            loc.labels = (torch.rand(n_local, num_classes, generator=gen, device=loc.device) < 0.1).float()
        else:
            loc.labels = torch.randint(0, num_classes, (n_local, 1), generator=gen, device=loc.device).float()
        return cls(loc, int(num_nodes), float(n_local), group=group, force_comm=force_comm)

    @classmethod
    def from_engine(cls, engine=None, node_type=-1, features=(), feature_dims=(), label=None, label_dim=None,
                    feature_dtype=torch.bfloat16, seed=0, device="cuda", group=None):
        """this rank's rows of the engine's graph: the node's ranks share ONE host export
        (``shared_export``: local rank 0 writes /dev/shm, every rank maps it) and each uploads
        only its rows — CSR, features, labels and root weights (HBM holds 1/W of the graph)"""
        from euler_amd.graph.device_graph import _export_local
        from euler_amd.ops import base

        eng = engine if engine is not None else base.get_engine()
        if getattr(eng, "mode", "local") != "local":
            raise ValueError("the sharded device graph loads from an in-process engine")
        names = [] if not features else ([features] if isinstance(features, (str, int)) else list(features))
        dims = [] if not features else ([feature_dims] if isinstance(feature_dims, int) else list(feature_dims))
        on = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
        W, r = (dist.get_world_size(group), dist.get_rank(group)) if on else (1, 0)
        arrays, done = shared_export(lambda: _export_local(eng, names, dims, label, label_dim))
        try:
            T = int(np.asarray(arrays["T"])[0])
            ids = np.array(arrays["ids"])
            lip, nbr, lw = shard_csr(arrays["indptr"], arrays["nbr"], arrays["w"], T, W, r)
            nw = np.asarray(arrays["nw"], np.float64)[r::W].copy()
            types = np.asarray(arrays["types"])[r::W]
            if node_type is not None and int(node_type) >= 0:
                nw = np.where(types == int(node_type), nw, 0.0)
            local = DeviceGraph.from_csr(lip, nbr, lw, T, node_weights=nw if nw.size else None,
                                         seed=seed, device=device)
            local.node_types = types.copy()
            if names:
                local.features = _upload(np.asarray(arrays["features"])[r::W], torch.float32, device).view(
                    len(nw), -1).to(feature_dtype)
            if label is not None:
                local.labels = _upload(np.asarray(arrays["labels"])[r::W], torch.float32, device).view(len(nw), -1)
        finally:
            del arrays
            done()
        return cls(local, len(ids), float(nw.sum()), ids=ids, group=group)

    @classmethod
    def from_engine_shard(cls, engine=None, node_type=-1, features=(), feature_dims=(), label=None, label_dim=None,
                          feature_dtype=torch.bfloat16, seed=0, device="cuda", group=None):
        """the sharded graph from engines that each hold ONE shard of the on-disk graph
        (``initialize_graph({"mode": "local", ..., "shard_idx": rank, "shard_num": W})``:
        the partitions p % W == rank, reference graph.cc:90-98) — host memory per rank is
        1/W of the graph, not the whole of it.  Rank r's nodes (sorted by id) become the
        global rows i * W + r; the ranks all-gather their id lists once to map every
        neighbour id to its row (``searchsorted`` on the device); shards with fewer nodes
        than the largest are padded with edgeless, zero-feature, zero-weight rows."""
        from euler_amd.ops import base

        eng = engine if engine is not None else base.get_engine()
        names = [] if not features else ([features] if isinstance(features, (str, int)) else list(features))
        dims = [] if not features else ([feature_dims] if isinstance(feature_dims, int) else list(feature_dims))
        on = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
        W, r = (dist.get_world_size(group), dist.get_rank(group)) if on else (1, 0)
        device = torch.device(device)
        cols = ["dense_" + str(n) for n in names] + ([] if label is None else ["dense_" + str(label)])
        widths = [int(d) for d in dims] + ([] if label is None else [int(label_dim)])
        parts = eng.export_shard(0, cols, widths)
        ids = np.asarray(parts[0], np.uint64).astype(np.int64)
        types = np.asarray(parts[1], np.int32)
        nw = np.asarray(parts[2], np.float64)
        indptr = np.asarray(parts[3], np.int64)
        n = ids.shape[0]
        T = max(1, (indptr.shape[0] - 1) // n) if n else 1
        # the ranks' node counts and id lists -> global rows (i * W + rank); the collectives
        # run on the device under RCCL and on the host under gloo
        cdev = device if on and dist.get_backend(group) == "nccl" else torch.device("cpu")
        cnt = torch.tensor([n], dtype=torch.int64, device=cdev)
        counts = [torch.zeros_like(cnt) for _ in range(W)] if on else [cnt]
        if on:
            dist.all_gather(counts, cnt, group=group)
        M = int(max(int(c.item()) for c in counts))
        mine = torch.full((M,), -1, dtype=torch.int64, device=cdev)
        mine[:n] = torch.from_numpy(ids).to(cdev)
        every = [torch.empty_like(mine) for _ in range(W)] if on else [mine]
        if on:
            dist.all_gather(every, mine, group=group)
        all_ids = torch.stack(every, 1).reshape(-1).to(device)  # row g = i * W + rank -> its id (-1: padding)
        row_of = torch.arange(all_ids.numel(), device=device)
        valid = all_ids >= 0
        sid, order = torch.sort(all_ids[valid])
        srow = row_of[valid][order]
        del every, mine
        nbr_ids = torch.from_numpy(np.asarray(parts[4], np.uint64).astype(np.int64)).to(device)
        pos = torch.searchsorted(sid, nbr_ids).clamp(max=max(sid.numel() - 1, 0))
        nbr_rows = torch.where(sid[pos] == nbr_ids, srow[pos], torch.full_like(pos, -1)).to(torch.int32)
        del nbr_ids, pos
        pad = (M - n) * T
        lip = np.concatenate([indptr, np.full(pad, indptr[-1] if indptr.size else 0, np.int64)]) if pad else indptr
        if node_type is not None and int(node_type) >= 0:
            nw = np.where(types == int(node_type), nw, 0.0)
        nwp = np.zeros(M, np.float64)
        nwp[:n] = nw
        local = DeviceGraph.from_csr(lip, nbr_rows.cpu().numpy(), np.asarray(parts[5], np.float32), T,
                                     node_weights=nwp if M else None, seed=seed, device=device)
        tabs = [np.asarray(t, np.float32).reshape(n, w) for t, w in zip(parts[6:], widths)]
        if names:
            f = torch.zeros(M, sum(widths[: len(names)]), dtype=torch.float32)
            f[:n] = torch.from_numpy(np.concatenate(tabs[: len(names)], 1))
            local.features = f.to(device=device, dtype=feature_dtype)
        if label is not None:
            lab = torch.zeros(M, int(label_dim), dtype=torch.float32)
            lab[:n] = torch.from_numpy(tabs[-1])
            local.labels = lab.to(device)
        obj = cls(local, W * M, float(nw.sum()), ids=None, group=group)
        obj._id_table = (sid, srow)
        obj.row_ids = all_ids
        return obj

    def set_root_weight(self, root_weight=None):
        """the owner alias table of the W shards' root-weight sums (all-gathered)"""
        wl = float(self.local.node_prob.numel() if root_weight is None else root_weight)
        # on the graph's device: the process group's backend may be nccl (RCCL)
        sums = torch.tensor([wl], dtype=torch.float64, device=self.device)
        if self.comm:
            out = [torch.zeros(1, dtype=torch.float64, device=self.device) for _ in range(self.world)]
            dist.all_gather(out, sums, group=self.group)
            sums = torch.cat(out)
        self.shard_weight = sums.cpu().numpy().copy()
        if not (self.shard_weight > 0).any():
            raise ValueError("no shard holds a root candidate")
        p, a = build_alias_table(self.shard_weight)
        self._owner_prob = torch.from_numpy(p).to(self.device)
        self._owner_alias = torch.from_numpy(a).to(self.device)

    # ------------------------------------------------------------------ DeviceGraph interface
    def rows_of(self, ids) -> torch.Tensor:
        tab = getattr(self, "_id_table", None)
        if tab is None:
            return DeviceGraph.rows_of(self, ids)
        sid, srow = tab  # from_engine_shard: rows are not in id order
        q = torch.as_tensor(np.asarray(ids, dtype=np.uint64).astype(np.int64)).reshape(-1).to(sid.device)
        pos = torch.searchsorted(sid, q).clamp(max=max(sid.numel() - 1, 0))
        return torch.where(sid[pos] == q, srow[pos], torch.full_like(pos, -1)).cpu()

    def advance(self, inc: int = 1):
        self.local.advance(inc)

    def manual_seed(self, seed: int):
        self.local.manual_seed(int(seed))

    def reseed_cpu(self):
        self.local.reseed_cpu()

    def _mask(self, edge_types) -> int:
        return self.local._mask(edge_types)

    def nbytes(self) -> int:
        g = self.local
        return sum(t.numel() * t.element_size() for t in (g.indptr, g.nbr, g.cumw, g.node_prob, g.node_alias))

    def capacity(self, n: int) -> int:
        """exchange slots per peer for n requests (mean + sigmas * sqrt(mean) + 64, 64-aligned)"""
        if self.world == 1:
            return int(n)
        mean = n / self.world
        return min(int(n), int(math.ceil((mean + self.sigmas * math.sqrt(mean) + 64) / 64.0)) * 64)

    def check_overflow(self):
        for name, o in (("graph", self.overflow), ("features", getattr(self.features, "overflow", None)),
                        ("labels", getattr(self.labels, "overflow", None))):
            if o is not None and int(o.item()):
                raise RuntimeError(f"ShardedDeviceGraph: the {name} exchange overflowed its per-peer slots "
                                   "(those requests read -1 / zeros); raise capacity_sigmas")

    def _a2a(self, send: torch.Tensor) -> torch.Tensor:
        """equal-split all-to-all of [W * C, ...] (block o -> rank o)"""
        if not self.comm:
            return send.clone()
        recv = torch.empty_like(send)
        comm.all_to_all_single(recv, send.contiguous(), group=self.group)
        return recv

    def _route(self, keys: torch.Tensor):
        """(slot of every key [n], this rank's received keys [W*C], C) of the owner exchange
        (owner = key % W)"""
        n = keys.numel()
        C = self.capacity(n)
        pos, send = route_by_owner(keys, self.world, C, self.overflow)
        return pos, self._a2a(send[: self.world * C]), C

    def _local_rows(self, recv):
        return torch.where(recv >= 0, torch.div(recv, self.world, rounding_mode="floor"), torch.full_like(recv, -1))

    def _back(self, vals: torch.Tensor, pos: torch.Tensor, fill):
        """the owners' answers [W*C, ...] returned to the requesters' order (trash -> fill)"""
        back = self._a2a(vals)
        pad = torch.full((1,) + tuple(back.shape[1:]), fill, dtype=back.dtype, device=back.device)
        return torch.cat([back, pad])[pos]

    def sample_node(self, count: int, stream_id: int = 1) -> torch.Tensor:
        """``count`` global rows drawn with the global root weights"""
        if self.world == 1:
            return self.local.sample_node(int(count), stream_id)
        owner = self._alias(self._owner_prob, self._owner_alias, int(count), stream_id).long()
        tickets = torch.arange(int(count), device=self.device, dtype=torch.long) * self.world + owner
        pos, recv, C = self._route(tickets)
        # this rank draws one local root per received ticket (the empty slots draw too and
        # are dropped: fixed shapes)
        if self.local.node_prob.numel():
            loc = self.local.sample_node(self.world * C, stream_id=stream_id + 64).long()
        else:
            loc = torch.full((self.world * C,), -1, dtype=torch.long, device=self.device)
        glob = torch.where((recv >= 0) & (loc >= 0), loc * self.world + self.rank, torch.full_like(loc, -1))
        return self._back(glob.int(), pos, -1)

    def _alias(self, prob, alias, count, stream_id):
        if use_hip(prob):
            return hip().alias_sample(prob, alias, None, int(count), self.local.rng, int(stream_id))
        g = self.local._cpu_gen
        k = torch.randint(0, prob.numel(), (count,), generator=g)
        u = torch.rand(count, generator=g)
        return torch.where(u < prob[k], k, alias[k].long()).int()

    def sample_neighbor(self, rows: torch.Tensor, count: int, edge_types=None, default: int = -1,
                        stream_id: int = 2, with_weights: bool = False):
        """``count`` weighted draws with replacement per row (``[n, count]``, global rows),
        each drawn by the row's owner from its local CSR"""
        rows = rows.reshape(-1).long()
        n, F = rows.numel(), int(count)
        if self.world == 1 and not self.comm:
            return self.local.sample_neighbor(rows, F, edge_types, default, stream_id, with_weights)
        ok = (rows >= 0) & (rows < self.num_rows)
        pos, recv, C = self._route(torch.where(ok, rows, torch.full_like(rows, -1)))
        local = self._local_rows(recv)
        nb, w, t = self.local.sample_neighbor(local, F, edge_types, -1, stream_id, True)
        nb = nb.view(-1, F).int()  # global rows < 2^31: int32 halves the return all-to-all
        out_nb = self._back(nb, pos, -1)
        if int(default) != -1:
            out_nb = torch.where(out_nb >= 0, out_nb, torch.full_like(out_nb, int(default)))
        if not with_weights:
            return out_nb
        return out_nb, self._back(w.view(-1, F).float(), pos, 0.0), self._back(t.view(-1, F).int(), pos, -1)

    # ------------------------------------------------------------------ full neighbourhoods
    def _masked_degree(self, local_rows: torch.Tensor, mask: int) -> torch.Tensor:
        """out-degree over the edge types of ``mask`` of local rows (``-1``: 0)"""
        g, T = self.local, self.num_types
        ok = local_rows >= 0
        r = torch.where(ok, local_rows, torch.zeros_like(local_rows)) * T
        deg = torch.zeros(local_rows.shape, dtype=torch.long, device=local_rows.device)
        if g.num_rows == 0:
            return deg
        for t in range(T):
            if (mask >> t) & 1:
                deg += (g.indptr[r + t + 1] - g.indptr[r + t]).long()
        return torch.where(ok, deg, torch.zeros_like(deg))

    def _reduce(self, t: torch.Tensor, op) -> torch.Tensor:
        if self.comm:
            comm.all_reduce(t, op, group=self.group)
        return t

    def degree_stats(self, mask: int, k: int = 1):
        """(largest out-degree, edge count, k-th largest out-degree) over the edge types of
        ``mask`` and every rank's rows — the inputs of the full-neighbourhood flow's
        capacities (dataflow/device_flow.py exact_caps / bounded_caps).  The k-th largest
        comes from the all-reduced degree histogram (exact, W-independent)."""
        n = self.local.num_rows
        deg = self._masked_degree(torch.arange(n, device=self.device), int(mask))
        agg = torch.stack([deg.max() if n else torch.zeros((), dtype=torch.long, device=self.device),
                           deg.sum()])
        mx = int(self._reduce(agg[:1].clone(), dist.ReduceOp.MAX).item()) if self.comm else int(agg[0].item())
        total = int(self._reduce(agg[1:].clone(), dist.ReduceOp.SUM).item())
        hist = self._reduce(torch.bincount(deg, minlength=mx + 1)[: mx + 1], dist.ReduceOp.SUM)
        at_least = torch.flip(torch.cumsum(torch.flip(hist, [0]), 0), [0])  # rows with degree >= d
        hit = torch.nonzero(at_least >= max(1, int(k))).reshape(-1)
        kth = int(hit[-1].item()) if hit.numel() else 0
        return mx, total, kth

    def full_neighbors(self, rows: torch.Tensor, mask: int, cap: int, overflow: torch.Tensor):
        """``full_neighbors`` over the sharded rows: (neighbours [cap], target index [cap],
        inclusive per-target offsets [n]) — every neighbour of every row of the edge types of
        ``mask``, target-major in storage order, ``-1`` padding, exactly the whole graph's
        expansion (dataflow/device_flow.py full_neighbors_cpu).  Each row is expanded by its
        owner; the lists come back over one fixed-capacity all-to-all (``capacity(cap)`` slots
        per peer) and are laid out target-major by ``full_neighbors`` over the received
        blocks.  No host read: the step captures.  More than ``cap`` entries, or more than a
        peer's slots, set ``overflow`` (the flow regrows its caps)."""
        rows = rows.reshape(-1).long()
        n, dev = rows.numel(), self.device
        if not self.comm:
            g = self.local
            if use_hip(rows):
                return hip().full_neighbors(g.indptr, g.nbr, g.num_rows, g.num_types, int(mask) & 0xFFFFFFFF, rows,
                                            int(cap), overflow)
            from euler_amd.dataflow.device_flow import full_neighbors_cpu

            return full_neighbors_cpu(g, int(mask), rows, int(cap), overflow)
        W = self.world
        ok = (rows >= 0) & (rows < self.num_rows)
        pos, recv, C = self._route(torch.where(ok, rows, torch.full_like(rows, -1)))
        loc = self._local_rows(recv)
        deg_l = self._masked_degree(loc, int(mask))  # [W*C], the owner's received slots
        # owner side: every received row expanded (slot order = requester-block order), each
        # requester's lists packed into its own Ce slots of one equal-split all-to-all
        Ce = self.capacity(int(cap))
        tot = deg_l.view(W, C).sum(1)
        blk0 = torch.cumsum(tot, 0) - tot  # where block o starts in the flat expansion
        own = torch.zeros(1, dtype=torch.int32, device=dev)
        nb_l, src_l, _ = _expand_full(self.local, int(mask), loc, W * Ce, own)
        o = torch.div(src_l.clamp(min=0), C, rounding_mode="floor")
        off = torch.arange(W * Ce, dtype=torch.long, device=dev) - blk0[o]
        keep = (src_l >= 0) & (off < Ce)
        dst = torch.where(keep, o * Ce + off, torch.full_like(off, W * Ce))
        send = torch.full((W * Ce + 1,), -1, dtype=torch.int32, device=dev)
        send.scatter_(0, dst, nb_l.int())
        # a requester's lists beyond its Ce slots: flagged on the flow (it regrows its caps)
        overflow.copy_(torch.maximum(overflow, (tot > Ce).any().reshape(1).to(overflow.dtype)))
        buf = self._a2a(send[: W * Ce])  # block o: this rank's lists from owner o
        deg_s = self._a2a(deg_l).view(W, C)
        # requester side: the received blocks are a CSR over this rank's request slots, one
        # gap row per block (rows o * (C + 1) + j; the gap spans the block's unused slots), so
        # placing the requests target-major is full_neighbors again over that CSR
        incl = torch.cumsum(deg_s, 1).clamp(max=Ce)
        excl = torch.cat([torch.zeros((W, 1), dtype=incl.dtype, device=dev), incl[:, :-1]], 1)
        base = (torch.arange(W, dtype=torch.long, device=dev) * Ce).unsqueeze(1)
        ptr = torch.cat([(torch.cat([excl, incl[:, -1:]], 1) + base).reshape(-1),
                         torch.full((1,), W * Ce, dtype=torch.long, device=dev)])
        pj = torch.div(pos, C, rounding_mode="floor")
        slots = torch.where(pos < W * C, pos + pj, torch.full_like(pos, -1))  # o * (C + 1) + j
        return _expand_csr(ptr, buf, slots, int(cap), overflow)


    # ------------------------------------------------------------------ features / labels
    def padded_features(self, mult: int = 16):
        """the feature exchange over a shard whose width is padded to ``mult`` columns
        (zeros; the fused SAGE kernels read 16-column groups)"""
        sf = self.features
        if sf is None or sf.dim % mult == 0:
            return sf
        if getattr(self, "_padded", None) is None:
            w = -(-sf.dim // mult) * mult
            shard = torch.zeros(sf.shard.shape[0], w, dtype=sf.shard.dtype, device=sf.shard.device)
            shard[:, : sf.dim] = sf.shard
            self._padded = ShardedFeatures(shard, self.num_rows, self.group, sf.comm)
        return self._padded

    def gather_features(self, rows: torch.Tensor) -> torch.Tensor:
        """feature rows [n, D] of global rows (``-1``: zeros), through the feature exchange"""
        return self._gather(self.features, rows)

    def gather_labels(self, rows: torch.Tensor) -> torch.Tensor:
        return self._gather(self.labels, rows)

    @staticmethod
    def _gather(sf, rows):
        if sf is None:
            raise ValueError("the sharded graph holds no such table")
        pos = sf.exchange(rows.reshape(-1).long())
        if use_hip(sf.cache):
            return mp_ops.gather(sf.cache, pos.long())
        return torch.where((pos >= 0).unsqueeze(1), sf.cache[pos.long().clamp(min=0)], torch.zeros(
            (), dtype=sf.cache.dtype))


def _expand_full(g, mask, rows, cap, overflow):
    """``full_neighbors`` of local rows over a DeviceGraph's CSR (HIP or the torch twin)"""
    if use_hip(rows):
        return hip().full_neighbors(g.indptr, g.nbr, g.num_rows, g.num_types, int(mask) & 0xFFFFFFFF, rows, int(cap),
                                    overflow)
    from euler_amd.dataflow.device_flow import full_neighbors_cpu

    return full_neighbors_cpu(g, int(mask), rows, int(cap), overflow)


def _expand_csr(indptr, nbr, rows, cap, overflow):
    """``full_neighbors`` over a one-type CSR (indptr int64 [n+1], nbr int32)"""
    if use_hip(rows):
        return hip().full_neighbors(indptr, nbr, indptr.numel() - 1, 1, 1, rows, int(cap), overflow)
    from types import SimpleNamespace

    from euler_amd.dataflow.device_flow import full_neighbors_cpu

    return full_neighbors_cpu(SimpleNamespace(indptr=indptr, nbr=nbr, num_types=1), 1, rows, int(cap), overflow)


def _alias_weights(g: DeviceGraph):
    """per-row root weights of a DeviceGraph's alias table (prob / alias -> weights)"""
    p = g.node_prob.detach().cpu().double()
    a = g.node_alias.detach().cpu().long()
    n = p.numel()
    w = p.clone()
    w.index_add_(0, a, 1.0 - p)
    out = torch.zeros(g.num_rows, dtype=torch.float64)
    if g.root_rows is not None:
        out[g.root_rows.cpu().long()] = w
    else:
        out[:n] = w
    return out.numpy()
