"""Full-neighbourhood dataflow built on the device, in fixed (capacity-padded) shapes.

The reference ``GCNDataFlow`` (``tf_euler/python/dataflow/gcn_dataflow.py:26-48``) expands
every hop with ``get_full_neighbor`` over the whole current node set and dedups with
``tf.unique`` (``neighbor_dataflow.py:84-110``), so its blocks change size every batch.  The
engine path (``dataflows.GCNDataFlow``) reproduces that on the CPU graph engine and ships
each block to the GPU.  Here the same blocks are built from the HBM copy of the graph
(:class:`~euler_amd.graph.device_graph.DeviceGraph`) with every shape fixed up front:

* node sets and edge lists have per-hop capacities; unused slots hold ``-1``.  The
  default ("exact") caps are upper bounds from the graph's maximum out-degree over the
  hop's edge types: hop 0's targets are the roots as drawn (repeats included), so its edge
  cap is ``B * max_out_degree``; later hops expand deduplicated sets, so theirs is also
  bounded by the masked edge count.  ``caps="bounded"`` sizes each hop from a degree
  quantile times a safety factor instead (:func:`bounded_caps`), which on a power-law graph
  is orders of magnitude smaller; a batch that exceeds a cap sets :attr:`overflow`, the
  trainer notices at its next boundary and grows the caps (``grow``) and re-captures;
* ``-1`` is the padding convention every message-passing op already honours
  (``mp_ops``: a ``-1`` destination / source edge is dropped, a ``-1`` gather row reads
  zeros), so the unchanged model convolutions run on the padded blocks and padded rows
  stay out of every real row;
* the expansion is ``full_neighbors`` (``csrc/hip/flow.hip``: degree, scan, binary-search
  expand; target-major edges in storage order, the reference's value order) and the dedup
  ``unique_first_padded`` (``csrc/hip/unique.hip``: first-occurrence order = ``tf.unique``);
  nothing syncs with the host, so sampling + model + backward + optimizer capture into
  one hipGraph (``models/full_trainer.py``).

Block layout equals ``UniqueDataFlow.produce_subgraph`` (``dataflows.py``): hop h's new
set is ``unique([neighbours, previous set])``, ``res_n_id`` = the previous set's positions
in it, edges = (target position, source position) for every neighbour occurrence and,
with self loops, one (t, position of t) per target.
"""
from __future__ import annotations

import os

import torch

from euler_amd.dataflow.dataflows import Block, DataFlow
from euler_amd.ops._native import hip, use_hip
from euler_amd.ops.mp_ops import SegmentIndex

__all__ = ["DeviceFullFlow", "DeviceLayerFlow", "DeviceRelationFlow", "DeviceSageFlow", "full_neighbors_cpu", "max_out_degree"]


def _round_up(x: int, m: int = 256) -> int:
    return -(-int(x) // m) * m


def max_out_degree(graph, mask: int) -> int:
    """largest out-degree of any row over the edge types of ``mask``"""
    if hasattr(graph, "degree_stats"):  # row-sharded: reduced over the ranks
        return graph.degree_stats(mask)[0]
    T = graph.num_types
    seg = (graph.indptr[1:] - graph.indptr[:-1]).view(graph.num_rows, T)
    sel = torch.tensor([(mask >> t) & 1 for t in range(T)], dtype=seg.dtype, device=seg.device)
    return int((seg * sel).sum(1).max().item()) if graph.num_rows else 0


def masked_edges(graph, mask: int) -> int:
    if hasattr(graph, "degree_stats"):
        return graph.degree_stats(mask)[1]
    T = graph.num_types
    seg = (graph.indptr[1:] - graph.indptr[:-1]).view(graph.num_rows, T)
    sel = torch.tensor([(mask >> t) & 1 for t in range(T)], dtype=seg.dtype, device=seg.device)
    return int((seg * sel).sum().item())


def full_neighbors_cpu(graph, mask: int, rows: torch.Tensor, cap: int, overflow: torch.Tensor):
    """torch twin of ``hip().full_neighbors`` (same order, same padding)"""
    T = graph.num_types
    rows = rows.reshape(-1).long()
    ok = rows >= 0
    r = torch.where(ok, rows, torch.zeros_like(rows))
    nbrs, srcs = [], []
    for i in range(rows.numel()):
        if not bool(ok[i]):
            continue
        for t in range(T):
            if not (mask >> t) & 1:
                continue
            a, b = int(graph.indptr[int(r[i]) * T + t]), int(graph.indptr[int(r[i]) * T + t + 1])
            if b > a:
                nbrs.append(graph.nbr[a:b].long())
                srcs.append(torch.full((b - a,), i, dtype=torch.long))
    nb = torch.cat(nbrs) if nbrs else torch.zeros(0, dtype=torch.long)
    sc = torch.cat(srcs) if srcs else torch.zeros(0, dtype=torch.long)
    if nb.numel() > cap:
        overflow.fill_(1)
        nb, sc = nb[:cap], sc[:cap]
    out_n = torch.full((cap,), -1, dtype=torch.long)
    out_s = torch.full((cap,), -1, dtype=torch.long)
    out_n[: nb.numel()] = nb
    out_s[: sc.numel()] = sc
    deg = torch.bincount(sc, minlength=rows.numel())[: rows.numel()] if sc.numel() else \
        torch.zeros(rows.numel(), dtype=torch.long)
    return out_n, out_s, torch.cumsum(deg, 0)


def _dst_csr(src, offs, n_targets, cap_e, cap_t, self_loops):
    """(perm, indptr) of the block's destination CSR, straight from the expansion: edges are
    target-major already, so target t's edges are its neighbours [offs[t-1], offs[t]) then
    (with self loops) its self edge cap_e + t — the order a stable sort of the reference
    edge list ([neighbours..., self loops...]) gives — and no sort is needed.  Padding
    edges fill the tail (the sentinel segment past indptr[cap_t])."""
    dev = src.device
    excl = torch.cat([torch.zeros(1, dtype=torch.long, device=dev), offs])  # [cap_t + 1]
    if not self_loops:
        return torch.arange(cap_e, dtype=torch.long, device=dev), excl
    t_ar = torch.arange(cap_t + 1, dtype=torch.long, device=dev)
    indptr = excl + torch.minimum(t_ar, n_targets)
    e_ar = torch.arange(cap_e, dtype=torch.long, device=dev)
    new_nbr = torch.where(src >= 0, e_ar + src, e_ar + n_targets)
    t = t_ar[:-1]
    new_self = torch.where(t < n_targets, excl[1:] + t, cap_e + t)
    new_pos = torch.cat([new_nbr, new_self])
    # zeros, not empty: after a capacity overflow (flagged, raised at the next check) the
    # positions may collide, and every entry must still be a valid edge index
    perm = torch.zeros_like(new_pos)
    perm.scatter_(0, new_pos, torch.arange(new_pos.numel(), dtype=torch.long, device=dev))
    return perm, indptr


_FUSED_BLOCK = os.environ.get("EULER_AMD_FLOW_FUSED", "1") == "1"


def _unique_padded(x: torch.Tensor):
    """(uniq padded with -1, inverse (-1 for -1 entries), count [1]) in first-occurrence order"""
    if use_hip(x):
        uniq, inv, cnt = hip().unique_first_padded(x.contiguous(), -1)
        return uniq, inv, cnt
    valid = x >= 0
    vals = x[valid]
    seen, order, inv_v = {}, [], []
    for v in vals.tolist():
        if v not in seen:
            seen[v] = len(order)
            order.append(v)
        inv_v.append(seen[v])
    uniq = torch.full_like(x, -1)
    uniq[: len(order)] = torch.tensor(order, dtype=x.dtype)
    inv = torch.full_like(x, -1)
    inv[valid] = torch.tensor(inv_v, dtype=x.dtype)
    return uniq, inv, torch.tensor([len(order)], dtype=torch.long)


def exact_caps(graph, masks, batch_size: int):
    """per-hop (edge, next-set) capacities no batch can exceed"""
    caps = []
    n = int(batch_size)
    N = graph.num_rows
    for h, m in enumerate(masks):
        e = n * max_out_degree(graph, m)
        if h > 0:  # a deduplicated set expands each node once
            e = min(masked_edges(graph, m), e)
        n_next = min(N, n + e)
        caps.append((_round_up(max(e, 1)), _round_up(n_next)))
        n = n_next
    return caps


def _bounded_args(spec: str):
    """"bounded" or "bounded:<quantile>:<safety>" -> (quantile, safety)"""
    parts = spec.split(":")
    q = float(parts[1]) if len(parts) > 1 else 0.99
    f = float(parts[2]) if len(parts) > 2 else 2.0
    return q, f


def bounded_caps(graph, masks, batch_size: int, quantile: float = 0.99, safety: float = 2.0):
    """Per-hop capacities from the degree distribution instead of its maximum: a hop over n
    targets is sized for n times the mean out-degree plus the ``quantile`` tail, times
    ``safety``, never above the exact bound (:func:`exact_caps`).  On a power-law graph one
    hub fixes ``max_out_degree`` and makes the exact caps reach the whole edge set by hop 2;
    these stay proportional to the work a typical batch does.  A batch over them is caught
    by the overflow flag (:meth:`DeviceFullFlow.grow`, re-capture)."""
    exact = exact_caps(graph, masks, batch_size)
    T = graph.num_types
    caps = []
    n = int(batch_size)
    N = graph.num_rows
    for (ex_e, ex_n), m in zip(exact, masks):
        k = max(1, int(N * (1.0 - quantile)))
        if hasattr(graph, "degree_stats"):  # row-sharded: mean and tail over every rank's rows
            _, total, tail = graph.degree_stats(m, k)
            mean = total / N if N else 0.0
        else:
            seg = (graph.indptr[1:] - graph.indptr[:-1]).view(graph.num_rows, T)
            sel = torch.tensor([(m >> t) & 1 for t in range(T)], dtype=seg.dtype, device=seg.device)
            deg = (seg * sel).sum(1).float()
            mean = float(deg.mean().item()) if deg.numel() else 0.0
            tail = float(torch.topk(deg, min(k, deg.numel())).values.min().item()) if deg.numel() else 0.0
        e = min(ex_e, _round_up(int(safety * (n * mean + tail)) + 1))
        n_next = min(ex_n, N, _round_up(n + e))
        caps.append((int(e), int(n_next)))
        n = n_next
    return caps


class DeviceFullFlow:
    """``GCNDataFlow`` on the device with fixed shapes.

    ``metapath``: one edge-type mask per hop (``DeviceGraph._mask``); ``batch_size``: the
    number of roots (set 0, unpadded: the roots as drawn, repeats included, as the
    reference).  ``caps`` (optional): per-hop (edge capacity, next-set capacity) pairs
    overriding the exact bounds (smaller caps cost less; an overflow sets :attr:`overflow`
    and :meth:`check` raises)."""

    def __init__(self, graph, masks, batch_size: int, add_self_loops: bool = True, caps=None):
        self.g = graph
        self.masks = [int(m) for m in masks]
        self.B = int(batch_size)
        self.self_loops = bool(add_self_loops)
        self.L = len(self.masks)
        N = graph.num_rows
        if caps is None or caps == "exact":
            caps = exact_caps(graph, self.masks, self.B)
        elif isinstance(caps, str) and caps.startswith("bounded"):
            caps = bounded_caps(graph, self.masks, self.B, *_bounded_args(caps))
        self.caps = [(int(e), int(n)) for e, n in caps]
        self.overflow = torch.zeros(1, dtype=torch.int32, device=graph.device)

    def node_caps(self):
        return [self.B] + [n for _, n in self.caps]

    def produce(self, roots: torch.Tensor) -> DataFlow:
        """the padded DataFlow of ``roots`` (int rows [B]); blocks carry fixed sizes
        ``[cap_prev, cap_next]``; ``df.valid[h]`` = device count of real nodes of set h"""
        g = self.g
        n_id = roots.reshape(-1).long()
        if n_id.numel() != self.B:
            raise ValueError(f"expected {self.B} roots, got {n_id.numel()}")
        dev = n_id.device
        df = DataFlow(n_id)
        last_idx = torch.arange(self.B, dtype=torch.long, device=dev)
        prev_cnt = torch.full((), self.B, dtype=torch.long, device=dev)
        cap_prev = self.B
        for h, mask in enumerate(self.masks):
            cap_e, cap_n = self.caps[h]
            nbr, src, offs = self._expand(n_id, mask, cap_e)
            kept = self._filter(h, n_id, nbr)
            if kept is not None:
                nbr = kept
            attr = self._hop_attr(h, n_id, src, offs)
            cat = torch.cat([nbr, n_id])
            uniq, inv, cnt = _unique_padded(cat)
            if use_hip(n_id) and _FUSED_BLOCK and kept is None:
                # the block assembly below as one launch (flow.hip flow_block_kernel)
                new_n_id, res_n_id, edge_index, perm, indptr, counts, last_idx, prev_cnt = hip().flow_block(
                    src, offs, uniq, inv, cnt.reshape(1), last_idx, prev_cnt.reshape(1), cap_n, self.self_loops,
                    self.overflow)
                seg = SegmentIndex(edge_index[0], cap_prev)
                seg._perm, seg._indptr, seg._counts = perm, indptr, counts
                edge_index._euler_cache = {"_euler_seg0_%d" % cap_prev: seg}
                df.blocks.append(Block(new_n_id, res_n_id, attr, edge_index, [cap_prev, cap_n]))
                df._last = new_n_id
                n_id = new_n_id
                cap_prev = cap_n
                continue
            # a set beyond its capacity: flag it and drop the excess (never index past it)
            self.overflow.copy_(torch.maximum(self.overflow, (cnt.reshape(1) > cap_n).to(self.overflow.dtype)))
            new_n_id = uniq[:cap_n] if uniq.numel() >= cap_n else torch.cat(
                [uniq, torch.full((cap_n - uniq.numel(),), -1, dtype=uniq.dtype, device=dev)])
            inv = torch.where(inv < cap_n, inv, torch.full_like(inv, -1))
            res_n_id = inv[cap_e:]
            if self.self_loops:
                edge_t = torch.cat([src, last_idx])
                edge_s = inv
            else:
                edge_t, edge_s = src, inv[:cap_e]
            # an edge whose source was dropped by an overflow must not keep its target
            edge_t = torch.where(edge_s >= 0, edge_t, torch.full_like(edge_t, -1))
            edge_index = torch.stack([edge_t, edge_s])
            if kept is None:
                # the destination CSR is known from the expansion: the convolutions' scatters
                # and SpMM reuse it instead of sorting (mp_ops.cached_segment); a filtered hop
                # has holes in its segments, so its index is built from edge_t as usual
                perm, indptr = _dst_csr(src, offs.clamp(max=cap_e), prev_cnt, cap_e, cap_prev, self.self_loops)
                edge_index._euler_cache = {"_euler_seg0_%d" % cap_prev: SegmentIndex.from_csr(edge_t, cap_prev,
                                                                                                 perm, indptr)}
            df.blocks.append(Block(new_n_id, res_n_id, attr, edge_index, [cap_prev, cap_n]))
            df._last = new_n_id
            ar = torch.arange(cap_n, dtype=torch.long, device=dev)
            prev_cnt = torch.clamp(cnt.reshape(()), max=cap_n)
            last_idx = torch.where(ar < prev_cnt, ar, torch.full_like(ar, -1))
            n_id = new_n_id
            cap_prev = cap_n
        return df

    def overflowed(self) -> bool:
        """True if any batch since the last :meth:`clear` exceeded a capacity (host sync)"""
        return int(self.overflow.item()) != 0

    def clear(self):
        self.overflow.zero_()

    def check(self):
        """raise if any batch so far exceeded a capacity (host sync)"""
        if self.overflowed():
            raise RuntimeError(f"device dataflow capacity exceeded (caps {self.caps}): raise the caps")

    def grow(self, factor: float = 2.0):
        """every capacity times ``factor`` (at most the exact bound); returns the new caps.
        The flow's fixed shapes change, so captured graphs over it must be re-captured."""
        exact = exact_caps(self.g, self.masks, self.B)
        self.caps = [(min(ex_e, _round_up(int(e * factor))), min(ex_n, _round_up(int(n * factor))))
                     for (e, n), (ex_e, ex_n) in zip(self.caps, exact)]
        self.overflow.zero_()
        return self.caps

    def _expand(self, n_id, mask, cap_e):
        """(neighbours, target index, inclusive offsets) of the hop's full expansion"""
        g = self.g
        if hasattr(g, "full_neighbors"):  # a row-sharded graph: the owners expand
            return g.full_neighbors(n_id, mask, cap_e, self.overflow)
        if use_hip(n_id):
            return hip().full_neighbors(g.indptr, g.nbr, g.num_rows, g.num_types, mask & 0xFFFFFFFF, n_id, cap_e,
                                        self.overflow)
        return full_neighbors_cpu(g, mask, n_id, cap_e, self.overflow)

    def _filter(self, h, n_id, nbr):
        """hook: the hop's neighbour list with dropped entries set to -1 (None: keep all)"""
        return None

    def _hop_attr(self, h, n_id, src, offs):
        """hook: a per-edge attribute of the hop (the block's ``e_id``; None: no attribute)"""
        return None

    def edge_positions(self, h, n_id, src, offs):
        """CSR position of every expansion entry (-1 for padding): entry e of target i is
        the k-th neighbour of i, k = e - (start of i's entries), walked through i's
        segments of the hop's edge types in ascending type order (``full_neighbors``'
        order)"""
        g = self.g
        T = g.num_types
        cap_e = src.numel()
        ok = src >= 0
        i = src.clamp(min=0)
        excl = torch.cat([torch.zeros(1, dtype=offs.dtype, device=offs.device), offs])[i]
        k = torch.arange(cap_e, dtype=torch.long, device=src.device) - excl.long()
        r = n_id.clamp(min=0)[i]
        pos = torch.full_like(k, -1)
        for t in range(T):
            if not (self.masks[h] >> t) & 1:
                continue
            a, b = g.indptr[r * T + t], g.indptr[r * T + t + 1]
            n = b - a
            pos = torch.where((pos < 0) & (k >= 0) & (k < n), a + k, pos)
            k = k - n
        return torch.where(ok, pos, torch.full_like(pos, -1))


class DeviceRelationFlow(DeviceFullFlow):
    """``RelationDataFlow`` (reference ``relation_dataflow.py:25-75``; engine twin in
    ``dataflows.py``) on the device: full neighbourhoods without self loops, each block's
    ``e_id`` the per-edge attribute ``edge_attr[CSR position]`` (``-1`` on padding) — the
    R-GCN relation of the (target, neighbour, type) edge, read once from the engine."""

    def __init__(self, graph, masks, batch_size: int, edge_attr: torch.Tensor, caps=None):
        super().__init__(graph, masks, batch_size, add_self_loops=False, caps=caps)
        self.edge_attr = edge_attr.to(graph.device).long()

    def _hop_attr(self, h, n_id, src, offs):
        pos = self.edge_positions(h, n_id, src, offs)
        return torch.where(pos >= 0, self.edge_attr[pos.clamp(min=0)], torch.full_like(pos, -1))


class DeviceLayerFlow(DeviceFullFlow):
    """``FastGCNDataFlow`` / ``LayerwiseDataFlow`` (reference ``fast_dataflow.py:25-57``,
    ``layerwise_dataflow.py:26-71``; engine twins in ``dataflows.py``) on the device with
    fixed shapes.  Every hop but the last keeps, of the current set's out-edges, those that
    land in a per-hop sampled layer; the last hop is the full neighbourhood:

    * ``"fast"``: the layer is ``sample_node(total_fanout, metapath[h][0])`` (the
      reference's node-type argument; ``samplers[h]``, a root sampler over that type), the
      kept edges are ``sparse_get_adj(set, unique(layer))``;
    * ``"layer"``: ``sampleLNB`` — ``total_fanout`` roots drawn from the current set in
      proportion to their out-edge weight, one weighted neighbour of each (Philox stream
      30 + h), the kept edges are the set's edges into that layer.

    A layer is a membership flag over the graph's rows, so an edge is kept once even when
    its destination was drawn several times (the engine path's adjacency repeats it per
    draw); node sets and the kept edges' (target, source) pairs otherwise equal the
    engine's blocks, in target-major storage order.  Capacities are the full flow's
    (exact upper bounds)."""

    def __init__(self, graph, masks, kinds, fanouts, batch_size: int, add_self_loops: bool = True, samplers=None):
        super().__init__(graph, masks, batch_size, add_self_loops)
        self.kinds = list(kinds)
        totals, t = [], 0
        for f in fanouts:
            t += int(f)
            totals.append(t)
        self.totals = totals
        self.samplers = list(samplers) if samplers is not None else [None] * len(self.kinds)
        if len(self.kinds) != self.L or any(k not in ("fast", "layer") for k in self.kinds[:-1]) or \
                len(self.totals) < self.L - 1:
            raise ValueError("kinds: 'fast' | 'layer' for every hop but the last")
        self._flag = torch.zeros(graph.num_rows + 1, dtype=torch.bool, device=graph.device)
        self._uflat_p = torch.ones(1 << 16, dtype=torch.float32, device=graph.device)
        self._uflat_a = torch.arange(1 << 16, dtype=torch.int32, device=graph.device)

    def _out_weight(self, rows, mask):
        g = self.g
        T = g.num_types
        r = rows.clamp(min=0)
        tot = torch.zeros(rows.numel(), dtype=torch.float32, device=rows.device)
        for t in range(T):
            if not (mask >> t) & 1:
                continue
            a, b = g.indptr[r * T + t], g.indptr[r * T + t + 1]
            tot = tot + torch.where(b > a, g.cumw[(b - 1).clamp(min=0)], torch.zeros_like(tot))
        return torch.where(rows >= 0, tot, torch.zeros_like(tot))

    def _layer(self, h, n_id):
        g, m = self.g, self.totals[h]
        if self.kinds[h] == "fast":
            return self.samplers[h].sample_node(m, stream_id=20 + h).long()
        w = self._out_weight(n_id, self.masks[h])
        # double prefix sums of the float weights (exact for any association, so the fused
        # GCN step's block scan picks the same roots: csrc/hip/gcn.hip gcn_layerwise_draw)
        cum = torch.cumsum(w.double(), 0)
        total = cum[-1]
        u = self._uniform(m, 40 + h) * total
        pick = torch.searchsorted(cum, u.contiguous(), right=True).clamp(max=n_id.numel() - 1)
        roots = torch.where(total > 0, n_id[pick], torch.full_like(pick, -1))
        types = [t for t in range(g.num_types) if (self.masks[h] >> t) & 1]
        return g.sample_neighbor(roots, 1, edge_types=types, default=-1, stream_id=30 + h).long().reshape(-1)

    def _uniform(self, n, stream_id):
        """n uniforms in [0, 1) keyed by the graph's (seed, counter) and ``stream_id``: two
        16-bit integer draws of the alias sampler over a flat table (Philox, capturable)"""
        g = self.g
        if use_hip(g.rng):
            hi = hip().alias_sample(self._uflat_p, self._uflat_a, None, int(n), g.rng, int(stream_id))
            lo = hip().alias_sample(self._uflat_p, self._uflat_a, None, int(n), g.rng, int(stream_id) + 100)
            return (hi.double() * 65536.0 + lo.double() + 0.5) / float(1 << 32)
        return torch.rand(int(n), generator=g._cpu_gen, dtype=torch.float64)

    def _filter(self, h, n_id, nbr):
        if h == self.L - 1:
            return None
        layer = self._layer(h, n_id)
        slot = torch.where(layer >= 0, layer, torch.full_like(layer, self.g.num_rows))
        self._flag.index_fill_(0, slot, True)  # slot num_rows (no draw) is never read below
        keep = self._flag[nbr.clamp(min=0)] & (nbr >= 0)
        self._flag.index_fill_(0, slot, False)
        return torch.where(keep, nbr, torch.full_like(nbr, -1))


class DeviceSageFlow:
    """``SageDataFlow`` on the device with fixed shapes (reference
    ``tf_euler/python/dataflow/sage_dataflow.py:35-50``; engine twin
    ``dataflows.SageDataFlow``): per hop ``fanouts[h]`` weighted draws with replacement per
    node (``DeviceGraph.sample_neighbor``, Philox stream 10 + h), then
    ``unique([neighbours, previous set])`` in first-occurrence order, the previous set's
    positions, target-major edges (F per target, then one self loop per target).

    Capacities are exact: hop h's set holds at most ``cap_{h-1} (F_h + 1)`` rows (capped by
    the graph size), its edge list ``cap_{h-1} F_h`` (+ ``cap_{h-1}`` self loops).  A node
    without an out-edge of the hop's types draws ``-1`` (the reference draws the padding
    node ``max_id + 1``, whose features are zero): the message-passing ops drop ``-1``
    edges, so such a node's mean is over nothing instead of over zero rows — the same 0."""

    def __init__(self, graph, edge_types, fanouts, batch_size: int, add_self_loops: bool = True):
        self.g = graph
        self.edge_types = [None if e is None else [int(t) for t in e] for e in edge_types]
        self.fanouts = [int(f) for f in fanouts]
        if len(self.edge_types) != len(self.fanouts):
            raise ValueError("one edge-type list per fanout")
        self.B = int(batch_size)
        self.self_loops = bool(add_self_loops)
        self.caps = []
        n = self.B
        for f in self.fanouts:
            e = n * f + (n if self.self_loops else 0)
            n_next = min(graph.num_rows, n * (f + 1))
            self.caps.append((e, n_next))
            n = n_next

    def node_caps(self):
        return [self.B] + [n for _, n in self.caps]

    def produce(self, roots: torch.Tensor) -> DataFlow:
        g = self.g
        n_id = roots.reshape(-1).long()
        if n_id.numel() != self.B:
            raise ValueError(f"expected {self.B} roots, got {n_id.numel()}")
        dev = n_id.device
        df = DataFlow(n_id)
        last_idx = torch.arange(self.B, dtype=torch.long, device=dev)
        cap_prev = self.B
        for h, (et, f) in enumerate(zip(self.edge_types, self.fanouts)):
            cap_e, cap_n = self.caps[h]
            nbr = g.sample_neighbor(n_id, f, edge_types=et, default=-1, stream_id=10 + h).long().reshape(-1)
            cat = torch.cat([nbr, n_id])
            uniq, inv, cnt = _unique_padded(cat)
            if use_hip(n_id) and _FUSED_BLOCK:
                # the block assembly below + the destination CSR as three launches (flow.hip
                # sage_block / sage_place): the convolutions' scatters and SpMM need no sort
                new_n_id, res_n_id, edge_index, perm, indptr, counts, last_idx, _ = hip().sage_block(
                    inv, uniq, cnt.reshape(1), last_idx, f, cap_n, self.self_loops)
                seg = SegmentIndex(edge_index[0], cap_prev)
                seg._perm, seg._indptr, seg._counts = perm, indptr, counts
                edge_index._euler_cache = {"_euler_seg0_%d" % cap_prev: seg}
                df.blocks.append(Block(new_n_id, res_n_id, None, edge_index, [cap_prev, cap_n]))
                df._last = new_n_id
                n_id = new_n_id
                cap_prev = cap_n
                continue
            new_n_id = uniq[:cap_n] if uniq.numel() >= cap_n else torch.cat(
                [uniq, torch.full((cap_n - uniq.numel(),), -1, dtype=uniq.dtype, device=dev)])
            res_n_id = inv[nbr.numel():]
            tgt = torch.arange(cap_prev, dtype=torch.long, device=dev).repeat_interleave(f)
            if self.self_loops:
                edge_t = torch.cat([tgt, last_idx])
                edge_s = inv
            else:
                edge_t, edge_s = tgt, inv[: nbr.numel()]
            # an edge of a -1 draw (or of a padding target) carries nothing
            edge_t = torch.where(edge_s >= 0, edge_t, torch.full_like(edge_t, -1))
            df.blocks.append(Block(new_n_id, res_n_id, None, torch.stack([edge_t, edge_s]), [cap_prev, cap_n]))
            df._last = new_n_id
            ar = torch.arange(cap_n, dtype=torch.long, device=dev)
            cnt_n = torch.clamp(cnt.reshape(()), max=cap_n)
            last_idx = torch.where(ar < cnt_n, ar, torch.full_like(ar, -1))
            n_id = new_n_id
            cap_prev = cap_n
        return df
