"""Graph queries answered from HBM: a scope in which the graph-op API (``ops/graph_api.py``)
serves a model's own forward from a :class:`~euler_amd.graph.device_graph.DeviceGraph`
instead of the C++ engine.

The reference's models reach the graph only through the ``tf_euler`` ops
(``tf_euler/python/euler_ops/{sample_ops,neighbor_ops,feature_ops}.py``); inside
``with device_graph_scope(scope):`` the ones the encoders use —

* ``sample_node(count, node_type)``         the graph's root alias table (Philox),
* ``sample_neighbor`` / ``sample_fanout``   the weighted with-replacement draw kernel,
* ``get_multi_hop_neighbor``               full neighbourhoods, first-occurrence unique
                                             sets and the weighted adjacency per hop,
* ``get_dense_feature``                    rows of the HBM feature / label tables —

return DEVICE tensors in node-id space (the engine's contract: ids in, ids out; ``-1``
and absent ids read zero features), with no host round trip for the fixed-shape ones, so
a step built from them can be captured in a hipGraph.  Every draw takes its own Philox
stream of the graph's (seed, counter) pair: the caller advances the counter once per step.

Used by :class:`~euler_amd.models.scalable_trainer.ScalableTrainer` to run the historical-
embedding encoders (ScalableSageEncoder / ScalableGCNEncoder) through their own forward on
the device path.
"""
from __future__ import annotations

import contextlib

import numpy as np
import torch

__all__ = ["DeviceGraphScope", "device_graph_scope", "active_scope"]

_ACTIVE = [None]


def active_scope():
    return _ACTIVE[0]


@contextlib.contextmanager
def device_graph_scope(scope):
    prev = _ACTIVE[0]
    _ACTIVE[0] = scope
    scope.calls = 0
    try:
        yield scope
    finally:
        _ACTIVE[0] = prev


class DeviceGraphScope:
    """``graph`` (DeviceGraph with ``features`` holding the columns ``feature_cols``
    {name: (offset, dim)} and ``labels`` the column ``label``), ``stream0``: the first
    Philox stream of the scope's draws (roots use stream 1 of the caller)."""

    def __init__(self, graph, feature_cols=None, label=None, stream0=24):
        self.g = graph
        self.dev = graph.device
        self.cols = dict(feature_cols or {})
        self.label = label  # (name, dim) or None
        self.stream0 = int(stream0)
        self.calls = 0
        ids = graph.ids
        if ids is None:
            self.ids = None
        else:
            a = np.asarray(ids).astype(np.int64)
            if a.size > 1 and not (a[1:] > a[:-1]).all():
                raise ValueError("device scope: graph ids must be sorted (engine rows are)")
            self.ids = torch.from_numpy(a).to(self.dev)
        self.record = None  # optional list: every draw's id tensors (tests)

    # ------------------------------------------------------------------ id <-> row
    def rows(self, ids):
        ids = torch.as_tensor(ids, device=self.dev).reshape(-1).long()
        if self.ids is None:
            ok = (ids >= 0) & (ids < self.g.num_rows)
            return torch.where(ok, ids, torch.full_like(ids, -1))
        n = self.ids.numel()
        pos = torch.searchsorted(self.ids, ids).clamp(max=max(n - 1, 0))
        hit = self.ids[pos] == ids
        return torch.where(hit, pos, torch.full_like(pos, -1))

    def ids_of(self, rows, default=-1):
        rows = rows.long()
        ok = rows >= 0
        r = torch.where(ok, rows, torch.zeros_like(rows))
        v = r if self.ids is None else self.ids[r]
        return torch.where(ok, v, torch.full_like(v, int(default)))

    def _stream(self):
        s = self.stream0 + self.calls
        self.calls += 1
        return s

    def _types(self, edge_types):
        from euler_amd.ops import graph_api as ge

        if edge_types is None:
            return None
        et = [int(t) for t in np.asarray(ge._et(edge_types)).reshape(-1)]
        return None if any(t < 0 for t in et) else et

    def _rec(self, kind, *ts):
        if self.record is not None:
            self.record.append((kind,) + tuple(t.detach().clone() for t in ts))

    # ------------------------------------------------------------------ API
    def sample_node(self, count, node_type=None):
        r = self.g.sample_node(int(count), stream_id=self._stream()).long()
        out = self.ids_of(r)
        self._rec("sample_node", out)
        return out

    def sample_neighbor(self, nodes, edge_types, count, default_node=-1):
        shape = tuple(torch.as_tensor(nodes).shape)
        rows = self.rows(nodes)
        nb, w, t = self.g.sample_neighbor(rows, int(count), edge_types=self._types(edge_types), default=-1,
                                          stream_id=self._stream(), with_weights=True)
        ids = self.ids_of(nb.long().reshape(-1), default_node).view(*shape, int(count))
        self._rec("sample_neighbor", ids)
        return ids, w.view(*shape, int(count)).float(), t.view(*shape, int(count)).int()

    def sample_fanout(self, nodes, edge_types, counts, default_node=-1):
        nb = [torch.as_tensor(nodes, device=self.dev).reshape(-1).long()]
        ws, ts = [], []
        for et, c in zip(edge_types, counts):
            i, w, t = self.sample_neighbor(nb[-1], et, int(c), default_node)
            nb.append(i.reshape(-1))
            ws.append(w.reshape(-1))
            ts.append(t.reshape(-1))
        return nb, ws, ts

    def _full_edges(self, rows, types):
        """every out-edge of ``rows`` in (row, type, storage) order: (source index, neighbour
        row, weight) — the engine's outV order (a host read of the edge count: eager only)"""
        g = self.g
        T = g.num_types
        tl = list(range(T)) if types is None else [t for t in types if 0 <= t < T]
        ok = rows >= 0
        r = torch.where(ok, rows, torch.zeros_like(rows))
        tt = torch.tensor(tl, dtype=torch.long, device=self.dev)
        seg = r.view(-1, 1) * T + tt.view(1, -1)
        starts = g.indptr[seg]
        cnt = (g.indptr[seg + 1] - starts) * ok.view(-1, 1)
        flat_cnt = cnt.reshape(-1)
        E = int(flat_cnt.sum().item())
        seg_id = torch.repeat_interleave(torch.arange(flat_cnt.numel(), device=self.dev), flat_cnt)
        excl = torch.cumsum(flat_cnt, 0) - flat_cnt
        off = torch.arange(E, device=self.dev) - excl[seg_id]
        pos = starts.reshape(-1)[seg_id] + off
        prev = torch.where(off > 0, g.cumw[(pos - 1).clamp(min=0)], torch.zeros((), device=self.dev))
        return seg_id // len(tl), g.nbr[pos].long(), g.cumw[pos] - prev

    def get_multi_hop_neighbor(self, nodes, edge_types):
        from euler_amd.ops.gnn_ops import unique_first
        from euler_amd.ops.graph_api import SparseTensor

        cur = torch.as_tensor(nodes, device=self.dev).reshape(-1).long()
        nodes_list, adj_list = [cur], []
        for et in edge_types:
            src, nrow, w = self._full_edges(self.rows(cur), self._types(et))
            nid = self.ids_of(nrow)
            nxt, inv = unique_first(nid)
            ind = torch.stack([src, inv.long()], 1)
            adj = SparseTensor(ind, w.float(), torch.tensor([cur.numel(), nxt.numel()], dtype=torch.int64))
            self._rec("multi_hop", nxt, ind, w)
            nodes_list.append(nxt)
            adj_list.append(adj)
            cur = nxt
        return nodes_list, adj_list

    def get_dense_feature(self, nodes, feature_names, dimensions):
        rows = self.rows(nodes)
        ok = (rows >= 0).unsqueeze(1)
        r = rows.clamp(min=0)
        out = []
        for name, d in zip(feature_names, dimensions):
            if self.label is not None and str(name) == str(self.label[0]) and self.g.labels is not None:
                tab, off = self.g.labels, 0
            elif str(name) in self.cols:
                tab, off = self.g.features, self.cols[str(name)][0]
            else:
                raise KeyError(f"device scope: feature {name!r} is not in the HBM tables")
            x = tab[r, off: off + int(d)].float()
            out.append(x * ok)
        return out
