"""Mini-batch subgraph builders (reference ``tf_euler/python/dataflow/*.py``).

A :class:`DataFlow` is a list of :class:`Block`s built hop by hop from the roots and
iterated in reverse (outermost hop first) by the GNN.  Each block holds

* ``n_id``       node ids of this hop's (larger) node set,
* ``res_n_id``   positions of the previous (smaller) set inside ``n_id``,
* ``edge_index`` [2, E]: row 0 = target position (smaller set), row 1 = source position,
* ``size``       [len(smaller set), len(n_id)],
* ``e_id``       optional per-edge attribute (edge types for RelationDataFlow).

Sampling runs through the graph engine (CPU, or remote shards); ``DataFlow.to(device)``
moves the int tensors to the GPU in one batch of non-blocking copies.
"""
from __future__ import annotations

import torch

import euler_amd.ops.graph_api as ge
from euler_amd.ops.gnn_ops import unique_first

__all__ = ["Block", "DataFlow", "NeighborDataFlow", "UniqueDataFlow", "SageDataFlow", "GCNDataFlow",
           "FastGCNDataFlow", "LayerwiseDataFlow", "LayerwiseEachDataFlow", "WholeDataFlow", "RelationDataFlow",
           "unique_with_inverse"]


def unique_with_inverse(x: torch.Tensor):
    """(unique values, inverse) — ``tf.unique`` semantics: first-occurrence order, so
    the previous hop's nodes keep their positions (GPU tensors: hash-table kernel
    ``unique.hip``; CPU: the engine's hash pass, same result)."""
    return unique_first(x)


class Block:
    """One hop of a DataFlow.  ``nbr`` (fixed-fanout flows only): int32 [n_target, F (+1)]
    positions of every target's sampled neighbours (and its self loop) in ``n_id`` —
    the edge list in the dense form the fused SAGE kernel consumes (K3, sage_ops)."""
    __slots__ = ("n_id", "res_n_id", "e_id", "edge_index", "size", "nbr", "_euler_cache")

    def __init__(self, n_id, res_n_id, e_id, edge_index, size, nbr=None):
        self.n_id = n_id
        self.res_n_id = res_n_id
        self.e_id = e_id
        self.edge_index = edge_index
        self.size = size
        self.nbr = nbr

    def to(self, device, non_blocking=True):
        mv = lambda t: None if t is None else t.to(device, non_blocking=non_blocking)  # noqa: E731
        return Block(mv(self.n_id), mv(self.res_n_id), mv(self.e_id), mv(self.edge_index), self.size, mv(self.nbr))

    def pin_memory(self):
        pm = lambda t: None if t is None else t.pin_memory()  # noqa: E731
        return Block(pm(self.n_id), pm(self.res_n_id), pm(self.e_id), pm(self.edge_index), self.size, pm(self.nbr))


class DataFlow:
    def __init__(self, n_id):
        self.n_id = n_id
        self._last = n_id
        self.blocks = []

    def append(self, n_id, res_n_id, e_id, edge_index):
        size = [int(self._last.numel()), int(n_id.numel())]
        self.blocks.append(Block(n_id, res_n_id, e_id, edge_index, size))
        self._last = n_id

    def __len__(self):
        return len(self.blocks)

    def __getitem__(self, idx):
        return self.blocks[::-1][idx]

    def __iter__(self):
        return iter(self.blocks[::-1])

    def to(self, device, non_blocking=True):
        out = DataFlow(self.n_id.to(device, non_blocking=non_blocking))
        out.blocks = [b.to(device, non_blocking) for b in self.blocks]
        out._last = self._last
        return out

    def pin_memory(self):
        out = DataFlow(self.n_id.pin_memory())
        out.blocks = [b.pin_memory() for b in self.blocks]
        out._last = self._last
        return out


class NeighborDataFlow:
    """Keep every sampled occurrence (no dedup)."""

    def __init__(self, num_hops, add_self_loops=True, **kwargs):
        self.num_hops = num_hops
        self.add_self_loops = add_self_loops

    def get_neighbors(self, n_id):
        raise NotImplementedError

    def produce_subgraph(self, n_id):
        n_id = torch.as_tensor(n_id).reshape(-1).long()
        last_idx = torch.arange(n_id.numel())
        df = DataFlow(n_id)
        neighbors, srcs = self.get_neighbors(n_id)
        for i in range(self.num_hops):
            new_n_id = torch.cat([neighbors[i], n_id])
            new_inv = torch.arange(new_n_id.numel())
            res_n_id = new_inv[-n_id.numel():] if n_id.numel() else new_inv[:0]
            edge_src = srcs[i]
            if self.add_self_loops:
                edge_src = torch.cat([edge_src, last_idx])
                last_idx = new_inv
            else:
                new_inv = new_inv[:new_inv.numel() - n_id.numel()]
                last_idx = new_inv
            n_id = new_n_id
            df.append(new_n_id, res_n_id, None, torch.stack([edge_src.long(), new_inv.long()]))
        return df

    def __call__(self, n_id):
        return self.produce_subgraph(n_id)


class UniqueDataFlow(NeighborDataFlow):
    """Dedup each hop's node set (reference neighbor_dataflow.py:84-110)."""

    def produce_subgraph(self, n_id):
        n_id = torch.as_tensor(n_id).reshape(-1).long()
        last_idx = torch.arange(n_id.numel())
        df = DataFlow(n_id)
        neighbors, srcs = self.get_neighbors(n_id)
        for i in range(self.num_hops):
            cat = torch.cat([neighbors[i], n_id])
            new_n_id, new_inv = unique_with_inverse(cat)
            res_n_id = new_inv[new_inv.numel() - n_id.numel():]
            edge_src = srcs[i]
            if self.add_self_loops:
                edge_src = torch.cat([edge_src, last_idx])
                last_idx = torch.arange(new_n_id.numel())
            else:
                new_inv = new_inv[:new_inv.numel() - n_id.numel()]
                last_idx = new_inv
            n_id = new_n_id
            df.append(new_n_id, res_n_id, None, torch.stack([edge_src.long(), new_inv.long()]))
        return df


class SageDataFlow(UniqueDataFlow):
    """Fixed-fanout sampling per hop (reference sage_dataflow.py:24-50)."""

    def __init__(self, fanouts, metapath, add_self_loops=True, max_id=-1, **kwargs):
        super().__init__(len(metapath), add_self_loops)
        self.fanouts = fanouts
        self.metapath = metapath
        self.max_id = max_id

    def produce_subgraph(self, n_id):
        n_id = torch.as_tensor(n_id).reshape(-1).long()
        hops = ge.sage_flow(n_id, self.metapath, self.fanouts, self.max_id + 1, self.add_self_loops)
        if hops is None:  # remote graph: per-hop GQL sampling + unique below
            df = super().produce_subgraph(n_id)
        else:
            # the engine built every hop in one native call (sampling, unique, edge index)
            df = DataFlow(n_id)
            for new_n_id, res_n_id, edge_index in hops:
                df.append(new_n_id, res_n_id, None, edge_index)
        self._attach_nbr(df)
        return df

    def _attach_nbr(self, df):
        """Both flows emit each hop's edges target-major (F sampled edges per target, then
        the n self loops): that is the dense [n, F (+1)] neighbour matrix, row-major."""
        for b, f in zip(df.blocks, self.fanouts):
            n, f = int(b.size[0]), int(f)
            e = int(b.edge_index.shape[1])
            if e != n * f + (n if self.add_self_loops else 0):
                continue
            src = b.edge_index[1]
            nbr = src[: n * f].view(n, f)
            if self.add_self_loops:
                nbr = torch.cat([nbr, src[n * f:].view(n, 1)], 1)
            b.nbr = nbr.to(torch.int32).contiguous()

    def get_neighbors(self, n_id):
        neighbors, srcs = [], []
        for et, count in zip(self.metapath, self.fanouts):
            n_id = n_id.reshape(-1)
            nb, _, _ = ge.sample_neighbor(n_id, et, int(count), default_node=self.max_id + 1)
            neighbors.append(nb.reshape(-1))
            srcs.append(torch.arange(n_id.numel()).repeat_interleave(int(count)))
            n_id, _ = unique_with_inverse(torch.cat([nb.reshape(-1), n_id]))
        return neighbors, srcs


class GCNDataFlow(UniqueDataFlow):
    """Full neighborhoods (reference gcn_dataflow.py:26-48)."""

    def __init__(self, metapath, add_self_loops=True, **kwargs):
        super().__init__(len(metapath), add_self_loops)
        self.metapath = metapath

    def get_neighbors(self, n_id):
        neighbors, srcs = [], []
        for et in self.metapath:
            n_id = n_id.reshape(-1)
            nb = ge.get_full_neighbor(n_id, et)[0]
            neighbors.append(nb.values.reshape(-1))
            srcs.append(nb.indices[:, 0].long())
            n_id, _ = unique_with_inverse(torch.cat([nb.values.reshape(-1), n_id]))
        return neighbors, srcs


class FastGCNDataFlow(UniqueDataFlow):
    """Global importance sampling per layer + induced adjacency (reference fast_dataflow.py:25-57)."""

    def __init__(self, fanouts, metapath, add_self_loops=True, **kwargs):
        super().__init__(len(metapath), add_self_loops)
        self.fanouts = fanouts
        self.metapath = metapath

    def get_neighbors(self, n_id):
        neighbors, srcs = [], []
        total = 0
        for i, et in enumerate(self.metapath):
            n_id = n_id.reshape(-1)
            if i == len(self.metapath) - 1:
                nb = ge.get_full_neighbor(n_id, et)[0]
                vals, src = nb.values.reshape(-1), nb.indices[:, 0].long()
            else:
                total += int(self.fanouts[i])
                cand, _ = unique_with_inverse(ge.sample_node(total, et[0] if isinstance(et, (list, tuple)) else et))
                adj = ge.sparse_get_adj(n_id, cand, et, -1, -1)
                vals, src = cand[adj.indices[:, 1].long()], adj.indices[:, 0].long()
            neighbors.append(vals)
            srcs.append(src)
            n_id, _ = unique_with_inverse(torch.cat([vals, n_id]))
        return neighbors, srcs


class LayerwiseDataFlow(UniqueDataFlow):
    """AdaptiveGCN layer-wise sampling (reference layerwise_dataflow.py:26-71)."""

    def __init__(self, fanouts, metapath, add_self_loops=True, **kwargs):
        super().__init__(len(metapath), add_self_loops)
        self.fanouts = fanouts
        self.metapath = metapath

    def get_neighbors(self, n_id):
        neighbors, srcs = [], []
        total = 0
        for i, et in enumerate(self.metapath):
            n_id = n_id.reshape(-1)
            if i == len(self.metapath) - 1:
                nb = ge.get_full_neighbor(n_id, et)[0]
                vals, src = nb.values.reshape(-1), nb.indices[:, 0].long()
            else:
                total += int(self.fanouts[i])
                layer, adj = ge.sample_neighbor_layerwise(n_id.reshape(1, -1), et, total)
                vals = layer.reshape(-1)[adj.indices[:, 2].long()]
                src = adj.indices[:, 1].long()
            neighbors.append(vals)
            srcs.append(src)
            n_id, _ = unique_with_inverse(torch.cat([vals, n_id]))
        return neighbors, srcs


class LayerwiseEachDataFlow(NeighborDataFlow):
    """First hop fanout sampling, then layer-wise per node group (reference layerwise_dataflow.py:74-119;
    its ``defulat_node`` keyword typo is not reproduced)."""

    def __init__(self, fanouts, metapath, add_self_loops=True, max_id=-1, **kwargs):
        super().__init__(len(metapath), add_self_loops)
        self.fanouts = fanouts
        self.metapath = metapath
        self.max_id = max_id

    def get_neighbors(self, n_id):
        n_id = n_id.reshape(-1)
        c0 = int(self.fanouts[0])
        nb, _, _ = ge.sample_neighbor(n_id, self.metapath[0], c0, default_node=self.max_id + 1)
        neighbors = [nb.reshape(-1)]
        srcs = [torch.arange(n_id.numel()).repeat_interleave(c0)]
        cur, last = nb.reshape(-1), c0
        for et, count in zip(self.metapath[1:], self.fanouts[1:]):
            layer, adj = ge.sample_neighbor_layerwise(cur.reshape(-1, last), et, int(count))
            ind = adj.indices.long()
            vals = layer.reshape(-1)[ind[:, 2] + ind[:, 0] * int(count)]
            neighbors.append(vals)
            srcs.append(ind[:, 1] + ind[:, 0] * last)
            cur, last = vals, int(count)
        return neighbors, srcs


class WholeDataFlow(NeighborDataFlow):
    """Induced subgraph of the batch, same block for every hop (reference whole_dataflow.py:26-62)."""

    def __init__(self, metapath, add_self_loops=True, **kwargs):
        super().__init__(len(metapath), add_self_loops)
        self.neighbor_type = metapath[0]
        for t in metapath:
            if t != self.neighbor_type:
                raise ValueError("Metapath should be the same in whole graph sampler.")

    def produce_subgraph(self, n_id):
        n_id = torch.as_tensor(n_id).reshape(-1).long()
        inv = torch.arange(n_id.numel())
        df = DataFlow(n_id)
        adj = ge.sparse_get_adj(n_id, n_id, self.neighbor_type, -1, -1)
        src, dst = adj.indices[:, 0].long(), adj.indices[:, 1].long()
        if self.add_self_loops:
            src, dst = torch.cat([src, inv]), torch.cat([dst, inv])
        ei = torch.stack([src, dst])
        for _ in range(self.num_hops):
            df.append(n_id, inv, None, ei)
        return df


class RelationDataFlow:
    """Full neighborhoods with edge types as ``e_id`` (reference relation_dataflow.py:25-75)."""

    def __init__(self, fanouts, metapath, add_self_loops=True, **kwargs):
        self.metapath = metapath

    def produce_subgraph(self, n_id):
        n_id = torch.as_tensor(n_id).reshape(-1).long()
        df = DataFlow(n_id)
        for et in self.metapath:
            nb, _, ty = ge.get_full_neighbor(n_id, et)
            cat = torch.cat([nb.values.reshape(-1), n_id])
            new_n_id, new_inv = unique_with_inverse(cat)
            res_n_id = new_inv[new_inv.numel() - n_id.numel():]
            dst = new_inv[:new_inv.numel() - n_id.numel()]
            df.append(new_n_id, res_n_id, ty.values.reshape(-1).long(),
                      torch.stack([nb.indices[:, 0].long(), dst.long()]))
            n_id = new_n_id
        return df

    def __call__(self, n_id):
        return self.produce_subgraph(n_id)
