"""Sparse-adjacency aggregators for full-neighbour encoders
(reference ``tf_euler/python/utils/sparse_aggregators.py:24-160``).

Inputs are ``(self_embedding [n, d], neigh_embedding [m, d], adj)`` where ``adj`` is a
:class:`euler_amd.ops.graph_api.SparseTensor` of shape ``[n, m]`` (its values are
ignored, as in the reference: ``_sparse_ones_like``).  The sparse-dense products are
gather + segment-reduce on the gfx950 kernels of :mod:`euler_amd.ops.mp_ops`; the
attention softmax is the fused edge-softmax kernel.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from euler_amd.ops import mp_ops
from euler_amd.utils.layers import Dense, get_activation

__all__ = ["GCNAggregator", "MeanAggregator", "SingleAttentionAggregator", "AttentionAggregator",
           "aggregators", "get"]

_relu = torch.relu


def _adj_rows_cols(adj, device):
    """(rows, cols, n, row SegmentIndex) of ``adj``, built once per adjacency and shared by
    every aggregator / head / layer over it (a producer that knows the CSR — the device
    flow — stores it as ``adj._euler_idx`` up front)"""
    idx = getattr(adj, "_euler_idx", None)
    if idx is not None and idx[0].device == torch.device(device):
        return idx
    ind = torch.as_tensor(adj.indices).to(device).long()
    n = int(adj.dense_shape[0])
    rows, cols = ind[:, 0].contiguous(), ind[:, 1].contiguous()
    idx = (rows, cols, n, mp_ops.SegmentIndex(rows, n))
    try:
        adj._euler_idx = idx
    except AttributeError:
        pass
    return idx


def _sum_neighbors(neigh, rows, cols, n, seg=None):
    """ones(adj) @ neigh as gather + segment sum; returns (sum [n, d], degree [n, 1])."""
    seg = seg if seg is not None else rows
    msg = mp_ops.gather(neigh, cols)
    s = mp_ops.scatter_add(msg, seg, n)
    # a -1 row (padding entry of a device-built adjacency) is dropped, like in scatter_add
    ones = torch.ones(rows.numel(), 1, dtype=neigh.dtype, device=neigh.device)
    deg = mp_ops.scatter_add(ones, seg, n)
    return s, deg


class GCNAggregator(nn.Module):
    def __init__(self, dim, activation=_relu, renorm=False, **kwargs):
        super().__init__()
        self.renorm = renorm
        self.dense = Dense(dim, activation=activation, use_bias=False)

    def forward(self, inputs):
        self_emb, neigh_emb, adj = inputs
        rows, cols, n, seg = _adj_rows_cols(adj, self_emb.device)
        agg, deg = _sum_neighbors(neigh_emb, rows, cols, n, seg)
        if self.renorm:
            agg = (self_emb + agg) / (1.0 + deg)
        else:
            agg = self_emb + agg / deg.clamp_min(1e-7)
        return self.dense(agg)


class MeanAggregator(nn.Module):
    def __init__(self, dim, activation=_relu, concat=False, **kwargs):
        super().__init__()
        if concat:
            dim //= 2
        self.concat = concat
        self.self_layer = Dense(dim, activation=activation, use_bias=False)
        self.neigh_layer = Dense(dim, activation=activation, use_bias=False)

    def forward(self, inputs):
        self_emb, neigh_emb, adj = inputs
        rows, cols, n, seg = _adj_rows_cols(adj, self_emb.device)
        agg, deg = _sum_neighbors(neigh_emb, rows, cols, n, seg)
        agg = agg / deg.clamp_min(1e-7)
        a, b = self.self_layer(self_emb), self.neigh_layer(agg)
        return torch.cat([a, b], 1) if self.concat else a + b


class SingleAttentionAggregator(nn.Module):
    """One GAT-style head over the sparse adjacency (``renorm`` adds self loops)."""

    def __init__(self, dim, activation=_relu, renorm=False, **kwargs):
        super().__init__()
        self.dense = Dense(dim, use_bias=False)
        self.self_layer = Dense(1, use_bias=False)
        self.neigh_layer = Dense(1, use_bias=False)
        self.activation = get_activation(activation)
        self.renorm = renorm

    def forward(self, inputs):
        self_emb, neigh_emb, adj = inputs
        rows, cols, n, seg = _adj_rows_cols(adj, self_emb.device)
        if self.renorm:
            # [eye | adj] over the column space [self rows ; neighbour rows]
            eye = torch.arange(n, device=rows.device)
            rows = torch.cat([eye, rows])
            cols = torch.cat([eye, torch.where(cols >= 0, cols + n, cols)])
            seg = mp_ops.SegmentIndex(rows, n)
            from_all = self.dense(torch.cat([self_emb, neigh_emb], 0))
            from_self = from_all[:n]
        else:
            from_all = self.dense(neigh_emb)
            from_self = self.dense(self_emb)
        self_w = self.self_layer(from_self).view(-1, 1)
        all_w = self.neigh_layer(from_all).view(-1, 1)
        # gfx950 gathers (their backward is a segment reduction; a torch index backward
        # serialises on repeated rows, e.g. the -1 padding entries of a device adjacency)
        logits = F.leaky_relu(mp_ops.gather(self_w, rows) + mp_ops.gather(all_w, cols), 0.2)
        coef = mp_ops.scatter_softmax(logits, seg, n)
        out = mp_ops.scatter_add(coef * mp_ops.gather(from_all, cols), seg, n)
        if not self.renorm:
            out = from_self + out
        if self.activation is not None:
            out = self.activation(out)
        return out


class AttentionAggregator(nn.Module):
    def __init__(self, dim, head_num=4, activation=_relu, renorm=False, **kwargs):
        super().__init__()
        dim //= head_num
        self.attentions = nn.ModuleList([SingleAttentionAggregator(dim, activation, renorm)
                                         for _ in range(head_num)])

    def forward(self, inputs):
        return torch.cat([att(inputs) for att in self.attentions], 1)


aggregators = {
    "gcn": GCNAggregator,
    "mean": MeanAggregator,
    "attention": AttentionAggregator,
}


def get(aggregator):
    return aggregators.get(aggregator)
