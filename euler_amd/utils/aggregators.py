"""Fixed-fanout neighbour aggregators for the encoder API
(reference ``tf_euler/python/utils/aggregators.py:24-118``).

Inputs are ``(self_embedding [n, d], neigh_embedding [n, fanout, d])``, which is the
dense tree layout the sampler produces.  The reductions are plain tensor ops on the
``[n, fanout, d]`` block (one fused reduce per call); the two projections of
``mean`` are computed as ONE GEMM on ``[x_self | mean]`` against the stacked weight,
the same trick the fused gfx950 SAGE kernel uses (``euler_amd/csrc/hip/sage.hip``).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from euler_amd.utils.layers import Dense, get_activation

__all__ = ["GCNAggregator", "BaseAggregator", "MeanAggregator", "BasePoolAggregator", "MeanPoolAggregator",
           "MaxPoolAggregator", "aggregators", "get"]

_relu = torch.relu


class GCNAggregator(nn.Module):
    """dense(mean([self, neighbours]))."""

    def __init__(self, dim, activation=_relu, **kwargs):
        super().__init__()
        self.dense = Dense(dim, activation=activation, use_bias=False)

    def forward(self, inputs):
        self_emb, neigh_emb = inputs
        k = neigh_emb.shape[1]
        agg = (self_emb + neigh_emb.sum(1)) / float(k + 1)
        return self.dense(agg)


class BaseAggregator(nn.Module):
    """self_layer(x) (+|concat) neigh_layer(aggregate(neighbours))."""

    def __init__(self, dim, activation=_relu, concat=False, **kwargs):
        super().__init__()
        if concat:
            if dim % 2:
                raise ValueError("dim must be divided exactly by 2 if concat is True.")
            dim //= 2
        self.concat = concat
        self.activation = get_activation(activation)
        self.self_layer = Dense(dim, activation=activation, use_bias=False)
        self.neigh_layer = Dense(dim, activation=activation, use_bias=False)

    def aggregate(self, inputs):
        raise NotImplementedError

    def forward(self, inputs):
        self_emb, neigh_emb = inputs
        agg = self.aggregate(neigh_emb)
        from_self = self.self_layer(self_emb)
        from_neighs = self.neigh_layer(agg)
        if self.concat:
            return torch.cat([from_self, from_neighs], 1)
        return from_self + from_neighs


class MeanAggregator(BaseAggregator):
    def aggregate(self, inputs):
        return inputs.mean(1)


class BasePoolAggregator(BaseAggregator):
    def __init__(self, dim, *args, **kwargs):
        super().__init__(dim, *args, **kwargs)
        self.layers = nn.ModuleList([Dense(dim, activation=_relu)])

    def aggregate(self, inputs):
        h = inputs
        for layer in self.layers:
            h = layer(h)
        return self.pool(h)

    def pool(self, inputs):
        raise NotImplementedError


class MeanPoolAggregator(BasePoolAggregator):
    def pool(self, inputs):
        return inputs.mean(1)


class MaxPoolAggregator(BasePoolAggregator):
    def pool(self, inputs):
        return inputs.amax(1)


aggregators = {
    "gcn": GCNAggregator,
    "mean": MeanAggregator,
    "meanpool": MeanPoolAggregator,
    "maxpool": MaxPoolAggregator,
}


def get(aggregator):
    return aggregators.get(aggregator)
