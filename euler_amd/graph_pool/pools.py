"""Graph pooling for graph classification (reference ``tf_euler/python/graph_pool/*.py``).

``pool(x [N, D], index [N] graph id, size)`` -> [size, D]; segment reductions and the
attention softmax run on the gfx950 segment kernels for GPU tensors.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from euler_amd.ops import mp_ops
from euler_amd.utils.layers import Dense

__all__ = ["Pooling", "AttentionPool", "Set2SetPool"]


def _size(index, size):
    return int(index.max().item()) + 1 if size is None else int(size)


class Pooling(nn.Module):
    def __init__(self, aggr="add"):
        super().__init__()
        assert aggr in ("add", "mean", "max")
        self.aggr = aggr

    def forward(self, inputs, index, size=None):
        return mp_ops.scatter_(self.aggr, inputs, index, _size(index, size))


class AttentionPool(Pooling):
    def __init__(self, gate_nn=None, nn_=None, aggr="add"):
        super().__init__(aggr)
        self.gate_nn = gate_nn if gate_nn is not None else Dense(1, use_bias=False)
        self.nn = nn_

    def forward(self, inputs, index, size=None):
        size = _size(index, size)
        gate = mp_ops.scatter_softmax(self.gate_nn(inputs), index, size)
        x = self.nn(inputs) if self.nn is not None else inputs
        return mp_ops.scatter_(self.aggr, gate * x, index, size)


class Set2SetPool(Pooling):
    def __init__(self, dim, processing_steps=3, num_layers=1, aggr="add"):
        super().__init__(aggr)
        self.dim, self.steps, self.num_layers = dim, processing_steps, num_layers
        self.lstm = nn.LSTM(2 * dim, dim, num_layers=num_layers)

    def forward(self, inputs, index, size=None):
        size = _size(index, size)
        q_star = torch.zeros(size, 2 * self.dim, device=inputs.device, dtype=inputs.dtype)
        h = (torch.zeros(self.num_layers, size, self.dim, device=inputs.device, dtype=inputs.dtype),
             torch.zeros(self.num_layers, size, self.dim, device=inputs.device, dtype=inputs.dtype))
        for _ in range(self.steps):
            q, h = self.lstm(q_star.unsqueeze(0), h)
            q = q.reshape(size, self.dim)
            e = (inputs * mp_ops.gather(q, index)).sum(-1, keepdim=True)
            a = mp_ops.scatter_softmax(e, index, size)
            r = mp_ops.scatter_(self.aggr, a * inputs, index, size)
            q_star = torch.cat([q, r], -1)
        return q_star
