"""Layers (reference ``tf_euler/python/utils/layers.py:35-270``) on PyTorch.

``Dense`` mirrors ``tf.layers.Dense``: the input width is inferred at the first call
(lazy), Glorot-uniform kernel, zero bias, optional activation.  ``Embedding`` /
``SparseEmbedding`` are id -> row lookups with the reference's ``max_id + 1`` rows
(the padding id ``max_id + 1`` is a valid, trainable row, like the reference);
on a GPU the row gather runs the gfx950 ``gather_rows`` kernel.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from euler_amd.ops import mp_ops

__all__ = ["Dense", "Embedding", "HashEmbedding", "SparseEmbedding", "HashSparseEmbedding", "AttLayer", "LSTMLayer",
           "get_activation"]

_ACTS = {None: None, "relu": F.relu, "tanh": torch.tanh, "sigmoid": torch.sigmoid, "elu": F.elu,
         "leaky_relu": F.leaky_relu}


def get_activation(act):
    if callable(act) or act is None:
        return act
    return _ACTS[act]


class Dense(nn.LazyLinear):
    cls_to_become = None  # keep the Dense class (and its activation) after materialisation

    def __init__(self, dim, activation=None, use_bias=True, **kwargs):
        super().__init__(dim, bias=use_bias)
        self.activation = get_activation(activation)

    def reset_parameters(self):
        if not self.has_uninitialized_params() and self.in_features != 0:
            nn.init.xavier_uniform_(self.weight)
            if self.bias is not None:
                nn.init.zeros_(self.bias)

    def forward(self, x):
        if self.has_uninitialized_params():
            return super().forward(x) if self.activation is None else self.activation(super().forward(x))
        w = self.weight if self.weight.dtype == x.dtype else self.weight.to(x.dtype)
        b = None if self.bias is None else (self.bias if self.bias.dtype == x.dtype else self.bias.to(x.dtype))
        if x.is_cuda and x.dim() == 2 and x.shape[0] >= 512:
            from euler_amd.ops.gnn_ops import splitk_linear

            y = splitk_linear(x, w, b)  # split-K weight gradient (GPU, tall batches)
        else:
            y = F.linear(x, w, b)
        return y if self.activation is None else self.activation(y)




def _trunc_normal(std):
    return lambda w: nn.init.trunc_normal_(w, std=std, a=-2 * std, b=2 * std)


class Embedding(nn.Module):
    """Id -> row lookup with ``max_id + 1`` rows (reference layers.py:119-149).

    Out-of-range ids (including the ``-1`` default node) map to the last row, so the
    sampler's padding id is a valid trainable row like the reference's ``max_id + 1``.
    """

    def __init__(self, max_id, dim, initializer=None, **kwargs):
        super().__init__()
        self.num = int(max_id) + 1
        self.dim = int(dim)
        self.weight = nn.Parameter(torch.empty(self.num, self.dim))
        (initializer or _trunc_normal(0.1))(self.weight)

    def _rows(self, ids):
        ids = torch.as_tensor(ids, device=self.weight.device).long()
        return torch.where((ids < 0) | (ids >= self.num), torch.full_like(ids, self.num - 1), ids)

    def forward(self, ids):
        ids = self._rows(ids)
        shape = ids.shape
        return mp_ops.gather(self.weight, ids.reshape(-1)).reshape(*shape, self.dim)


class HashEmbedding(Embedding):
    """Embedding over ``hash(id) % num_buckets`` rows (the reference names this class in
    encoders.py:107 but never defines it; here it is a real multiplicative hash)."""

    def _rows(self, ids):
        ids = torch.as_tensor(ids, device=self.weight.device).long()
        h = (ids * 0x9E3779B1) & 0x7FFFFFFF
        return h % self.num


class SparseEmbedding(Embedding):
    """Embedding-bag over a SparseTensor of ids, combiner sum | mean
    (reference layers.py:152-169, ``embedding_lookup_sparse``)."""

    def __init__(self, max_id, dim, initializer=None, combiner="sum", **kwargs):
        super().__init__(max_id, dim, initializer or _trunc_normal(0.0002))
        self.combiner = combiner

    def forward(self, sp):
        rows = torch.as_tensor(sp.indices)[:, 0].to(self.weight.device).long()
        n = int(sp.dense_shape[0])
        ids = self._rows(torch.as_tensor(sp.values).to(torch.int64))
        # one fused embedding-bag (CSR SpMM over the table) instead of gather + scatter
        order = torch.argsort(rows, stable=True)
        return mp_ops.embedding_bag(self.weight, ids.reshape(-1)[order], rows[order], n,
                                    "mean" if self.combiner == "mean" else "sum")


class HashSparseEmbedding(SparseEmbedding):
    _rows = HashEmbedding._rows


class AttLayer(nn.Module):
    """Multi-head self-attention over a sequence, returning position 0
    (reference layers.py:172-238).

    input [B, L, D]; hidden layers of ``hidden_dim[i]`` x ``head_num[i]`` heads, then
    ``head_num[-1]`` output heads of width ``out_dim`` averaged.  Each head is
    ``softmax(leaky_relu(f1 + f2^T)) @ (x W) + b``.
    """

    def __init__(self, out_dim, activation=F.elu, activation_out=None, hidden_dim=(), head_num=(1,), **kwargs):
        super().__init__()
        hidden_dim, head_num = list(hidden_dim), list(head_num)
        if len(head_num) < 1 or len(head_num) != len(hidden_dim) + 1:
            raise ValueError("head_num must have len(hidden_dim) + 1 entries, got {},{}".format(head_num, hidden_dim))
        self.out_dim, self.hidden_dim, self.head_num = out_dim, hidden_dim, head_num
        self.activation = get_activation(activation)
        self.activation_out = get_activation(activation_out)
        widths = hidden_dim + [out_dim]
        self.heads = nn.ModuleList([nn.ModuleList([_AttHead(w) for _ in range(h)])
                                    for w, h in zip(widths, head_num)])

    def forward(self, x):
        if x.dim() != 3:
            raise ValueError("inputs rank must be 3 for AttLayer, got shape %s" % (tuple(x.shape),))
        h = x
        for heads in self.heads[:-1]:
            h = torch.cat([hd(h, self.activation) for hd in heads], -1)
        out = sum(hd(h, self.activation_out) for hd in self.heads[-1]) / len(self.heads[-1])
        return out[:, 0, :]


class _AttHead(nn.Module):
    def __init__(self, out_size):
        super().__init__()
        self.proj = Dense(out_size, use_bias=False)
        self.f1 = Dense(1, use_bias=False)
        self.f2 = Dense(1, use_bias=False)
        self.bias = nn.Parameter(torch.zeros(out_size))

    def forward(self, seq, act):
        fts = self.proj(seq)
        logits = self.f1(fts) + self.f2(fts).transpose(1, 2)
        coefs = torch.softmax(F.leaky_relu(logits, 0.2), -1)
        out = torch.bmm(coefs, fts) + self.bias
        return out if act is None else act(out)


class LSTMLayer(nn.Module):
    """Sequence LSTM ``[B, T, D] -> (outputs [B, T, out_dim], (h, c))``
    (reference layers.py:241-270)."""

    def __init__(self, out_dim, activation=None, **kwargs):
        super().__init__()
        self.out_dim = out_dim
        self.activation = get_activation(activation)
        self.lstm = None

    def forward(self, x, state=None):
        if self.lstm is None:
            self.lstm = nn.LSTM(x.shape[-1], self.out_dim, batch_first=True).to(x.device)
        out, st = self.lstm(x, state)
        if self.activation is not None:
            out = self.activation(out)
        return out, st
