"""Supervised GraphSAGE on the fused, fixed-shape "tree layout" path.

Model = reference ``SupervisedGraphSage`` (``examples/graphsage/graphsage.py:56-67``):
``dims = [hidden] * (layers + 1)``, one ``SAGEConv`` (self_fc + neigh_fc, no bias,
mean aggregation, ``add_self_loops=False``) + ReLU per hop, then ``fc`` (with bias)
and ``out_fc`` (no bias) and a sigmoid cross-entropy on the label
(``tf_euler/python/mp_utils/base.py:24-47``).

Mini-batch layout (MI355X-first): instead of ``tf.unique`` relabelling per hop
(dynamic shapes, host syncs), every hop keeps one row per *sampled occurrence*:

    level_0 = roots                                  [B]
    level_i = concat(nbr_i.flatten(), level_{i-1})   [B * prod(f_j + 1)]

so the neighbors of target ``t`` of an inner layer are rows ``t*f .. t*f+f-1`` and
its self row is ``|nbr_i| + t`` — static index tensors, disjoint rows (backward
needs no atomics).  Every shape is static, so sampling + forward + backward +
optimizer are captured into ONE hipGraph and replayed per step.  Without dedup
each occurrence draws its own hop samples: the same estimator as the reference's
``SageDataFlow`` (weighted with-replacement sampling per node), with no merging of
repeated ids.  The outermost layer gathers straight from the HBM feature table
inside the fused kernel: the [rows, D] input block is never materialised.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from euler_amd.ops.sage_ops import sage_layer

__all__ = ["FusedSupervisedGraphSage", "TreeBatchIndex", "synthetic_features", "synthetic_labels", "expected_rows"]


class TreeBatchIndex:
    """Static index tensors of the tree layout for a given (batch, fanouts)."""

    def __init__(self, batch_size: int, fanouts, device):
        self.batch_size = int(batch_size)
        self.fanouts = [int(f) for f in fanouts]
        self.level_sizes = [self.batch_size]
        for f in self.fanouts:
            self.level_sizes.append(self.level_sizes[-1] * (f + 1))
        # inner layer i (targets = level i, sources = level i+1)
        self.inner = []
        for i in range(len(self.fanouts) - 1):
            n_t = self.level_sizes[i]
            f = self.fanouts[i]
            nbr = torch.arange(n_t * f, dtype=torch.int32, device=device).view(n_t, f)
            self_idx = torch.arange(n_t * f, n_t * f + n_t, dtype=torch.int32, device=device)
            self.inner.append((self_idx, nbr))


class FusedSupervisedGraphSage(nn.Module):
    def __init__(self, feature_dim: int, hidden_dim: int, label_dim: int, fanouts, add_self_loops: bool = False):
        super().__init__()
        self.fanouts = [int(f) for f in fanouts]
        self.num_layers = len(self.fanouts)
        self.add_self_loops = add_self_loops
        dims = [feature_dim] + [hidden_dim] * self.num_layers
        self.conv_weights = nn.ParameterList()
        for i in range(self.num_layers):
            w = torch.empty(dims[i + 1], 2 * dims[i])
            # glorot like tf.layers.Dense; self_fc / neigh_fc halves initialised independently
            nn.init.xavier_uniform_(w[:, : dims[i]])
            nn.init.xavier_uniform_(w[:, dims[i]:])
            self.conv_weights.append(nn.Parameter(w))
        self.fc = nn.Linear(hidden_dim, hidden_dim, bias=True)
        self.out_fc = nn.Linear(hidden_dim, label_dim, bias=False)
        nn.init.xavier_uniform_(self.fc.weight)
        nn.init.zeros_(self.fc.bias)
        nn.init.xavier_uniform_(self.out_fc.weight)
        self._tree = None

    def tree(self, batch_size, device):
        if self._tree is None or self._tree.batch_size != batch_size:
            self._tree = TreeBatchIndex(batch_size, self.fanouts, device)
        return self._tree

    def sample(self, graph, roots, edge_types=None):
        """Per-hop neighbor samples in tree layout.  Returns [level_0, ..., level_L] and nbr blocks."""
        levels = [roots.reshape(-1).int()]
        nbrs = []
        for i, f in enumerate(self.fanouts):
            nb = graph.sample_neighbor(levels[-1], f, edge_types=edge_types, default=-1, stream_id=16 + i)
            nbrs.append(nb)
            levels.append(torch.cat([nb.reshape(-1), levels[-1]]))
        return levels, nbrs

    def embed(self, features, levels, nbrs):
        L = self.num_layers
        tree = self.tree(levels[0].numel(), levels[0].device)
        # outermost layer: gather straight from the feature table
        h = sage_layer(features, levels[L - 1], nbrs[L - 1], self.conv_weights[0], None,
                       include_self=self.add_self_loops, relu=True, disjoint=False)
        for j in range(1, L):
            self_idx, nbr = tree.inner[L - 1 - j]
            h = sage_layer(h, self_idx, nbr, self.conv_weights[j], None,
                           include_self=self.add_self_loops, relu=True, disjoint=True)
        emb = F.linear(h, self.fc.weight.to(h.dtype), self.fc.bias.to(h.dtype))
        return emb

    def forward(self, features, levels, nbrs):
        emb = self.embed(features, levels, nbrs)
        return F.linear(emb, self.out_fc.weight.to(emb.dtype))

    def loss(self, logits, labels):
        """Sigmoid CE on one-hot labels (reference SuperviseModel)."""
        # scatter-based one-hot: no host-side range check (hipGraph-capturable)
        target = torch.zeros(logits.shape, dtype=torch.float32, device=logits.device)
        target.scatter_(1, labels.long().view(-1, 1), 1.0)
        return F.binary_cross_entropy_with_logits(logits.float(), target)


def synthetic_labels(features: torch.Tensor, label_dim: int, chunk: int = 1 << 22) -> torch.Tensor:
    """Learnable synthetic labels: argmax of the first ``label_dim`` feature columns."""
    n = features.shape[0]
    out = torch.empty(n, dtype=torch.int16, device=features.device)
    for s in range(0, n, chunk):
        out[s:s + chunk] = features[s:s + chunk, :label_dim].float().argmax(1).to(torch.int16)
    return out


def synthetic_features(n: int, dim: int, seed: int, device, dtype=torch.bfloat16, chunk: int = 1 << 22):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    out = torch.empty((n, dim), dtype=dtype, device=device)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        out[s:e] = torch.randn((e - s, dim), generator=g, device=device, dtype=torch.float32).to(dtype)
    return out


def expected_rows(batch_size, fanouts):
    return batch_size * math.prod(f + 1 for f in fanouts)
