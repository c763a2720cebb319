"""Unsupervised / self-supervised embedding models (reference ``examples/*``).

=====================  ===================================================  =====================================
model                  objective                                            reference
=====================  ===================================================  =====================================
UnsupervisedGraphSage  1 sampled neighbour vs sampled negatives, sigmoid CE  examples/graphsage/graphsage.py:70-98
DeepWalk / Node2Vec    random_walk + gen_pair skip-gram, negatives          examples/deepwalk/deepwalk.py:27-99
LINE                   first / second order proximity                       examples/line/line.py:27-71
DGI                    deep graph infomax with a corrupted view             examples/dgi/dgi.py:24-90
GraphAutoEncoder       GCN/SAGE encoder, link reconstruction                examples/gae/gae.py:52-92
VGAE                   variational GAE (+ KL)                               examples/gae/gae.py:94-153
UnsupervisedRGCN       RelationConv + RelationDataFlow                      examples/rgcn/rgcn.py:30-105
=====================  ===================================================  =====================================

Id embedding tables can be row-sharded across data-parallel ranks
(``sharded=True`` -> :class:`~euler_amd.parallel.embedding.ShardedEmbedding`), the
MI355X replacement for the reference's PS-partitioned variables.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

import euler_amd.ops.graph_api as ge
from euler_amd.mp_utils.models import BaseGNNNet, BaseGraphAutoEncoder, UnsuperviseModel
from euler_amd.models.node_classification import FeatureGNN
from euler_amd.parallel.embedding import ShardedEmbedding
from euler_amd.utils import encoders
from euler_amd.utils import metrics as M
from euler_amd.utils.layers import Dense

__all__ = ["UnsupervisedGraphSage", "BaseNode2Vec", "DeepWalk", "Node2Vec", "Line", "DGI", "GraphAutoEncoder",
           "VariationalGraphAutoEncoder", "UnsupervisedRGCN", "IdEncoder"]


class IdEncoder(nn.Module):
    """id -> embedding, optionally row-sharded over the process group.  Both forms hold
    ``max_id + 2`` rows: row ``max_id + 1`` is the trainable pad row of the walks' and
    samplers' default node (reference ``max_id + 1``), never an alias of node ``max_id``."""

    def __init__(self, max_id, dim, sharded=False):
        super().__init__()
        self.table = ShardedEmbedding(max_id + 1, dim) if sharded else None
        self.enc = None if sharded else encoders.ShallowEncoder(dim=dim, feature_idx=-1, max_id=max_id,
                                                                 embedding_dim=dim, combiner="add")

    def forward(self, ids):
        return self.table(ids) if self.table is not None else self.enc(ids)


def _embed3(fn, n_id, dim):
    n_id = torch.as_tensor(n_id)
    b = n_id.shape[0]
    return fn(n_id.reshape(-1)).reshape(b, -1, dim)


class UnsupervisedGraphSage(UnsuperviseModel):
    def __init__(self, dims, fanouts, metapath, feature_idx, feature_dim, node_type, edge_type, max_id, num_negs=5,
                 metric_name="mrr"):
        super().__init__(node_type, edge_type, max_id, num_negs, metric_name)
        self.gnn = FeatureGNN("sage", "sage", dims, fanouts, metapath, feature_idx, feature_dim, max_id=max_id)
        self.context_gnn = FeatureGNN("sage", "sage", dims, fanouts, metapath, feature_idx, feature_dim,
                                      max_id=max_id)
        self.dim = dims[-1]

    def embed(self, n_id):
        return _embed3(self.gnn, n_id, self.dim)

    def embed_context(self, n_id):
        return _embed3(self.context_gnn, n_id, self.dim)

    def forward(self, inputs):
        emb, loss, name, metric = super().forward(inputs)
        return emb.reshape(-1, self.dim), loss, name, metric


class BaseNode2Vec(UnsuperviseModel):
    """random walk -> skip-gram pairs -> negatives (deepwalk.py:27-70)."""

    def __init__(self, node_type, edge_type, max_id, walk_len=3, walk_p=1, walk_q=1, left_win_size=1,
                 right_win_size=1, num_negs=5, metric="mrr", neg_condition=""):
        super().__init__(node_type, edge_type, max_id, num_negs, metric)
        self.walk_len, self.walk_p, self.walk_q = walk_len, walk_p, walk_q
        self.left_win_size, self.right_win_size = left_win_size, right_win_size
        self.neg_condition = neg_condition
        self.batch_size_ratio = int(ge.gen_pair(torch.zeros((0, walk_len + 1), dtype=torch.int64), left_win_size,
                                                right_win_size).shape[1])

    def to_sample(self, inputs):
        inputs = torch.as_tensor(inputs).reshape(-1)
        b = inputs.numel()
        path = ge.random_walk(inputs, [self.edge_type] * self.walk_len, p=self.walk_p, q=self.walk_q,
                              default_node=self.max_id + 1)
        pair = torch.as_tensor(ge.gen_pair(path, self.left_win_size, self.right_win_size))
        n_pairs = pair.shape[1]
        src = pair[..., 0].reshape(b * n_pairs, 1)
        pos = pair[..., 1].reshape(b * n_pairs, 1)
        negs = ge.sample_node(b * n_pairs * self.num_negs, self.node_type, condition=self.neg_condition)
        return src, pos, torch.as_tensor(negs).reshape(b * n_pairs, self.num_negs)


class DeepWalk(BaseNode2Vec):
    def __init__(self, node_type, edge_type, max_id, dim, walk_len=3, walk_p=1, walk_q=1, left_win_size=1,
                 right_win_size=1, num_negs=5, feature_idx=-1, feature_dim=0, use_id=True, embedding_dim=16,
                 metric="mrr", combiner="add", neg_condition="", sharded=False):
        super().__init__(node_type, edge_type, max_id, walk_len, walk_p, walk_q, left_win_size, right_win_size,
                         num_negs, metric, neg_condition)
        self.dim = dim
        if sharded and use_id and feature_idx == -1:
            self._target_encoder = IdEncoder(max_id, dim, sharded=True)
            self._context_encoder = IdEncoder(max_id, dim, sharded=True)
        else:
            mk = lambda: encoders.ShallowEncoder(dim=dim, feature_idx=feature_idx, feature_dim=feature_dim,  # noqa
                                                 max_id=max_id if use_id else -1, embedding_dim=embedding_dim,
                                                 combiner=combiner)
            self._target_encoder, self._context_encoder = mk(), mk()

    def embed(self, inputs):
        return self._target_encoder(inputs)

    def embed_context(self, inputs):
        return self._context_encoder(inputs)


class Node2Vec(DeepWalk):
    """DeepWalk with biased (p, q) walks; the defaults of the reference runner are p=q=1."""


class Line(UnsuperviseModel):
    def __init__(self, node_type, edge_type, max_id, dim, num_negs=5, order=1, feature_idx=-1, feature_dim=0,
                 use_id=True, sparse_feature_idx=-1, sparse_feature_max_id=-1, embedding_dim=16,
                 use_hash_embedding=False, combiner="add", metric="mrr", sharded=False):
        super().__init__(node_type, edge_type, max_id, num_negs, metric)
        order = {1: "first", 2: "second"}.get(order, order)
        if order not in ("first", "second"):
            raise ValueError('Line order must be one of 1, 2, "first", or "second" got {}:'.format(order))

        def mk():
            if sharded and use_id and feature_idx == -1 and sparse_feature_idx == -1:
                return IdEncoder(max_id, dim, sharded=True)
            return encoders.ShallowEncoder(dim=dim, feature_idx=feature_idx, feature_dim=feature_dim,
                                           max_id=max_id if use_id else -1, sparse_feature_idx=sparse_feature_idx,
                                           sparse_feature_max_id=sparse_feature_max_id, embedding_dim=embedding_dim,
                                           use_hash_embedding=use_hash_embedding, combiner=combiner)

        self.dim = dim
        self._target_encoder = mk()
        self._context_encoder = self._target_encoder if order == "first" else mk()

    def embed(self, inputs):
        return self._target_encoder(inputs)

    def embed_context(self, inputs):
        return self._context_encoder(inputs)


class DGI(nn.Module):
    """Deep Graph Infomax (dgi.py:24-90): a bilinear discriminator separates real
    embeddings from embeddings of a feature-shuffled view, against the sigmoid of the
    batch-mean readout."""

    def __init__(self, node_type, edge_type, max_id, metapath, fanouts, dim, aggregator="mean", concat=False,
                 feature_idx=-1, feature_dim=0, use_feature=None, use_id=False, sparse_feature_idx=-1,
                 sparse_feature_max_id=-1, embedding_dim=16, use_hash_embedding=False, use_residual=False,
                 num_negs=5, metric="mrr"):
        super().__init__()
        self.node_type, self.edge_type, self.max_id, self.num_negs, self.dim = node_type, edge_type, max_id, \
            num_negs, dim
        self.kernel = Dense(dim, use_bias=False)
        self.metric = M.get(metric)
        self.metric_name = metric
        self._target_encoder = encoders.ShuffleSageEncoder(
            metapath, fanouts, dim, aggregator, concat, feature_idx=feature_idx, feature_dim=feature_dim,
            max_id=max_id, use_id=use_id, sparse_feature_idx=sparse_feature_idx,
            sparse_feature_max_id=sparse_feature_max_id, embedding_dim=embedding_dim,
            use_hash_embedding=use_hash_embedding, use_residual=use_residual)

    def target_encoder(self, inputs):
        return self._target_encoder(inputs)

    @staticmethod
    def readout_func(inputs):
        res = torch.sigmoid(inputs.mean(0, keepdim=True))
        return res.expand(inputs.shape[0], *res.shape[1:])

    def decoder(self, emb, emb_pos, emb_negs):
        logits = torch.matmul(self.kernel(emb), emb_pos.transpose(-1, -2)).float()
        neg_logits = torch.matmul(self.kernel(emb_negs), emb_pos.transpose(-1, -2)).float()
        metric = self.metric(logits.detach().cpu(), neg_logits.detach().cpu())
        t = F.binary_cross_entropy_with_logits(logits, torch.ones_like(logits), reduction="sum")
        n = F.binary_cross_entropy_with_logits(neg_logits, torch.zeros_like(neg_logits), reduction="sum")
        return (t + n) / float(logits.numel() + neg_logits.numel()), metric

    def forward(self, inputs):
        src = torch.as_tensor(inputs).reshape(-1, 1)
        emb, emb_negs = self.target_encoder(src)
        loss, metric = self.decoder(emb, self.readout_func(emb), emb_negs)
        return emb.reshape(-1, self.dim), loss, self.metric_name, metric


class GraphAutoEncoder(BaseGraphAutoEncoder):
    def __init__(self, node_encoder, dims, fanouts, metapath, feature_idx, feature_dim, node_type, edge_type, max_id,
                 num_negs=5):
        super().__init__(node_type, edge_type, max_id, num_negs)
        if node_encoder == "gcn":
            self.gnn = FeatureGNN("gcn", "full", dims, None, metapath, feature_idx, feature_dim)
        else:
            self.gnn = FeatureGNN("sage", "sage", dims, fanouts, metapath, feature_idx, feature_dim, max_id=max_id)
        self.dim = dims[-1]

    def embed(self, n_id):
        return _embed3(self.gnn, n_id, self.dim)

    def forward(self, inputs):
        emb, loss, name, metric = super().forward(inputs)
        return emb.reshape(-1, self.dim), loss, name, metric


class VariationalGraphAutoEncoder(BaseGraphAutoEncoder):
    def __init__(self, radius, node_encoder, dims, fanouts, metapath, feature_idx, feature_dim, node_type,
                 edge_type, max_id, num_negs=5, train=True):
        super().__init__(node_type, edge_type, max_id, num_negs)
        self.log_var_encoder = encoders.ShallowEncoder(dim=dims[-1], feature_idx=-1, max_id=max_id, combiner="add")
        if node_encoder == "gcn":
            self.gnn = FeatureGNN("gcn", "full", dims, None, metapath, feature_idx, feature_dim)
        else:
            self.gnn = FeatureGNN("sage", "sage", dims, fanouts, metapath, feature_idx, feature_dim, max_id=max_id)
        self.dim, self.radius = dims[-1], radius

    @staticmethod
    def kl(mu, log_var):
        return (-0.5 * (log_var - torch.exp(log_var) - mu.pow(2) + 1)).reshape(-1)

    def embed(self, n_id):
        n_id = torch.as_tensor(n_id)
        b = n_id.shape[0]
        flat = n_id.reshape(-1)
        mu = self.gnn(flat)
        log_var = self.log_var_encoder(flat)
        if self.training:
            emb = mu + self.radius * torch.randn_like(log_var) * torch.exp(0.5 * log_var)
        else:
            emb = mu
        return mu, log_var, emb.reshape(b, -1, self.dim)

    def forward(self, inputs):
        src, pos, negs = self.to_sample(inputs)
        mu, lv, emb = self.embed(src)
        mu_p, lv_p, emb_p = self.embed(pos)
        mu_n, lv_n, emb_n = self.embed(negs)
        logits = torch.matmul(emb, emb_p.transpose(1, 2)).float()
        neg_logits = torch.matmul(emb, emb_n.transpose(1, 2)).float()
        t = F.binary_cross_entropy_with_logits(logits, torch.ones_like(logits), reduction="sum")
        n = F.binary_cross_entropy_with_logits(neg_logits, torch.zeros_like(neg_logits), reduction="sum")
        loss = (t + n) / float(logits.numel() + neg_logits.numel())
        loss = loss + torch.cat([self.kl(mu, lv), self.kl(mu_p, lv_p), self.kl(mu_n, lv_n)]).float().mean()
        pred = torch.cat([torch.sigmoid(logits), torch.sigmoid(neg_logits)], 2).detach().cpu()
        lab = torch.cat([torch.ones_like(logits), torch.zeros_like(neg_logits)], 2).cpu()
        acc = self.metric(lab, pred)
        mu_out = self.gnn(torch.as_tensor(inputs).reshape(-1))
        return mu_out, loss, "acc", acc


class _RGCNNet(BaseGNNNet):
    """RelationConv stack over id embeddings; edge relations from the dense edge
    feature ``feature_idx`` (rgcn.py:30-78)."""

    def __init__(self, dims, metapath, rel_num, node_max_id, feature_idx, feature_dim, embedding_dim):
        self._fea_dim = embedding_dim
        self._rel_num = rel_num
        super().__init__("relation", "relation", dims, None, metapath, add_self_loops=False)
        self._encoder = encoders.ShallowEncoder(dim=embedding_dim, feature_idx=-1, max_id=node_max_id,
                                                embedding_dim=embedding_dim)
        self.feature_idx = feature_idx if isinstance(feature_idx, list) else [feature_idx]
        self.feature_dim = feature_dim if isinstance(feature_dim, list) else [feature_dim]

    def get_conv(self, conv_class, dim):
        conv = conv_class(self._fea_dim, dim, None, self._rel_num)
        self._fea_dim = dim
        return conv

    def to_x(self, n_id):
        return self._encoder(n_id)

    def to_edge(self, n_id_src, n_id_dst, e_id):
        edges = torch.stack([n_id_src.cpu(), n_id_dst.cpu(), e_id.cpu().long()], 1)
        rel = ge.get_edge_dense_feature(edges, self.feature_idx, self.feature_dim)[0]
        return rel.reshape(-1).long().to(n_id_src.device)


class UnsupervisedRGCN(UnsuperviseModel):
    def __init__(self, node_type, edge_type, max_id, dims, metapath, relation_num, feature_idx, feature_dim,
                 embedding_dim, num_negs=5, metric="mrr"):
        super().__init__(node_type, edge_type, max_id, num_negs, metric)
        self.dim = dims[-1]
        self.gnn = _RGCNNet(dims, metapath, relation_num, max_id, feature_idx, feature_dim, embedding_dim)

    def embed(self, n_id):
        n_id = torch.as_tensor(n_id)
        return self.gnn(n_id.reshape(-1)).reshape(*n_id.shape, self.dim)

    def embed_context(self, n_id):
        return self.embed(n_id)
