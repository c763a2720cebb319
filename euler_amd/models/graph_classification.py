"""Graph-classification models (reference ``examples/{gin,gated_graph,graphgcn,set2set}``,
SURVEY §2.6).  Node inputs are sparse-feature embedding bags; a conv stack over the
induced ("full") subgraph of every batch of graphs is followed by graph pooling
(segment-reduce kernels on the GPU).  Used with :class:`~euler_amd.estimator.GraphEstimator`.
"""
from __future__ import annotations

import torch

import euler_amd.ops.graph_api as ge
from euler_amd.graph_pool import AttentionPool, Pooling, Set2SetPool
from euler_amd.mp_utils.models import BaseGNNNet, GraphModel
from euler_amd.utils.layers import SparseEmbedding

__all__ = ["SparseFeatureGNN", "GIN", "GatedGraph", "GraphGCN", "Set2SetModel"]


class SparseFeatureGNN(BaseGNNNet):
    def __init__(self, conv, flow, dims, fanouts, metapath, feature_idx, feature_max_id, conv_kwargs=None,
                 add_self_loops=False):
        self._conv_kwargs = dict(conv_kwargs or {})
        super().__init__(conv, flow, dims, fanouts, metapath, add_self_loops=add_self_loops)
        self.feature_idx = feature_idx if isinstance(feature_idx, list) else [feature_idx]
        self.encoder = SparseEmbedding(feature_max_id, dims[0])

    def get_conv(self, conv_class, dim):
        return conv_class(dim, **self._conv_kwargs)

    def to_x(self, n_id):
        sp = ge.get_sparse_feature(n_id.cpu() if torch.is_tensor(n_id) else n_id, self.feature_idx)[0]
        return self.encoder(sp)


class _PooledGraphModel(GraphModel):
    def embed(self, n_id, graph_index):
        node_emb = self.gnn(torch.as_tensor(n_id))
        gi = torch.as_tensor(graph_index, device=node_emb.device).long()
        return self.pool(node_emb, gi)


class GIN(_PooledGraphModel):
    def __init__(self, dims, metapath, label_dim, feature_idx, feature_max_id, mlp=None, eps=0.0, train_eps=False):
        super().__init__(label_dim)
        self.gnn = SparseFeatureGNN("gin", "full", dims, None, metapath, feature_idx, feature_max_id,
                                    conv_kwargs={"mlp": mlp, "eps": eps, "train_eps": train_eps})
        self.pool = Pooling("add")


class GatedGraph(_PooledGraphModel):
    def __init__(self, dims, metapath, label_dim, feature_idx, feature_max_id, processing_steps=4, lstm_layers=2):
        super().__init__(label_dim)
        self.gnn = SparseFeatureGNN("gated", "full", dims, None, metapath, feature_idx, feature_max_id,
                                    conv_kwargs={"processing_steps": processing_steps, "lstm_layers": lstm_layers})
        self.pool = AttentionPool()


class GraphGCN(_PooledGraphModel):
    def __init__(self, dims, metapath, label_dim, feature_idx, feature_max_id):
        super().__init__(label_dim)
        # the reference's GraphGCN flow adds self loops (examples/graphgcn/graphgcn.py:32), the
        # other graph models' flows do not
        self.gnn = SparseFeatureGNN("graphgcn", "full", dims, None, metapath, feature_idx, feature_max_id,
                                    add_self_loops=True)
        self.pool = Pooling("add")


class Set2SetModel(_PooledGraphModel):
    def __init__(self, dims, metapath, label_dim, feature_idx, feature_max_id, processing_steps=4, lstm_layers=2):
        super().__init__(label_dim)
        self.gnn = SparseFeatureGNN("sage", "full", dims, None, metapath, feature_idx, feature_max_id)
        self.pool = Set2SetPool(dims[-1], processing_steps=processing_steps, num_layers=lstm_layers)
