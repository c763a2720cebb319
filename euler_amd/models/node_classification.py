"""Supervised node-classification model zoo (reference ``examples/*``).

Every model is a :class:`~euler_amd.mp_utils.models.SuperviseModel` returning
``(embedding, loss, metric_name, metric)``; the message passing runs on the gfx950
gather / segment-reduce / edge-softmax kernels when the model is on the GPU.

=============  ======================================  =====================================
model          conv + dataflow / encoder               reference
=============  ======================================  =====================================
GraphSAGE      SAGEConv + SageDataFlow                 examples/graphsage/graphsage.py:56-67
GCN            GCNConv + full                          examples/gcn/gcn.py:52-58
GAT            MultiHeadGATConv + full                 examples/gat/gat.py:27-86
FastGCN        GCNConv + FastGCNDataFlow               examples/fastgcn/fastgcn.py:51-57
AdaptiveGCN    GCNConv + LayerwiseDataFlow             examples/adaptivegcn/adaptivegcn.py:51-57
AGNN           AGNNConv + full                         examples/agnn/agnn.py:58
APPNP          APPNPConv(K, alpha) + full              examples/appnp/appnp.py:69
ARMA           ARMAConv(K, T) + full                   examples/arma/arma.py:67
DNA            DNAConv(heads, groups) + full           examples/dna/dna.py:66
SGCN           SGCNConv(K) + full                      examples/sgcn/sgcn.py:63
TAGCN          TAGConv(K) + full                       examples/tagcn/tagcn.py:63
GeniePath      GenieEncoder                            examples/geniepath/geniepath.py:26-49
LGCN           LGCEncoder                              examples/lgcn/lgcn.py:26-37
=============  ======================================  =====================================
"""
from __future__ import annotations

import torch

import euler_amd.ops.graph_api as ge
from euler_amd.convolution import convs as C
from euler_amd.mp_utils.models import BaseGNNNet, SuperviseModel
from euler_amd.utils import encoders

__all__ = ["FeatureGNN", "SupervisedGraphSage", "SupervisedGCN", "GAT", "FastGCN", "AdaptiveGCN", "AGNN", "APPNP",
           "ARMA", "DNA", "SGCN", "TAGCN", "GeniePath", "LGCN", "SupervisedGNN", "ScalableSage", "ScalableGCN"]


def _lst(x):
    return list(x) if isinstance(x, (list, tuple)) else [x]


class FeatureGNN(BaseGNNNet):
    """BaseGNNNet whose node inputs are dense features; ``conv_kwargs`` go to every conv."""

    def __init__(self, conv, flow, dims, fanouts, metapath, feature_idx, feature_dim, add_self_loops=False,
                 max_id=-1, conv_kwargs=None, **kwargs):
        self._conv_kwargs = dict(conv_kwargs or {})
        super().__init__(conv, flow, dims, fanouts, metapath, add_self_loops=add_self_loops, max_id=max_id)
        self.feature_idx, self.feature_dim = _lst(feature_idx), _lst(feature_dim)

    def get_conv(self, conv_class, dim):
        return conv_class(dim, **self._conv_kwargs)

    def to_x(self, n_id):
        return torch.cat(ge.get_dense_feature(n_id, self.feature_idx, self.feature_dim), -1)


class SupervisedGNN(SuperviseModel):
    """Generic ``conv + flow`` supervised model."""

    def __init__(self, conv, flow, dims, fanouts, metapath, feature_idx, feature_dim, label_idx, label_dim,
                 max_id=-1, metric_name="f1", conv_kwargs=None, add_self_loops=False):
        super().__init__(label_idx, label_dim, metric_name)
        self.gnn = FeatureGNN(conv, flow, dims, fanouts, metapath, feature_idx, feature_dim,
                              add_self_loops=add_self_loops, max_id=max_id, conv_kwargs=conv_kwargs)

    def embed(self, n_id):
        return self.gnn(n_id)

    def prepare_embed(self, n_id):
        return self.gnn.sample_inputs(n_id)


class SupervisedGraphSage(SupervisedGNN):
    def __init__(self, dims, fanouts, metapath, feature_idx, feature_dim, label_idx, label_dim, max_id=-1,
                 metric_name="f1"):
        super().__init__("sage", "sage", dims, fanouts, metapath, feature_idx, feature_dim, label_idx, label_dim,
                         max_id, metric_name)


class SupervisedGCN(SupervisedGNN):
    def __init__(self, dims, metapath, feature_idx, feature_dim, label_idx, label_dim, metric_name="f1"):
        super().__init__("gcn", "full", dims, None, metapath, feature_idx, feature_dim, label_idx, label_dim,
                         metric_name=metric_name)


class GAT(SupervisedGNN):
    def __init__(self, dims, metapath, feature_idx, feature_dim, label_idx, label_dim, head_num=1, concat=True,
                 improved=False, metric_name="f1"):
        super().__init__(C.MultiHeadGATConv, "full", dims, None, metapath, feature_idx, feature_dim, label_idx,
                         label_dim, metric_name=metric_name,
                         conv_kwargs={"heads": head_num, "concat": concat, "improved": improved})


class FastGCN(SupervisedGNN):
    def __init__(self, dims, fanouts, metapath, feature_idx, feature_dim, label_idx, label_dim, metric_name="f1"):
        super().__init__("gcn", "fast", dims, fanouts, metapath, feature_idx, feature_dim, label_idx, label_dim,
                         metric_name=metric_name)


class AdaptiveGCN(SupervisedGNN):
    def __init__(self, dims, fanouts, metapath, feature_idx, feature_dim, label_idx, label_dim, metric_name="f1"):
        super().__init__("gcn", "adapt", dims, fanouts, metapath, feature_idx, feature_dim, label_idx, label_dim,
                         metric_name=metric_name)


class AGNN(SupervisedGNN):
    def __init__(self, metric, dims, metapath, feature_idx, feature_dim, label_idx, label_dim):
        super().__init__("agnn", "full", dims, None, metapath, feature_idx, feature_dim, label_idx, label_dim,
                         metric_name=metric)


class APPNP(SupervisedGNN):
    def __init__(self, dims, metapath, feature_idx, feature_dim, label_idx, label_dim, K=10, alpha=0.1,
                 metric_name="f1"):
        super().__init__("appnp", "full", dims, None, metapath, feature_idx, feature_dim, label_idx, label_dim,
                         metric_name=metric_name, conv_kwargs={"K": K, "alpha": alpha})


class ARMA(SupervisedGNN):
    def __init__(self, dims, metapath, feature_idx, feature_dim, label_idx, label_dim, K=1, num_layers=1,
                 metric_name="f1"):
        super().__init__("arma", "full", dims, None, metapath, feature_idx, feature_dim, label_idx, label_dim,
                         metric_name=metric_name, conv_kwargs={"K": K, "num_layers": num_layers})


class DNA(SupervisedGNN):
    def __init__(self, dims, metapath, feature_idx, feature_dim, label_idx, label_dim, head_num=1, group_num=1,
                 metric_name="f1"):
        super().__init__("dna", "full", dims, None, metapath, feature_idx, feature_dim, label_idx, label_dim,
                         metric_name=metric_name, conv_kwargs={"heads": head_num, "groups": group_num})


class SGCN(SupervisedGNN):
    def __init__(self, dims, metapath, feature_idx, feature_dim, label_idx, label_dim, K=1, metric_name="f1"):
        super().__init__("sgcn", "full", dims, None, metapath, feature_idx, feature_dim, label_idx, label_dim,
                         metric_name=metric_name, conv_kwargs={"K": K})


class TAGCN(SupervisedGNN):
    def __init__(self, dims, metapath, feature_idx, feature_dim, label_idx, label_dim, K=3, metric_name="f1"):
        super().__init__("tag", "full", dims, None, metapath, feature_idx, feature_dim, label_idx, label_dim,
                         metric_name=metric_name, conv_kwargs={"K": K})


class GeniePath(SuperviseModel):
    def __init__(self, dim, metapath, label_idx, label_dim, max_id=-1, feature_idx=-1, feature_dim=0, use_id=False,
                 sparse_feature_idx=-1, sparse_feature_max_id=-1, embedding_dim=16, use_hash_embedding=False,
                 use_residual=False, head_num=4, metric_name="f1"):
        super().__init__(label_idx, label_dim, metric_name)
        self._encoder = encoders.GenieEncoder(
            metapath, dim, "attention", feature_idx=feature_idx, feature_dim=feature_dim, max_id=max_id,
            use_id=use_id, sparse_feature_idx=sparse_feature_idx, sparse_feature_max_id=sparse_feature_max_id,
            embedding_dim=embedding_dim, use_hash_embedding=use_hash_embedding, use_residual=use_residual,
            head_num=head_num)

    def embed(self, n_id):
        return self._encoder(n_id)


class LGCN(SuperviseModel):
    def __init__(self, dim, metapath, label_idx, label_dim, feature_idx=-1, feature_dim=0, k=3, nb_num=10,
                 out_dim=64, metric_name="f1"):
        super().__init__(label_idx, label_dim, metric_name)
        self._encoder = encoders.LGCEncoder(metapath, feature_idx, feature_dim, k, dim, nb_num, out_dim)

    def embed(self, n_id):
        return self._encoder(n_id)


class ScalableSage(SuperviseModel):
    """Supervised node classification over ``ScalableSageEncoder`` (reference
    tf_euler/python/utils/encoders.py:629-748): one sampled hop per step, deeper layers from
    per-layer stores of stale embeddings (device path: models/scalable_trainer.py)."""

    def __init__(self, edge_type, fanout, num_layers, dim, label_idx, label_dim, feature_idx, feature_dim, max_id,
                 aggregator="mean", store_learning_rate=0.001, metric_name="f1"):
        super().__init__(label_idx, label_dim, metric_name)
        self._encoder = encoders.ScalableSageEncoder(edge_type, fanout, num_layers, dim, aggregator=aggregator,
                                                     feature_idx=feature_idx, feature_dim=feature_dim, max_id=max_id,
                                                     store_learning_rate=store_learning_rate)

    def embed(self, n_id):
        return self._encoder(n_id)


class ScalableGCN(SuperviseModel):
    """Supervised node classification over ``ScalableGCNEncoder`` (reference
    tf_euler/python/utils/encoders.py:294-408): the roots' full 1-hop neighbourhood per step,
    deeper layers from stale-embedding stores."""

    def __init__(self, edge_type, num_layers, dim, label_idx, label_dim, feature_idx, feature_dim, max_id,
                 aggregator="mean", store_learning_rate=0.001, metric_name="f1"):
        super().__init__(label_idx, label_dim, metric_name)
        self._encoder = encoders.ScalableGCNEncoder(edge_type, num_layers, dim, aggregator=aggregator,
                                                    feature_idx=feature_idx, feature_dim=feature_dim, max_id=max_id,
                                                    store_learning_rate=store_learning_rate)

    def embed(self, n_id):
        return self._encoder(n_id)

