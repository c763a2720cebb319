"""Device-path training of the *encoder* models — GeniePath (``GenieEncoder``), any
``SuperviseModel`` whose ``_encoder`` is a ``GCNEncoder``, LGCN (``LGCEncoder``,
:class:`LgcnTrainer`) and ``SuperviseSolution`` over a ``SageEncoder``
(:class:`SolutionTrainer`) — under ``NodeEstimator(device_graph=True)``.

Reference: ``examples/geniepath/geniepath.py:26-49``, ``tf_euler/python/utils/
encoders.py:174-291`` (``get_multi_hop_neighbor`` node sets and sparse adjacencies, the
sparse aggregators, GeniePath's per-depth projections and LSTM).

The hop sets and adjacencies come from :class:`~euler_amd.dataflow.device_flow.
DeviceFullFlow` (no self loops): hop h+1's set is ``unique([neighbours, set h])`` — the
reference's neighbour set plus the previous set's nodes, which have no adjacency entry
unless they are neighbours, so every root's aggregation is the reference's — padded with
``-1`` in fixed capacities; the adjacency of hop h is the block's (target, source) edge
list as a ``[cap_h, cap_h+1]`` SparseTensor whose padding entries are ``(-1, -1)``, which
the sparse aggregators drop (``utils/sparse_aggregators.py``).  The model's own
``encode`` (``utils/encoders.py``), ``out_fc``, loss and F1 counts then run as in
:class:`~euler_amd.models.full_trainer.FullFlowTrainer`, several steps per hipGraph.
"""
from __future__ import annotations

import numpy as np
import torch

from euler_amd.dataflow.device_flow import DeviceFullFlow
from euler_amd.models.full_trainer import FullFlowTrainer
from euler_amd.ops import mp_ops

__all__ = ["EncoderFlowTrainer", "LgcnTrainer", "SolutionTrainer"]


class EncoderFlowTrainer(FullFlowTrainer):
    @classmethod
    def from_model(cls, model, graph, batch_size, optimizer="adam", learning_rate=0.01, **kw):
        import euler_amd.ops.graph_api as ge
        from euler_amd.utils.encoders import GCNEncoder

        enc = getattr(model, "_encoder", None)
        ne = getattr(enc, "_node_encoder", None)
        if not isinstance(enc, GCNEncoder) or ne is None or ne.use_id or ne.use_sparse_feature or \
                not ne.use_feature:
            raise ValueError("EncoderFlowTrainer trains GCNEncoder / GenieEncoder models over dense features")
        masks = []
        for m in enc.metapath:
            ids = None if m is None else [int(t) for t in np.asarray(ge.get_edge_type_id(m)).reshape(-1)]
            masks.append(graph._mask(None if ids is None or any(t < 0 for t in ids) else ids))
        flow = DeviceFullFlow(graph, masks, int(batch_size), add_self_loops=False)
        tr = cls(model, graph, batch_size, masks, add_self_loops=False, optimizer=optimizer,
                 learning_rate=learning_rate, flow=flow, **kw)
        return tr

    def _node_features(self, rows):
        ne = self.model._encoder._node_encoder
        x = mp_ops.gather(self.features, rows.clamp(min=0)).float()
        x = x * (rows >= 0).unsqueeze(1).to(x.dtype)
        return ne.dense(x) if ne.combiner == "add" else x

    def _forward(self, roots):
        from euler_amd.ops.graph_api import SparseTensor

        df = self.flow.produce(roots)
        sets = [roots.reshape(-1).long()] + [b.n_id for b in df.blocks]
        hidden = [self._node_features(s) for s in sets]
        adjs = []
        for b in df.blocks:
            ei = b.edge_index
            adj = SparseTensor(ei.t(), torch.ones(ei.shape[1], device=ei.device), list(b.size))
            # the block's destination CSR is known from the expansion (mp_ops.cached_segment)
            n = int(b.size[0])
            adj._euler_idx = (ei[0], ei[1], n, mp_ops.cached_segment(ei, 0, n))
            adjs.append(adj)
        emb = self.model._encoder.encode(hidden, adjs)
        return self.model.out_fc(emb).float(), df


class LgcnTrainer(FullFlowTrainer):
    """LGCN (reference ``examples/lgcn/lgcn.py:26-37``, ``encoders.py:872-922``): ``nb_num``
    weighted neighbour draws per root on the HBM graph (Philox stream 6; a root without an
    out-edge draws ``-1``, whose features are zero like the engine's default node), node
    and neighbour features gathered in HBM, then the model's own top-k + 1-D convolutions
    (``LGCEncoder.encode``), ``out_fc``, loss and F1 counts; several steps per hipGraph."""

    @classmethod
    def from_model(cls, model, graph, batch_size, optimizer="adam", learning_rate=0.01, **kw):
        import euler_amd.ops.graph_api as ge
        from euler_amd.utils.encoders import LGCEncoder

        enc = getattr(model, "_encoder", None)
        if not isinstance(enc, LGCEncoder):
            raise ValueError("LgcnTrainer trains LGCN (LGCEncoder)")
        ids = [int(t) for t in np.asarray(ge.get_edge_type_id(enc.edge_type)).reshape(-1)]
        tr = cls.__new__(cls)
        tr.types = None if any(t < 0 for t in ids) else ids
        FullFlowTrainer.__init__(tr, model, graph, batch_size, [], add_self_loops=False, optimizer=optimizer,
                                 learning_rate=learning_rate, **kw)
        return tr

    def _forward(self, roots):
        enc = self.model._encoder
        roots = roots.reshape(-1).long()
        nbrs = self.graph.sample_neighbor(roots, enc.nb_num, edge_types=self.types, default=-1,
                                          stream_id=6).long().reshape(-1)

        def feats(rows):
            x = mp_ops.gather(self.features, rows.clamp(min=0)).float()
            return x * (rows >= 0).unsqueeze(1).to(x.dtype)

        nb_f = feats(nbrs).view(roots.numel(), enc.nb_num, -1)
        emb = enc.encode(feats(roots), nb_f)
        return self.model.out_fc(emb).float(), None


class SolutionTrainer(FullFlowTrainer):
    """``solution.SuperviseSolution`` (reference ``euler_estimator`` solution API,
    ``examples/solution/run_solution.py``) over a dense-feature ``SageEncoder``, labels from
    a dense feature (``GetLabelFromFea``), the default sigmoid loss: the fan-out tree drawn
    per hop on the HBM graph (Philox stream 4 + h; ``-1`` for a node without an out-edge,
    zero features like the engine's default node), features gathered once, the encoder's own
    aggregators (``SageEncoder._aggregate``), the solution's ``logit_fn``, the fused loss +
    F1 counts; several steps per hipGraph."""

    @classmethod
    def from_model(cls, model, graph, batch_size, optimizer="adam", learning_rate=0.01, **kw):
        import euler_amd.ops.graph_api as ge
        from euler_amd import solution as S
        from euler_amd.utils.encoders import SageEncoder

        enc = getattr(model, "encoder", None)
        ne = getattr(enc, "_node_encoder", None)
        if not isinstance(model, S.SuperviseSolution) or type(enc) is not SageEncoder or ne is None or \
                ne.use_id or ne.use_sparse_feature or not ne.use_feature or model.loss_fn is not S.sigmoid_loss or \
                not isinstance(model.get_label_fn, S.GetLabelFromFea):
            raise ValueError("SolutionTrainer trains SuperviseSolution(GetLabelFromFea, dense-feature SageEncoder, "
                             "logit_fn) with the default sigmoid loss")
        tr = cls.__new__(cls)
        tr.types = []
        for m in enc.metapath:
            ids = [int(t) for t in np.asarray(ge.get_edge_type_id(m)).reshape(-1)]
            tr.types.append(None if any(t < 0 for t in ids) else ids)
        FullFlowTrainer.__init__(tr, model, graph, batch_size, [], add_self_loops=False, optimizer=optimizer,
                                 learning_rate=learning_rate, **kw)
        return tr

    def _forward(self, roots):
        enc = self.model.encoder
        hops = [roots.reshape(-1).long()]
        for i, (f, et) in enumerate(zip(enc.fanouts, self.types)):
            hops.append(self.graph.sample_neighbor(hops[-1], int(f), edge_types=et, default=-1,
                                                   stream_id=4 + i).long().reshape(-1))
        hidden = []
        for rows in hops:
            x = mp_ops.gather(self.features, rows.clamp(min=0)).float()
            hidden.append(x * (rows >= 0).unsqueeze(1).to(x.dtype))
        emb = enc._aggregate(hidden)
        return self.model.logit_fn(emb).float(), None
