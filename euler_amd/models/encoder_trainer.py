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
from euler_amd.models.captured import CapturedTrainer
from euler_amd.models.full_trainer import FullFlowTrainer
from euler_amd.ops import mp_ops

__all__ = ["EncoderFlowTrainer", "LgcnTrainer", "SolutionTrainer", "UnsupSolutionTrainer"]


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


def _check_sage_encoder(enc):
    from euler_amd.utils.encoders import SageEncoder

    ne = getattr(enc, "_node_encoder", None)
    if type(enc) is not SageEncoder or ne is None or ne.use_id or ne.use_sparse_feature or not ne.use_feature:
        raise ValueError("the solution device paths take dense-feature SageEncoders")
    return ne


def _type_list(ge, et):
    ids = [int(t) for t in np.asarray(ge.get_edge_type_id(et)).reshape(-1)]
    return None if any(t < 0 for t in ids) else ids


def _sage_tree_encode(enc, graph, features, types, roots, stream_base):
    """SageEncoder.forward on the HBM graph: per-hop draws (Philox stream_base + h), one
    feature gather per hop, the encoder's aggregators"""
    hops = [roots.reshape(-1).long()]
    for i, (f, et) in enumerate(zip(enc.fanouts, types)):
        hops.append(graph.sample_neighbor(hops[-1], int(f), edge_types=et, default=-1,
                                          stream_id=stream_base + i).long().reshape(-1))
    hidden = []
    for rows in hops:
        x = mp_ops.gather(features, rows.clamp(min=0)).float()
        hidden.append(x * (rows >= 0).unsqueeze(1).to(x.dtype))
    return enc._aggregate(hidden)


class UnsupSolutionTrainer(CapturedTrainer):
    """``solution.UnsuperviseSolution`` (reference ``base_unsupervise.py:27-73``) with
    dense-feature ``SageEncoder`` target / context encoders, ``SamplePosWithTypes``
    positives and single-type ``SampleNegWithTypes`` negatives: roots, positives and
    negatives drawn on the HBM graph, both encoders' trees built there, the solution's own
    ``logit_fn`` and ``loss_fn``, MRR on the device; several steps per hipGraph."""

    metric_name = "mrr"

    def __init__(self, model, graph, batch_size, optimizer="adam", learning_rate=0.01):
        import copy

        import euler_amd.ops.graph_api as ge
        from euler_amd import solution as S

        ne = _check_sage_encoder(model.target_encoder)
        ne_c = _check_sage_encoder(model.context_encoder)
        pos_fn, neg_fn = model.pos_sample_fn, model.neg_sample_fn
        if not isinstance(pos_fn, S.SamplePosWithTypes) or not isinstance(neg_fn, S.SampleNegWithTypes) or \
                len(neg_fn.neg_type) != 1 or list(ne_c.feature_idx) != list(ne.feature_idx):
            raise ValueError("UnsupSolutionTrainer takes SamplePosWithTypes / single-type SampleNegWithTypes "
                             "samplers and encoders over the same dense features")
        if graph.features is None:
            raise ValueError("the device graph needs the encoders' dense features (DeviceGraph.from_engine)")
        self.graph, self.B = graph, int(batch_size)
        self.P, self.K = int(pos_fn.num_pos), int(neg_fn.num_negs)
        self.pos_types = _type_list(ge, pos_fn.edge_type)
        self.t_types = [_type_list(ge, m) for m in model.target_encoder.metapath]
        self.c_types = [_type_list(ge, m) for m in model.context_encoder.metapath]
        self.features = graph.features
        nt = neg_fn.neg_type[0]
        tid = -1 if nt in (None, -1, "-1") else int(np.asarray(ge.get_node_type_id(nt)).reshape(-1)[0])
        _, _, nw = ge.get_engine().export_nodes()
        self.neg_sampler = copy.copy(graph)
        self.neg_sampler.set_root_type(tid, node_weights=np.asarray(nw))
        self.mrr = torch.zeros(2, dtype=torch.float64, device=graph.device)
        super().__init__(model, graph, graph.device, optimizer, learning_rate)

    def _materialize(self):
        if not any(isinstance(p, torch.nn.parameter.UninitializedParameter) for p in self.model.parameters()):
            return
        state = self.graph.rng.clone()
        with torch.no_grad():
            self._logits(torch.zeros(self.B, dtype=torch.long, device=self.features.device))
        self.graph.rng.copy_(state)

    def _logits(self, src):
        m, g, B = self.model, self.graph, self.B
        pos = g.sample_neighbor(src, self.P, edge_types=self.pos_types, default=-1, stream_id=4).long().reshape(-1)
        neg = self.neg_sampler.sample_node(B * self.K, stream_id=5).long()
        emb = _sage_tree_encode(m.target_encoder, g, self.features, self.t_types, src, 10).view(B, 1, -1)
        ctx = _sage_tree_encode(m.context_encoder, g, self.features, self.c_types, torch.cat([pos, neg]), 20)
        d = ctx.shape[-1]
        self._samples = (src, pos, neg)
        return m.logit_fn(emb, ctx[: B * self.P].view(B, self.P, d), ctx[B * self.P:].view(B, self.K, d))

    def _forward_loss(self):
        self._draw()
        B = self.B
        logits, neg_logits = self._logits(self.graph.sample_node(B, stream_id=1).long())
        loss = self.model.loss_fn(logits, neg_logits)
        with torch.no_grad():
            lp = logits.float().reshape(B, -1)[:, :1]
            ln = neg_logits.float().reshape(B, -1)
            rank = 1.0 + (ln >= lp).sum(-1).double()
            self.mrr += torch.stack([(1.0 / rank).sum(), torch.full_like(rank[0], float(B))])
        return loss

    def metric(self) -> float:
        s, n = self.mrr.tolist()
        return s / max(n, 1.0)

    def reset_metric(self):
        self.mrr.zero_()
