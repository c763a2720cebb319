"""Device-path training of first-order LINE (one id table for both roles) under
``NodeEstimator(device_graph=True)``.

Reference: ``examples/line/line.py:27-71`` (order 1: ``context_encoder = target_encoder``)
through ``tf_euler/python/mp_utils/base.py:50-91`` (positive = one weighted neighbour of
each root, ``num_negs`` negatives from ``sample_node``, sigmoid cross-entropy, MRR).

Second-order LINE (separate context table) runs on the row-sparse SGNS path
(:class:`~euler_amd.models.deepwalk_step.DeepWalkEstimatorTrainer`).  With one shared
table a row can be a target and a context in the same step, which that in-place update
does not allow; here the step is the model's own embedding lookups, the fused
``sgns_loss`` kernel, autograd and the flat optimizer, captured several steps per hipGraph
(:class:`~euler_amd.models.captured.CapturedTrainer`).
"""
from __future__ import annotations

import numpy as np
import torch

from euler_amd.models.captured import CapturedTrainer
from euler_amd.ops import gnn_ops

__all__ = ["IdPairTrainer"]


class IdPairTrainer(CapturedTrainer):
    metric_name = "mrr"

    def __init__(self, model, graph, batch_size, optimizer="adam", learning_rate=0.01):
        import euler_amd.ops.graph_api as ge

        for e in (getattr(model, "_target_encoder", None), getattr(model, "_context_encoder", None)):
            if e is None or not getattr(e, "use_id", False) or getattr(e, "use_feature", True) or \
                    getattr(e, "use_sparse_feature", True):
                raise ValueError("IdPairTrainer trains pure id embeddings (no dense / sparse features)")
        self.graph = graph
        self.B, self.K = int(batch_size), int(model.num_negs)
        et = model.edge_type
        self.types = None if et in (None, -1, "-1") else \
            [int(t) for t in np.asarray(ge.get_edge_type_id(et)).reshape(-1)]
        ids = graph.ids if graph.ids is not None else np.arange(graph.num_rows)
        self._ids = torch.as_tensor(np.asarray(ids).astype(np.int64), device=graph.device)
        self._pad_id = int(model.max_id) + 1
        self.mrr = torch.zeros(2, dtype=torch.float64, device=graph.device)  # sum, count
        super().__init__(model, graph, graph.device, optimizer, learning_rate)

    def _node_ids(self, rows):
        return torch.where(rows >= 0, self._ids[rows.clamp(min=0)], torch.full_like(rows, self._pad_id))

    def _forward_loss(self):
        self._draw()
        g, B, K = self.graph, self.B, self.K
        src = g.sample_node(B, stream_id=1).long()
        pos = g.sample_neighbor(src, 1, edge_types=self.types, default=-1, stream_id=4).long().reshape(-1)
        neg = g.sample_node(B * K, stream_id=5).long()
        m = self.model
        emb = m.embed(self._node_ids(src)).reshape(B, -1)
        emb_pos = m.embed_context(self._node_ids(pos)).reshape(B, 1, -1)
        emb_neg = m.embed_context(self._node_ids(neg)).reshape(B, K, -1)
        loss, logits, neg_logits = gnn_ops.sgns_loss(emb, emb_pos, emb_neg)
        with torch.no_grad():
            lp, ln = logits.float().view(B, 1), neg_logits.float().view(B, K)
            rank = 1.0 + (ln >= lp).sum(-1).double()
            self.mrr += torch.stack([(1.0 / rank).sum(), torch.full_like(rank[0], float(B))])
        self._samples = (src, pos, neg)
        return loss

    def metric(self) -> float:
        s, n = self.mrr.tolist()
        return s / max(n, 1.0)

    def reset_metric(self):
        self.mrr.zero_()
