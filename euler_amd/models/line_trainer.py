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

from euler_amd.models.captured import CapturedTrainer, RowSparseTableMixin
from euler_amd.ops import gnn_ops

__all__ = ["IdPairTrainer", "RowSparseIdPairTrainer"]


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


def _id_table_module(enc):
    """the id embedding module of a pure-id encoder (ShallowEncoder with only ids, or the
    sharded IdEncoder), else None"""
    table = getattr(enc, "table", None)
    if table is not None:
        return table  # IdEncoder(sharded=True): a ShardedEmbedding
    inner = getattr(enc, "enc", None)
    if inner is not None:
        enc = inner
    if getattr(enc, "use_id", False) and not getattr(enc, "use_feature", True) and \
            not getattr(enc, "use_sparse_feature", True) and getattr(enc, "combiner", "add") == "add" and \
            not hasattr(enc, "dense"):
        return getattr(enc, "embedding", None)
    return None


class RowSparseIdPairTrainer(RowSparseTableMixin, IdPairTrainer):
    """First-order LINE with its one id table row-sharded and row-sparse
    (:class:`~euler_amd.parallel.sparse_table.ShardedTable`): per step the batch's source,
    positive and negative ids are de-duplicated on the device, their rows gathered (from
    the owner ranks over one fixed-capacity all-to-all when world > 1), the fused
    ``sgns_loss`` runs on the gathered rows, and the row gradients go back to the owners'
    row-sparse Adam / Adagrad / SGD.  Per-step work is independent of |V|; a row that is a
    target and a context in one step gets one merged gradient (the shared-table case the
    in-place SGNS update cannot take).  Table ownership and per-rank shard checkpoints:
    :class:`~euler_amd.models.captured.RowSparseTableMixin`.  Reference:
    examples/line/line.py:27-71, tf_euler/python/utils/embedding.py:24-68."""

    def __init__(self, model, graph, batch_size, optimizer="adam", learning_rate=0.01, group=None):
        import euler_amd.ops.graph_api as ge

        mod = _id_table_module(getattr(model, "_target_encoder", None))
        if mod is None or model._context_encoder is not model._target_encoder:
            raise ValueError("RowSparseIdPairTrainer trains first-order LINE over one pure id table")
        self.graph = graph
        self.B, self.K = int(batch_size), int(model.num_negs)
        et = model.edge_type
        self.types = None if et in (None, -1, "-1") else \
            [int(t) for t in np.asarray(ge.get_edge_type_id(et)).reshape(-1)]
        ids = graph.ids if graph.ids is not None else np.arange(graph.num_rows)
        self._ids = torch.as_tensor(np.asarray(ids).astype(np.int64), device=graph.device)
        self._pad_id = int(model.max_id) + 1
        self.mrr = torch.zeros(2, dtype=torch.float64, device=graph.device)
        model.to(graph.device)
        self._adopt_table(model, mod, graph.device, group, optimizer, learning_rate)
        CapturedTrainer.__init__(self, model, graph, graph.device, optimizer, learning_rate)
        self.world = self.id_table.world

    def _step(self, grad_sync=None):
        from euler_amd.ops.gnn_ops import unique_first_padded

        self._draw()
        g, B, K = self.graph, self.B, self.K
        src = g.sample_node(B, stream_id=1).long()
        pos = g.sample_neighbor(src, 1, edge_types=self.types, default=-1, stream_id=4).long().reshape(-1)
        neg = g.sample_node(B * K, stream_id=5).long()
        t = self.id_table
        ids = self._node_ids(torch.cat([src, pos, neg]))
        ids = torch.where((ids < 0) | (ids >= t.num_rows), torch.full_like(ids, t.num_rows - 1), ids)
        uids, inv, _ = unique_first_padded(ids)
        rows, h = t.lookup_static(uids, trash_row=True)
        leaf = rows.detach().requires_grad_(True)
        p = h.pos[inv]
        emb = leaf[p[:B]]
        emb_pos = leaf[p[B: 2 * B]].view(B, 1, -1)
        emb_neg = leaf[p[2 * B:]].view(B, K, -1)
        loss, logits, neg_logits = gnn_ops.sgns_loss(emb, emb_pos, emb_neg)
        self.opt.zero_grad()
        loss.backward()
        with torch.no_grad():
            lp, ln = logits.float().view(B, 1), neg_logits.float().view(B, K)
            rank = 1.0 + (ln >= lp).sum(-1).double()
            self.mrr += torch.stack([(1.0 / rank).sum(), torch.full_like(rank[0], float(B))])
        scale = 1.0
        if grad_sync is not None and self.flat.flat.numel():
            s = grad_sync(self.flat.grad)
            scale = 1.0 if s is None else float(s)
        self.opt.step(scale)
        gr = leaf.grad if leaf.grad is not None else torch.zeros_like(leaf)
        n = gr.shape[0] - 1
        t.apply_static(h, gr[:n] / self.world if self.world > 1 else gr[:n])
        self._samples = (src, pos, neg)
        self.loss_out.copy_(loss.detach())
        return self.loss_out

