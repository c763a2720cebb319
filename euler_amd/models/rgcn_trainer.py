"""Device-path training of the estimator's ``UnsupervisedRGCN`` (``models/unsupervised.py``)
under ``NodeEstimator(device_graph=True)``.

Reference: ``examples/rgcn/rgcn.py:30-105`` (RelationConv stack over id embeddings,
``RelationDataFlow`` full neighbourhoods, the edge relation read from a dense edge
feature, the unsupervised positive / negative objective of ``mp_utils/base.py:50-91``).

On the device: the relation of every stored edge is read from the engine once (one
``get_edge_dense_feature`` over the CSR) and kept in HBM; a step draws the roots, one
weighted neighbour per root and the negatives, builds the blocks of all of them with
:class:`~euler_amd.dataflow.device_flow.DeviceRelationFlow` (relations as the blocks'
``e_id``), and runs the model's own id embedding, relation weights and ``fc``.  The
relation transform on the padded blocks is transform-then-gather: one GEMM gives every
source row under every relation (``[S, R * dim]``, small R), each edge gathers its
(source, relation) row (``-1`` padding reads zeros), a segment mean per target — no
relation-sorted tiles, which need the edge count on the host.  Several steps per hipGraph.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from euler_amd.dataflow.device_flow import DeviceRelationFlow
from euler_amd.models.captured import CapturedTrainer, RowSparseTableMixin
from euler_amd.ops import gnn_ops, mp_ops

__all__ = ["UnsupRgcnTrainer", "RowSparseRgcnTrainer", "edge_relations"]


def edge_relations(graph, feature_idx, feature_dim):
    """the dense edge feature (first column, as ``_RGCNNet.to_edge``) of every CSR position
    of ``graph`` (built with ``DeviceGraph.from_engine``), read from the engine once"""
    import euler_amd.ops.graph_api as ge

    T = graph.num_types
    indptr = graph.indptr.cpu().numpy()
    nbr = graph.nbr.cpu().numpy().astype(np.int64)
    ids = np.asarray(graph.ids).astype(np.int64) if graph.ids is not None else np.arange(graph.num_rows)
    seg = np.repeat(np.arange(indptr.size - 1), np.diff(indptr))
    edges = np.stack([ids[seg // T], ids[nbr], seg % T], 1)
    if edges.shape[0] == 0:
        return torch.zeros(0, dtype=torch.long)
    rel = ge.get_edge_dense_feature(torch.as_tensor(edges), feature_idx, feature_dim)[0]
    return torch.as_tensor(np.asarray(rel)).reshape(edges.shape[0], -1)[:, 0].long()


class UnsupRgcnTrainer(CapturedTrainer):
    metric_name = "mrr"

    def __init__(self, model, graph, batch_size, optimizer="adam", learning_rate=0.01):
        import euler_amd.ops.graph_api as ge

        gnn = model.gnn
        self.graph, self.gnn = graph, gnn
        self.B, self.K = int(batch_size), int(model.num_negs)
        et = model.edge_type
        self.types = None if et in (None, -1, "-1") else \
            [int(t) for t in np.asarray(ge.get_edge_type_id(et)).reshape(-1)]
        masks = []
        for m in gnn.sampler.metapath:
            tids = None if m is None else [int(t) for t in np.asarray(ge.get_edge_type_id(m)).reshape(-1)]
            masks.append(graph._mask(None if tids is None or any(t < 0 for t in tids) else tids))
        rel = edge_relations(graph, gnn.feature_idx, gnn.feature_dim)
        self.flow = DeviceRelationFlow(graph, masks, self.B * (2 + self.K), rel)
        ids = graph.ids if graph.ids is not None else np.arange(graph.num_rows)
        self._ids = torch.as_tensor(np.asarray(ids).astype(np.int64), device=graph.device)
        self._pad_id = int(model.max_id) + 1
        self.mrr = torch.zeros(2, dtype=torch.float64, device=graph.device)
        super().__init__(model, graph, graph.device, optimizer, learning_rate)

    def _node_ids(self, rows):
        return torch.where(rows >= 0, self._ids[rows.clamp(min=0)], torch.full_like(rows, self._pad_id))

    @staticmethod
    def _relation_conv(conv, x_t, x, edge_index, rel, size):
        """RelationConv.forward on a padded block: fc(x_t) + mean_e W[rel_e] x[src_e]"""
        W = conv.relation_matrices()                               # [R, D, K]
        R, D, K = W.shape
        xw = (x.float() @ W.reshape(R * D, K).t().float()).reshape(-1, D)   # row s * R + r
        src, dst = edge_index[1], edge_index[0]
        ok = (src >= 0) & (rel >= 0) & (rel < R)
        idx = torch.where(ok, src * R + rel, torch.full_like(src, -1))
        dst = torch.where(ok, dst, torch.full_like(dst, -1))
        agg = mp_ops.scatter_mean(mp_ops.gather(xw, idx), dst, int(size[0]))
        return conv.fc(x_t) + agg.to(x_t.dtype)

    def _embed(self, rows):
        df = self.flow.produce(rows)
        x = self.gnn.to_x(self._node_ids(df[0].n_id)).float()
        for conv, block in zip(self.gnn.convs, df):
            x_t = mp_ops.gather(x, block.res_n_id)
            x = F.relu(self._relation_conv(conv, x_t, x, block.edge_index, block.e_id, block.size))
        return self.gnn.fc(x)

    def _materialize(self):
        if not any(isinstance(p, torch.nn.parameter.UninitializedParameter) for p in self.model.parameters()):
            return
        state = self.graph.rng.clone()
        with torch.no_grad():
            self._embed(torch.zeros(self.B * (2 + self.K), dtype=torch.long, device=self._ids.device))
        self.graph.rng.copy_(state)

    def _forward_loss(self):
        self._draw()
        g, B, K = self.graph, self.B, self.K
        src = g.sample_node(B, stream_id=1).long()
        pos = g.sample_neighbor(src, 1, edge_types=self.types, default=-1, stream_id=4).long().reshape(-1)
        neg = g.sample_node(B * K, stream_id=5).long()
        emb = self._embed(torch.cat([src, pos, neg]))
        d = emb.shape[-1]
        loss, logits, neg_logits = gnn_ops.sgns_loss(emb[:B].reshape(B, d), emb[B:2 * B].view(B, 1, d),
                                                     emb[2 * B:].view(B, K, d))
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


class _RowsAt(torch.nn.Module):
    """Stand-in for the id embedding during a row-sparse step: returns the rows of the
    step's gathered leaf at the positions the step computed for the one id tensor the
    encoder embeds (the block's node set)."""

    def __init__(self, num, dim):
        super().__init__()
        self.num, self.dim = int(num), int(dim)
        self.rows = self.p = None

    def forward(self, ids):
        if self.p is None or ids.numel() != self.p.numel():
            raise RuntimeError("row-sparse R-GCN step: unexpected id lookup")
        return self.rows[self.p].reshape(*ids.shape, self.dim)


class RowSparseRgcnTrainer(RowSparseTableMixin, UnsupRgcnTrainer):
    """UnsupRgcnTrainer with the id embedding table row-sharded and row-sparse
    (:class:`~euler_amd.parallel.sparse_table.ShardedTable`): per step the blocks' node set
    (unique by construction, padding collapsed) is gathered from the table — from the
    owner ranks over one fixed-capacity all-to-all when world > 1 — runs through the
    encoder's own projection and the relation convolutions, and its row gradients go back
    to the owners' row-sparse optimizer.  The relation weights and ``fc`` stay in the flat
    buffer.  Per-step work is independent of |V| (reference examples/rgcn/rgcn.py:30-105,
    tf_euler/python/utils/embedding.py:24-68)."""

    def __init__(self, model, graph, batch_size, optimizer="adam", learning_rate=0.01, group=None):

        enc = model.gnn._encoder
        mod = getattr(enc, "embedding", None)
        if mod is None or not hasattr(mod, "num"):
            raise ValueError("RowSparseRgcnTrainer needs the encoder's id embedding")
        model.to(graph.device)
        self._adopt_table(model, mod, graph.device, group, optimizer, learning_rate)
        self._enc = enc
        enc.embedding = _RowsAt(mod.num, mod.dim)  # position lookups into the step's gathered rows
        self._pending = None
        super().__init__(model, graph, batch_size, optimizer, learning_rate)
        self.world = self.id_table.world

    def _swap_in(self):
        if not isinstance(self._enc.embedding, _RowsAt):
            self._enc.embedding = _RowsAt(self._mod.num, self._mod.dim)

    def _embed(self, rows):
        from euler_amd.ops.gnn_ops import unique_first_padded

        self._swap_in()
        t = self.id_table
        df = self.flow.produce(rows)
        ids = self._node_ids(df[0].n_id)
        ids = torch.where((ids < 0) | (ids >= t.num_rows), torch.full_like(ids, t.num_rows - 1), ids)
        uids, inv, _ = unique_first_padded(ids)
        tab_rows, h = t.lookup_static(uids, trash_row=True)
        leaf = tab_rows.detach().requires_grad_(torch.is_grad_enabled())
        stub = self._enc.embedding
        stub.rows, stub.p = leaf, h.pos[inv]
        self._pending = (h, leaf)
        x = self.gnn.to_x(ids).float()
        for conv, block in zip(self.gnn.convs, df):
            x_t = mp_ops.gather(x, block.res_n_id)
            x = F.relu(self._relation_conv(conv, x_t, x, block.edge_index, block.e_id, block.size))
        return self.gnn.fc(x)

    def _step(self, grad_sync=None):
        loss = self._forward_loss()
        self.opt.zero_grad()
        loss.backward()
        scale = 1.0
        if grad_sync is not None:
            s = grad_sync(self.flat.grad)
            scale = 1.0 if s is None else float(s)
        self.opt.step(scale)
        h, leaf = self._pending
        g = leaf.grad if leaf.grad is not None else torch.zeros_like(leaf)
        n = g.shape[0] - 1
        self.id_table.apply_static(h, g[:n] / self.world if self.world > 1 else g[:n])
        stub = self._enc.embedding
        stub.rows = stub.p = None
        self._pending = None
        self.loss_out.copy_(loss.detach())
        return self.loss_out

    # ------------------------------------------------------------------ state
    def finish(self):
        """the encoder's own id embedding back in place, holding the trained table"""
        self._enc.embedding = self._mod
        RowSparseTableMixin.finish(self)
