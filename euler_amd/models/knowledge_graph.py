"""Knowledge-graph embedding models (reference ``examples/TransX/*.py``,
``examples/distmult/distmult.py``).

Data convention (the reference's, kept for compatibility): the edge *type* is the data
split and the relation id is the dense edge feature ``id``; training batches are
``sample_edge`` triples ``[n, 3] = (src, dst, edge_type)``.

The scoring of the positive and all corrupted triples is one batched tensor
expression over ``[B, 1 + 2*negs, dim]`` (no per-negative tiling copies); on the GPU
the entity rows come from the gfx950 gather kernel.  Returns
``([src_emb, rel_emb, dst_emb], loss, metric_name, metric)`` so ``EdgeEstimator``
can pick node_src / edge / node_dst embeddings.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

import euler_amd.ops.graph_api as ge
from euler_amd.ops import gnn_ops
from euler_amd.parallel.embedding import ShardedEmbedding
from euler_amd.utils import metrics as M
from euler_amd.utils.layers import Embedding

__all__ = ["TransX", "TransE", "TransH", "TransR", "TransD", "DistMult"]


class TransX(nn.Module):
    def __init__(self, node_type, edge_type, node_max_id, edge_max_id, ent_dim, rel_dim, num_negs=5, l1=True,
                 metric_name="mrr", corrupt="both", sharded=False, **kwargs):
        super().__init__()
        self.node_type, self.edge_type = node_type, edge_type
        self.node_max_id, self.edge_max_id = node_max_id, edge_max_id
        self.ent_dim, self.rel_dim = ent_dim, rel_dim
        self.num_negs, self.l1, self.metric_name, self.corrupt = num_negs, l1, metric_name, corrupt
        if metric_name not in ("mrr", "mr", "hit10"):
            raise ValueError("Metric name :{} not in list [mrr, mr, hit10]".format(metric_name))
        self.metric = M.get(metric_name)
        # the reference passes node_max_id + 1 to an Embedding that adds one more row
        self.entity_encoder = ShardedEmbedding(node_max_id + 1, ent_dim) if sharded else \
            Embedding(node_max_id + 1, ent_dim)
        self.relation_encoder = Embedding(edge_max_id + 1, rel_dim)

    def _dev(self):
        return self.relation_encoder.weight.device

    def generate_negative(self, batch_size):
        return ge.sample_node(batch_size * self.num_negs, self.node_type)

    def generate_triplets(self, inputs):
        inputs = torch.as_tensor(inputs)
        b = inputs.shape[0]
        rel = ge.get_edge_dense_feature(inputs, ["id"], [1])[0].reshape(b, 1).long()
        neg = torch.as_tensor(self.generate_negative(b)).reshape(b, self.num_negs)
        return inputs[:, 0:1], inputs[:, 1:2], neg, rel

    @staticmethod
    def norm_emb(x):
        return F.normalize(x, dim=-1)

    def calculate_scores(self, src, rel, dst):
        d = src + rel - dst
        return -(d.abs().sum(-1) if self.l1 else d.norm(dim=-1))

    def loss_fn(self, pos_scores, neg_scores):
        """margin ranking against the MEAN negative score (transE.py:49-65)."""
        return F.relu(self.margin + neg_scores.mean(-1, keepdim=True) - pos_scores).mean()

    def energy_scores(self, src, dst, neg, rel):
        """(positive scores [B, 1, 1], corrupted scores [B, 1, k]) of embedded triples"""
        pos = self.calculate_scores(src, rel, dst).reshape(-1, 1, 1)
        if self.corrupt == "front":
            neg_s = self.calculate_scores(neg, rel, dst)
        elif self.corrupt == "tail":
            neg_s = self.calculate_scores(src, rel, neg)
        else:
            neg_s = torch.cat([self.calculate_scores(neg, rel, dst), self.calculate_scores(src, rel, neg)], -1)
        return pos, neg_s.reshape(pos.shape[0], 1, -1)

    def calculate_energy(self, src, dst, neg, rel):
        pos, neg_s = self.energy_scores(src, dst, neg, rel)
        loss = self.loss_fn(pos, neg_s)
        metric = self.metric(pos.detach().float().cpu(), neg_s.detach().float().cpu())
        return loss, metric

    def _fused_ok(self, dev, rows=None):
        return self.fused_kind is not None and dev.type == "cuda" and (
            isinstance(self.entity_encoder, Embedding) or rows is not None)

    def loss_scores(self, src, dst, neg, rel, rows=None):
        """(loss, positive scores [B, 1, 1], corrupted scores [B, 1, k]) of device id tensors
        src / dst / rel [B, 1], neg [B, num_negs], with no host round trip: the step of the
        device-path trainer (models/kg_trainer.py) is captured into a hipGraph.

        ``rows``: a row-sparse step (RowSparseKGTrainer) passes its gathered entity rows
        (``{"entity_encoder": [n, D], "entity_transfer": ...}``) and src / dst / neg are
        POSITIONS into them; the fused kinds then score and differentiate straight on those
        rows (the kg_fwd / kg_bwd kernels, the row gradients land on the gathered rows)."""
        if self._fused_ok(src.device, rows):
            ent, rtab = self.entity_encoder, self.relation_encoder
            if rows is not None:
                table, s, d, n = rows["entity_encoder"], src, dst, neg
            else:
                table, s, d, n = ent.weight, ent._rows(src), ent._rows(dst), ent._rows(neg)
            pos_s, neg_s = gnn_ops.kg_score(table, rtab.weight, s, d, rtab._rows(rel), n, self.fused_kind,
                                            self.corrupt, True)
            pos, neg_s = pos_s.view(-1, 1, 1), neg_s.view(pos_s.shape[0], 1, -1)
        else:
            pos, neg_s = self.energy_scores(*self.generate_embedding(src, dst, neg, rel, rows=rows))
        return self.loss_fn(pos, neg_s), pos, neg_s

    def generate_embedding(self, src, dst, neg, rel, rows=None):
        raise NotImplementedError

    def _lookup(self, name, rows=None):
        """the id -> row function of table ``name``: the module itself, or — in a row-sparse
        step (``rows[name]``: the step's gathered rows) — a gather at the positions the
        trainer passes instead of ids"""
        if rows is None or name not in rows:
            return getattr(self, name)
        r = rows[name]
        return lambda p: r[p.reshape(-1)].reshape(*p.shape, r.shape[-1])


    # score kind of the fused gfx950 kernel (embed.hip kg_fwd / kg_bwd), None = unfused
    fused_kind = None

    def _fused_forward(self, src, dst, neg, rel):
        """gather + l2-normalise + score of the positive and every corrupted triple, and
        the whole backward into the two tables, in two kernels."""
        ent, rtab = self.entity_encoder, self.relation_encoder
        loss, pos, neg_s = self.loss_scores(src, dst, neg, rel)
        metric = self.metric(pos.detach().float().cpu(), neg_s.detach().float().cpu())
        with torch.no_grad():
            s, d, r = self.norm_emb(ent(src)), self.norm_emb(ent(dst)), self.norm_emb(rtab(rel))
        return [s.reshape(-1, s.shape[-1]), r.reshape(-1, r.shape[-1]), d.reshape(-1, d.shape[-1])], loss, \
            self.metric_name, metric

    def forward(self, inputs):
        src, dst, neg, rel = self.generate_triplets(inputs)
        dev = self._dev()
        src, dst, neg, rel = src.to(dev), dst.to(dev), neg.to(dev), rel.to(dev)
        if self._fused_ok(dev):
            return self._fused_forward(src, dst, neg, rel)
        s, d, n, r = self.generate_embedding(src, dst, neg, rel)
        loss, metric = self.calculate_energy(s, d, n, r)
        return [s.reshape(-1, s.shape[-1]), r.reshape(-1, r.shape[-1]), d.reshape(-1, d.shape[-1])], loss, \
            self.metric_name, metric


class TransE(TransX):
    def __init__(self, node_type, edge_type, node_max_id, edge_max_id, ent_dim, rel_dim, num_negs=5, margin=1.0,
                 l1=True, metric_name="mrr", corrupt="both", sharded=False):
        super().__init__(node_type, edge_type, node_max_id, edge_max_id, ent_dim, rel_dim, num_negs, l1,
                         metric_name, corrupt, sharded)
        if ent_dim != rel_dim:
            raise ValueError("Entity dim and Relation dim should be equal in TransE")
        self.margin = margin
        # subclasses with projections (TransH / TransD) override generate_embedding and
        # keep the unfused path
        if type(self).generate_embedding is TransE.generate_embedding:
            self.fused_kind = "l1" if l1 else "l2"

    def generate_embedding(self, src, dst, neg, rel, rows=None):
        e = self._lookup("entity_encoder", rows)
        return (self.norm_emb(e(src)), self.norm_emb(e(dst)), self.norm_emb(e(neg)),
                self.norm_emb(self.relation_encoder(rel)))


class TransH(TransE):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.hyper_vector = Embedding(self.edge_max_id + 1, self.ent_dim)

    @staticmethod
    def projection(x, hyper):
        h = F.normalize(hyper, dim=-1)
        return x - (x * h).sum(-1, keepdim=True) * h

    def generate_embedding(self, src, dst, neg, rel, rows=None):
        e = self._lookup("entity_encoder", rows)
        hyper = self.hyper_vector(rel)  # [B, 1, D] broadcasts over negatives
        return (self.projection(e(src), hyper), self.projection(e(dst), hyper), self.projection(e(neg), hyper),
                self.norm_emb(self.relation_encoder(rel)))


class TransR(TransX):
    def __init__(self, node_type, edge_type, node_max_id, edge_max_id, ent_dim, rel_dim, num_negs=5, margin=1.0,
                 l1=True, metric_name="mrr", corrupt="both", sharded=False):
        super().__init__(node_type, edge_type, node_max_id, edge_max_id, ent_dim, rel_dim, num_negs, l1,
                         metric_name, corrupt, sharded)
        self.margin = margin
        self.transfer_matrix = Embedding(edge_max_id + 1, ent_dim * rel_dim)

    def projection(self, x, mat):
        # x [B, k, ent] @ mat [B, ent, rel] -> one batched GEMM per batch (rocBLAS strided batched)
        return F.normalize(torch.bmm(x, mat), dim=-1)

    def generate_embedding(self, src, dst, neg, rel, rows=None):
        e = self._lookup("entity_encoder", rows)
        mat = self.transfer_matrix(rel).reshape(-1, self.ent_dim, self.rel_dim)
        return (self.projection(e(src), mat), self.projection(e(dst), mat), self.projection(e(neg), mat),
                self.norm_emb(self.relation_encoder(rel)))


class TransD(TransE):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.entity_transfer = Embedding(self.node_max_id + 1, self.ent_dim)
        self.relation_transfer = Embedding(self.edge_max_id + 1, self.rel_dim)

    @staticmethod
    def projection(x, ent_t, rel_t):
        return F.normalize(x + (x * ent_t).sum(-1, keepdim=True) * rel_t, dim=-1)

    def generate_embedding(self, src, dst, neg, rel, rows=None):
        e, et = self._lookup("entity_encoder", rows), self._lookup("entity_transfer", rows)
        rt = self.relation_transfer(rel)
        return (self.projection(e(src), et(src), rt), self.projection(e(dst), et(dst), rt),
                self.projection(e(neg), et(neg), rt), self.norm_emb(self.relation_encoder(rel)))


class DistMult(TransX):
    """score = sum(h * r * t) (distmult.py:74-77: diag(r) t then dot with h)."""

    def __init__(self, node_type, edge_type, node_max_id, edge_max_id, ent_dim, rel_dim, num_negs=5, margin=1,
                 metric_name="mrr", corrupt="both", l2_regular=False, regular_param=0.0001, sharded=False):
        super().__init__(node_type, edge_type, node_max_id, edge_max_id, ent_dim, rel_dim, num_negs, True,
                         metric_name, corrupt, sharded)
        self.margin, self.l2_regular, self.regular_param = margin, l2_regular, regular_param
        self.fused_kind = "distmult"

    def calculate_scores(self, src, rel, dst):
        return (src * rel * dst).sum(-1)

    def loss_fn(self, pos_scores, neg_scores):
        loss = super().loss_fn(pos_scores, neg_scores)
        if self.l2_regular:
            loss = loss + self.regular_param * (self.entity_encoder.weight.pow(2).sum()
                                                + self.relation_encoder.weight.pow(2).sum())
        return loss

    def generate_embedding(self, src, dst, neg, rel, rows=None):
        e = self._lookup("entity_encoder", rows)
        return (self.norm_emb(e(src)), self.norm_emb(e(dst)), self.norm_emb(e(neg)),
                self.norm_emb(self.relation_encoder(rel)))
