"""The fused GraphSAGE step (models/sage_trainer.py, csrc/hip/sage_tree.hip) over a graph
row-sharded across the data-parallel ranks (graph/sharded_graph.py).

The whole-graph :class:`~euler_amd.models.sage_trainer.SageTrainer` draws each step's
slotted tree inside its kernels from the CSR in HBM.  Here no rank holds the whole CSR, so
the tree is drawn across the ranks before the forward — the reference's distributed
``SageDataFlow`` (``tf_euler/python/dataflow/sage_dataflow.py:35-50`` over
``remote_op.cc:60-146``):

* roots: :meth:`ShardedDeviceGraph.sample_node` (global node weights);
* every hop: :meth:`ShardedDeviceGraph.sample_neighbor` — each row's owner draws its
  fanout from its local CSR, the draws come back over the all-to-all — laid out in the
  kernels' slotted tree (sibling group: F draws, then the parent itself, then padding);
* input features: the trainer's row-sharded feature exchange (``feature_shard``,
  graph/sharded_features.py) fills the forward's feature cache;
* labels: the roots' label rows come over the label exchange into a [B] table, and the
  head reads it through roots 0 .. B-1 (TreePlan ``label_rows``).

Forward, head, backward, split-K dW, gradient all-reduce and the optimizer are the
whole-graph trainer's launches unchanged.  Evaluate / infer run on the device too, with the
ranks in lockstep (:meth:`ShardedSageTrainer.infer_logits`; the engine of an
``engine_shards`` job holds only its own partitions, so it could not answer them).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from euler_amd.models.sage_trainer import SageTrainer

__all__ = ["ShardedSageTrainer"]

_STREAM0 = 40  # Philox streams of the tree draws (roots 40, hop k: 41 + k)


class ShardedSageTrainer(SageTrainer):
    # evaluate / infer on the device, collectively: every rank calls with batches of the same
    # padded size in lockstep (estimator/base.py _lockstep_batches)
    collective_infer = True

    def __init__(self, graph, batch_size, fanouts, dims, label_dim, **kw):
        self.sgraph = graph
        loc = graph.local
        if graph.labels is None or graph.features is None:
            raise ValueError("the sharded graph needs features and labels")
        lab = graph.labels.shard
        self._class_labels = lab.shape[1] == 1 and int(label_dim) > 1
        B = int(batch_size)
        dummy = torch.zeros(B, dtype=torch.int32) if self._class_labels else torch.zeros(B, int(label_dim))
        kw.pop("features", None)
        kw.pop("labels", None)
        kw.pop("feature_shard", None)
        if graph.comm:
            fs = dict(feature_shard=graph.padded_features(16), feature_dim=graph.features.dim)
        else:
            # one rank without collectives: global rows are local rows, the forward gathers
            # from the table itself (no exchange, no dedup pass)
            fs = dict(features=loc.features)
        super().__init__(loc, batch_size, fanouts, dims, label_dim, labels=dummy, **fs, **kw)
        self.pipelined = False
        if self.on_gpu:
            self.roots.copy_(torch.arange(self.B, dtype=torch.int32, device=self.device))

    def _alloc_gpu(self):
        # the head reads the batch's label table through roots 0 .. B-1
        self._label_rows = self.B
        super()._alloc_gpu()

    # ------------------------------------------------------------------ the tree draw
    def _types(self, mask):
        return [t for t in range(self.sgraph.num_types) if (mask >> t) & 1]

    def _draw_tree(self):
        """(global roots [B], slotted hop-(L-1) rows [M], leaf draws [M, F_L]) across the
        ranks, int32 throughout (the kernels' row type: no conversion passes)"""
        g = self.sgraph
        roots = g.sample_node(self.B, stream_id=_STREAM0).int()
        level = roots
        for k in range(1, self.L):
            f, P = self.fanouts[k - 1], 1 << self.logP[k]
            nb = g.sample_neighbor(level, f, self._types(self.masks[k - 1]), -1, stream_id=_STREAM0 + k).view(-1, f)
            slots = torch.full((level.numel(), P), -1, dtype=torch.int32, device=level.device)
            slots[:, :f] = nb
            slots[:, f] = level
            level = slots.view(-1)
        leaf = g.sample_neighbor(level, self.fanouts[-1], self._types(self.masks[-1]), -1,
                                 stream_id=_STREAM0 + self.L).view(-1, self.fanouts[-1])
        return roots, level, leaf

    def _batch_labels(self, roots):
        g = self.sgraph
        if g.comm:
            y = g.gather_labels(roots)  # [B, C] fp32 (or [B, 1] class ids) over the exchange
        else:
            y = g.local.labels[roots.long()]  # one rank: global rows are local rows
        if self._class_labels:
            return y.reshape(-1).to(torch.int32)
        return y

    def _sample_sharded(self):
        roots, level, leaf = self._draw_tree()
        y = self._batch_labels(roots)
        self._global_roots = roots
        self._batch_y = y
        if not self.on_gpu:
            return roots.long(), level.long(), leaf.long(), y
        self.nodes.copy_(level)
        self.leaf.copy_(leaf.reshape(-1))
        if self.label_mode == 2:
            self.labels[:, : self.C].copy_(y)
        else:
            self.labels.copy_(y)
        return None

    # ------------------------------------------------------------------ GPU step
    def _prime(self):
        if not self._primed:
            self._sample_sharded()
            self._primed = True
            self._gathered = False

    def step(self, grad_sync=None):
        """draw the tree across the ranks, then the whole-graph trainer's launches (no
        in-kernel sampler blocks)"""
        self.step_count += 1
        if not self.on_gpu:
            return self._cpu_step(grad_sync)
        p = self.plan
        self._prime()
        self._fwd()
        p.head(None, False)
        p.bwd()
        if grad_sync is None:
            p.dw(self._dw_all)
            p.opt(2, 1.0, False, False)
        elif len(self.grad_buckets()) == 1:
            p.dw(self._dw_all)
            p.opt(0, 1.0, False, False)
            g = self.grad if getattr(self, "grad16", None) is None else self.grad16
            scale = grad_sync(g)
            p.opt(1, 1.0 if scale is None else float(scale))
        else:
            self._dist_backward(grad_sync, False)
        self._primed = False
        self._gathered = False

    # ------------------------------------------------------------------ inference
    @torch.no_grad()
    def infer_logits(self, ids, pad_to=None):
        """(embeddings [n, E], logits [n, C], labels [n, C]) of raw node ids: a fresh tree
        per root drawn through the owners (Philox streams 8.., training's untouched), the
        features over the exchange and the fp32 model on the trained parameters (the
        whole-graph trainer's ``infer_logits`` on the sharded graph).  Collective: every rank
        calls it with the same ``pad_to`` (rows padded with -1, which touch nothing)."""
        g = self.sgraph
        rows = g.rows_of(ids).to(self.device).long().reshape(-1)
        n = rows.numel()
        B = max(n, int(pad_to or 0), 1)
        if B > n:
            rows = torch.cat([rows, torch.full((B - n,), -1, dtype=torch.long, device=rows.device)])
        level = rows.int()
        for k in range(1, self.L):
            f, P = self.fanouts[k - 1], 1 << self.logP[k]
            nb = g.sample_neighbor(level, f, self._types(self.masks[k - 1]), -1, stream_id=7 + k).view(-1, f)
            slots = torch.full((level.numel(), P), -1, dtype=torch.int32, device=level.device)
            slots[:, :f] = nb
            slots[:, f] = level
            level = slots.view(-1)
        leaf = g.sample_neighbor(level, self.fanouts[-1], self._types(self.masks[-1]), -1,
                                 stream_id=7 + self.L).view(-1, self.fanouts[-1])
        g.advance()
        params = {k: v.float() for k, v in self.logical_params().items()}
        nodes, leaf = level.long(), leaf.long()
        if self.fshard is not None:
            pos = self.fshard.exchange(torch.cat([nodes, leaf.reshape(-1)])).long()
            emb = self.logical_embed(params, pos[: nodes.numel()], pos[nodes.numel():].view_as(leaf),
                                     self.fshard.cache)
        else:
            emb = self.logical_embed(params, nodes, leaf)
        logits = emb @ params["out_fc.weight"].t().to(emb.device)
        y = self._batch_labels(rows if g.comm else rows.clamp(min=0))  # -1 rows: zeros over the exchange
        if self._class_labels:
            y = torch.zeros((B, self.C), dtype=torch.float32, device=y.device).scatter_(1, y.long().view(-1, 1), 1.0)
        return emb[:n], logits[:n], y[:n].float().to(emb.device)

    def infer_embed(self, ids, pad_to=None):
        return self.infer_logits(ids, pad_to)[0]

    def _labels_of(self, roots):
        """the last drawn batch's labels [B, C] (fp32; the batch's roots are rows 0 .. B-1
        of the label table the head reads)"""
        y = self._batch_y
        if self._class_labels:
            out = torch.zeros((y.numel(), self.C), dtype=torch.float32, device=y.device)
            out.scatter_(1, y.long().view(-1, 1), 1.0)
            return out
        return y.float()

    def samples(self):
        """(global roots [B], hop rows [M], leaf draws [M, F_L]) of the last step"""
        if self.on_gpu:
            return (self._global_roots.long(), self.nodes.long(), self.leaf.view(-1, self.fanouts[-1]).long())
        return self._cpu_samples

    # ------------------------------------------------------------------ CPU twin
    def _cpu_forward_backward(self):
        self.sgraph.reseed_cpu()
        roots, nodes, leaf, y = self._sample_sharded()
        self._cpu_samples = (roots, nodes, leaf)
        P = self._cpu_params
        for t in P.values():
            t.grad = None
        if self.fshard is not None:
            pos = self.fshard.exchange(torch.cat([nodes, leaf.reshape(-1)])).long()
            nodes_p, leaf_p = pos[: nodes.numel()], pos[nodes.numel():].view_as(leaf)
            logits = self.logical_forward(P, roots, nodes_p, leaf_p, self.fshard.cache)
        else:
            logits = self.logical_forward(P, roots, nodes, leaf)
        if self._class_labels:
            yy = torch.zeros((roots.numel(), self.C), dtype=torch.float32)
            yy.scatter_(1, y.long().view(-1, 1), 1.0)
            y = yy
        y = y.float().to(logits.device)
        loss = F.binary_cross_entropy_with_logits(logits, y)
        loss.backward()
        with torch.no_grad():
            pred, pos_ = logits >= 0, y > 0.5
            self._cpu_counts[0] += int((pred & pos_).sum())
            self._cpu_counts[1] += int((pred & ~pos_).sum())
            self._cpu_counts[2] += int((~pred & pos_).sum())
        self.graph.rng[1] += 1
        return loss.detach()
