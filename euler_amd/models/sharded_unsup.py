"""Unsupervised GraphSAGE (two 2-hop towers, skip-gram pairs with sampled negatives) on a
graph row-sharded over the data-parallel ranks (graph/sharded_graph.py).

The whole-graph :class:`~euler_amd.models.sage_tower.UnsupSageTrainer` samples inside its
tower kernels from the CSR in HBM.  Here no rank holds the whole CSR, so every draw of the
reference's unsupervised step (``tf_euler/python/mp_utils/base.py`` UnsuperviseModel:
``sample_node`` sources, one ``sample_neighbor`` positive per source over the model's edge
type, ``sample_node`` negatives; each tower's ``SageDataFlow`` over ``remote_op.cc:60-146``)
goes through the rows' owners:

* sources / negatives: :meth:`ShardedDeviceGraph.sample_node` (global node weights);
* positives and both towers' trees: :meth:`ShardedDeviceGraph.sample_neighbor` (owner-side
  draws over the all-to-all), laid out in the towers' slotted trees;
* input features: one exchange for all four trees' rows (``padded_features``: the
  parameters' padded layer-0 width).

The towers, the pair loss and the flat Adam are the trainer's fp32 torch path (the oracle
of the fused kernels) over the exchanged feature rows; over RCCL the whole step captures
into a hipGraph (fixed-size exchanges), over gloo it runs eagerly.  ``infer_embed`` embeds
raw ids collectively for the estimator's lockstep infer.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from euler_amd.models.sage_tower import UnsupSageTrainer
from euler_amd.ops import mp_ops

__all__ = ["ShardedUnsupSageTrainer"]

_S = 50  # Philox streams: sources 50, positives 51, negatives 52, trees 53-56, infer 57-58


class ShardedUnsupSageTrainer(UnsupSageTrainer):
    _device_towers = False  # the towers' in-kernel samplers need a whole CSR
    collective_infer = True

    def __init__(self, graph, batch_size, fanouts, dims, **kw):
        if graph.features is None:
            raise ValueError("the sharded graph needs node features")
        self.sgraph = graph
        kw.pop("features", None)
        kw.pop("fused", None)
        # the local table gives the feature width (and is the table itself at one rank)
        super().__init__(graph, batch_size, fanouts, dims, features=graph.local.features, fused=False, **kw)
        self.fshard = graph.padded_features(16) if graph.comm else None
        self._grad_sync = None

    # ------------------------------------------------------------------ draws
    def sample_roots(self):
        """(sources [B], positives [B], negatives [B*K]) global rows, drawn through the owners"""
        g = self.sgraph
        g.advance()
        if self.device.type != "cuda":
            g.reseed_cpu()
        src = g.sample_node(self.B, stream_id=_S)
        pos = g.sample_neighbor(src, 1, self._types(self.pos_mask), -1, stream_id=_S + 1).reshape(-1)
        negs = g.sample_node(self.B * self.K, stream_id=_S + 2)
        return src.int(), pos.int(), negs.int()

    def _tree(self, roots, stream):
        """a tower's slotted tree of ``roots``: nodes [R * P], leaf [R * P, F2] (global rows)"""
        g = self.sgraph
        F1, F2, P = self.fanouts[0], self.fanouts[1], 1 << self.logP
        nb = g.sample_neighbor(roots.int(), F1, self._types(self.masks[0]), -1, stream_id=stream).view(-1, F1).long()
        slots = torch.full((roots.numel(), P), -1, dtype=torch.int64, device=nb.device)
        slots[:, :F1] = nb
        slots[:, F1] = roots.long().to(nb.device)
        nodes = slots.reshape(-1)
        leaf = g.sample_neighbor(nodes.int(), F2, self._types(self.masks[1]), -1, stream_id=stream + 1)
        return nodes, leaf.view(-1, F2).long()

    def _features_of(self, *idx):
        """(feature table, the rows of ``idx`` as positions in it): one exchange for all"""
        if self.fshard is None:
            return self.features, idx
        flat = torch.cat([i.reshape(-1) for i in idx])
        pos = self.fshard.exchange(flat).long()
        out, o = [], 0
        for i in idx:
            out.append(pos[o:o + i.numel()].view_as(i))
            o += i.numel()
        return self.fshard.cache, out

    def _tower_reference(self, W0, nodes, leaf, table=None):
        """the towers' layer 0 + slot aggregation (UnsupSageTrainer._tower_reference) with
        the tree's rows gathered first (``-1``: zeros) and only those converted to fp32 —
        never the whole table (100M rows at one rank)"""
        table = self.features if table is None else table
        xs = mp_ops.gather(table, nodes.reshape(-1)).float()
        agg = mp_ops.gather_sum(table, leaf.reshape(leaf.shape[0], -1))  # fp32, -1 leaves add nothing
        cnt = self.fanouts[1]
        if self.include_self:
            agg, cnt = agg + xs, cnt + 1
        h0 = torch.relu(torch.cat([xs, agg / cnt], 1) @ W0.t())
        P, f = 1 << self.logP, self.fanouts[0]
        hg = h0.view(-1, P, h0.shape[1])
        s, a = hg[:, f], hg[:, :f].sum(1)
        c = f
        if self.include_self:
            a, c = a + s, c + 1
        return torch.cat([s, a / c], 1)

    # ------------------------------------------------------------------ step
    def _forward_loss(self):
        src, pos, negs = self.sample_roots()
        ctx = torch.cat([pos, negs])
        ns, ls = self._tree(src, _S + 3)
        nc, lc = self._tree(ctx, _S + 5)
        self._samples = (src.long(), ctx.long(), ns, ls, nc, lc)
        table, (ns_p, ls_p, nc_p, lc_p) = self._features_of(ns, ls, nc, lc)
        P = self.params
        A1s = self._tower_reference(P["gnn.W0"], ns_p, ls_p, table)
        A1c = self._tower_reference(P["context_gnn.W0"], nc_p, lc_p, table)
        return self._pair_loss(self._head("gnn", A1s), self._head("context_gnn", A1c))

    def _step(self, grad_sync=None):
        loss, mrr = self._forward_loss()
        self.opt.zero_grad()
        loss.backward()
        scale = 1.0
        if grad_sync is not None:
            s = grad_sync(self.flat.grad)
            scale = 1.0 if s is None else float(s)
        self.opt.step(scale)
        self.loss_out.copy_(loss.detach())
        self.mrr_sum.add_(mrr)
        return self.loss_out

    def tower_samples(self, tower):
        src, ctx, ns, ls, nc, lc = self._samples
        return (src, ns, ls) if tower == "gnn" else (ctx, nc, lc)

    # ------------------------------------------------------------------ hipGraph
    def capturable(self) -> bool:
        """on the GPU without exchanges or over RCCL (fixed-size exchanges capture like any
        kernel); gloo stages through host memory: eager"""
        g = self.sgraph
        if self.device.type != "cuda":
            return False
        return not g.comm or dist.get_backend(g.group) != "gloo"

    def capture(self, grad_sync=None, warmup: int = 2, steps: int = 1, extra_sizes=()):
        self._grad_sync = grad_sync
        if self.capturable():
            return super().capture(grad_sync, warmup, steps, extra_sizes)
        for _ in range(int(warmup)):
            self.step_count += 1
            self._step(grad_sync)
        self._graphs, self._graph_exec = {}, None
        return None

    def replay(self, n: int = 1):
        if self._graph_exec is not None:
            return super().replay(n)
        self.replay_steps(n)

    def replay_steps(self, n: int):
        if self._graphs:
            return super().replay_steps(n)
        for _ in range(int(n)):
            self._step(self._grad_sync)
        self.step_count += int(n)

    # ------------------------------------------------------------------ inference
    @torch.no_grad()
    def embed(self, rows, tower="gnn", seed_offset=0):
        """embeddings [n, E] of global rows through a tower on a fresh tree drawn through
        the owners (collective: every rank calls it with the same row count)"""
        rows = torch.as_tensor(rows).reshape(-1).to(self.device)
        nodes, leaf = self._tree(rows, _S + 7)
        self.sgraph.advance()
        table, (n_p, l_p) = self._features_of(nodes, leaf)
        A1 = self._tower_reference(self.params[f"{tower}.W0"].detach(), n_p, l_p, table)
        return self._head(tower, A1)[:, : self.E]

    @torch.no_grad()
    def infer_embed(self, ids, pad_to=None):
        """source-tower embeddings of raw node ids (the estimator's infer), rows padded with
        -1 to ``pad_to`` so every rank's exchanges match"""
        rows = self.sgraph.rows_of(ids).to(self.device).long().reshape(-1)
        n = rows.numel()
        B = max(n, int(pad_to or 0), 1)
        if B > n:
            rows = torch.cat([rows, torch.full((B - n,), -1, dtype=torch.long, device=rows.device)])
        return self.embed(rows)[:n]
