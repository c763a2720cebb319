"""DeepWalk / node2vec(p = q = 1) skip-gram training step on the GPU with row-sharded
embedding tables (BASELINE config 4: 128-d embeddings, 100M nodes, DP over RCCL with an
embedding all-to-all).

Reference model: examples/deepwalk/deepwalk.py:27-99 — ``random_walk`` (walk_len, p, q)
-> ``gen_pair`` (left/right window) -> negatives from ``sample_node`` (batch x pairs x
num_negs) -> target embedding of the centre, context embedding of the positive and the
negatives -> sigmoid CE (mp_utils/base.py:80-91) -> Adam on the (PS-partitioned) tables.

One step here, per rank (no autograd, no dense table gradient):

  1. walks    : ``random_walk_kernel`` from ``batch`` alias-sampled start nodes
  2. pairs    : skip-gram (centre, context) pairs of every walk; negatives per pair
  3. unique   : hash-table unique of the centre ids and of the context+negative ids
  4. lookup   : ShardedTable.lookup — RCCL all-to-all of ids and rows (world > 1)
  5. loss     : gather rows per pair, fused dot + sigmoid-CE fwd/bwd (embed.hip K11)
  6. grads    : per-unique-row gradient sums (index_add_rows kernel)
  7. update   : ShardedTable.apply — all-to-all of row grads to the owners, merge,
                row-sparse Adam (optim.hip) on the owner's shard

Padding: a walk that hits a node without out-edges continues with the pad row
``num_nodes`` (the reference's ``max_id + 1`` default node).
"""
from __future__ import annotations

import torch

import euler_amd.ops.graph_api as ge
from euler_amd.ops import gnn_ops
from euler_amd.ops._native import hip, use_hip
from euler_amd.parallel.sparse_table import ShardedTable

__all__ = ["DeepWalkTrainer"]


def _pair_positions(walk_len, left, right):
    pairs = ge.gen_pair(torch.arange(walk_len + 1).view(1, -1), left, right)[0]
    return pairs[:, 0].clone(), pairs[:, 1].clone()


class DeepWalkTrainer:
    def __init__(self, graph, num_nodes, dim=128, walk_len=3, left_win_size=1, right_win_size=1, num_negs=5,
                 batch_size=1024, lr=0.01, optimizer="adam", group=None, seed=0, emb_dtype=torch.float32,
                 force_comm=False):
        self.graph = graph
        self.num_nodes = int(num_nodes)
        self.pad = self.num_nodes  # rows: num_nodes + 1 (pad row like the reference's max_id + 1)
        self.dim, self.walk_len, self.num_negs, self.batch = int(dim), int(walk_len), int(num_negs), int(batch_size)
        dev = graph.device
        self.device = dev
        self.target = ShardedTable(self.num_nodes + 1, dim, dev, group, optimizer, lr, seed=seed,
                                   force_comm=force_comm)
        self.context = ShardedTable(self.num_nodes + 1, dim, dev, group, optimizer, lr, seed=seed + 1,
                                    force_comm=force_comm)
        pi, pj = _pair_positions(walk_len, left_win_size, right_win_size)
        self.pi, self.pj = pi.to(dev), pj.to(dev)
        self.pairs_per_walk = int(pi.numel())
        self.emb_dtype = emb_dtype
        self.loss = torch.zeros((), device=dev)

    def _gather(self, rows, inv):
        if use_hip(rows, inv):
            return hip().gather_rows(rows, inv.contiguous())
        return rows[inv]

    def _grad_rows(self, n, inv, g):
        acc = torch.zeros(n, self.dim, dtype=torch.float32, device=g.device)
        g2 = g.reshape(-1, self.dim).float().contiguous()
        if use_hip(acc, inv, g2):
            hip().index_add_rows_(acc, inv.reshape(-1).contiguous(), g2)
        else:
            acc.index_add_(0, inv.reshape(-1), g2)
        return acc

    def sample(self):
        """(centre [P], positive [P], negatives [P, K]) global ids of one step."""
        g = self.graph
        g.advance()
        starts = g.sample_node(self.batch, stream_id=1)
        walks = g.random_walk(starts, self.walk_len, default=-1, stream_id=3).long()
        walks = torch.where(walks < 0, torch.full_like(walks, self.pad), walks)
        src = walks[:, self.pi].reshape(-1)
        pos = walks[:, self.pj].reshape(-1)
        negs = g.sample_node(src.numel() * self.num_negs, stream_id=4).long().view(-1, self.num_negs)
        return src, pos, negs

    def step(self):
        src, pos, negs = self.sample()
        P, K = src.numel(), self.num_negs
        # unique ids per table (first-occurrence order; hash kernel on the GPU)
        u_t, inv_t = gnn_ops.unique_first(src)
        u_c, inv_c = gnn_ops.unique_first(torch.cat([pos, negs.reshape(-1)]))
        rows_t, h_t = self.target.lookup(u_t)
        rows_c, h_c = self.context.lookup(u_c)
        rt, rc = rows_t.to(self.emb_dtype), rows_c.to(self.emb_dtype)
        emb = self._gather(rt, inv_t)                                       # [P, D]
        pos_rows = self._gather(rc, inv_c[:P]).view(P, 1, self.dim)         # [P, 1, D]
        neg_rows = self._gather(rc, inv_c[P:]).view(P, K, self.dim)         # [P, K, D]
        if use_hip(emb, pos_rows, neg_rows):
            logits, loss_rows = hip().sgns_fwd(emb, pos_rows, neg_rows)
            demb, dpos, dneg = hip().sgns_bwd(emb, pos_rows, neg_rows, logits, 1.0 / (P * (1 + K)))
            self.loss = loss_rows.sum() / (P * (1 + K))
        else:
            e = emb.float().requires_grad_(True)
            p_ = pos_rows.float().requires_grad_(True)
            n_ = neg_rows.float().requires_grad_(True)
            loss, _, _ = gnn_ops.sgns_loss_reference(e, p_, n_)
            demb, dpos, dneg = torch.autograd.grad(loss, (e, p_, n_))
            self.loss = loss.detach()
        g_t = self._grad_rows(u_t.numel(), inv_t, demb)
        # inv_c is ordered [positives (P), negatives (P*K)]: stack the grads the same way
        g_c = self._grad_rows(u_c.numel(), inv_c,
                              torch.cat([dpos.reshape(P, self.dim), dneg.reshape(P * K, self.dim)], 0))
        self.target.apply(h_t, g_t)
        self.context.apply(h_c, g_c)
        return self.loss

    def pairs_per_step(self):
        return self.batch * self.pairs_per_walk

    def embedding(self, ids):
        """target embeddings of global ids (inference)."""
        u, inv = gnn_ops.unique_first(ids.reshape(-1).long())
        rows, _ = self.target.lookup(u)
        return rows[inv].view(*ids.shape, self.dim)
