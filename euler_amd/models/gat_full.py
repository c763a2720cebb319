"""Full-graph multi-head GAT training (BASELINE config 3) in the product: the model, the
trainer and its captured step.

Model (reference ``examples/gat/gat.py:27-86``: GATConv layers with ``head_num`` heads,
concatenated, ELU, then the classifier; here all heads of a layer are ONE convolution):

    layer l: z = h W_l -> [N, H, C];  al = <z, a_src>, ar = <z, a_dst> per head
             h = ELU(edge-softmax aggregation of z)          (gat.hip, one pass per node)
    logits = h W_out + b  on the rows the loss reads

Trainer (:class:`FullGraphGatTrainer`): one epoch = forward over every node in bf16
autocast, softmax cross-entropy on the training rows, backward, the flat Adam
(``parallel/flat.py``: one launch over one parameter buffer); the epoch is captured once
into a hipGraph and replayed (``CapturedTrainer``).  The per-edge work is entirely in the
HIP kernels (``gnn_ops.gat_conv``: attention terms + online softmax + aggregation forward,
CSR + CSC passes backward, no atomics), the projections on the tall split-K GEMM
(``gnn_ops.tall_linear``).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from euler_amd.models.captured import CapturedTrainer
from euler_amd.ops import gnn_ops, mp_ops

__all__ = ["FullGraphGAT", "FullGraphGatTrainer", "add_self_loops"]


def add_self_loops(indptr, col):
    """a destination CSR with a self-loop prepended to every row (the reference's full
    flow adds them)"""
    n = indptr.numel() - 1
    dev = indptr.device
    deg = torch.diff(indptr)
    new_indptr = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(deg + 1, 0, out=new_indptr[1:])
    new_col = torch.empty(int(col.numel()) + n, dtype=torch.int32, device=dev)
    new_col[new_indptr[:-1]] = torch.arange(n, dtype=torch.int32, device=dev)
    row = torch.repeat_interleave(torch.arange(n, device=dev), deg)
    pos = torch.arange(col.numel(), device=dev) - indptr[row] + new_indptr[row] + 1
    new_col[pos] = col
    return new_indptr, new_col


class FullGraphGAT(nn.Module):
    """``layers`` multi-head GAT convolutions (``heads`` x ``ch``, concatenated, ELU) and a
    linear classifier.  ``impl="composed"``: the reference's op sequence (gather logits,
    segment softmax, gather messages, segment sum) on the message-passing ops instead of
    the fused kernel (the numerics / speed comparison of ``benchmarks/bench_gat.py``)."""

    def __init__(self, in_dim, heads, ch, n_cls, layers=2, impl="fused", slope=0.2):
        super().__init__()
        self.heads, self.ch, self.impl, self.slope = heads, ch, impl, slope
        dims = [in_dim] + [heads * ch] * layers
        self.lin = nn.ModuleList([nn.Linear(dims[i], dims[i + 1], bias=False) for i in range(layers)])
        self.att_src = nn.ParameterList([nn.Parameter(torch.randn(heads, ch) * 0.1) for _ in range(layers)])
        self.att_dst = nn.ParameterList([nn.Parameter(torch.randn(heads, ch) * 0.1) for _ in range(layers)])
        self.out = nn.Linear(heads * ch, n_cls)

    def forward(self, x, csr, rows=None):
        h = x
        H, C = self.heads, self.ch
        for lin, a_s, a_d in zip(self.lin, self.att_src, self.att_dst):
            if self.impl == "fused":
                z = gnn_ops.tall_linear(h, lin.weight).view(-1, H, C)
                agg = gnn_ops.gat_conv(z, a_s, a_d, csr, self.slope)
            else:
                z = lin(h).view(-1, H, C)
                al = (z.float() * a_s).sum(-1)
                ar = (z.float() * a_d).sum(-1)
                ei = csr.edge_index
                seg = _csr_seg(csr)
                logit = F.leaky_relu(mp_ops.gather(ar, ei[0]) + mp_ops.gather(al, ei[1]), self.slope)
                alpha = mp_ops.scatter_softmax(logit, seg, csr.n_dst)
                # fp32 messages and sums, like the fused kernel's accumulators
                msg = mp_ops.gather(z.reshape(-1, H * C), ei[1]).view(-1, H, C).float() * alpha.unsqueeze(-1).float()
                agg = mp_ops.scatter_add(msg.reshape(-1, H * C), seg, csr.n_dst).view(-1, H, C).to(z.dtype)
            h = F.elu(agg.reshape(-1, H * C))
        # the classifier runs on the rows the loss reads only (same loss and gradients)
        hr = h if rows is None else h[rows]
        return gnn_ops.tall_linear(hr, self.out.weight, self.out.bias)


def _csr_seg(csr):
    if not hasattr(csr, "_seg"):
        csr._seg = mp_ops.SegmentIndex(csr.edge_index[0].long(), csr.n_dst)
    return csr._seg


class _NoDraws:
    """full-graph training draws nothing: the trainer's RNG source is a fixed pair"""

    def __init__(self, device):
        self.rng = torch.zeros(2, dtype=torch.int64, device=device)

    def advance(self, inc: int = 1):
        pass

    def reseed_cpu(self):
        pass


class FullGraphGatTrainer(CapturedTrainer):
    """``x`` [N, F] node features, ``csr`` the graph (``gnn_ops.EdgeCSR``, self loops
    included), ``labels`` [N] classes, ``train_idx`` the rows of the loss."""

    metric_name = "acc"

    def __init__(self, model, x, csr, labels, train_idx, optimizer="adam", learning_rate=5e-3, amp=True):
        self.x, self.csr = x, csr
        self.labels = labels
        self.train_idx = train_idx
        self.y_train = labels[train_idx].contiguous()
        self.amp = bool(amp) and x.is_cuda
        super().__init__(model, _NoDraws(x.device), x.device, optimizer, learning_rate)

    def _logits(self, rows):
        if self.amp:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                return self.model(self.x, self.csr, rows)
        return self.model(self.x, self.csr, rows)

    def _forward_loss(self):
        return gnn_ops.xent(self._logits(self.train_idx), self.y_train)

    @torch.no_grad()
    def accuracy(self, rows):
        """accuracy on ``rows`` (eval mode: no state changes)"""
        logits = self._logits(rows)
        return float((logits.float().argmax(1) == self.labels[rows]).float().mean())

    def metric(self) -> float:
        return float(self.loss_out.item())
