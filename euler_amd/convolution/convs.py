"""Message-passing convolutions (reference ``tf_euler/python/convolution/*.py``).

Contract (unchanged from the reference ``conv.py:27-53``)::

    out = conv(x, edge_index, size, edge_attr=None)

* ``x = (x_target, x_source)``: rows of the smaller (target, ``size[0]``) and larger
  (source, ``size[1]``) node sets of a dataflow block;
* ``edge_index`` [2, E]: row 0 indexes targets, row 1 indexes sources;
* every gather / scatter goes through :mod:`euler_amd.ops.mp_ops`, i.e. the gfx950
  segment-reduce / edge-softmax kernels on GPU tensors.

Destination CSRs are built once per ``edge_index`` and cached on the block
(``SegmentIndex``), so the degree normalisations, softmax and aggregation of one
layer all reuse one sort.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from euler_amd.ops import gnn_ops, mp_ops
from euler_amd.ops._native import hip, use_hip
from euler_amd.utils.layers import Dense

__all__ = ["Conv", "GCNConv", "SAGEConv", "GATConv", "TAGConv", "AGNNConv", "SGCNConv", "GINConv", "GraphConv",
           "APPNPConv", "ARMAConv", "DNAConv", "RelationConv", "GatedConv", "MultiHeadGATConv", "restricted_softmax"]


def _seg(edge_index, i, size):
    """destination CSR of edge_index[i] (cached on the tensor object, shared with the SpMM)."""
    return mp_ops.cached_segment(edge_index, i, size)


class Conv(nn.Module):
    def __init__(self, aggr="add"):
        super().__init__()
        assert aggr in ("add", "mean", "max")
        self.aggr = aggr

    @staticmethod
    def gather_feature(features, edge_index):
        out = []
        for feature in features:
            assert isinstance(feature, (tuple, list)) and len(feature) == 2
            feature = list(feature)
            if feature[1] is None:
                feature[1] = feature[0]
            out.append([None if t is None else mp_ops.gather(t, edge_index[i]) for i, t in enumerate(feature)])
        return out

    def scatter(self, values, edge_index, size, aggr=None):
        return mp_ops.scatter_(aggr or self.aggr, values, _seg(edge_index, 0, size[0]), size[0])

    @staticmethod
    def norm(edge_index, size):
        """deg^-1/2 on both ends (reference gcn_conv.py:32-40)."""
        ones = torch.ones(edge_index.shape[1], 1, device=edge_index.device)

        def dis(i):
            # the in-degree of every segment is its CSR count (the reference's sum of ones)
            deg = _seg(edge_index, i, size[i]).counts.to(ones.dtype).unsqueeze(1)
            return deg.clamp(min=1e-12).pow(-0.5)

        return dis(0), dis(1)

    def aggregate(self, src, edge_index, size, aggr=None):
        """aggr (add | mean) of the source rows over each destination's in-edges as one SpMM
        (mean: weight 1 / in-degree); max keeps the gather + segment-max kernels."""
        aggr = aggr or self.aggr
        if aggr == "max":
            return self.scatter(mp_ops.gather(src, edge_index[1]), edge_index, size, "max")
        w = None
        if aggr == "mean":
            seg = _seg(edge_index, 0, size[0])
            inv = 1.0 / seg.counts.clamp(min=1).float()
            w = inv[edge_index[0].long().clamp(min=0)]
        return mp_ops.weighted_aggregate(src, edge_index, size, w)

    def edge_weight(self, edge_index, size):
        """n0[dst] * n1[src] per edge (the symmetric GCN normalisation)."""
        if use_hip(edge_index) and edge_index.dim() == 2 and edge_index.dtype == torch.int64 \
                and edge_index.is_contiguous():
            # one launch over the two (cached) segment-count vectors; padding edges get 0
            c0 = _seg(edge_index, 0, size[0]).counts.long().contiguous()
            c1 = _seg(edge_index, 1, size[1]).counts.long().contiguous()
            return hip().gcn_norm_weight(edge_index, c0, c1)
        n0, n1 = self.norm(edge_index, size)
        return (mp_ops.gather(n0, edge_index[0]) * mp_ops.gather(n1, edge_index[1])).reshape(-1)

    def apply_edge(self, x_j):
        return x_j

    def apply_node(self, aggr_out):
        return aggr_out


def _pair(x):
    return list(x) if isinstance(x, (list, tuple)) else [x, None]


class GCNConv(Conv):
    def __init__(self, dim, **kwargs):
        super().__init__("add")
        self.fc = Dense(dim, use_bias=False)

    def forward(self, x, edge_index, size=None, **kwargs):
        x = _pair(x)
        src = x[1] if x[1] is not None else x[0]
        # deg^-1/2 on both ends folded into per-edge weights: one SpMM instead of three
        # gathers, a product and a scatter
        return self.fc(mp_ops.weighted_aggregate(src, edge_index, size, self.edge_weight(edge_index, size)))


class SAGEConv(Conv):
    """self_fc(x) + neigh_fc(mean_j x_j) (reference sage_conv.py:26-44).

    :meth:`fused_relu` is the fixed-fanout GPU form the GNN loops dispatch to when a block
    carries a dense neighbour matrix (SageDataFlow): gather + mean + both linears + ReLU
    in the K3 kernel (``sage_fwd``, csrc/hip/sage.hip: LDS-staged gather, bf16 MFMA,
    fp32 accumulation), backward through ``sage_bwd_scatter`` — no edge list, no
    segment reduce, no separate GEMMs."""

    fused_calls = 0  # class-wide counter of fused dispatches (tests / tracing)

    def __init__(self, dim, **kwargs):
        super().__init__("mean")
        self.self_fc = Dense(dim, use_bias=False)
        self.neigh_fc = Dense(dim, use_bias=False)

    def forward(self, x, edge_index, size=None, **kwargs):
        x = _pair(x)
        xs = x[1] if x[1] is not None else x[0]
        agg = self.aggregate(xs, edge_index, size)
        return self.self_fc(x[0]) + self.neigh_fc(agg)

    def can_fuse(self, x_all, block) -> bool:
        import os

        if block.nbr is None or not x_all.is_cuda or os.environ.get("EULER_AMD_FUSED_CONV", "1") == "0":
            return False
        if self.self_fc.has_uninitialized_params() or self.neigh_fc.has_uninitialized_params():
            return False  # the first (materialising) call takes the generic path
        return x_all.shape[1] <= 512

    def fused_relu(self, x_all, block):
        """relu(self_fc(x_all[res_n_id]) + neigh_fc(mean_j x_all[nbr[:, j]])) in one kernel.
        Widths that are not a multiple of the kernel's 16-column K step (e.g. 50-d input
        features) are zero-padded on x and on both weights' input columns."""
        from euler_amd.ops.sage_ops import sage_layer

        SAGEConv.fused_calls += 1
        xb, ws, wn = x_all.to(torch.bfloat16), self.self_fc.weight, self.neigh_fc.weight
        pad = -x_all.shape[1] % 16
        if pad:
            xb, ws, wn = F.pad(xb, (0, pad)), F.pad(ws, (0, pad)), F.pad(wn, (0, pad))
        w = torch.cat([ws, wn], 1)
        out = sage_layer(xb, block.res_n_id.to(torch.int32), block.nbr, w, None,
                         include_self=False, relu=True, disjoint=False)
        return out.to(x_all.dtype)


class GATConv(Conv):
    """Single-head GAT (reference gat_conv.py:41-78); the logits softmax per destination
    runs in the edge_softmax kernel."""

    def __init__(self, dim, improved=False, aggr="add", **kwargs):
        super().__init__(aggr)
        self.dim = dim
        self.improved = improved
        self.fc = Dense(dim, use_bias=False)
        self.att_i = Dense(1, use_bias=False)
        self.att_j = Dense(1, use_bias=False)

    def forward(self, x, edge_index, size=None, **kwargs):
        x = _pair(x)
        x = [None if t is None else self.fc(t) for t in x]
        if self.aggr == "add":
            # fused logits + edge softmax + weighted aggregation (gat.hip)
            xs = x[1] if x[1] is not None else x[0]
            out = gnn_ops.gat_aggregate(xs.unsqueeze(1), self.att_j(xs).float(), self.att_i(x[0]).float(),
                                        edge_index, size, 0.2).squeeze(1)
            return x[0] + out if self.improved else out
        gx = self.gather_feature([x], edge_index)[0]
        x_i, x_j = gx
        alpha = F.leaky_relu(self.att_i(x_i) + self.att_j(x_j), 0.2)
        alpha = mp_ops.scatter_softmax(alpha, _seg(edge_index, 0, size[0]), size[0])
        out = self.scatter(x_j * alpha.reshape(-1, 1), edge_index, size)
        if self.improved:
            out = x[0] + out
        return out


class TAGConv(Conv):
    def __init__(self, dim, K=3, **kwargs):
        super().__init__("add")
        self.K = K
        self.fc = Dense(dim, use_bias=False)

    def forward(self, x, edge_index, size=None, **kwargs):
        x = _pair(x)
        w = self.edge_weight(edge_index, size)
        xs = [x[0]]
        src = x[1] if x[1] is not None else x[0]
        for _ in range(self.K):
            xs.append(mp_ops.weighted_aggregate(src, edge_index, size, w))
        return self.fc(torch.cat(xs, -1))


class AGNNConv(Conv):
    def __init__(self, dim=None, **kwargs):
        super().__init__("add")
        self.beta = nn.Parameter(torch.ones(1))

    def forward(self, x, edge_index, size=None, **kwargs):
        x = _pair(x)
        norm = [None if t is None else F.normalize(t, dim=-1) for t in x]
        gx, gn = self.gather_feature([x, norm], edge_index)
        alpha = (self.beta * gn[0] * gn[1]).sum(-1, keepdim=True)
        alpha = mp_ops.scatter_softmax(alpha, _seg(edge_index, 0, size[0]), size[0])
        return self.scatter(gx[1] * alpha.reshape(-1, 1), edge_index, size)


class SGCNConv(Conv):
    def __init__(self, dim, K=1, **kwargs):
        super().__init__("add")
        self.K = K
        self.fc = Dense(dim, use_bias=False)

    def forward(self, x, edge_index, size=None, **kwargs):
        x = _pair(x)
        w = self.edge_weight(edge_index, size)
        out = x[0]
        src = x[1] if x[1] is not None else x[0]
        for _ in range(self.K):
            out = mp_ops.weighted_aggregate(src, edge_index, size, w)
        return self.fc(out)


class GINConv(Conv):
    def __init__(self, dim, mlp=None, eps=0.0, train_eps=True, **kwargs):
        super().__init__("add")
        self.mlp = mlp if mlp is not None else Dense(dim, use_bias=False)
        if train_eps:
            self.eps = nn.Parameter(torch.tensor([float(eps)]))
        else:
            self.register_buffer("eps", torch.tensor([float(eps)]))

    def forward(self, x, edge_index, size=None, **kwargs):
        x = _pair(x)
        src = x[1] if x[1] is not None else x[0]
        agg = self.aggregate(src, edge_index, size)
        return self.mlp((1 + self.eps) * x[0] + agg)


class GraphConv(Conv):
    def __init__(self, dim, **kwargs):
        super().__init__("mean")
        self.fc = Dense(dim, use_bias=False)
        self.liner = Dense(dim, use_bias=True)

    def forward(self, x, edge_index, size=None, **kwargs):
        x = _pair(x)
        src = x[1] if x[1] is not None else x[0]
        agg = self.aggregate(self.fc(src), edge_index, size)
        return self.liner(x[0]) + agg


class APPNPConv(Conv):
    def __init__(self, dim, K=10, alpha=0.1, **kwargs):
        super().__init__("add")
        self.K = K
        self.alpha = alpha

    def forward(self, x, edge_index, size=None, **kwargs):
        x = _pair(x)
        hidden = list(x)
        w = self.edge_weight(edge_index, size)
        cur = x
        out = x[0]
        for _ in range(self.K):
            src = cur[1] if cur[1] is not None else cur[0]
            out = mp_ops.weighted_aggregate(src, edge_index, size, w)
            out = out * (1 - self.alpha) + self.alpha * hidden[0]
            cur = [out, hidden[1]]
        return out


class ARMAConv(Conv):
    def __init__(self, dim, K=1, num_layers=1, shared_weights=False, act=F.relu, **kwargs):
        super().__init__("add")
        self.K, self.T, self.dim = K, num_layers, dim
        self.shared_weights = shared_weights
        self.act = act
        n = 1 if shared_weights else num_layers
        self.ws = nn.ModuleList([Dense(K * dim, use_bias=False) for _ in range(n)])
        self.vs = nn.ModuleList([Dense(K * dim, use_bias=False) for _ in range(n)])

    def forward(self, x, edge_index, size=None, **kwargs):
        x = _pair(x)
        origin = list(x)
        w = self.edge_weight(edge_index, size)
        cur = x
        out = None
        for t in range(self.T):
            k = 0 if self.shared_weights else t
            src = cur[1] if cur[1] is not None else cur[0]
            # W (A x) == A (W x): the linear runs on the source rows, not on every edge
            out = mp_ops.weighted_aggregate(self.ws[k](src), edge_index, size, w) + self.vs[k](origin[0])
            if self.act is not None:
                out = self.act(out)
            cur = [out, origin[1]]
        return out.reshape(-1, self.K, self.dim).mean(1)


class GroupDense(nn.Module):
    """Grouped linear (reference dna_conv.py GroupDense)."""

    def __init__(self, dim, groups=1, use_bias=True):
        super().__init__()
        self.dim, self.groups = dim, groups
        self.kernel = nn.UninitializedParameter()
        self.bias = nn.Parameter(torch.zeros(dim)) if use_bias else None

    def forward(self, x):
        if isinstance(self.kernel, nn.UninitializedParameter):
            self.kernel.materialize((self.groups, x.shape[-1] // self.groups, self.dim // self.groups),
                                    device=x.device)
            with torch.no_grad():
                nn.init.xavier_uniform_(self.kernel.view(-1, self.dim // self.groups))
        shp = x.shape
        xg = x.reshape(-1, self.groups, shp[-1] // self.groups).transpose(0, 1)
        out = torch.bmm(xg, self.kernel).transpose(0, 1).reshape(*shp[:-1], self.dim)
        return out + self.bias if self.bias is not None else out


def restricted_softmax(inputs, dim=-1, margin=0.0):
    m = inputs.max(dim=dim, keepdim=True).values.clamp(min=0)
    out = torch.exp(inputs - m)
    return out / (out.sum(dim=dim, keepdim=True) + torch.exp(margin - m))


class DNAConv(Conv):
    def __init__(self, dim, heads=1, groups=1, use_bias=True, **kwargs):
        super().__init__("mean")
        assert dim % heads == 0 and dim % groups == 0
        self.dim, self.heads, self.groups = dim, heads, groups
        self.in_fc = Dense(dim, use_bias=False)
        self.lin_q = GroupDense(dim, groups, use_bias)
        self.lin_k = GroupDense(dim, groups, use_bias)
        self.lin_v = GroupDense(dim, groups, use_bias)

    def multi_head(self, q, k, v):  # [E, 1, D]
        q, k, v = self.lin_q(q), self.lin_k(k), self.lin_v(v)
        E = q.shape[0]
        ch = self.dim // self.heads
        if q.shape[1] == 1 and k.shape[1] == 1:
            # one key per query (the conv's case): the attention products are per-head dot
            # products and a scale — elementwise over the edges instead of E tiny batched
            # matmuls (which dominated capacity-padded device blocks)
            qh, kh, vh = (t.reshape(E, self.heads, ch) for t in (q, k, v))
            s = restricted_softmax((qh * kh).sum(-1, keepdim=True) / math.sqrt(ch), dim=-1)
            return (s * vh).reshape(E, 1, self.dim)
        q = q.reshape(E, -1, self.heads, ch).transpose(1, 2)
        k = k.reshape(E, -1, self.heads, ch).transpose(1, 2)
        v = v.reshape(E, -1, self.heads, ch).transpose(1, 2)
        s = restricted_softmax(q @ k.transpose(-1, -2) / math.sqrt(ch), dim=-1)
        return (s @ v).transpose(1, 2).reshape(E, -1, self.dim)

    def forward(self, x, edge_index, size=None, **kwargs):
        x = _pair(x)
        x = [None if t is None else self.in_fc(t) for t in x]
        n0, n1 = self.norm(edge_index, size)
        gx, gn = self.gather_feature([x, [n0, n1]], edge_index)
        out = self.multi_head(gx[0].unsqueeze(1), gx[1].unsqueeze(1), gx[1].unsqueeze(1)).squeeze(1)
        return self.scatter(gn[0] * gn[1] * out, edge_index, size)


class _BasisCompose(torch.autograd.Function):
    """W [R, N*K] = coef [R, B] @ bases [B, N*K] and its gradients on the tiled MFMA GEMM"""

    @staticmethod
    def forward(ctx, coef, bases):
        ctx.save_for_backward(coef, bases)
        return gnn_ops.gemm(coef, bases)

    @staticmethod
    def backward(ctx, dw):
        coef, bases = ctx.saved_tensors
        dw = dw.contiguous().float()
        dcoef = gnn_ops.gemm(dw, bases, trans_b=True)
        dbases = gnn_ops.gemm(coef, dw, trans_a=True,
                              splits=gnn_ops._gemm_splits(coef.shape[0], -(-bases.shape[1] // 64)))
        return dcoef, dbases


class RelationConv(Conv):
    """R-GCN relation transform (reference relation_conv.py:33-73).  Instead of gathering
    an [E, dim, fea_dim] matrix per edge, edges are grouped by relation and each group
    does one GEMM.

    ``num_bases`` > 0 (an extension; the reference keeps one full matrix per relation):
    the basis decomposition of the R-GCN paper, W_r = sum_b a_rb V_b with B shared bases —
    rare relations of a power-law KG then share what the frequent ones learn instead of
    memorising their few triples.  :attr:`matrix` is then composed every forward (one GEMM)."""

    def __init__(self, fea_dim, dim, metapath=None, total_relation_num=1, num_bases=0, **kwargs):
        super().__init__("mean")
        self.fea_dim, self.dim, self.relation_num = fea_dim, dim, total_relation_num
        self.num_bases = int(num_bases)
        if self.num_bases > 0:
            self.bases = nn.Parameter(torch.empty(self.num_bases, dim, fea_dim))
            nn.init.kaiming_uniform_(self.bases.view(self.num_bases * dim, fea_dim), a=math.sqrt(5))
            self.coef = nn.Parameter(torch.randn(total_relation_num, self.num_bases) / math.sqrt(self.num_bases))
        else:
            self.matrix = nn.Parameter(torch.empty(total_relation_num, dim, fea_dim))
            nn.init.kaiming_uniform_(self.matrix.view(total_relation_num * dim, fea_dim), a=math.sqrt(5))
        self.fc = Dense(dim, use_bias=False)

    def relation_matrices(self):
        """[R, dim, fea_dim] relation transforms"""
        if self.num_bases == 0:
            return self.matrix
        if self.bases.is_cuda:
            w = _BasisCompose.apply(self.coef, self.bases.view(self.num_bases, -1))
        else:
            w = self.coef @ self.bases.view(self.num_bases, -1)
        return w.view(self.relation_num, self.dim, self.fea_dim)

    def forward(self, x, edge_index, size=None, edge_attr=None, **kwargs):
        assert edge_attr is not None
        x = _pair(x)
        src = x[1] if x[1] is not None else x[0]
        # relation-grouped MFMA GEMM with the gather and the mean aggregation fused (rgcn.hip)
        agg = gnn_ops.relation_transform(src, edge_attr, self.relation_matrices(), edge_index, size, "mean")
        fc, x0 = self.fc, x[0]
        if x0.is_cuda and x0.dim() == 2 and not fc.has_uninitialized_params() and fc.bias is None \
                and fc.activation is None:
            # self-loop transform on the tiled MFMA GEMM, bf16 operands like the relation
            # GEMMs (hipBLASLt ran it on a few 128 x 128 tiles)
            return gnn_ops.linear(x0, fc.weight) + agg.to(src.dtype)
        return fc(x0) + agg.to(src.dtype)


class GatedConv(Conv):
    """Gated graph conv with a stacked GRU (reference gated_graph_conv.py:26-60)."""

    def __init__(self, dim, processing_steps=2, lstm_layers=2, **kwargs):
        super().__init__("add")
        self.dim = dim
        self.steps = processing_steps
        self.layers = lstm_layers
        self.fc = nn.ModuleList([Dense(dim, use_bias=False) for _ in range(processing_steps)])
        self.cells = nn.ModuleList([nn.GRUCell(dim, dim) for _ in range(lstm_layers)])

    def forward(self, x, edge_index, size=None, **kwargs):
        h = _pair(x)
        out = None
        for i in range(self.steps):
            src = h[1] if h[1] is not None else h[0]
            m = mp_ops.gather(self.fc[i](src), edge_index[1])
            out = self.scatter(m, edge_index, size)
            state = h[0]
            inp = out
            for cell in self.cells:
                inp = cell(inp, state)
            out = inp
            h = [out, h[1]]
        return out


class MultiHeadGATConv(Conv):
    """All GAT heads in one pass (the reference builds ``head_num`` separate GATConv
    objects and concatenates, examples/gat/gat.py:56-70).

    One GEMM projects to ``[N, H*C]``; the ``[E, H]`` logits go through ONE
    edge-softmax launch (the kernel treats the H columns as independent softmaxes);
    one gather + one segment-sum aggregate every head.  ``concat=False`` averages the
    heads (the reference's reshape-then-mean over the feature axis is a bug, §2.10).
    """

    def __init__(self, dim, heads=1, concat=True, improved=False, negative_slope=0.2, **kwargs):
        super().__init__("add")
        if concat:
            assert dim % heads == 0, "dim must be divisible by heads when concat=True"
        self.heads, self.concat, self.improved = heads, concat, improved
        self.ch = dim // heads if concat else dim
        self.slope = negative_slope
        self.fc = Dense(heads * self.ch, use_bias=False)
        self.att_i = nn.Parameter(torch.empty(heads, self.ch))
        self.att_j = nn.Parameter(torch.empty(heads, self.ch))
        nn.init.xavier_uniform_(self.att_i)
        nn.init.xavier_uniform_(self.att_j)

    def forward(self, x, edge_index, size=None, **kwargs):
        x = _pair(x)
        H, Ch = self.heads, self.ch
        h_dst = self.fc(x[0])
        h_src = self.fc(x[1]) if x[1] is not None else h_dst
        a_i = (h_dst.view(-1, H, Ch).float() * self.att_i.float()).sum(-1)
        a_j = (h_src.view(-1, H, Ch).float() * self.att_j.float()).sum(-1)
        # one fused kernel: logits, per-head edge softmax and weighted aggregation (gat.hip)
        out = gnn_ops.gat_aggregate(h_src.view(-1, H, Ch), a_j, a_i, edge_index, size, self.slope)
        out = out.reshape(-1, H * Ch)
        if self.improved:
            out = out + h_dst
        if self.concat:
            return out
        return out.view(-1, H, Ch).mean(1)
