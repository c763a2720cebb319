"""R-GCN encoder + TransE decoder (BASELINE config 5) and its fused training step.

Model (reference ``examples/rgcn/rgcn.py:30-105`` RelationConv encoder,
``examples/TransX/transE.py`` / ``transX.py:63-145`` margin loss):

    h_0 = entity table [Ne, D]
    h_{l+1} = act(mean_{e: dst(e) = i} W_{rel(e)} h_l[src(e)] + h_l W_self^T)    (RelationConv)
    loss    = mean_i relu(margin + mean_k score(corruption_ik) - score(triple_i))

with TransE-l2 scores on l2-normalised rows and both front and tail corruptions.

:class:`RgcnTransE` is the plain autograd module (``forward`` = one loss).
:class:`RgcnTransEStep` runs the same step — triple / corruption draws, encoder, loss,
backward, optimizer — as hand-written launches only, for hipGraph capture:

* draws: ``kg_step`` (embed.hip K10b) picks the B triples and K corruptions per triple with
  Philox(seed, optimizer step, row) inside the scoring kernel;
* encoder: per layer one bf16 cast, ``rel_weight_bf16`` (both W and W^T operands),
  ``rel_gemm`` (relation-grouped MFMA GEMM, gather fused), the per-destination mean
  (``segment_reduce_wave``) and the self-loop GEMM with the relation aggregate added in its
  epilogue (gemm.hip ``addend``; relu fused for inner layers);
* backward: ``kg_step``'s backward kernel writes d loss / d h (atomics into a zeroed buffer)
  and d loss / d rel straight into the relation table's flat-gradient view; per layer the
  transposed relation GEMM + source sums, one GEMM for d h_l = dH W_self + relation part
  (relu' of the layer input fused as the rmask), the split-K self-loop weight gradient and
  ``rel_gemm_dw`` into the relation weights' flat-gradient view;
* the flat optimizer (one launch, plus the step-count increment for large buffers).

Basis-decomposed relations (``num_bases`` > 0) compose W = coef @ bases with one GEMM per
layer and step and take d coef / d bases from the composed dW with two more; self-loop
dropout draws its per-row keep mask with Philox(seed, step, layer) (``drop_rows``) and
scales the self-loop product's rows with it in the backward GEMM's epilogue.

``deterministic=True`` (or ``EULER_AMD_DETERMINISTIC=1``) makes the step atomic-free and
bit-reproducible: the scoring backward writes one gradient row per entity / relation
occurrence (and its row key; a triple whose margin holds writes none), summed per row in
occurrence order (``det_occ``: counted CSR whose lists one wave sorts, then
``det_segment_sum``, one block per row), and the relation-weight gradient of a relation with several
edge chunks is added from per-chunk slabs in chunk order (``rel_gemm_dw`` slot mode).

No torch elementwise kernel runs in the default step; gradients are zeroed with one memset.  The
draws come from a different generator than ``torch.randint`` (Philox keyed by the
optimizer's device step count), so the batch stream differs from the autograd path's;
the step's loss and gradients on the same batch match it (tests/test_kg_step.py).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

import os

from euler_amd.convolution import RelationConv
from euler_amd.ops import gnn_ops
from euler_amd.ops._native import hip

__all__ = ["RgcnTransE", "RgcnTransEStep"]


class RgcnTransE(nn.Module):
    """entity / relation tables, ``layers`` RelationConvs, TransE-l2 margin loss"""

    self_drop = 0.0  # training: probability of dropping an entity's own (self-loop) input
    self_keep = None  # evaluation: [Ne] bool, entities whose own embedding is used (None: all)
    norm = True

    def __init__(self, num_ent, num_rel, dim, layers=1, margin=1.0, num_bases=0):
        super().__init__()
        self.ent = nn.Parameter(torch.randn(num_ent, dim) * 0.1)
        self.rel = nn.Parameter(torch.randn(num_rel, dim) * 0.1)
        self.convs = nn.ModuleList([RelationConv(dim, dim, total_relation_num=num_rel, num_bases=num_bases)
                                    for _ in range(layers)])
        self.margin = margin

    def encode(self, edge_index, edge_rel):
        n = self.ent.shape[0]
        h = self.ent
        for i, conv in enumerate(self.convs):
            x0 = h
            if self.training and self.self_drop > 0:
                # self-loop dropout (the R-GCN paper drops self-loop edges more than others):
                # an entity whose own input is dropped must be placed by its neighbours, so the
                # relation transforms learn to carry type information (inductive use)
                x0 = h * (torch.rand(n, 1, device=h.device) >= self.self_drop).to(h.dtype)
            elif not self.training and self.self_keep is not None:
                x0 = h * self.self_keep.view(n, 1).to(h.dtype)
            h = conv([x0, h], edge_index, (n, n), edge_attr=edge_rel)
            if i + 1 < len(self.convs):
                h = F.relu(h)
        return h

    def forward(self, edge_index, edge_rel, src, rel, dst, negs):
        h = self.encode(edge_index, edge_rel).float()
        pos, neg = gnn_ops.kg_score(h, self.rel, src, dst, rel, negs, "l2", "both", self.norm)
        return F.relu(self.margin + neg.mean(-1) - pos).mean()


class RgcnTransEStep:
    """The fused step of an :class:`RgcnTransE` whose parameters live in ``flat``
    (:class:`~euler_amd.parallel.flat.FlatParams`, updated by ``opt``).

    ``triples`` = (src, rel, dst) int64 device tensors of the training triples, ``pool``
    the rows of them the loss draws from; ``edge_index`` [2, E] (row 0 destination) and
    ``edge_rel`` [E] the encoder graph.  ``grad_sync`` (optional) all-reduces the flat
    gradient between backward and update and returns the gradient scale."""

    def __init__(self, model: RgcnTransE, flat, opt, edge_index, edge_rel, triples, pool, batch: int,
                 num_negs: int, seed: int = 0, grad_sync=None, deterministic=None):
        dev = model.ent.device
        if dev.type != "cuda":
            raise ValueError("the fused KG step runs on the GPU")
        self.model, self.flat, self.opt = model, flat, opt
        self.grad_sync = grad_sync
        self.N, self.D = model.ent.shape
        self.R = model.rel.shape[0]
        self.B, self.K = int(batch), int(num_negs)
        if self.D % 8 != 0 or self.D > 256:
            raise ValueError("the fused KG step needs dim % 8 == 0 and dim <= 256")
        self.seed = int(seed) & ((1 << 63) - 1)
        self.margin = float(model.margin)
        self.normalize = bool(model.norm)
        t_src, t_rel, t_dst = (t.reshape(-1).long().contiguous() for t in triples)
        self.pool = pool.reshape(-1).long().contiguous()
        # the kernels index without range checks: validate the tables once, here
        T = t_src.numel()
        if not (t_rel.numel() == T and t_dst.numel() == T and self.pool.numel() > 0):
            raise ValueError("triple tables of different lengths or an empty pool")
        for name, t, hi in (("src", t_src, self.N), ("dst", t_dst, self.N), ("rel", t_rel, self.R),
                            ("pool", self.pool, T)):
            if int(t.min()) < 0 or int(t.max()) >= hi:
                raise ValueError(f"triple {name} ids out of range [0, {hi})")
        self.t_src, self.t_rel, self.t_dst = t_src, t_rel, t_dst
        self.layers = []
        self.drop = float(model.self_drop)
        n = self.N
        params = [model.ent, model.rel]
        for conv in model.convs:
            if conv.fc.has_uninitialized_params() or conv.fc.bias is not None or conv.fc.activation is not None:
                raise ValueError("the fused KG step needs a bias-free, materialised self-loop fc")
            Wfc = conv.fc.weight
            if tuple(Wfc.shape) != (self.D, self.D):
                raise ValueError("the fused KG step needs square [dim, dim] layers")
            tiles = gnn_ops.relation_tiles(edge_index, edge_rel, (n, n), self.R, self.D, self.D, "mean")
            # the relation matrices: a parameter, or composed from bases every step (coef @ bases)
            basis = (conv.coef, conv.bases) if conv.num_bases > 0 else None
            self.layers.append((conv.matrix if basis is None else None, Wfc, tiles, basis))
            params += [Wfc] + ([conv.matrix] if basis is None else list(basis))
        for p in params:
            if p.grad is None or not p.grad.is_contiguous():
                raise ValueError("every parameter needs its flat-gradient view (FlatParams)")
        L = len(self.layers)
        f32 = dict(device=dev, dtype=torch.float32)
        nb = sum(1 for lay in self.layers if lay[3] is not None)
        # composed relation matrices and their gradient (basis layers; one buffer pair, reused)
        self.Wc = torch.empty(self.R, self.D, self.D, **f32) if nb else None
        self.dWc = torch.empty(self.R, self.D, self.D, **f32) if nb else None
        # self-loop dropout: the masked layer input and its per-row keep mask
        self.x0 = [torch.empty(self.N, self.D, **f32) for _ in range(L)] if self.drop > 0 else None
        self.keep = [torch.empty(self.N, **f32) for _ in range(L)] if self.drop > 0 else None
        bf = dict(device=dev, dtype=torch.bfloat16)
        i64 = dict(device=dev, dtype=torch.int64)
        self.xb = [torch.empty(self.N, self.D, **bf) for _ in range(L)]
        self.h = [torch.empty(self.N, self.D, **f32) for _ in range(L)]
        self.dh = [torch.empty(self.N, self.D, **f32) for _ in range(L)]
        self.gb = torch.empty(self.N, self.D, **bf)
        E = max((lay[2].num_edges for lay in self.layers), default=0)
        self.msg = torch.empty(max(E, 1), self.D, **bf)
        self.o_src = torch.empty(self.B, **i64)
        self.o_dst = torch.empty(self.B, **i64)
        self.o_rel = torch.empty(self.B, **i64)
        self.o_neg = torch.empty(self.B, self.K, **i64)
        self.coef = torch.empty(self.B, **f32)
        self.part = torch.empty(int(hip().kg_step_parts(self.B, self.D)), **f32)
        self.loss = torch.zeros(1, **f32)
        # relation-gradient replicas for the backward scoring kernel's hot relations
        # (EULER_AMD_KG_REL_REP=0: add straight into the relation table's gradient)
        rep = int(os.environ.get("EULER_AMD_KG_REL_REP", "16"))
        self.drel_rep = torch.empty(rep, self.R, self.D, **f32) if rep > 0 else None
        self._fc_splits = gnn_ops._gemm_splits(self.N, -(-self.D // 64) ** 2)
        if deterministic is None:
            deterministic = os.environ.get("EULER_AMD_DETERMINISTIC", "0") == "1"
        self.deterministic = bool(deterministic)
        if self.deterministic:
            # atomic-free backward: the scoring kernel writes one gradient row per entity /
            # relation occurrence, summed per row in a fixed order (occurrences stably sorted
            # by row, wave-per-row segment sums); multi-chunk relations store per-chunk dW
            # slabs, added in chunk order (rel_gemm_dw slot mode)
            nocc = self.B * (2 + self.K)
            self.occ_e = torch.empty(nocc, self.D, **f32)
            self.occ_r = torch.empty(self.B, self.D, **f32)
            self.key_e = torch.empty(nocc, **i64)
            self.key_r = torch.empty(self.B, **i64)
            slots = max((lay[2].det_slots()[3] for lay in self.layers), default=0)
            self.dw_part = torch.empty(max(slots, 1), self.D, self.D, **f32)

    # ------------------------------------------------------------------ step
    def _relation_matrices(self, li):
        W, _, _, basis = self.layers[li]
        if basis is None:
            return W.detach()
        coef, bases = basis
        B = bases.shape[0]
        gnn_ops.gemm(coef.detach(), bases.detach().view(B, -1), out=self.Wc.view(self.R, -1))
        return self.Wc

    _check = os.environ.get("EULER_AMD_KG_STEP_CHECK", "0") == "1"  # eager debugging: finiteness per stage

    def _chk(self, stage, *ts):
        if self._check and not all(bool(torch.isfinite(t).all()) for t in ts):
            raise FloatingPointError(f"fused KG step {int(self.opt.step_count.item())}: non-finite after {stage}")

    def forward_backward(self):
        """draws, encoder, loss and every gradient into the flat gradient buffer"""
        H = hip()
        m = self.model
        self._chk("previous update", self.flat.flat)
        H.zero_(self.flat.grad)
        x = m.ent.detach()
        saved = []
        L = len(self.layers)
        for li, (_, Wfc, tiles, _) in enumerate(self.layers):
            H.cast_bf16(x, self.xb[li])
            wb, wt = H.rel_weight_bf16(self._relation_matrices(li))
            tr, ts, tl = tiles.tiles()
            msg = self.msg[: tiles.num_edges]
            H.rel_gemm(self.xb[li], tiles.src, tr, ts, tl, wb, None, tiles.slot_dst, 0, tiles.tile, msg)
            agg = gnn_ops._seg_sum(msg, tiles.dst_seg.indptr, 1)
            x0 = x
            if self.drop > 0:
                # self-loop dropout (RgcnTransE.encode): the self term of a dropped row is 0
                x0 = self.x0[li]
                H.drop_rows(x, self.drop, self.seed ^ 0x5E1F, self.opt.step_count, li, x0, self.keep[li])
            gnn_ops.gemm(x0, Wfc.detach(), out=self.h[li], trans_b=True, addend=agg, relu=li + 1 < L)
            self._chk("layer %d forward" % li, agg, self.h[li], wb)
            saved.append((x, x0, wt))
            x = self.h[li]
        dtop = m.ent.grad if L == 0 else self.dh[L - 1]
        if L:
            H.zero_(dtop)
        occ = (self.occ_e, self.occ_r, self.key_e, self.key_r) if self.deterministic else (None,) * 4
        H.kg_step(x, m.rel.detach(), self.pool, self.t_src, self.t_dst, self.t_rel, self.opt.step_count, self.seed,
                  gnn_ops.KG_KINDS["l2"], self.normalize, self.margin, self.o_src, self.o_dst, self.o_rel, self.o_neg,
                  self.coef, self.part, self.loss, dtop, m.rel.grad, self.drel_rep, *occ)
        if self.deterministic:
            self._occurrence_sums(dtop, m.rel.grad)
        self._chk("scores", dtop, m.rel.grad, self.loss)
        for li in range(L - 1, -1, -1):
            W, Wfc, tiles, basis = self.layers[li]
            x_l, x0_l, wt = saved[li]
            g = self.dh[li]
            H.cast_bf16(g, self.gb)
            tr, ts, tl = tiles.tiles()
            msg = self.msg[: tiles.num_edges]
            H.rel_gemm(self.gb, tiles.dst, tr, ts, tl, wt, tiles.scale, tiles.slot_src, 0, tiles.tile, msg)
            dxr = gnn_ops._seg_sum(msg, tiles.src_seg.indptr, 0)
            out = m.ent.grad if li == 0 else self.dh[li - 1]
            # d h_l = keep * (dH W_self) + relation part, times relu'(h_l) below the top layer
            gnn_ops.gemm(g, Wfc.detach(), out=out, addend=dxr, rmask=x_l if li > 0 else None,
                         row_scale=self.keep[li] if self.drop > 0 else None)
            gnn_ops.gemm(g, x0_l, out=Wfc.grad, trans_a=True, splits=self._fc_splits)
            self._chk("layer %d input gradients" % li, dxr, out, Wfc.grad)
            cr, cs, cl = tiles.chunks()
            det = {}
            if self.deterministic:
                slot, mrel, mrp, _ = tiles.det_slots()
                det = dict(slot=slot, part=self.dw_part, mrel=mrel, mrp=mrp)
            if basis is None:
                H.rel_gemm_dw(self.gb, tiles.dst, self.xb[li], tiles.src, tiles.scale, cr, cs, cl, tiles.chunk_solo,
                              W.grad, accumulate=False, **det)
                continue
            # dW of the composed matrices, then d coef = dW bases^T, d bases = coef^T dW
            coef, bases = basis
            nbs = bases.shape[0]
            H.zero_(self.dWc)
            H.rel_gemm_dw(self.gb, tiles.dst, self.xb[li], tiles.src, tiles.scale, cr, cs, cl, tiles.chunk_solo,
                          self.dWc, accumulate=False, **det)
            dw = self.dWc.view(self.R, -1)
            sp = int(os.environ.get("EULER_AMD_KG_DCOEF_SPLITS", "0")) or \
                gnn_ops._gemm_splits(dw.shape[1], -(-self.R // 64))
            gnn_ops.gemm(dw, bases.detach().view(nbs, -1), out=coef.grad, trans_b=True, splits=sp)
            gnn_ops.gemm(coef.detach(), dw, out=bases.grad.view(nbs, -1), trans_a=True,
                         splits=gnn_ops._gemm_splits(self.R, -(-dw.shape[1] // 64)))
            self._chk("layer %d basis gradients" % li, self.dWc, coef.grad, bases.grad)
        return self.loss

    def _occurrence_sums(self, dent, drel):
        """deterministic mode: d h and d rel as fixed-order sums of the scoring kernel's
        occurrence rows (keyed by the kernel: [h, t, neg_0 .. neg_{K-1}] per triple, one
        relation row per triple, -1 for triples without gradient); each row's occurrences
        are summed in occurrence order (det_occ: counted CSR, lists sorted in one wave)"""
        H = hip()
        for keys, S, occ, out in ((self.key_e, self.N, self.occ_e, dent), (self.key_r, self.R, self.occ_r, drel)):
            ptr, perm = H.det_occ(keys, S)
            H.det_segment_sum(occ, ptr, perm, out)

    def keep_masks(self):
        """per-layer [N] keep masks of the last step's self-loop dropout (None without)"""
        return self.keep

    def optimizer_step(self):
        scale = 1.0
        if self.grad_sync is not None:
            s = self.grad_sync(self.flat.grad)
            scale = 1.0 if s is None else float(s)
        self.opt.step(scale)

    def step(self):
        self.forward_backward()
        self.optimizer_step()
        return self.loss

    def batch(self):
        """(src, rel, dst, negs) of the last step's draws"""
        return self.o_src, self.o_rel, self.o_dst, self.o_neg
