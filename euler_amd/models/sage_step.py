"""Fused supervised-GraphSAGE training step: ten gfx950 kernels per step, no autograd.

The same model as :class:`~euler_amd.models.fused_sage.FusedSupervisedGraphSage`
(reference ``examples/graphsage/graphsage.py:56-67``: two mean-SAGEConv hops + ReLU,
``fc`` with bias, ``out_fc`` without, sigmoid cross-entropy, Adam — the reference
runner's defaults ``tf_euler/python/utils/optimizers.py``), executed as::

    st_roots      alias-sample B roots (+ labels, Adam step++)        csrc/hip/sage_train.hip
    hop1, hop2    weighted neighbour sampling into the tree layout    csrc/hip/sampling.hip
    fwd L0        gather x + mean + MFMA + ReLU   -> h0, A0 (kt)      sage_train.hip
    fwd L1        gather h0 + mean + MFMA + ReLU  -> h1, A1 (kt)
    head          fc, out_fc, loss, dlogits, demb, dbfc, g1, dA1 = g1 W1
    route         dA1 -> tree routing -> ReLU mask -> g0 (kt)
    dW            grouped split-K MFMA: dW0, dW1, dWfc, dWout
    reduce        split-K partials -> flat gradient
    adam          flat Adam + bf16 (and transposed) weight shadows, RNG advance

Every buffer is allocated once; the whole step is hipGraph-capturable and replays
with fresh samples (the RNG counter lives on the device).  For data parallelism the
flat gradient is all-reduced between :meth:`forward_backward` and :meth:`optimizer_step`.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from euler_amd.models.fused_sage import FusedSupervisedGraphSage
from euler_amd.ops._native import hip

__all__ = ["FusedSageTrainer"]

_S_ROOTS, _S_HOP = 1, 16


def fm_to_dense(t: torch.Tensor) -> torch.Tensor:
    """Row-major view of a weight shadow stored in the kernels' fragment-major layout
    Wf[N/16][K/32][4][16][8] (sage_train.hip fm_off); ``t`` has the logical shape [N, K]."""
    N, K = t.shape
    return t.reshape(N // 16, K // 32, 4, 16, 8).permute(0, 3, 1, 2, 4).reshape(N, K)


class FusedSageTrainer:
    def __init__(self, graph, features: torch.Tensor, labels: torch.Tensor, batch_size: int, fanouts,
                 hidden_dim: int, label_dim: int, lr: float = 0.01, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, add_self_loops: bool = False, init_model: FusedSupervisedGraphSage = None):
        if len(fanouts) != 2:
            raise ValueError("the fused step implements the 2-hop model (fanouts [f1, f2])")
        dev = features.device
        if dev.type != "cuda":
            raise ValueError("FusedSageTrainer runs on the GPU")
        self.graph, self.features, self.labels = graph, features, labels
        if features.dtype != torch.bfloat16:
            raise ValueError("features must be bfloat16")
        if labels.dtype != torch.int16:
            raise ValueError("labels must be int16 class ids")
        B, (F1, F2) = int(batch_size), (int(fanouts[0]), int(fanouts[1]))
        D, H, C = features.shape[1], int(hidden_dim), int(label_dim)
        if B % 32 or D % 16 or H % 64 or C % 32:
            raise ValueError("need batch%32 == 0, feature_dim%16 == 0, hidden%64 == 0, label_dim%32 == 0")
        self.B, self.F1, self.F2, self.D, self.H, self.C = B, F1, F2, D, H, C
        self.M1 = B * (F1 + 1)
        self.include_self = bool(add_self_loops)
        self.lr, self.betas, self.eps, self.wd = float(lr), betas, float(eps), float(weight_decay)
        self.device = dev

        # ------------------------------------------------------------- parameters (flat fp32)
        model = init_model if init_model is not None else FusedSupervisedGraphSage(D, H, C, [F2, F1])
        sizes = [H * 2 * D, H * 2 * H, H * H, H, C * H]
        self.offsets = [0]
        for s in sizes:
            self.offsets.append(self.offsets[-1] + s)
        n = self.offsets[-1]
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(n, dtype=torch.float32, device=dev)
        self.m = torch.zeros(n, dtype=torch.float32, device=dev)
        self.v = torch.zeros(n, dtype=torch.float32, device=dev)
        with torch.no_grad():
            src = [model.conv_weights[0], model.conv_weights[1], model.fc.weight, model.fc.bias, model.out_fc.weight]
            for (a, b), t in zip(zip(self.offsets[:-1], self.offsets[1:]), src):
                self.flat[a:b].copy_(t.detach().reshape(-1).float())
        o = self.offsets
        self.W0 = self.flat[o[0]:o[1]].view(H, 2 * D)
        self.W1 = self.flat[o[1]:o[2]].view(H, 2 * H)
        self.Wfc = self.flat[o[2]:o[3]].view(H, H)
        self.bfc = self.flat[o[3]:o[4]]
        self.Wout = self.flat[o[4]:o[5]].view(C, H)
        self.gW0 = self.grad[o[0]:o[1]]
        self.gW1 = self.grad[o[1]:o[2]]
        self.gWfc = self.grad[o[2]:o[3]]
        self.gbfc = self.grad[o[3]:o[4]]
        self.gWout = self.grad[o[4]:o[5]]

        # bf16 shadows in the kernels' fragment-major layout (see fm_to_dense); same shapes
        bf = dict(dtype=torch.bfloat16, device=dev)
        self.W0b = torch.empty(H, 2 * D, **bf)
        self.W1b = torch.empty(H, 2 * H, **bf)
        self.W1T = torch.empty(2 * H, H, **bf)
        self.Wfcb = torch.empty(H, H, **bf)
        self.WfcT = torch.empty(H, H, **bf)
        self.Woutb = torch.empty(C, H, **bf)
        self.WoutT = torch.empty(H, C, **bf)
        self._sh = ([o[0], o[1], o[2], o[4]], [2 * D, 2 * H, H, H], [self.W0b, self.W1b, self.Wfcb, self.Woutb],
                    [None, self.W1T, self.WfcT, self.WoutT])
        self.refresh_shadows()

        # ------------------------------------------------------------- step buffers
        i32 = dict(dtype=torch.int32, device=dev)
        M1 = self.M1
        # Adam step = _stepbuf[1] (a 2-word buffer so rng_advance can bump it on the device)
        self._stepbuf = torch.zeros(2, dtype=torch.int64, device=dev)
        self.step_count = self._stepbuf[1:2]
        self._dummy_step = torch.zeros(1, dtype=torch.int64, device=dev)
        # sample buffers, double-buffered: with pipelined sampling (EULER_AMD_PIPELINE_SAMPLING=1)
        # the roots and both hops of step t+1 are drawn on a side stream while step t's kernels
        # run (sampling does not depend on the weights), joined before the optimizer so the RNG
        # counter advance stays ordered after them.  Measured on MI355X (100M nodes, B=1024,
        # hipGraph): 0.1275 ms/step pipelined vs 0.1222 ms serial -- the latency-bound sampling
        # gathers slow the concurrent forward more than they save, so serial is the default
        self._sets = []
        for _ in range(2):
            level1 = torch.empty(M1, **i32)
            self._sets.append(dict(roots=torch.empty(B, **i32), level1=level1, nb1=level1[: B * F1],
                                   nb2=torch.empty(M1, F2, **i32), label_idx=torch.empty(B, **i32)))
        self.pipelined = os.environ.get("EULER_AMD_PIPELINE_SAMPLING", "0") == "1"
        self._cur = 0          # set holding the samples of the next forward_backward
        self._primed = False   # pipelined: set _cur has been sampled
        self._side = torch.cuda.Stream(device=dev) if self.pipelined else None
        self._join = None
        self._bind(0)
        self.h0 = torch.empty(M1, H, **bf)
        self.A0_kt = torch.empty(M1 * 2 * D, **bf)
        self.A1 = torch.empty(B, 2 * H, **bf)
        self.A1_kt = torch.empty(B * 2 * H, **bf)
        self.h1_kt = torch.empty(B * H, **bf)
        self.emb_kt = torch.empty(B * H, **bf)
        self.dlog_kt = torch.empty(B * C, **bf)
        self.demb_kt = torch.empty(B * H, **bf)
        self.g1_kt = torch.empty(B * H, **bf)
        self.dA1 = torch.empty(B, 2 * H, dtype=torch.float32, device=dev)
        # outer-layer gradient g0: the route kernel materialises it in kt layout from dA1, the
        # tree layout and the forward's ReLU mask bits.  EULER_AMD_FUSE_ROUTE=1 instead rebuilds
        # g0 fragments inside the dW kernel (no g0 round trip, but 8 scalar loads per MFMA
        # operand: measured 105 us vs 19 + 19 us for route + dW on MI355X, so off by default)
        self.fuse_route = F1 >= 2 and os.environ.get("EULER_AMD_FUSE_ROUTE", "0") == "1"
        self.mask0 = torch.empty((M1 // 32) * H, **i32)
        self.g0_kt = None if self.fuse_route else torch.empty(M1 * H, **bf)
        self.loss_acc = torch.zeros(1, dtype=torch.float32, device=dev)
        self.loss_out = torch.zeros(1, dtype=torch.float32, device=dev)
        # split-K plan: ~1024 reduction rows per workgroup (tunable for sweeps)
        kps = int(os.environ.get("EULER_AMD_DW_KPS", "32"))
        self._dw = [  # (G_kt, X_kt, P, Q, M)
            (self.g0_kt, self.A0_kt, H, 2 * D, M1),
            (self.g1_kt, self.A1_kt, H, 2 * H, B),
            (self.demb_kt, self.h1_kt, H, H, B),
            (self.dlog_kt, self.emb_kt, C, H, B),
        ]
        self._splits = [-(-(m // 32) // kps) for (_, _, _, _, m) in self._dw]
        self._kps = kps
        self.parts = [torch.empty(s * p * q, dtype=torch.float32, device=dev)
                      for s, (_, _, p, q, _) in zip(self._splits, self._dw)]
        self._grad_views = [self.gW0, self.gW1, self.gWfc, self.gWout]
        self.bm0 = int(os.environ.get("EULER_AMD_BM0", "32"))  # rows per block of the outer layer

    # ------------------------------------------------------------------ kernels
    def refresh_shadows(self):
        """Rebuild the bf16 weight shadows from the fp32 flat parameters (after an
        external write such as the data-parallel broadcast)."""
        hip().st_shadow(self.flat, *self._sh)

    def _bind(self, i):
        st = self._sets[i]
        self.roots, self.level1, self.nb1, self.nb2, self.label_idx = (st["roots"], st["level1"], st["nb1"],
                                                                        st["nb2"], st["label_idx"])

    def sample(self, i=None, step=None):
        """roots + both hops into sample set ``i`` (default: the bound one)."""
        st = self._sets[self._cur if i is None else i]
        g, h = self.graph, hip()
        h.st_roots(g.node_prob, g.node_alias, g.rng, _S_ROOTS, self.labels, st["roots"], st["level1"],
                   st["label_idx"], self.step_count if step is None else step)
        h.sample_neighbor_into(g.indptr, g.nbr, g.cumw, g.num_rows, g.num_types, -1, st["roots"], self.F1, -1, g.rng,
                               _S_HOP, st["nb1"])
        h.sample_neighbor_into(g.indptr, g.nbr, g.cumw, g.num_rows, g.num_types, -1, st["level1"], self.F2, -1,
                               g.rng, _S_HOP + 1, st["nb2"])

    def forward_backward(self, phase: str = "all"):
        """One step's sampling, forward and backward into :attr:`grad`.

        ``phase`` splits the step for data parallelism with overlapped gradient sync:
        ``"head"`` ends once the gradients of W1 / fc / out_fc (:attr:`grad_bucket_head`,
        77 % of the bytes) are final, ``"outer"`` then computes the outer layer's dW0
        (:attr:`grad_bucket_outer`), so the all-reduce of the first bucket runs while the
        second is computed.  ``"all"`` = both, with one grouped dW launch."""
        if phase in ("all", "head"):
            self._forward_and_head()
        if phase == "all":
            self._dw_reduce([0, 1, 2, 3])
        elif phase == "head":
            self._dw_reduce([1, 2, 3])
        elif phase == "outer":
            self._dw_reduce([0])
        else:
            raise ValueError("phase must be all | head | outer")
        if phase in ("all", "outer") and self._join is not None:
            # the optimizer advances the RNG counter: the next step's draws must precede it
            torch.cuda.current_stream(self.device).wait_event(self._join)
            self._join = None

    def _forward_and_head(self):
        h = hip()
        use = self._cur
        self._bind(use)
        self._join = None
        if not self.pipelined:
            self.sample(use)
        else:
            if not self._primed:  # first step: this step's own samples, in order, then a counter
                self.sample(use, self._dummy_step)  # advance so the side-stream draws below differ
                hip().rng_advance(self.graph.rng, 1)
                self._primed = True
            # next step's samples on the side stream, concurrent with this step's kernels
            # (set 1-use was last read by the previous step, which precedes this fork)
            main = torch.cuda.current_stream(self.device)
            fork = torch.cuda.Event()
            fork.record(main)
            self._side.wait_event(fork)
            with torch.cuda.stream(self._side):
                self.sample(1 - use, self._dummy_step)
                self._join = torch.cuda.Event()
                self._join.record(self._side)
            self._cur = 1 - use
        h.st_sage_fwd(self.features, self.level1, self.nb2, self.F2, self.include_self, self.W0b, self.h0,
                      self.A0_kt, self.mask0, self.bm0)
        # inner hop: tree layout, neighbours of root t are level-1 rows t*F1 .. t*F1+F1-1; its
        # GEMM (h1 = relu(A1 W1^T)) runs inside the head kernel
        h.st_tree_mean(self.h0, self.B, self.F1, self.include_self, self.A1)
        h.st_head(self.A1, self.W1b, self.Wfcb, self.WfcT, self.bfc, self.Woutb, self.WoutT, self.W1T,
                  self.label_idx, self.A1_kt, self.h1_kt, self.emb_kt, self.dlog_kt, self.demb_kt, self.g1_kt,
                  self.dA1, self.gbfc, self.loss_acc)

    def _dw_reduce(self, probs):
        """grouped split-K dW of the listed problems (0 = outer layer W0, routed from dA1)
        and their split-K reduction into the flat gradient"""
        h = hip()
        dw = [self._dw[i] for i in probs]
        route = 0 in probs
        if route and not self.fuse_route:
            h.st_route(self.dA1, self.F1, self.include_self, self.mask0, self.g0_kt)
        fused = route and self.fuse_route
        h.st_dw([d[0] for d in dw], [d[1] for d in dw], [self.parts[i] for i in probs], [d[2] for d in dw],
                [d[3] for d in dw], [d[4] for d in dw], [self._kps] * len(probs), self.mask0 if fused else None,
                self.dA1 if fused else None, self.F1 if fused else 0, self.include_self if fused else False)
        h.st_reduce([self.parts[i] for i in probs], [self._grad_views[i] for i in probs],
                    [self._splits[i] for i in probs])

    @property
    def grad_bucket_head(self) -> torch.Tensor:
        """W1, fc (weight + bias) and out_fc gradients: final after phase "head"."""
        return self.grad[self.offsets[1]:self.offsets[5]]

    @property
    def grad_bucket_outer(self) -> torch.Tensor:
        """W0 gradient: final after phase "outer"."""
        return self.grad[self.offsets[0]:self.offsets[1]]

    def optimizer_step(self, grad_scale: float = 1.0):
        o = self.offsets
        if self.pipelined:
            hip().rng_advance(self._stepbuf, 1)  # Adam step++ (st_roots did it in the serial order)
        hip().st_adam(self.flat, self.grad, self.m, self.v, self.step_count, self.lr, self.betas[0], self.betas[1],
                      self.eps, self.wd, float(grad_scale), *self._sh, o[3], o[4] - o[3], self.loss_acc,
                      self.loss_out, self.graph.rng)

    def step(self):
        self.forward_backward()
        self.optimizer_step()

    @property
    def parity(self) -> int:
        """Sample set the next step computes on.  A captured hipGraph bakes in the set it
        was captured with, so with pipelined sampling capture one graph per parity and
        replay ``graphs[trainer.parity]``, then call :meth:`advance_parity`."""
        return self._cur if self.pipelined else 0

    def advance_parity(self):
        if self.pipelined:
            self._cur = 1 - self._cur

    @property
    def loss(self) -> torch.Tensor:
        """loss of the last completed step (device scalar)."""
        return self.loss_out

    # ------------------------------------------------------------------ fp32 oracle
    def reference_forward_backward(self):
        """Recompute the current step's loss and parameter gradients with fp32 torch
        autograd on the SAME sampled indices and parameters (numerics oracle)."""
        B, F1, F2, H = self.B, self.F1, self.F2, self.H
        ps = [t.detach().clone().requires_grad_(True) for t in (self.W0, self.W1, self.Wfc, self.bfc, self.Wout)]
        W0, W1, Wfc, bfc, Wout = ps
        x = torch.cat([self.features.float(), torch.zeros(1, self.D, device=self.device)], 0)
        n = self.features.shape[0]  # row n of x is the zero row for padding (-1) ids
        lv1 = self.level1.long()
        nb2 = self.nb2.long()
        lv1z = torch.where(lv1 < 0, torch.full_like(lv1, n), lv1)
        nb2z = torch.where(nb2 < 0, torch.full_like(nb2, n), nb2)
        xs = x[lv1z]
        agg = x[nb2z].sum(1)
        cnt = F2
        if self.include_self:
            agg, cnt = agg + xs, cnt + 1
        h0 = torch.relu(torch.cat([xs, agg / cnt], 1) @ W0.t())
        s1 = h0[B * F1:]
        a1 = h0[: B * F1].view(B, F1, H).sum(1)
        c1 = F1
        if self.include_self:
            a1, c1 = a1 + s1, c1 + 1
        h1 = torch.relu(torch.cat([s1, a1 / c1], 1) @ W1.t())
        emb = h1 @ Wfc.t() + bfc
        logits = emb @ Wout.t()
        y = torch.zeros_like(logits)
        y.scatter_(1, self.labels[self.roots.long()].long().view(-1, 1), 1.0)
        loss = F.binary_cross_entropy_with_logits(logits, y)
        loss.backward()
        return float(loss), [p.grad.reshape(-1) for p in ps]
