"""Fused device-path training step for SupervisedGCN-shaped models (GCN over the
full-neighbourhood flow): one fixed sequence of hand-written gfx950 launches per step
(``csrc/hip/gcn.hip``, plan ``csrc/hip/binding_gcn.cpp``), captured in hipGraphs like every
other device trainer.

Reference model: ``examples/gcn/gcn.py:52-58`` — ``GNN('gcn', 'full', dims)`` over
``tf_euler/python/dataflow/gcn_dataflow.py:26-48`` (every hop's full neighbourhood, unique,
self loops), ``convolution/gcn_conv.py:26-54`` (``fc(sum_e deg_t^-1/2 deg_s^-1/2 x_s)``),
ReLU after each conv, ``fc`` + ``out_fc`` and the sigmoid cross-entropy of
``mp_utils/base.py:24-47``.

What one step launches (L = 2 convs; 3 L + 4 = 10 on one process, the flat optimizer
folded into the reduce; 11 with a data-parallel all-reduce between them):

* per hop: expand (hop 0's also draws the roots: the alias table on Philox stream 1 of the
  graph's (seed, counter), the same draw as ``alias_sample``; degrees, look-back scan,
  neighbour list, one counter atomic per edge whose first taker claims the node), mark (positions of the new nodes), place (edge
  sources, in-block source counts from the claimers);
* the outer conv: edge-parallel aggregation + MFMA linear + ReLU;
* the head: last conv, fc, out_fc, loss, F1 counts and the whole row-local backward, the
  weight-gradient partials of its rows and d(agg) of the roots;
* d(W0) partials as one GEMM over hop 0's edges (the ReLU mask is per source row, so
  d(h1) is never formed: no scatter); the reduce into the flat gradient (+ loss, counts,
  RNG counter) — on one process it also applies the flat optimizer to every element it
  sums (``optim_math.h``; the head launch advances FlatOptimizer's step count first);
* with data parallelism: the all-reduce, then the flat optimizer launch
  (``parallel/flat.py``).

The generic path (``models/full_trainer.py``) runs the user's convolution modules on
``DeviceFullFlow`` blocks: ~100 launches per step.  Both draw the same roots from the same
graph RNG state and build the same node sets (in a different order: here each set is the
previous one followed by its new neighbours in claim order), so their losses agree to bf16
rounding;
``tests/test_gcn_trainer.py`` checks that and an fp32 oracle.

FastGCN (``examples/fastgcn``: the same convs over ``fast_dataflow.py:25-57``) takes the same
launches plus one per sampled hop: ``gcn_layer_draw`` stamps the step's layer (the generic
``DeviceLayerFlow``'s ``sample_node`` draw) and that hop's expand keeps only the edges into
it (per target: the kept count for the offsets, then one wave per target compacts its
neighbour list with a ballot).

Capacities: the flow's edge / node-set caps come from ``dataflow/device_flow.py``
(``"bounded"`` by default through the estimator); a batch beyond them sets the overflow
word, and the estimator rolls the chunk back, grows the caps and re-plans.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from euler_amd.dataflow.device_flow import bounded_caps, exact_caps, _bounded_args, _round_up
from euler_amd.models.captured import CapturedTrainer
from euler_amd.ops._native import hip

__all__ = ["GcnTrainer", "GcnFlowCaps"]


class GcnFlowCaps:
    """Per-hop (edge, node-set) capacities of the fused GCN flow and its overflow word
    (the DeviceFullFlow capacity API the estimator's regrow loop uses)."""

    def __init__(self, graph, masks, batch_size, caps="bounded"):
        self.g = graph
        self.masks = [int(m) for m in masks]
        self.B = int(batch_size)
        if caps is None or caps == "exact":
            caps = exact_caps(graph, self.masks, self.B)
        elif isinstance(caps, str) and caps.startswith("bounded"):
            caps = bounded_caps(graph, self.masks, self.B, *_bounded_args(caps))
        self.caps = [(int(e), int(n)) for e, n in caps]
        self.overflow = torch.zeros(1, dtype=torch.int32, device=graph.device)
        self.on_clear = None  # the plan's node-counter reset (a discarded step may leave some set)

    def overflowed(self) -> bool:
        return int(self.overflow.item()) != 0

    def clear(self):
        self.overflow.zero_()
        if self.on_clear is not None:
            self.on_clear()

    def check(self):
        if self.overflowed():
            raise RuntimeError(f"fused GCN flow capacity exceeded (caps {self.caps})")

    def grow(self, factor: float = 2.0):
        exact = exact_caps(self.g, self.masks, self.B)
        self.caps = [(min(ex_e, _round_up(int(e * factor))), min(ex_n, _round_up(int(n * factor))))
                     for (e, n), (ex_e, ex_n) in zip(self.caps, exact)]
        self.clear()
        return self.caps


def _gcn_shape(model):
    """the GCNConvs of a SupervisedGCN-shaped model (the full-neighbourhood flow, or
    FastGCN's layer-sampled one), or None"""
    from euler_amd.convolution.convs import GCNConv
    from euler_amd.dataflow.dataflows import FastGCNDataFlow, GCNDataFlow, LayerwiseDataFlow

    gnn = getattr(model, "gnn", None)
    if gnn is None or not isinstance(getattr(gnn, "sampler", None), (GCNDataFlow, FastGCNDataFlow, LayerwiseDataFlow)):
        return None
    convs = list(getattr(gnn, "convs", []))
    if not 1 <= len(convs) <= 2 or not all(type(c) is GCNConv for c in convs):
        return None
    from euler_amd.mp_utils.models import BaseGNNNet

    if type(gnn).forward is not BaseGNNNet.forward or type(gnn).calculate_conv is not BaseGNNNet.calculate_conv:
        return None  # e.g. JKGNNNet: another layer combination
    if any(getattr(l, "activation", None) is not None for l in [c.fc for c in convs] + [gnn.fc, model.out_fc]):
        return None
    if any(getattr(c.fc, "bias", None) is not None for c in convs):
        return None
    if getattr(model.out_fc, "bias", None) is not None or getattr(gnn.fc, "bias", None) is None:
        return None
    return convs


class GcnTrainer(CapturedTrainer):
    metric_name = "f1"

    def __init__(self, model, graph, batch_size, masks, caps="bounded", optimizer="adam", learning_rate=0.01,
                 layer_draws=None):
        if graph.device.type != "cuda":
            raise ValueError("the fused GCN step runs on the GPU (the generic FullFlowTrainer covers the CPU)")
        self.gnn = model.gnn
        self.graph = graph
        self.B = int(batch_size)
        if graph.features is None or graph.labels is None:
            raise ValueError("the device graph needs dense features and labels (DeviceGraph.from_engine)")
        feats = graph.features
        self.D = int(feats.shape[1])
        dp = _round_up(self.D, 32)
        if dp != self.D or not feats.is_contiguous():  # rows padded for 16-byte loads
            padded = torch.zeros((feats.shape[0], dp), dtype=feats.dtype, device=feats.device)
            padded[:, : self.D] = feats
            feats = padded
        self.features = feats
        self.labels = graph.labels.to(graph.device).float().contiguous()
        self.flow = GcnFlowCaps(graph, masks, self.B, caps)
        self.masks = list(masks)
        # FastGCN: per hop None or the layer draw {prob, alias, root_rows, count, stream}
        self.layer_draws = list(layer_draws) if layer_draws is not None else None
        self.counts = torch.zeros(3, dtype=torch.int64, device=graph.device)
        self._stamp = torch.zeros(1, dtype=torch.int32, device=graph.device)
        super().__init__(model, graph, graph.device, optimizer, learning_rate)
        self.plan = None
        self._plan_caps = None
        self._build_plan()

    # ------------------------------------------------------------------ construction
    @staticmethod
    def supports(model, graph=None, batch_size=None) -> bool:
        """SupervisedGCN-shaped: 1-2 bias-free GCNConvs on GCNDataFlow with self loops, fc with
        bias, out_fc without; conv widths <= 64, inputs <= 128, fc / label widths <= 128"""
        if os.environ.get("EULER_AMD_GCN_FUSED", "1") == "0":
            return False
        convs = _gcn_shape(model)
        if convs is None:
            return False
        try:
            widths = [int(c.fc.weight.shape[0]) for c in convs]
            ins = [int(c.fc.weight.shape[1]) for c in convs]
            E = int(model.gnn.fc.weight.shape[0])
            C = int(model.out_fc.weight.shape[0])
        except (AttributeError, ValueError, RuntimeError):
            return False  # lazy layers not materialised
        if graph is not None and (graph.labels is None or graph.features is None or graph.device.type != "cuda"):
            return False
        from euler_amd.dataflow.dataflows import LayerwiseDataFlow

        if isinstance(model.gnn.sampler, LayerwiseDataFlow) and batch_size is not None and int(batch_size) > 4096:
            return False  # the layer-wise draw keeps the roots' prefix sums in one block's LDS
        return (max(widths) <= 64 and max(ins) <= 128 and _round_up(E, 32) <= 128 and _round_up(C, 32) <= 128)

    @classmethod
    def from_model(cls, model, graph, batch_size, optimizer="adam", learning_rate=0.01, caps="bounded"):
        import copy

        import euler_amd.ops.graph_api as ge
        from euler_amd.dataflow.dataflows import FastGCNDataFlow, LayerwiseDataFlow

        flow = model.gnn.sampler
        ets = []
        for m in flow.metapath:
            ids = None if m is None else [int(t) for t in np.asarray(ge.get_edge_type_id(m)).reshape(-1)]
            ets.append(None if ids is None or any(t < 0 for t in ids) else ids)
        draws = None
        if isinstance(flow, FastGCNDataFlow):
            # every hop but the last keeps the edges into a layer of sum(fanouts[:h + 1])
            # rows drawn by sample_node(.., metapath[h][0]) on Philox stream 20 + h: the
            # generic DeviceLayerFlow's "fast" hops (models/full_trainer.py)
            _, _, nw = ge.get_engine().export_nodes()
            draws, total = [], 0
            for h, m in enumerate(flow.metapath):
                if h == len(flow.metapath) - 1:  # the last hop: the full neighbourhood
                    draws.append(None)
                    continue
                total += int(flow.fanouts[h])
                nt = m[0] if isinstance(m, (list, tuple)) else m
                tid = int(np.asarray(ge.get_node_type_id(nt)).reshape(-1)[0])
                smp = copy.copy(graph)
                smp.set_root_type(tid if tid >= 0 else -1, node_weights=np.asarray(nw))
                draws.append({"prob": smp.node_prob, "alias": smp.node_alias, "root_rows": smp.root_rows,
                              "count": total, "stream": 20 + h})
        elif isinstance(flow, LayerwiseDataFlow) and len(flow.metapath) >= 2:
            # AdaptiveGCN (sampleLNB): hop 0's layer = fanouts[0] roots picked in proportion
            # to their out-weight, one weighted neighbour each (DeviceLayerFlow "layer"; the
            # last hop is the full neighbourhood)
            draws = [{"kind": "layer", "count": int(flow.fanouts[0]), "stream": 30, "stream_u": 40}] + \
                [None] * (len(flow.metapath) - 1)
        return cls(model, graph, batch_size, [graph._mask(e) for e in ets], caps=caps, optimizer=optimizer,
                   learning_rate=learning_rate, layer_draws=draws)

    def _build_plan(self):
        m = self.model
        convs = list(self.gnn.convs)
        L = len(convs)
        if len(self.masks) != L:
            raise ValueError("one metapath entry per GCN layer")
        g = self.graph
        w = [c.fc.weight for c in convs]
        d = {"L": L, "B": self.B, "self_loops": int(bool(self.gnn.sampler.add_self_loops)), "indptr": g.indptr, "nbr": g.nbr, "num_types": g.num_types,
             "masks": [int(x) & 0xFFFFFFFF for x in self.masks],
             "cap_e": [e for e, _ in self.flow.caps], "cap_n": [n for _, n in self.flow.caps],
             "node_prob": g.node_prob, "node_alias": g.node_alias, "root_rows": g.root_rows, "rng": g.rng,
             "cumw": g.cumw,
             "stamp": self._stamp, "overflow": self.flow.overflow,
             "features": self.features, "labels": self.labels, "D": self.D,
             "H0": int(w[0].shape[0]), "E": int(self.gnn.fc.weight.shape[0]), "C": int(m.out_fc.weight.shape[0]),
             "w0": w[0].detach(), "g_w0": w[0].grad,
             "wfc": self.gnn.fc.weight.detach(), "g_wfc": self.gnn.fc.weight.grad,
             "bfc": self.gnn.fc.bias.detach(), "g_bfc": self.gnn.fc.bias.grad,
             "wout": m.out_fc.weight.detach(), "g_wout": m.out_fc.weight.grad,
             "loss_out": self.loss_out, "counts": self.counts, "layer_draws": self.layer_draws}
        if L == 2:
            d.update({"H1": int(w[1].shape[0]), "w1": w[1].detach(), "g_w1": w[1].grad})
        self.plan = hip().GcnPlan(d)
        self.flow.on_clear = self.plan.reset_counters
        self._plan_caps = list(self.flow.caps)
        self._fused_opt = self._set_fused_optimizer()

    def _set_fused_optimizer(self, grad_scale: float = 1.0) -> bool:
        """hand the flat optimizer to the plan so one process's step applies it in the
        reduce launch (no separate optimizer launch); False when the optimizer has a
        per-range weight decay or the reduce does not cover the flat buffer"""
        from euler_amd.parallel.flat import _KINDS

        o = self.opt
        if o.decay_range[1] > o.decay_range[0] or o._ticket is None:
            return False
        return bool(self.plan.set_optimizer({
            "flat": self.flat.flat, "grad": self.flat.grad, "m": o.m, "v": o.v, "step": o.step_count,
            "used": int(self.flat.numel), "kind": _KINDS[o.kind], "lr": o.lr, "b1": o.b1, "b2": o.b2, "eps": o.eps,
            "wd": o.wd, "grad_scale": float(grad_scale)}))

    def set_learning_rate(self, lr):
        super().set_learning_rate(lr)
        self._fused_opt = self._set_fused_optimizer()

    # ------------------------------------------------------------------ step
    def _step(self, grad_sync=None):
        if self._plan_caps != self.flow.caps:  # grown after an overflow: new fixed shapes
            self._build_plan()
        if grad_sync is None and self._fused_opt:  # one process: the update rides the reduce launch
            self.plan.step(True)
            return self.loss_out
        self.plan.step()
        scale = 1.0
        if grad_sync is not None:
            s = grad_sync(self.flat.grad)
            scale = 1.0 if s is None else float(s)
        self.opt.step(scale)
        return self.loss_out

    def capture(self, grad_sync=None, warmup: int = 2, steps: int = 1, extra_sizes=()):
        if self._plan_caps != self.flow.caps:
            self._build_plan()
        return super().capture(grad_sync, warmup, steps, extra_sizes)

    @property
    def launches_per_step(self) -> int:
        """launches of one single-process step (the optimizer folded into the reduce)"""
        return int(self.plan.launches) + (0 if self._fused_opt else 1)

    # ------------------------------------------------------------------ metric
    def metric(self) -> float:
        tp, fp, fn = self.counts.tolist()
        return 2.0 * tp / max(2.0 * tp + fp + fn, 1e-12)

    def reset_metric(self):
        self.counts.zero_()

    def samples(self):
        return (self.plan.flow()["roots"],)

    # ------------------------------------------------------------------ inference
    @torch.no_grad()
    def infer_logits(self, ids):
        """(embeddings, logits, labels) of raw node ids: the model's own modules (their
        parameters are the trained flat buffer's views) on an exact full-neighbourhood block
        of exactly these roots (models/full_trainer.py full_flow_embed)"""
        from euler_amd.models.full_trainer import full_flow_embed, infer_flow

        if self.layer_draws is not None:
            # FastGCN / AdaptiveGCN sample their layers (reference fast_dataflow /
            # LayerwiseDataFlow): an exact block would report other metrics than the engine path
            raise NotImplementedError("layer-sampled GCN models infer on the engine path")
        n = int(torch.as_tensor(ids).numel())
        flow = infer_flow(self, self.graph, self.masks, bool(self.gnn.sampler.add_self_loops), n)
        rows = self.graph.rows_of(ids).to(self.graph.device)
        emb, _ = full_flow_embed(self.gnn, flow, self.graph.features, rows)
        logits = self.model.out_fc(emb).float()
        return emb.float(), logits, self.labels[rows.clamp(min=0)]

    def infer_embed(self, ids):
        return self.infer_logits(ids)[0]

    # ------------------------------------------------------------------ oracle
    def reference_loss_and_grads_bf16(self):
        """The bf16-aware fp32 oracle of the last step, in pure CPU torch (no HIP op): the
        model's GCN on the blocks the fused flow built (``plan.flow()``: the same roots,
        node sets and edge lists), every operand rounded to bf16 exactly where gcn.hip
        rounds it and everything else fp32 — so the kernels must match it to fp32
        accumulation order, not to bf16 noise.  Rounding points:

        * weights: bf16 images of the fp32 masters (conv W, fc W, out W);
        * agg_t = bf(sum_e x_s deg_t^-1/2 deg_s^-1/2) over the target's block edges (+ the
          self loop), deg_t = its edge count (+1), deg_s = the source's in-block count;
          h = bf(relu(agg W^T)) (the outer conv's h1 kept bf16 for the next hop);
        * head: emb = bf(h Wfc^T + bfc), logits = emb Wout^T (fp32),
          d = bf((sigmoid - y) / (B C)), demb = d Wout, dz = bf(relu'(h) (bf(demb) Wfc));
          dWout = d^T emb, dWfc = bf(demb)^T h, dbfc = sum demb, dW = dz^T agg;
        * L = 2: dagg = dz W (fp32); per hop-0 edge e: bf(relu'(h1_s) w_e dagg_t) against
          agg1_s (gcn_dw_kernel: d h1 is never formed).

        Semantics: tf_euler/python/convolution/gcn_conv.py:42-54, mp_utils/base.py:24-47."""
        f32 = torch.float32
        cpu = torch.device("cpu")

        def bf(t):
            return t.to(torch.bfloat16).to(f32)

        fl = self.plan.flow()
        L = len(self.gnn.convs)
        sl = int(bool(self.gnn.sampler.add_self_loops))
        roots = fl["roots"].to(cpu).long()
        B = roots.numel()
        cnt = [int(c) for c in fl["cnt"].to(cpu).tolist()]
        node_set = fl["set"].to(cpu).long()
        rself = fl["rself"].to(cpu).long()
        x = self.features[:, : self.D].to(cpu).to(f32)
        convs = [bf(c.fc.weight.detach().to(cpu).float()) for c in self.gnn.convs]
        Wfc = bf(self.gnn.fc.weight.detach().to(cpu).float())
        bfc = self.gnn.fc.bias.detach().to(cpu).float()
        Wout = bf(self.model.out_fc.weight.detach().to(cpu).float())

        def block(h, nt, self_pos):
            """(target, source position, coefficient) of hop h's edges + self loops"""
            hop = {k: v.to(cpu).long() for k, v in fl["hops"][h].items()}
            off = hop["off"][: nt + 1]
            E = int(off[-1])
            t = hop["etgt"][:E]
            sp = hop["esrc"][:E]
            node = hop["enode"][:E]
            keep = sp >= 0
            t, sp, node = t[keep], sp[keep], node[keep]
            if sl:
                tt = torch.arange(nt)
                t, sp = torch.cat([t, tt]), torch.cat([sp, self_pos])
                node = torch.cat([node, node_set[self_pos]])
            deg_t = (off[1:] - off[:-1] + sl).to(f32)
            deg_s = hop["deg_s"].to(f32)
            coef = deg_t[t].rsqrt() * deg_s[sp].rsqrt()
            return t, sp, node, coef

        def aggregate(nt, t, vals, coef):
            return torch.zeros(nt, vals.shape[1]).index_add_(0, t, vals * coef[:, None])

        if L == 2:
            n1 = cnt[1]
            t1, sp1, node1, c1 = block(1, n1, torch.arange(n1))
            agg1 = bf(aggregate(n1, t1, x[node1], c1))
            h1 = bf(torch.relu(agg1 @ convs[0].t()))
            t0, sp0, node0, c0 = block(0, B, rself)
            agg = bf(aggregate(B, t0, h1[sp0], c0))
        else:
            t0, sp0, node0, c0 = block(0, B, rself)
            agg = bf(aggregate(B, t0, x[node0], c0))
        Wl = convs[-1]
        H0 = bf(torch.relu(agg @ Wl.t()))
        emb = bf(H0 @ Wfc.t() + bfc)
        logits = emb @ Wout.t()
        y = self.labels[roots.to(self.labels.device)].to(cpu).float()
        loss = torch.nn.functional.binary_cross_entropy_with_logits(logits, y)
        d = bf((torch.sigmoid(logits) - y) / float(y.numel()))
        demb = d @ Wout
        De = bf(demb)
        dz = bf((H0 > 0).to(f32) * (De @ Wfc))
        names = {id(p): n for n, p in self.model.named_parameters()}
        g = {names[id(self.model.out_fc.weight)]: d.t() @ emb, names[id(self.gnn.fc.weight)]: De.t() @ H0,
             names[id(self.gnn.fc.bias)]: demb.sum(0), names[id(self.gnn.convs[-1].fc.weight)]: dz.t() @ agg}
        if L == 2:
            dagg = dz @ Wl
            rows = bf((h1[sp0] > 0).to(f32) * (c0[:, None] * dagg[t0]))
            g[names[id(self.gnn.convs[0].fc.weight)]] = rows.t() @ agg1[sp0]
        return float(loss), g


    def forward_backward_only(self):
        """plan step without the optimizer (tests): loss_out and the flat gradient"""
        if self._plan_caps != self.flow.caps:
            self._build_plan()
        self.plan.step()
        return self.loss_out
