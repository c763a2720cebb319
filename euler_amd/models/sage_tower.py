"""Unsupervised GraphSAGE on an HBM-resident graph: the device path of the reference's
other flagship GraphSAGE configuration.

Model = the reference ``UnsupervisedGraphSage`` (``examples/graphsage/graphsage.py:70-98``,
``tf_euler/python/mp_utils/base.py:49-91``): a source tower ``gnn`` and a context tower
``context_gnn``, each ``dims[:-1]`` SAGEConv layers (``self_fc(x) + neigh_fc(mean_j x_j)``,
ReLU; ``convolution/sage_conv.py:33-44``) + ``fc`` = Dense(dims[-1]) with bias; a batch of
``sample_node`` sources, one ``sample_neighbor`` positive per source (padding when it has
no out-edge, the reference's ``max_id + 1``) and ``num_negs`` ``sample_node`` negatives;
logits = <src, pos> and <src, neg_k>, sigmoid cross-entropy averaged over the B + B*K
logits, MRR of the positive as the metric (``utils/metrics.py`` mrr).

Execution (MI355X), per step, one hipGraph:
  * roots: alias-table sources, the positive neighbour draw and the negatives on the GPU
    (``DeviceGraph.sample_node`` / ``sample_neighbor``, Philox);
  * layer 0 of each tower is the fused tree step of ``csrc/hip/sage_tree.hip`` over the
    given roots (``TowerPlan``): hop-1 + leaf sampling, the leaf-row gather + mean, the
    layer-0 MFMA GEMM + ReLU and the tree mean of hop 1 in one launch, producing the last
    conv's input rows [R][2H0]; its backward routes dA1 through the tree and the ReLU bits
    inside the split-K dW kernel (no per-row gradient tensor is materialised);
  * the last conv and fc of a tower form ONE autograd node with its layer 0
    (``models/_tower_ops.py`` tower_head: split-K head dW, every gradient written into its
    flat-gradient view, no zero fill, no accumulation pass); the pair logits + sigmoid CE are
    one more node (pair_loss); one flat Adam launch (``csrc/hip/optim.hip``) updates both
    towers.

Widths are padded (features to 16, conv widths to 64, fc to 32) with zero rows / columns
that stay zero.  On a CPU device the same model, sampling layout and optimizer run in fp32
torch (:meth:`_tower_reference` is also the GPU kernels' numerics oracle).
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as F

from euler_amd.models._tower_ops import pair_loss, tower_head
from euler_amd.ops import mp_ops
from euler_amd.ops._native import hip
from euler_amd.parallel.flat import FlatOptimizer, FlatParams
from euler_amd.models.captured import new_graph

# the fused 7-launch step (PairPlan) on GPUs; EULER_AMD_PAIR_FUSED_STEP=0 keeps the
# per-op autograd step (tower kernels + GEMM autograd nodes)
_FUSED = os.environ.get("EULER_AMD_PAIR_FUSED_STEP", "1") == "1"

__all__ = ["UnsupSageTrainer", "unsup_param_names"]


def _ceil(x: int, m: int) -> int:
    return -(-int(x) // m) * m


def _slot(f: int) -> int:
    p = 4
    while (1 << p) < f + 1:
        p += 1
    return p


def unsup_param_names():
    """Reference parameter names (euler_amd.models.UnsupervisedGraphSage, 2 hops)."""
    out = []
    for t in ("gnn", "context_gnn"):
        for k in range(2):
            out += [f"{t}.convs.{k}.self_fc.weight", f"{t}.convs.{k}.neigh_fc.weight"]
        out += [f"{t}.fc.weight", f"{t}.fc.bias"]
    return out


def _xavier(shape, gen):
    fan_out, fan_in = shape
    a = math.sqrt(6.0 / (fan_in + fan_out))
    return (torch.rand(shape, generator=gen, dtype=torch.float64) * 2 - 1).mul_(a).float()


class _Tower:
    """Layer 0 of one 2-hop tower over R given roots (csrc/hip/binding_tree.cpp TowerPlan)."""

    def __init__(self, graph, features, R, F1, F2, H0, masks, include_self, W0, device):
        self.R, self.F1, self.F2, self.H0 = int(R), int(F1), int(F2), int(H0)
        self.logP = _slot(F1)
        self.M = self.R << self.logP
        self.D = int(features.shape[1])
        i32 = dict(dtype=torch.int32, device=device)
        self.roots_in = torch.full((self.R,), -1, **i32)
        self.roots_out = torch.full((self.R,), -1, **i32)  # the roots the sampler used
        self.nodes = torch.zeros(self.M, **i32)
        self.leaf = torch.zeros(self.M * self.F2, **i32)
        self.A1 = torch.zeros(self.R * 2 * self.H0, dtype=torch.bfloat16, device=device)
        self.dA1 = torch.zeros(self.R * 2 * self.H0, dtype=torch.float32, device=device)
        # the routed layer-0 dW is reduced straight into W0's flat-gradient view when there
        # is one (FlatParams), else into a buffer of its own
        g = W0.grad
        self.gW0 = (g.view(-1) if g is not None and g.is_contiguous() and g.dtype == torch.float32
                    else torch.zeros(W0.numel(), dtype=torch.float32, device=device))
        self.plan = None
        if device.type == "cuda":
            g = graph
            d = {"R": self.R, "F1": self.F1, "F2": self.F2, "logP": self.logP, "D": self.D, "H": self.H0,
                 "include_self": int(include_self), "mask1": int(masks[0]) & 0xFFFFFFFF,
                 "mask2": int(masks[1]) & 0xFFFFFFFF, "indptr": g.indptr, "nbr": g.nbr, "cumw": g.cumw,
                 "num_types": g.num_types, "node_prob": g.node_prob, "node_alias": g.node_alias, "rng": g.rng,
                 "roots_in": self.roots_in, "roots_out": self.roots_out, "nodes": self.nodes, "leaf": self.leaf,
                 "features": features,
                 "root_rows": g.root_rows,
                 "W0": W0, "W0_sh": torch.zeros(W0.numel(), dtype=torch.bfloat16, device=device),
                 "A0_kt": torch.empty(self.M * 2 * self.D, dtype=torch.bfloat16, device=device),
                 "mask0": torch.zeros((self.M // 32) * self.H0, **i32), "A1": self.A1, "dA1": self.dA1,
                 "gW0": self.gW0}
            self._keep = d
            self.plan = hip().TowerPlan(d)


class UnsupSageTrainer:
    _device_towers = True

    def __init__(self, graph, batch_size, fanouts, dims, features=None, num_negs=5, pos_edge_types=None,
                 metapath=None, add_self_loops=False, optimizer="adam", learning_rate=0.01, init=None, init_seed=0,
                 fused=True):
        self.graph = graph
        self.device = graph.device
        self.B = int(batch_size)
        self.K = int(num_negs)
        self.fanouts = [int(f) for f in fanouts]
        if len(self.fanouts) != 2:
            raise ValueError("the device unsupervised GraphSAGE trains 2-hop towers")
        dims = [int(d) for d in dims]
        if len(dims) != 3:
            raise ValueError("dims = two conv widths + the embedding width")
        if self.B % 32:
            raise ValueError("batch_size must be a multiple of 32")
        feats = features if features is not None else graph.features
        if feats is None:
            raise ValueError("node features are required")
        self.conv_dims, self.E = dims[:2], dims[2]
        self.D = int(feats.shape[1])
        self.Dp = _ceil(self.D, 16)
        self.Hp = [_ceil(h, 64) for h in self.conv_dims]
        self.Ep = _ceil(self.E, 32)
        self.include_self = bool(add_self_loops)
        mp = metapath if metapath is not None else [None, None]
        self.masks = [graph._mask(m) for m in mp]
        self.pos_mask = graph._mask(pos_edge_types)
        self.logP = _slot(self.fanouts[0])
        f = feats.to(self.device)
        if f.shape[1] != self.Dp or f.dtype not in (torch.bfloat16, torch.float32):
            pad = torch.zeros(f.shape[0], self.Dp, dtype=f.dtype if f.dtype in (torch.bfloat16, torch.float32)
                              else torch.float32, device=self.device)
            pad[:, : self.D] = f.to(pad.dtype)
            f = pad
        self.features = f.contiguous()
        # parameters (padded, fp32) of both towers -> one flat buffer
        logical = self._init_logical(init, init_seed)
        self.params = {}
        for t in ("gnn", "context_gnn"):
            H0, H1 = self.Hp
            shapes = {"W0": (H0, 2 * self.Dp), "W1": (H1, 2 * H0), "Wfc": (self.Ep, H1), "bfc": (self.Ep,)}
            for k, shp in shapes.items():
                self.params[f"{t}.{k}"] = torch.zeros(shp, device=self.device, requires_grad=True)
        self.flat = FlatParams(list(self.params.values()), self.device)
        self.load_logical(logical)
        self.opt = FlatOptimizer(self.flat, optimizer, learning_rate)
        R = {"gnn": self.B, "context_gnn": self.B * (1 + self.K)}
        # the towers' in-kernel samplers read a whole CSR in HBM (a row-sharded graph's
        # trainer draws its trees across the ranks instead: models/sharded_unsup.py)
        self.towers = {t: _Tower(graph, self.features, R[t], self.fanouts[0], self.fanouts[1], self.Hp[0],
                                 self.masks, self.include_self, self.params[f"{t}.W0"], self.device)
                       for t in ("gnn", "context_gnn")} if self._device_towers else {}
        self.loss_out = torch.zeros((), device=self.device)
        self.mrr_sum = torch.zeros((), device=self.device)
        self.mrr_n = 0
        self.step_count = 0
        self._graph_exec = None
        self._graphs = {}
        self._samples = None
        self.pair = None
        if self.device.type == "cuda" and fused and _FUSED and self.towers:
            try:
                self._build_pair(optimizer)
            except RuntimeError as e:  # shapes the pair head does not take (LDS): per-op step
                self.pair = None
                self.fused_error = str(e)

    metric_name = "mrr"

    # ------------------------------------------------------------------ fused step (GPU)
    def _build_pair(self, optimizer):
        """the 7-launch step (csrc/hip/binding_tree.cpp PairPlan): both towers' layer 0, the
        pair head kernel, one dW launch, one optimizer launch over the flat buffer"""
        dev = self.device
        bf = dict(dtype=torch.bfloat16, device=dev)
        H0, H1 = self.Hp
        E = self.Ep
        names = [f"{t}.{k}" for t in ("gnn", "context_gnn") for k in ("W0", "W1", "Wfc", "bfc")]
        where = {id(p): i for i, p in enumerate(self.flat.params)}
        offs = [self.flat.offsets[where[id(self.params[n])]][0] for n in names] + [self.flat.numel]
        if offs != sorted(offs):
            raise RuntimeError("flat parameter order is not the pair plan's segment order")
        d = {"B": self.B, "K": self.K, "H1": H1, "E": E, "pos_mask": int(self.pos_mask) & 0xFFFFFFFF,
             "flat": self.flat.flat, "grad": self.flat.grad, "m": self.opt.m, "v": self.opt.v,
             "step": self.opt.step_count, "offsets": offs, "loss_acc": torch.zeros(1, device=dev),
             "loss_out": self.loss_out, "mrr_sum": self.mrr_sum, "lr": self.opt.lr, "beta1": self.opt.b1,
             "beta2": self.opt.b2, "eps": self.opt.eps, "weight_decay": self.opt.wd,
             "opt_kind": {"adam": 0, "adagrad": 1, "sgd": 2, "momentum": 3}[optimizer]}
        for x, t in (("s", "gnn"), ("c", "context_gnn")):
            d[f"W1_sh_{x}"] = torch.zeros(H1 * 2 * H0, **bf)
            d[f"W1_shT_{x}"] = torch.zeros(H1 * 2 * H0, **bf)
            d[f"Wfc_sh_{x}"] = torch.zeros(E * H1, **bf)
            d[f"Wfc_shT_{x}"] = torch.zeros(E * H1, **bf)
            d[f"bfc_{x}"] = self.params[f"{t}.bfc"]
        self._pair_keep = d
        self.pair = hip().PairPlan(self.towers["gnn"].plan, self.towers["context_gnn"].plan, d)
        self.pair.opt(3)  # bf16 shadows of every weight

    def _fused_step(self, grad_sync=None):
        p = self.pair
        p.sample()
        p.fwd()
        p.head()
        p.dw()
        if grad_sync is None:
            p.opt(2)
        else:
            p.opt(0)
            s = grad_sync(self.flat.grad)
            p.opt(1, 1.0 if s is None else float(s))
        return self.loss_out

    @classmethod
    def from_model(cls, model, graph, batch_size, optimizer="adam", learning_rate=0.01, **kw):
        """Trainer for a (materialised) 2-hop ``UnsupervisedGraphSage``: widths, fanouts,
        metapath, the positives' edge types and the negatives from the model; weights
        copied.  Negatives come from the graph's root sampler (``set_root_type`` of the
        model's node type, as the reference's ``sample_node(node_type)``)."""
        from euler_amd.convolution.convs import SAGEConv
        from euler_amd.dataflow.dataflows import SageDataFlow
        import euler_amd.ops.graph_api as ge
        import numpy as np

        gnn = model.gnn
        if (not all(isinstance(c, SAGEConv) for c in gnn.convs) or not isinstance(gnn.sampler, SageDataFlow)
                or len(gnn.convs) != 2):
            raise ValueError("the device path trains 2-hop SAGEConv + SageDataFlow towers (UnsupervisedGraphSage)")

        def types(m):
            if m is None:
                return None
            ids = [int(t) for t in np.asarray(ge.get_edge_type_id(m)).reshape(-1)]
            return None if any(t < 0 for t in ids) else ids

        dims = [c.self_fc.out_features for c in gnn.convs] + [gnn.fc.out_features]
        metapath = [types(m) for m in gnn.sampler.metapath]
        return cls(graph, batch_size, gnn.sampler.fanouts, dims, num_negs=model.num_negs,
                   pos_edge_types=types(model.edge_type), metapath=metapath,
                   add_self_loops=bool(getattr(gnn.sampler, "add_self_loops", False)), optimizer=optimizer,
                   learning_rate=learning_rate, init=model, **kw)

    def write_to_model(self, model):
        sd = model.state_dict()
        with torch.no_grad():
            for k, v in self.logical_params().items():
                if k in sd:
                    sd[k].copy_(v.to(sd[k]))

    def set_learning_rate(self, lr):
        self.opt.lr = float(lr)
        if self.pair is not None:
            self.pair.set_lr(float(lr))

    # ------------------------------------------------------------------ parameters
    def _logical_shapes(self):
        s = {}
        for t in ("gnn", "context_gnn"):
            hin = self.D
            for k, h in enumerate(self.conv_dims):
                s[f"{t}.convs.{k}.self_fc.weight"] = (h, hin)
                s[f"{t}.convs.{k}.neigh_fc.weight"] = (h, hin)
                hin = h
            s[f"{t}.fc.weight"] = (self.E, hin)
            s[f"{t}.fc.bias"] = (self.E,)
        return s

    def _init_logical(self, init, seed):
        if init is not None and not isinstance(init, dict):
            init = init.state_dict()
        gen = torch.Generator().manual_seed(int(seed))
        out = {}
        for k, shp in self._logical_shapes().items():
            if init is not None and k in init:
                out[k] = torch.as_tensor(init[k]).detach().float().cpu().clone()
            elif k.endswith("bias"):
                out[k] = torch.zeros(shp)
            else:
                out[k] = _xavier(shp, gen)
        return out

    def load_logical(self, logical):
        with torch.no_grad():
            for t in ("gnn", "context_gnn"):
                P = {k: self.params[f"{t}.{k}"] for k in ("W0", "W1", "Wfc", "bfc")}
                for v in P.values():
                    v.zero_()
                hin, hinp = self.D, self.Dp
                for k, (name, w) in enumerate((("W0", P["W0"]), ("W1", P["W1"]))):
                    h = self.conv_dims[k]
                    w[:h, :hin] = torch.as_tensor(logical[f"{t}.convs.{k}.self_fc.weight"]).to(w)
                    w[:h, hinp:hinp + hin] = torch.as_tensor(logical[f"{t}.convs.{k}.neigh_fc.weight"]).to(w)
                    hin, hinp = h, self.Hp[k]
                P["Wfc"][: self.E, :hin] = torch.as_tensor(logical[f"{t}.fc.weight"]).to(P["Wfc"])
                P["bfc"][: self.E] = torch.as_tensor(logical[f"{t}.fc.bias"]).to(P["bfc"])

    def logical_params(self):
        out = {}
        for t in ("gnn", "context_gnn"):
            P = {k: self.params[f"{t}.{k}"].detach() for k in ("W0", "W1", "Wfc", "bfc")}
            hin, hinp = self.D, self.Dp
            for k, name in enumerate(("W0", "W1")):
                h = self.conv_dims[k]
                out[f"{t}.convs.{k}.self_fc.weight"] = P[name][:h, :hin].clone()
                out[f"{t}.convs.{k}.neigh_fc.weight"] = P[name][:h, hinp:hinp + hin].clone()
                hin, hinp = h, self.Hp[k]
            out[f"{t}.fc.weight"] = P["Wfc"][: self.E, :hin].clone()
            out[f"{t}.fc.bias"] = P["bfc"][: self.E].clone()
        return out

    def state_dict(self):
        return {k: v.cpu() for k, v in self.logical_params().items()}

    def trainer_state(self):
        return {"m": self.opt.m.cpu().clone(), "v": self.opt.v.cpu().clone(),
                "step": int(self.opt.step_count.item()), "rng": self.graph.rng.detach().cpu().clone()}

    def dp_state_tensors(self):
        """tensors equal on every data-parallel rank (what a re-synchronisation broadcasts)"""
        return [self.flat.flat, self.opt.m, self.opt.v, self.opt.step_count]

    def load_trainer_state(self, st):
        self.opt.m.copy_(torch.as_tensor(st["m"]).to(self.opt.m))
        self.opt.v.copy_(torch.as_tensor(st["v"]).to(self.opt.v))
        self.opt.step_count.fill_(int(st["step"]))
        self.graph.rng.copy_(torch.as_tensor(st["rng"]).to(self.graph.rng))
        self.step_count = int(st["step"])
        self.refresh_shadows()

    def refresh_shadows(self):
        """rebuild the fused step's bf16 weight shadows (after a load or a broadcast)"""
        if self.pair is not None:
            self.pair.opt(3)

    # ------------------------------------------------------------------ sampling
    def sample_roots(self):
        """(sources [B], positives [B], negatives [B*K]) int32 rows; -1 = no positive"""
        g = self.graph
        g.advance()
        if self.device.type != "cuda":
            g.reseed_cpu()
        src = g.sample_node(self.B, stream_id=5)
        pos = g.sample_neighbor(src, 1, self._types(self.pos_mask), -1, stream_id=6).reshape(-1)
        negs = g.sample_node(self.B * self.K, stream_id=7)
        return src.int(), pos.int(), negs.int()

    def _cpu_tree(self, roots):
        """slotted tree of a tower on the CPU twin: nodes [R * P], leaf [R * P, F2]"""
        g = self.graph
        F1, F2, P = self.fanouts[0], self.fanouts[1], 1 << self.logP
        nb = g._sample_neighbor_cpu(roots.int(), F1, self.masks[0], -1, False).long()
        slots = torch.full((roots.numel(), P), -1, dtype=torch.int64)
        slots[:, :F1] = nb
        slots[:, F1] = roots.long()
        nodes = slots.reshape(-1)
        leaf = g._sample_neighbor_cpu(nodes.int(), F2, self.masks[1], -1, False).long()
        return nodes, leaf

    # ------------------------------------------------------------------ model
    def _tower_reference(self, W0, nodes, leaf, table=None):
        """fp32 A1 rows of a tower from its sampled tree (oracle / CPU path); ``table``: the
        feature rows ``nodes`` / ``leaf`` index (default the trainer's feature table)"""
        tab = self.features if table is None else table
        nodes, leaf = nodes.to(tab.device).long(), leaf.to(tab.device).long()
        # the tree's rows first (-1: zero rows), then fp32: never the whole table in fp32
        xs = mp_ops.gather(tab, nodes).float()
        agg = mp_ops.gather(tab, leaf).float().sum(1)
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

    def _head(self, t, A1, P=None):
        P = self.params if P is None else P
        h1 = torch.relu(A1 @ P[f"{t}.W1"].t())
        return h1 @ P[f"{t}.Wfc"].t() + P[f"{t}.bfc"]

    def _pair_loss(self, es, ec):
        # context rows: the B positives, then the B x K negatives (source-major)
        ec = torch.cat([ec[: self.B].unsqueeze(1), ec[self.B:].view(self.B, self.K, -1)], 1)
        logits = (es.unsqueeze(1) * ec).sum(-1)  # [B, 1 + K]: positive first
        y = torch.zeros_like(logits)
        y[:, 0] = 1.0
        loss = F.binary_cross_entropy_with_logits(logits, y)
        with torch.no_grad():
            rank = 1 + (logits[:, 1:] >= logits[:, :1]).sum(1).float()
            mrr = (1.0 / rank).sum()
        return loss, mrr

    def _forward_loss(self):
        src, pos, negs = self.sample_roots()
        ts, tc = self.towers["gnn"], self.towers["context_gnn"]
        if self.device.type == "cuda":
            ts.roots_in.copy_(src)
            tc.roots_in[: self.B].copy_(pos)
            tc.roots_in[self.B:].copy_(negs)
            P = self.params
            # fused towers (one autograd node each: layer 0 + last conv + fc, gradients
            # written into the flat-gradient views) and the fused pair loss
            es = tower_head(P["gnn.W0"], P["gnn.W1"], P["gnn.Wfc"], P["gnn.bfc"], ts)
            ec = tower_head(P["context_gnn.W0"], P["context_gnn.W1"], P["context_gnn.Wfc"], P["context_gnn.bfc"],
                            tc)
            loss, logits, counted = pair_loss(es, ec, self.B, self.K, self.mrr_sum)
            if counted:
                return loss, None  # the kernel added the batch's reciprocal ranks to mrr_sum
            with torch.no_grad():
                rank = 1 + (logits[:, 1:] >= logits[:, :1]).sum(1).float()
                mrr = (1.0 / rank).sum()
            return loss, mrr
        else:
            ctx = torch.cat([pos, negs]).long()
            ns, ls = self._cpu_tree(src.long())
            nc, lc = self._cpu_tree(ctx)
            self._samples = (src, ctx, ns, ls, nc, lc)
            A1s = self._tower_reference(self.params["gnn.W0"], ns, ls)
            A1c = self._tower_reference(self.params["context_gnn.W0"], nc, lc)
        return self._pair_loss(self._head("gnn", A1s), self._head("context_gnn", A1c))

    def step(self, grad_sync=None):
        """One training step; ``grad_sync(flat_grad)`` (an in-place all-reduce returning
        the 1/world scale) runs between the backward and the optimizer (data parallel)."""
        self.step_count += 1
        if self._graph_exec is not None:
            self._graph_exec.replay()
            return self.loss_out
        return self._step(grad_sync)

    def replay(self, n: int = 1):
        for _ in range(int(n)):
            self._graph_exec.replay()
        self.step_count += int(n)

    def replay_steps(self, n: int):
        """exactly n steps, greedily from the largest captured graph down"""
        left = int(n)
        for k in sorted(self._graphs, reverse=True):
            while left >= k:
                self._graphs[k].replay()
                left -= k
        self.step_count += int(n)

    def release_graphs(self):
        for gr in self._graphs.values():
            gr.reset()
        self._graphs = {}
        self._graph_exec = None

    def _step(self, grad_sync=None):
        if self.pair is not None:
            return self._fused_step(grad_sync)
        loss, mrr = self._forward_loss()
        if self.device.type != "cuda":
            self.opt.zero_grad()  # the GPU towers overwrite every gradient view instead
        loss.backward()
        scale = 1.0
        if grad_sync is not None:
            s = grad_sync(self.flat.grad)
            scale = 1.0 if s is None else float(s)
        self.opt.step(scale)
        self.loss_out.copy_(loss.detach())
        if mrr is not None:
            self.mrr_sum.add_(mrr)
        return self.loss_out

    def capture(self, grad_sync=None, warmup: int = 2, steps: int = 1, extra_sizes=()):
        """Record ``steps`` complete steps (sampling, both towers, loss, backward,
        [all-reduce,] optimizer) into one hipGraph after ``warmup`` eager steps on a side
        stream; graphs of 1 step and of each ``extra_sizes`` entry are kept too
        (:meth:`replay_steps`; :meth:`step` / :meth:`replay` replay the 1-step graph)."""
        if self.device.type != "cuda":
            return None
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.step_count += 1
                self._step(grad_sync)
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        self.flat.rebind_grads()
        self._graphs = {}
        for k in sorted({1, int(steps)} | {int(e) for e in extra_sizes if int(e) > 0}, reverse=True):
            g = new_graph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                for _ in range(k):
                    self._step(grad_sync)
            self._graphs[k] = g
        self._graph_exec = self._graphs[1]
        return self._graphs[int(steps)]

    @property
    def loss(self):
        return self.loss_out

    def metric(self):
        """mean reciprocal rank of the positive since the last reset"""
        n = max(self.mrr_n_steps(), 1)
        return float(self.mrr_sum.item()) / (n * self.B)

    def mrr_n_steps(self):
        return self.step_count - getattr(self, "_mrr_reset_at", 0)

    def reset_metric(self):
        self.mrr_sum.zero_()
        self._mrr_reset_at = self.step_count

    # ------------------------------------------------------------------ inference
    @torch.no_grad()
    def embed(self, rows, tower="gnn", seed_offset=0):
        """embeddings [n, E] of graph rows through a tower (its own fp32 torch forward on a
        freshly sampled tree: the reference's infer path)"""
        rows = torch.as_tensor(rows).reshape(-1).to(self.device)
        out = []
        W0 = self.params[f"{tower}.W0"].detach()
        cpu_graph = self.device.type != "cuda"
        for a in range(0, rows.numel(), 4096):
            r = rows[a:a + 4096]
            if cpu_graph:
                nodes, leaf = self._cpu_tree(r.long())
            else:
                nodes, leaf = self._gpu_tree(r.int())
            A1 = self._tower_reference(W0, nodes, leaf)
            out.append(self._head(tower, A1)[:, : self.E])
        return torch.cat(out)

    def _gpu_tree(self, roots):
        g = self.graph
        F1, F2, P = self.fanouts[0], self.fanouts[1], 1 << self.logP
        nb = g.sample_neighbor(roots, F1, self._types(self.masks[0]), -1, stream_id=8).view(-1, F1).long()
        slots = torch.full((roots.numel(), P), -1, dtype=torch.int64, device=roots.device)
        slots[:, :F1] = nb
        slots[:, F1] = roots.long()
        nodes = slots.reshape(-1)
        leaf = g.sample_neighbor(nodes.int(), F2, self._types(self.masks[1]), -1, stream_id=9).view(-1, F2).long()
        g.advance()
        return nodes, leaf

    def _types(self, mask):
        return [t for t in range(self.graph.num_types) if (mask >> t) & 1]

    # ------------------------------------------------------------------ oracle
    def tower_samples(self, tower):
        """(roots, nodes [R*P], leaf [R*P, F2]) of the last forward of a tower"""
        if self.device.type != "cuda":
            src, ctx, ns, ls, nc, lc = self._samples
            return (src, ns, ls) if tower == "gnn" else (ctx, nc, lc)
        t = self.towers[tower]
        roots = t.roots_out if self.pair is not None else t.roots_in
        return roots.long(), t.nodes.long(), t.leaf.view(-1, self.fanouts[1]).long()

    def reference_loss_and_grads(self):
        """fp32 torch autograd loss and gradients (padded parameter names) on the samples
        of the last forward (call after forward_backward, before the optimizer)"""
        P = {k: v.detach().float().clone().requires_grad_(True) for k, v in self.params.items()}
        _, ns, ls = self.tower_samples("gnn")
        _, nc, lc = self.tower_samples("context_gnn")
        A1s = self._tower_reference(P["gnn.W0"], ns, ls)
        A1c = self._tower_reference(P["context_gnn.W0"], nc, lc)
        loss, _ = self._pair_loss(self._head("gnn", A1s, P), self._head("context_gnn", A1c, P))
        loss.backward()
        return float(loss), {k: v.grad.detach() for k, v in P.items()}

    def forward_backward(self):
        """sampling, forward, backward of one step (no optimizer): :meth:`gradients`"""
        if self.pair is not None:
            p = self.pair
            p.sample()
            p.fwd()
            p.head()
            p.dw()
            p.opt(0)  # split-K reduce into the flat gradient, no update
            return float(self._pair_keep["loss_acc"].item())
        loss, _ = self._forward_loss()
        if self.device.type != "cuda":
            self.opt.zero_grad()
        loss.backward()
        return float(loss)

    def gradients(self):
        return {k: v.grad.detach().clone() for k, v in self.params.items()}
