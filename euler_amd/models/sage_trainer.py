"""Supervised GraphSAGE training on an HBM-resident graph: the framework's device path.

Model = the reference ``SupervisedGraphSage`` (``examples/graphsage/graphsage.py:56-67``):
``dims[:-1]`` SAGEConv layers (``self_fc(x) + neigh_fc(mean_j x_j)``, no bias, ReLU;
``convolution/sage_conv.py:33-44``), ``fc`` = Dense(dims[-1]) with bias, ``out_fc`` =
Dense(label_dim) without, sigmoid cross-entropy averaged over ``[batch, label_dim]``
(``mp_utils/base.py:24-47``), roots drawn by ``sample_node(batch, train_node_type)``
(``euler_estimator/python/node_estimator.py``) and neighbours by the reference
``SageDataFlow`` (``sage_dataflow.py:35-50``: every hop re-samples all nodes of the
previous hops), trained with adam / adagrad / sgd / momentum (``utils/optimizers.py``).

Execution (MI355X): the graph (CSR + prefix-sum weights), the feature table and the
labels live in HBM (:meth:`DeviceGraph.from_engine` uploads a loaded dataset;
:meth:`DeviceGraph.synthetic` builds one on the GPU).  A training step is 4 gfx950
launches for 2 hops (``csrc/hip/sage_tree.hip``): sampling + gather + GEMM + tree mean,
the fused head (last conv, fc, out_fc, loss, backward), the grouped split-K dW with the
tree routing of the outer layer's gradient built in, and the reduce + optimizer + bf16
weight shadows.  All state (RNG counter, optimizer step) is on the device, so the step
is captured once into a hipGraph and replayed; with data parallelism the flat gradient
is all-reduced (RCCL) between the split-K reduce and the optimizer.

Layout: dims are padded (features to 16, conv widths to 64, fc / labels to 32) with
zero rows / columns that provably stay zero (their gradients are exactly zero), and the
mini-batch is the "slotted tree" of ``csrc/hip/tree_args.h`` (power-of-two sibling
groups of F + 1 used slots).  Without dedup every occurrence draws its own neighbours:
the same estimator as the reference flow, in static shapes.

On a CPU device the same model, sampling layout and optimizer run in fp32 torch
(:meth:`_cpu_step`); that implementation is also the numerics oracle of the kernels
(:meth:`reference_loss_and_grads`).  Checkpoints hold the weights in the reference
``SupervisedGraphSage`` parameter names (unpadded), the optimizer slots in the same
names, the step and the Philox ``(seed, counter)``, so training resumes bit-for-bit
on the same sample stream and a checkpoint loads into the torch model for evaluate /
infer.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch
import torch.nn.functional as F

from euler_amd.ops import mp_ops
from euler_amd.ops._native import hip
from euler_amd.models.captured import new_graph

__all__ = ["SageTrainer", "sage_param_names"]

_OPT_KIND = {"adam": 0, "adagrad": 1, "sgd": 2, "momentum": 3}


def _ceil(x: int, m: int) -> int:
    return -(-int(x) // m) * m


def _slot(f: int) -> int:
    """log2 of the sibling-group size of a hop with fanout f (>= 16 rows, >= f + 1 slots)."""
    p = 4
    while (1 << p) < f + 1:
        p += 1
    return p


def sage_param_names(num_layers: int):
    """Parameter names of the reference model (euler_amd.models.SupervisedGraphSage)."""
    names = []
    for k in range(num_layers):
        names += [f"gnn.convs.{k}.self_fc.weight", f"gnn.convs.{k}.neigh_fc.weight"]
    return names + ["gnn.fc.weight", "gnn.fc.bias", "out_fc.weight"]


def _xavier(shape, gen):
    fan_out, fan_in = shape
    a = math.sqrt(6.0 / (fan_in + fan_out))
    return (torch.rand(shape, generator=gen, dtype=torch.float64) * 2 - 1).mul_(a).float()


# which launch carries the next step's sampler blocks: the head (default) or the optimizer
_SAMPLE_IN_OPT = os.environ.get("EULER_AMD_SAMPLE_IN", "head") == "opt"
# pipelined step (2 hops): the optimizer launch gathers the next step's layer-0 inputs on
# the CUs its parameter blocks leave idle, the forward is then GEMM-only
_PIPELINE = os.environ.get("EULER_AMD_PIPELINE", "0") == "1"


class SageTrainer:
    def __init__(self, graph, batch_size, fanouts, dims, label_dim, features=None, labels=None, metapath=None,
                 add_self_loops=False, optimizer="adam", learning_rate=0.01, betas=(0.9, 0.999), eps=1e-8,
                 weight_decay=0.0, init=None, init_seed=0, keep_samples=True, grad_buckets=1, feature_shard=None,
                 feature_dim=None):
        self.graph = graph
        # row-sharded features (graph/sharded_features.py): this rank holds rows r % W; each
        # step's sampled rows come over the all-to-all into a fixed cache the forward reads
        self.fshard = feature_shard
        self.device = graph.device
        self.B = int(batch_size)
        self.fanouts = [int(f) for f in fanouts]
        self.L = len(self.fanouts)
        if not 1 <= self.L <= 3:
            raise ValueError("1 to 3 hops are supported")
        dims = [int(d) for d in dims]
        if len(dims) != self.L + 1:
            raise ValueError("dims = conv widths (one per hop) + the fc width (reference dims[:-1] / dims[-1])")
        if self.B % 32:
            raise ValueError("batch_size must be a multiple of 32")
        self.conv_dims, self.E = dims[:-1], dims[-1]
        if grad_buckets not in (1, 2):
            raise ValueError("grad_buckets must be 1 or 2")
        self.n_buckets = int(grad_buckets)
        self.C = int(label_dim)
        self.include_self = bool(add_self_loops)
        self.opt_name = optimizer
        if optimizer not in _OPT_KIND:
            raise ValueError(f"optimizer must be one of {sorted(_OPT_KIND)}")
        self.lr, self.betas, self.eps, self.wd = float(learning_rate), tuple(betas), float(eps), float(weight_decay)
        if optimizer == "momentum" and betas == (0.9, 0.999):
            self.betas = (0.9, 0.0)  # momentum coefficient (reference MomentumOptimizer(lr, 0.9))
        if optimizer == "adagrad" and eps == 1e-8:
            self.eps = 1e-10
        feats = features if features is not None else graph.features
        if feature_shard is not None:
            feats = feature_shard.shard
            if feats.shape[1] % 16 or feats.dtype not in (torch.bfloat16, torch.float32):
                raise ValueError("sharded features must be bf16 / fp32 with a width padded to 16")
            if feature_dim is not None and _ceil(int(feature_dim), 16) != feats.shape[1]:
                raise ValueError(f"feature_dim {feature_dim} does not pad to the shard's {feats.shape[1]} columns")
        labs = labels if labels is not None else graph.labels
        if feats is None or labs is None:
            raise ValueError("features and labels are required (or a graph built with from_engine)")
        self.D = int(feature_dim) if feature_dim is not None else int(feats.shape[1])  # real width (padded: Dp)
        masks = metapath if metapath is not None else [None] * self.L
        if len(masks) != self.L:
            raise ValueError("one metapath entry (edge types) per hop")
        self.masks = [graph._mask(m) for m in masks]

        # padded widths and the slotted tree
        self.Dp = _ceil(self.D, 16)
        self.Hp = [_ceil(h, 64) for h in self.conv_dims]
        self.Ep, self.Cp = _ceil(self.E, 32), _ceil(self.C, 32)
        self.logP = [0] + [_slot(self.fanouts[k - 1]) for k in range(1, self.L)]
        self.M = [self.B]
        for k in range(1, self.L):
            self.M.append(self.M[-1] << self.logP[k])
        self.on_gpu = self.device.type == "cuda"

        # feature / label tables in the kernels' layout (padded copies only when needed)
        self.features = self._pad_cols(feats, self.Dp, feats.dtype if feats.dtype in (torch.bfloat16,
                                                                                  torch.float32) else torch.float32)
        self.label_mode, self.labels = self._label_table(labs)

        # logical parameters -> padded flat layout
        self._shapes = self._logical_shapes()
        logical = self._init_logical(init, init_seed)
        self._build_flat()
        self.keep_samples = keep_samples  # accepted for compatibility: the sample buffers always exist
        self.step_count = 0  # host mirror (the device counter is authoritative on the GPU)
        if self.on_gpu:
            self._alloc_gpu()
            self.load_logical(logical)
        else:
            self._cpu_params = {k: v.clone().to(self.device).requires_grad_(True) for k, v in logical.items()}
            self._cpu_m = {k: torch.zeros_like(v) for k, v in logical.items()}
            self._cpu_v = {k: torch.full_like(v, 0.1 if optimizer == "adagrad" else 0.0) for k, v in
                           logical.items()}
            self._cpu_loss = torch.zeros(())
            self.pipelined, self._gathered = False, False
            self._cpu_counts = [0, 0, 0]
            self._cpu_samples = None
        self._graph_exec = None

    # ------------------------------------------------------------------ construction helpers
    @classmethod
    def from_model(cls, model, graph, batch_size, optimizer="adam", learning_rate=0.01, **kw):
        """Trainer for a (materialised) ``SupervisedGraphSage``: dims, fanouts, metapath,
        self loops, feature / label names come from the model, weights are copied."""
        from euler_amd.convolution.convs import SAGEConv
        from euler_amd.dataflow.dataflows import SageDataFlow
        import euler_amd.ops.graph_api as ge

        gnn = model.gnn
        if not all(isinstance(c, SAGEConv) for c in gnn.convs) or not isinstance(gnn.sampler, SageDataFlow):
            raise ValueError("the device path trains SAGEConv + SageDataFlow models (SupervisedGraphSage)")
        dims = [c.self_fc.out_features for c in gnn.convs] + [gnn.fc.out_features]
        metapath = []
        for m in gnn.sampler.metapath:
            ids = None if m is None else [int(t) for t in np.asarray(ge.get_edge_type_id(m)).reshape(-1)]
            metapath.append(None if ids is None or any(t < 0 for t in ids) else ids)  # -1 = every type
        return cls(graph, batch_size, gnn.sampler.fanouts, dims, model.label_dim, metapath=metapath,
                   add_self_loops=bool(getattr(gnn.sampler, "add_self_loops", False)), optimizer=optimizer,
                   learning_rate=learning_rate, init=model, **kw)

    def _pad_cols(self, t, width, dtype):
        t = t.to(self.device)
        if t.shape[1] == width and t.dtype == dtype and t.is_contiguous():
            return t
        out = torch.zeros((t.shape[0], width), dtype=dtype, device=self.device)
        out[:, : t.shape[1]] = t.to(dtype)
        return out

    def _label_table(self, labs):
        labs = labs.to(self.device)
        if labs.dim() == 1 or (labs.dim() == 2 and labs.shape[1] == 1 and not labs.is_floating_point()):
            labs = labs.reshape(-1)
            if labs.dtype == torch.int16:
                return 0, labs.contiguous()
            return 1, labs.to(torch.int32).contiguous()
        if labs.shape[1] != self.C:
            raise ValueError(f"label table has {labs.shape[1]} columns, label_dim is {self.C}")
        self._labels_dense = labs.float()
        return 2, self._pad_cols(labs, self.Cp, torch.bfloat16)

    def _logical_shapes(self):
        shapes = {}
        hin = self.D
        for k, h in enumerate(self.conv_dims):
            shapes[f"gnn.convs.{k}.self_fc.weight"] = (h, hin)
            shapes[f"gnn.convs.{k}.neigh_fc.weight"] = (h, hin)
            hin = h
        shapes["gnn.fc.weight"] = (self.E, hin)
        shapes["gnn.fc.bias"] = (self.E,)
        shapes["out_fc.weight"] = (self.C, self.E)
        return shapes

    def _init_logical(self, init, seed):
        if init is not None and not isinstance(init, dict):
            sd = init.state_dict()
            init = {k: sd[k] for k in self._shapes if k in sd}
        gen = torch.Generator().manual_seed(int(seed))
        out = {}
        for k, shp in self._shapes.items():
            if init is not None and k in init:
                v = torch.as_tensor(init[k]).detach().float().cpu()
                if tuple(v.shape) != tuple(shp):
                    raise ValueError(f"{k}: shape {tuple(v.shape)} != {shp}")
                out[k] = v.clone()
            elif k.endswith("bias"):
                out[k] = torch.zeros(shp)
            else:
                out[k] = _xavier(shp, gen)
        return out

    def _build_flat(self):
        """offsets of the padded flat parameter buffer: convs, fc W, fc b, out W"""
        sizes = []
        hin = self.Dp
        for h in self.Hp:
            sizes.append(h * 2 * hin)
            hin = h
        sizes += [self.Ep * hin, self.Ep, self.Cp * self.Ep]
        self.offsets = [0]
        for s in sizes:
            self.offsets.append(self.offsets[-1] + s)

    def _flat_views(self, flat):
        """padded views of a flat buffer: [conv_0 .. conv_{L-1}, fc_w, fc_b, out_w]"""
        o = self.offsets
        views = []
        hin = self.Dp
        for k, h in enumerate(self.Hp):
            views.append(flat[o[k]:o[k + 1]].view(h, 2 * hin))
            hin = h
        L = self.L
        views.append(flat[o[L]:o[L + 1]].view(self.Ep, hin))
        views.append(flat[o[L + 1]:o[L + 2]])
        views.append(flat[o[L + 2]:o[L + 3]].view(self.Cp, self.Ep))
        return views

    def _pack(self, logical, flat):
        """logical (unpadded) tensors -> padded flat buffer (padding zero)"""
        flat.zero_()
        v = self._flat_views(flat)
        hin, hinp = self.D, self.Dp
        for k, h in enumerate(self.conv_dims):
            v[k][:h, :hin] = logical[f"gnn.convs.{k}.self_fc.weight"].to(flat)
            v[k][:h, hinp:hinp + hin] = logical[f"gnn.convs.{k}.neigh_fc.weight"].to(flat)
            hin, hinp = h, self.Hp[k]
        L = self.L
        v[L][: self.E, :hin] = logical["gnn.fc.weight"].to(flat)
        v[L + 1][: self.E] = logical["gnn.fc.bias"].to(flat)
        v[L + 2][: self.C, : self.E] = logical["out_fc.weight"].to(flat)

    def _unpack(self, flat):
        v = self._flat_views(flat)
        out = {}
        hin, hinp = self.D, self.Dp
        for k, h in enumerate(self.conv_dims):
            out[f"gnn.convs.{k}.self_fc.weight"] = v[k][:h, :hin].clone()
            out[f"gnn.convs.{k}.neigh_fc.weight"] = v[k][:h, hinp:hinp + hin].clone()
            hin, hinp = h, self.Hp[k]
        L = self.L
        out["gnn.fc.weight"] = v[L][: self.E, :hin].clone()
        out["gnn.fc.bias"] = v[L + 1][: self.E].clone()
        out["out_fc.weight"] = v[L + 2][: self.C, : self.E].clone()
        return out

    # ------------------------------------------------------------------ GPU buffers + plan
    def _alloc_gpu(self):
        dev, B, L = self.device, self.B, self.L
        bf = dict(dtype=torch.bfloat16, device=dev)
        f32 = dict(dtype=torch.float32, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        n = self.offsets[-1]
        self.flat = torch.zeros(n, **f32)
        self.grad = torch.zeros(n, **f32)
        self.m = torch.zeros(n, **f32)
        self.v = torch.zeros(n, **f32)
        self._step = torch.zeros(1, dtype=torch.int64, device=dev)
        self.loss_acc = torch.zeros(1, **f32)
        self.loss_out = torch.zeros(1, **f32)
        self.counts = torch.zeros(3, **i32)
        if self.opt_name == "adagrad":
            self.v.fill_(0.1)  # reference AdagradOptimizer initial_accumulator_value
        g = self.graph
        d = {"L": L, "B": B, "F": [0] + self.fanouts, "logP": self.logP[:L] if L > 1 else [0],
             "masks": [0] + [int(m) & 0xFFFFFFFF for m in self.masks], "H": self.Hp, "D": self.Dp,
             "E": self.Ep, "C": self.Cp, "C_real": self.C, "include_self": int(self.include_self),
             "indptr": g.indptr, "nbr": g.nbr, "cumw": g.cumw, "num_types": g.num_types, "node_prob": g.node_prob,
             "node_alias": g.node_alias, "root_rows": g.root_rows, "rng": g.rng,
             "labels": self.labels, "label_mode": self.label_mode,
             "step": self._step, "flat": self.flat, "grad": self.grad, "m": self.m, "v": self.v,
             "label_rows": getattr(self, "_label_rows", None),
             "offsets": self.offsets, "loss_acc": self.loss_acc, "loss_out": self.loss_out, "counts": self.counts,
             "lr": self.lr, "beta1": self.betas[0], "beta2": self.betas[1], "eps": self.eps,
             "weight_decay": self.wd, "opt_kind": _OPT_KIND[self.opt_name]}
        for key in ("EULER_AMD_DW_TARGET_WG", "EULER_AMD_DW_MIN_KPS", "EULER_AMD_DW_ROUTE_WG", "EULER_AMD_FWD_BM",
                    "EULER_AMD_DW_ROUTE_IMPL"):
            if os.environ.get(key):
                d[key[len("EULER_AMD_"):].lower()] = int(os.environ[key])
        M_last = self.M[L - 1]
        FL = self.fanouts[-1]
        self.roots = torch.zeros(B, **i32)
        d["roots"] = self.roots
        # the sampler's output (the batch of the next forward)
        self.nodes = torch.zeros(M_last, **i32)
        self.leaf = torch.zeros(M_last * FL, **i32)
        d["nodes"], d["leaf"] = self.nodes, self.leaf
        if self.fshard is None:
            d["features"] = self.features
            if _PIPELINE and L == 2:
                d["A0_rows"] = torch.empty(M_last * 2 * self.Dp, **bf)
        else:
            # the forward gathers from the exchange's cache through cache positions
            n = M_last * (1 + FL)
            self.fshard.alloc_cache(n)
            self._fpos = torch.full((n,), -1, **i32)
            d["fwd_features"] = self.fshard.cache
            d["fwd_nodes"], d["fwd_leaf"] = self._fpos[:M_last], self._fpos[M_last:]
        # layer inputs: A rows (row-major) feed the next layer / head, A_kt the dW GEMMs
        hin = [self.Dp] + self.Hp[:-1]
        for k in range(L):
            rows = self.M[L - 1 - k]
            d[f"A{k}_kt"] = torch.empty(rows * 2 * hin[k], **bf)
            if k >= 1 or L == 1:
                d[f"A{k}"] = torch.empty(rows * 2 * hin[k], **bf)
            if k < L - 1:
                d[f"mask{k}"] = torch.zeros((rows // 32) * self.Hp[k], **i32)
                d[f"dA{k + 1}"] = torch.empty(self.M[L - 2 - k] * 2 * self.Hp[k], **f32)
        H = self.Hp[-1]
        for name, cols in (("h_kt", H), ("emb_kt", self.Ep), ("dlog_kt", self.Cp), ("demb_kt", self.Ep),
                           ("g_kt", H)):
            d[name] = torch.empty(B * cols, **bf)
        views = self._flat_views(self.flat)
        for k in range(L):
            d[f"W{k}_sh"] = torch.empty(views[k].numel(), **bf)
            if k >= 1:
                d[f"W{k}_shT"] = torch.empty(views[k].numel(), **bf)
        for name, t in (("Wfc", views[L]), ("Wout", views[L + 2])):
            d[f"{name}_sh"] = torch.empty(t.numel(), **bf)
            d[f"{name}_shT"] = torch.empty(t.numel(), **bf)
        d["bfc"] = views[L + 1]
        self._buf = d
        self.plan = hip().TreePlan(d)
        self._dw_all = list(range(self.plan.num_problems()))
        self._primed = False  # the sample buffers hold the batch of counter graph.rng[1]
        self.pipelined = bool(self.plan.pipeline_ok())
        self._gathered = False  # A0_rows / A0_kt hold the layer-0 inputs of the sampled batch

    # ------------------------------------------------------------------ parameters / state
    def load_logical(self, logical):
        """Set the weights from logical (unpadded, reference-named) tensors."""
        if self.on_gpu:
            self._pack({k: torch.as_tensor(v) for k, v in logical.items()}, self.flat)
            self.refresh_shadows()
        else:
            with torch.no_grad():
                for k, v in logical.items():
                    self._cpu_params[k].copy_(torch.as_tensor(v).to(self._cpu_params[k]))

    def refresh_shadows(self):
        """Rebuild the bf16 weight shadows from the fp32 parameters (after an external
        write such as a load or the data-parallel broadcast)."""
        if self.on_gpu:
            self.plan.opt(3)

    def logical_params(self):
        if self.on_gpu:
            return self._unpack(self.flat.detach())
        return {k: v.detach().clone() for k, v in self._cpu_params.items()}

    def state_dict(self):
        """Weights in the reference model's names (unpadded)."""
        return {k: v.cpu() for k, v in self.logical_params().items()}

    def write_to_model(self, model):
        """Copy the trained weights into a (materialised) SupervisedGraphSage."""
        sd = model.state_dict()
        with torch.no_grad():
            for k, v in self.logical_params().items():
                sd[k].copy_(v.to(sd[k]))

    def trainer_state(self):
        """Optimizer slots (reference names), step and the device RNG (seed, counter)."""
        if self.on_gpu:
            m, v = self._unpack(self.m), self._unpack(self.v)
            step = int(self._step.item())
        else:
            m = {k: t.clone() for k, t in self._cpu_m.items()}
            v = {k: t.clone() for k, t in self._cpu_v.items()}
            step = self.step_count
        return {"m": {k: t.cpu() for k, t in m.items()}, "v": {k: t.cpu() for k, t in v.items()}, "step": step,
                "rng": self.graph.rng.detach().cpu().clone(), "optimizer": self.opt_name}

    def dp_state_tensors(self):
        """tensors that must be equal on every data-parallel rank (parameters, optimizer
        slots, step): what a re-synchronisation broadcasts from rank 0"""
        if self.on_gpu:
            return [self.flat, self.m, self.v, self._step]
        return [t.data for t in self._cpu_params.values()] + list(self._cpu_m.values()) + list(self._cpu_v.values())

    def load_trainer_state(self, st):
        self.graph.rng.copy_(torch.as_tensor(st["rng"]).to(self.graph.rng))
        self.step_count = int(st["step"])
        self._primed = False
        self._gathered = False
        if self.on_gpu:
            self._pack({k: torch.as_tensor(t) for k, t in st["m"].items()}, self.m)
            self._pack({k: torch.as_tensor(t) for k, t in st["v"].items()}, self.v)
            self._step.fill_(int(st["step"]))
        else:
            for k in self._cpu_m:
                self._cpu_m[k].copy_(torch.as_tensor(st["m"][k]))
                self._cpu_v[k].copy_(torch.as_tensor(st["v"][k]))

    # ------------------------------------------------------------------ training step
    def _prime(self):
        if not self._primed:
            self.plan.sample()
            self._primed = True
            self._gathered = False

    def _fwd(self):
        if self.fshard is not None:
            self.fshard.exchange(torch.cat([self.nodes, self.leaf]), pos_out=self._fpos)
        self.plan.fwd()

    def forward_backward(self):
        """Sampling, forward and backward of one step; the split-K partials are reduced
        into :attr:`grad` (the all-reduce point of data parallelism).  The sample buffers
        keep this step's batch (:meth:`samples`); the next call samples again."""
        p = self.plan
        self._prime()
        self._fwd()
        p.head()
        self._primed = False
        self._gathered = False
        p.bwd()
        p.dw(self._dw_all)
        p.opt(0)

    def optimizer_step(self, grad_scale: float = 1.0):
        self.plan.opt(1, float(grad_scale))

    def grad_buckets(self):
        """(name, start, end) of the data-parallel gradient buckets in the flat layout, in
        the order ``grad_sync`` receives them.  One bucket (default): the whole flat
        gradient.  Two (``grad_buckets=2``): "head" = the last conv, fc and out_fc (their dW
        needs only the head's outputs), then "routed" = the inner convs, whose dW (the
        tree-routed split-K problems, the longest launch of the backward) the head
        bucket's reduce and all-reduce overlap on a side stream."""
        o = self.offsets
        if self.n_buckets == 1 or self.L == 1:
            return [("all", 0, o[-1])]
        return [("head", o[self.L - 1], o[-1]), ("routed", 0, o[self.L - 1])]

    def step(self, grad_sync=None):
        """One training step.  ``grad_sync(bucket)`` (e.g. an in-place RCCL all-reduce)
        is called once per gradient bucket (:meth:`grad_buckets`, in that order) and
        returns the scale applied to the summed gradient (1 / world); None = single
        process (fused reduce + optimizer launch).

        One bucket (default): fwd -> head -> [bwd] -> dW -> reduce -> grad_sync -> optimizer
        on one stream — four graph nodes plus the collective.  Inside a hipGraph a
        side-stream fork / join costs ~5 us per edge on MI355X (measured:
        profiles/r3_dist/), as much as the all-reduce it would hide at one rank.

        Single process: one stream, no forks (a hipGraph branch join costs more than the
        work it would overlap): fwd -> head -> [bwd] -> every dW in one launch ->
        optimizer.  The head launch also carries the sampler of the NEXT step's batch in
        extra blocks, on the CUs the head's B/16 blocks leave idle (sampling reads only the
        graph and the RNG counter the forward advanced; the head reads the forward's copy
        of the roots), so the sampler's dependent-load chain is off the critical path.

        Two buckets: the dW of the "head" bucket (last conv, fc, out_fc) runs on a side
        stream next to the routed inner-layer dW; its split-K reduce and all-reduce then
        overlap the routed dW, and only the routed bucket's (smaller) all-reduce is on the
        critical path.  Both collectives are issued on the side stream in bucket order, so
        every rank enqueues them identically."""
        self.step_count += 1
        if not self.on_gpu:
            return self._cpu_step(grad_sync)
        p = self.plan
        self._prime()
        if self.pipelined and self._gathered:
            p.fwd(None, True)  # layer-0 inputs gathered by the previous optimizer launch
        else:
            self._fwd()
        smp_opt = _SAMPLE_IN_OPT and grad_sync is None
        p.head(None, not smp_opt)
        p.bwd()
        gat = self.pipelined  # this launch gathers the batch the head just sampled
        if grad_sync is None:
            p.dw(self._dw_all)
            p.opt(2, 1.0, smp_opt, gat)
        elif len(self.grad_buckets()) == 1:
            p.dw(self._dw_all)
            p.opt(0, 1.0, False, gat)  # independent of the all-reduce that follows
            g = self.grad if getattr(self, "grad16", None) is None else self.grad16
            scale = grad_sync(g)
            p.opt(1, 1.0 if scale is None else float(scale))
        else:
            self._dist_backward(grad_sync, gat)
        self._primed = True
        self._gathered = gat

    def _dist_backward(self, grad_sync, gather=False):
        p = self.plan
        if not hasattr(self, "_comm_stream"):
            self._comm_stream = torch.cuda.Stream(device=self.device)
            nseg = self.L + 3
            self._segs_head = list(range(self.L - 1, nseg))
            self._segs_routed = list(range(0, self.L - 1))
        g = self.grad if getattr(self, "grad16", None) is None else self.grad16
        (_, a0, a1), (_, b0, b1) = self.grad_buckets()
        main, side = torch.cuda.current_stream(self.device), self._comm_stream
        side.wait_stream(main)
        with torch.cuda.stream(side):
            p.dw(p.problems(False))
            p.opt_segments(0, self._segs_head, True)
            scale = grad_sync(g[a0:a1])
        if self._segs_routed:
            p.dw(p.problems(True))
            p.opt_segments(0, self._segs_routed, False)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                grad_sync(g[b0:b1])
        main.wait_stream(side)
        p.opt(1, 1.0 if scale is None else float(scale), False, gather)

    def plan_launches(self):
        """(name, callable) of every launch of one pipelined step, for per-kernel timing"""
        p = self.plan
        out = [("sample", p.sample), ("fwd", self._fwd), ("head", p.head),
               ("head+sample", lambda: p.head(None, True))]
        if self.L == 3:
            out.append(("bwd", p.bwd))
        out += [("dw", lambda: p.dw(self._dw_all)), ("opt", lambda: p.opt(2))]
        if self.pipelined:
            out += [("opt+gather", lambda: p.opt(2, 1.0, False, True)), ("fwd_gemm", lambda: p.fwd(None, True))]
        return out

    def capture(self, grad_sync=None, warmup: int = 2, steps: int = 1, extra_sizes=()):
        """Record ``steps`` consecutive training steps into one hipGraph (after ``warmup``
        eager steps on a side stream); :meth:`replay` then runs it.  ``grad_sync`` is
        captured too (RCCL collectives are capturable).  ``steps > 1`` amortises the
        per-replay launch gap (~5 us between back-to-back replays of a ~74 us graph,
        profiles/r3_headline/) over several complete steps; a 1-step graph is kept as well,
        and one graph per entry of ``extra_sizes`` (e.g. the remainder of a known step
        count), so :meth:`replay_steps` covers any count with few replays."""
        if not self.on_gpu:
            return None
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.step(grad_sync)
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        self._graphs = {}
        for k in sorted({1, int(steps)} | {int(e) for e in extra_sizes if int(e) > 0}, reverse=True):
            g = new_graph()
            # thread-local capture: RCCL's watchdog thread keeps querying the events of
            # collectives that just finished; under the default global mode such a query
            # during the capture invalidates it and aborts the process (seen on a box:
            # profiles/r3_xgmi/xgmi_bench_capture_race.log)
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                for _ in range(k):
                    self.step(grad_sync)
            self.step_count -= k  # the captured steps did not run
            self._graphs[k] = g
        self._graph_steps = int(steps)
        self._graph_exec = self._graphs[1]
        return self._graphs[int(steps)]

    def replay(self, n: int = 1):
        """n replays of the 1-step graph"""
        for _ in range(int(n)):
            self._graph_exec.replay()
        self.step_count += int(n)

    def replay_steps(self, n: int):
        """exactly n training steps, greedily from the largest captured graph down (the
        multi-step graph as often as it fits, then the remainder graphs, 1-step last)"""
        left = int(n)
        for k in sorted(self._graphs, reverse=True):
            while left >= k:
                self._graphs[k].replay()
                left -= k
        self.step_count += int(n)

    def release_graphs(self):
        """drop the captured graphs (before destroying a process group whose collectives
        they recorded)"""
        for g in getattr(self, "_graphs", {}).values():
            g.reset()
        self._graphs = {}
        self._graph_exec = None

    def set_grad_sync_dtype(self, dtype):
        """Data parallel: the gradient handed to ``grad_sync`` as fp32 (default) or bf16
        (the reduce launch writes bf16, the optimizer reads it back: the all-reduce moves
        half the bytes; an 8-rank all-reduce of this ~1 MB gradient is latency/bandwidth
        bound on the critical path of an ~80 us step)."""
        if not self.on_gpu:
            self.set_grad_sync_dtype_cpu(dtype)
            return
        if dtype in (torch.bfloat16, "bf16", "bfloat16"):
            self.grad16 = torch.zeros(self.grad.numel(), dtype=torch.bfloat16, device=self.device)
            self.plan.set_grad16(self.grad16)
        else:
            self.grad16 = None
            self.plan.set_grad16(None)

    def use_grad_buffer(self, t: torch.Tensor):
        """Data parallel: make ``t`` the gradient buffer that the reduce launch writes and
        ``grad_sync`` receives (fp32 :attr:`grad`, or bf16 :attr:`grad16` after
        ``set_grad_sync_dtype("bf16")``) — e.g. the xGMI all-reduce's IPC input region, so
        the all-reduce runs in place without a staging copy (parallel/xgmi.py)."""
        if not self.on_gpu:
            raise RuntimeError("use_grad_buffer: GPU trainers only")
        if t.dtype == torch.bfloat16:
            if getattr(self, "grad16", None) is None:
                raise ValueError("bf16 gradient buffer without set_grad_sync_dtype('bf16')")
            t.copy_(self.grad16)
            self.grad16 = t
            self.plan.set_grad16(t)
        else:
            t.copy_(self.grad)
            self.grad = t
            self.plan.set_grad(t)

    def set_learning_rate(self, lr: float):
        self.lr = float(lr)
        if self.on_gpu:
            self.plan.set_lr(self.lr)

    @property
    def loss(self) -> torch.Tensor:
        """loss of the last completed step (device scalar)"""
        return self.loss_out if self.on_gpu else self._cpu_loss

    def metric(self) -> float:
        """streaming micro-F1 (threshold 0.5) since the last :meth:`reset_metric`
        (reference metrics.f1_score)"""
        tp, fp, fn = (self.counts.tolist() if self.on_gpu else self._cpu_counts)
        return 2.0 * tp / max(2.0 * tp + fp + fn, 1e-12)

    def reset_metric(self):
        if self.on_gpu:
            self.counts.zero_()
        else:
            self._cpu_counts = [0, 0, 0]

    # ------------------------------------------------------------------ samples + fp32 model
    def samples(self):
        """(roots [B], nodes of the outer layer's target slots [M], leaf draws [M, F_L]) of
        the last step, as int64"""
        if self.on_gpu:
            if self._primed:
                raise RuntimeError("samples() describes the batch of the last forward_backward(); step() has "
                                   "already drawn the next batch into the sample buffers")
            return (self.roots.long(), self.nodes.long(), self.leaf.view(-1, self.fanouts[-1]).long())
        return self._cpu_samples

    def _cpu_sample(self):
        g, B = self.graph, self.B
        g.reseed_cpu()
        roots = g.sample_node(B).long()
        level = roots
        for k in range(1, self.L):
            f, P = self.fanouts[k - 1], 1 << self.logP[k]
            nb = g._sample_neighbor_cpu(level.int(), f, self.masks[k - 1], -1, False).long()
            slots = torch.full((level.numel(), P), -1, dtype=torch.int64)
            slots[:, :f] = nb
            slots[:, f] = level
            level = slots.reshape(-1)
        leaf = g._sample_neighbor_cpu(level.int(), self.fanouts[-1], self.masks[-1], -1, False).long()
        return roots, level, leaf

    def _labels_of(self, roots):
        if self.label_mode == 2:
            return self._labels_dense[roots.to(self._labels_dense.device)].float()
        y = torch.zeros((roots.numel(), self.C), dtype=torch.float32, device=self.labels.device)
        y.scatter_(1, self.labels[roots.to(self.labels.device)].long().view(-1, 1), 1.0)
        return y

    # ------------------------------------------------------------------ inference
    def _tree_of(self, roots):
        """a slotted sample tree (nodes, leaf) of the given rows on the trainer's graph
        (device sampler on the GPU; Philox streams 8.. so training's streams are untouched)"""
        g = self.graph
        level = roots.long()
        types = lambda m: [t for t in range(g.num_types) if (m >> t) & 1]  # noqa: E731
        for k in range(1, self.L):
            f, P = self.fanouts[k - 1], 1 << self.logP[k]
            nb = g.sample_neighbor(level.int(), f, types(self.masks[k - 1]), -1, stream_id=7 + k).view(-1, f).long()
            slots = torch.full((level.numel(), P), -1, dtype=torch.int64, device=level.device)
            slots[:, :f] = nb
            slots[:, f] = level
            level = slots.reshape(-1)
        leaf = g.sample_neighbor(level.int(), self.fanouts[-1], types(self.masks[-1]), -1,
                                 stream_id=7 + self.L).view(-1, self.fanouts[-1]).long()
        g.advance()
        return level, leaf

    @torch.no_grad()
    def infer_logits(self, ids):
        """(embeddings [n, E], logits [n, C], labels [n, C]) of raw node ids: a fresh sample
        tree per root (the reference's infer path samples as its train path does) and the
        fp32 model on the trained parameters"""
        rows = self.graph.rows_of(ids).to(self.graph.device)
        params = self.logical_params()
        nodes, leaf = self._tree_of(rows.clamp(min=0))
        emb = self.logical_embed(params, nodes, leaf)
        logits = emb @ params["out_fc.weight"].float().t().to(emb.device)
        return emb, logits, self._labels_of(rows.clamp(min=0)).to(emb.device)

    def infer_embed(self, ids):
        return self.infer_logits(ids)[0]

    def logical_forward(self, params, roots, nodes, leaf, table=None):
        """fp32 logits of the model for one sampled slotted tree (``table``: the feature rows
        ``nodes`` / ``leaf`` index; default the whole feature table)"""
        emb = self.logical_embed(params, nodes, leaf, table)
        return emb @ params["out_fc.weight"].t()

    def logical_embed(self, params, nodes, leaf, table=None):
        """fp32 gnn embedding (``gnn.fc`` output) of one sampled slotted tree"""
        dev = params["gnn.fc.weight"].device
        tab = self.features if table is None else table
        # the tree's rows are gathered first (-1: zero rows) and only they go to fp32: the
        # whole table in fp32 would be 51 GB at 100M rows (device evaluate / infer)
        xs = mp_ops.gather(tab, nodes.to(tab.device).long())[:, : self.D].float().to(dev)
        agg = mp_ops.gather(tab, leaf.to(tab.device).long())[..., : self.D].float().to(dev).sum(1)
        cnt = self.fanouts[-1]
        if self.include_self:
            agg, cnt = agg + xs, cnt + 1
        w0 = torch.cat([params["gnn.convs.0.self_fc.weight"], params["gnn.convs.0.neigh_fc.weight"]], 1)
        h = torch.relu(torch.cat([xs, agg / cnt], 1) @ w0.t())
        for k in range(1, self.L):
            lvl = self.L - 1 - k
            P, f = 1 << self.logP[lvl + 1], self.fanouts[lvl]
            hg = h.view(-1, P, h.shape[1])
            s, a = hg[:, f], hg[:, :f].sum(1)
            c = f
            if self.include_self:
                a, c = a + s, c + 1
            wk = torch.cat([params[f"gnn.convs.{k}.self_fc.weight"], params[f"gnn.convs.{k}.neigh_fc.weight"]], 1)
            h = torch.relu(torch.cat([s, a / c], 1) @ wk.t())
        return h @ params["gnn.fc.weight"].t() + params["gnn.fc.bias"]

    def reference_loss_and_grads(self, params=None, samples=None):
        """fp32 torch autograd loss and parameter gradients on the last step's samples
        (before its optimizer update: call after :meth:`forward_backward`)"""
        params = {k: v.detach().float().clone().requires_grad_(True)
                  for k, v in (params or self.logical_params()).items()}
        roots, nodes, leaf = samples if samples is not None else self.samples()
        logits = self.logical_forward(params, roots, nodes, leaf)
        y = self._labels_of(roots).to(logits.device)
        loss = F.binary_cross_entropy_with_logits(logits, y)
        loss.backward()
        return float(loss), {k: v.grad.detach() for k, v in params.items()}

    def reference_loss_and_grads_bf16(self, params=None, samples=None, table=None):
        """The bf16-aware fp32 oracle of one tree step: the same model, with every operand
        rounded to bf16 exactly where the fused kernels round it (csrc/hip/sage_tree.hip) and
        everything else in fp32 — so the kernels' step must match it to fp32 accumulation
        order (~1e-6), not to bf16 noise.  Rounding points (bf = round to bf16, RNE):

        * weights: bf16 shadows Wk, Wfc, Wout; Wc = bf(Wout_bf @ Wfc_bf) (tr_comb_wave);
          bc = Wout @ bfc in fp32 (masters);
        * layer 0: A0 = [bf(x_self) | bf(sum(x_leaf (+ x_self)) * inv_leaf)];
          h_k = bf(relu(A_k @ W_k,bf^T)); A_k+1 = [h_self | bf(sum_{j<F} h_j (+ h_self) * inv_grp)];
        * head: logits = h @ Wc^T + bc (fp32), loss = mean BCE (fp32),
          d = bf((sigmoid - y) / (B C)), emb = bf(h @ Wfc_bf^T + bfc), demb = d @ Wout_bf,
          g = bf(relu'(h) * (d @ Wc)), dA = g @ W_bf (fp32);
        * routed gradients (tr_dw_route / tr_bwd): g_k-1 = bf(relu'(h_k-1) * route(dA_k)),
          neighbour slots dA[:, H:] * inv_grp, the self slot dA[:, :H] (+ that share with
          self loops);
        * dW_k = g_k^T @ A_k, dWfc = bf(demb)^T @ h, dWout = d^T @ emb, dbfc = sum demb.

        Reference model semantics: tf_euler/python/convolution/sage_conv.py:33-44,
        mp_utils/base_gnn.py:75-92, mp_utils/base.py:24-47."""
        f32 = torch.float32

        def bf(t):
            return t.to(torch.bfloat16).to(f32)

        P = {k: v.detach().to(f32) for k, v in (params or self.logical_params()).items()}
        roots, nodes, leaf = samples if samples is not None else self.samples()
        dev = P["gnn.fc.weight"].device
        x = (self.features if table is None else table)[:, : self.D].to(dev).to(f32)
        x = torch.cat([x, torch.zeros(1, self.D, device=dev)], 0)
        n = x.shape[0] - 1
        nodes, leaf = nodes.to(dev), leaf.to(dev)
        xs = x[torch.where(nodes < 0, torch.full_like(nodes, n), nodes)]
        agg = x[torch.where(leaf < 0, torch.full_like(leaf, n), leaf)].sum(1)
        inc = 1 if self.include_self else 0
        if inc:
            agg = agg + xs
        inv_leaf = torch.tensor(1.0 / (self.fanouts[-1] + inc), dtype=f32)
        W = [bf(torch.cat([P[f"gnn.convs.{k}.self_fc.weight"], P[f"gnn.convs.{k}.neigh_fc.weight"]], 1))
             for k in range(self.L)]
        A = [torch.cat([bf(xs), bf(agg * inv_leaf)], 1)]
        h = [bf(torch.relu(A[0] @ W[0].t()))]
        groups = []
        for k in range(1, self.L):
            lvl = self.L - 1 - k
            Pg, f = 1 << self.logP[lvl + 1], self.fanouts[lvl]
            hg = h[-1].view(-1, Pg, h[-1].shape[1])
            sf, a = hg[:, f], hg[:, :f].sum(1)
            if inc:
                a = a + sf
            inv = torch.tensor(1.0 / (f + inc), dtype=f32)
            A.append(torch.cat([sf, bf(a * inv)], 1))
            h.append(bf(torch.relu(A[-1] @ W[k].t())))
            groups.append((Pg, f, inv))
        Wfc, bfc, Wout = bf(P["gnn.fc.weight"]), P["gnn.fc.bias"], bf(P["out_fc.weight"])
        Wc = bf(Wout @ Wfc)
        hl = h[-1]
        logits = hl @ Wc.t() + P["out_fc.weight"] @ bfc
        y = self._labels_of(roots).to(dev)
        loss = torch.nn.functional.binary_cross_entropy_with_logits(logits, y)
        d = bf((torch.sigmoid(logits) - y) / float(y.numel()))
        emb = bf(hl @ Wfc.t() + bfc)
        demb = d @ Wout
        grads = {"out_fc.weight": d.t() @ emb, "gnn.fc.weight": bf(demb).t() @ hl, "gnn.fc.bias": demb.sum(0)}
        g = bf((hl > 0).to(f32) * (d @ Wc))
        for k in range(self.L - 1, -1, -1):
            dW = g.t() @ A[k]
            hin = A[k].shape[1] // 2
            grads[f"gnn.convs.{k}.self_fc.weight"] = dW[:, :hin]
            grads[f"gnn.convs.{k}.neigh_fc.weight"] = dW[:, hin:]
            if k == 0:
                break
            dA = g @ W[k]
            Pg, f, inv = groups[k - 1]
            dn = dA[:, hin:] * inv
            ds = dA[:, :hin] + (dn if inc else 0.0)
            route = torch.zeros(dA.shape[0], Pg, hin, device=dev)
            route[:, :f] = dn.unsqueeze(1)
            route[:, f] = ds
            g = bf((h[k - 1] > 0).to(f32) * route.view(-1, hin))
        return float(loss), grads

    def gradients(self):
        """logical view of :attr:`grad` after :meth:`forward_backward` (GPU)"""
        return self._unpack(self.grad)

    def set_grad_sync_dtype_cpu(self, dtype):
        self._cpu_sync_bf16 = dtype in (torch.bfloat16, "bf16", "bfloat16")

    def _cpu_forward_backward(self):
        """fp32 autograd forward + backward of a fresh batch: p.grad of every parameter"""
        roots, nodes, leaf = self._cpu_sample()
        self._cpu_samples = (roots, nodes, leaf)
        P = self._cpu_params
        for t in P.values():
            t.grad = None
        table = None
        if self.fshard is not None:
            pos = self.fshard.exchange(torch.cat([nodes, leaf.reshape(-1)])).long()
            nodes, leaf = pos[: nodes.numel()], pos[nodes.numel():].view_as(leaf)
            table = self.fshard.cache
        logits = self.logical_forward(P, roots, nodes, leaf, table)
        y = self._labels_of(roots).to(logits.device)
        loss = F.binary_cross_entropy_with_logits(logits, y)
        loss.backward()
        with torch.no_grad():
            pred, pos = logits >= 0, y > 0.5
            self._cpu_counts[0] += int((pred & pos).sum())
            self._cpu_counts[1] += int((pred & ~pos).sum())
            self._cpu_counts[2] += int((~pred & pos).sum())
        self.graph.rng[1] += 1
        return loss.detach()

    def _cpu_grad_sync(self, grad_sync):
        """the GPU path's data-parallel hand-off on the CPU twin: the gradients in the flat
        (logical) parameter order, the same buckets in the same order, fp32 or bf16"""
        names = list(self._shapes)
        flat = torch.cat([self._cpu_params[k].grad.reshape(-1) for k in names])
        buf = flat.to(torch.bfloat16) if getattr(self, "_cpu_sync_bf16", False) else flat
        if len(self.grad_buckets()) == 1:
            scale = grad_sync(buf)
        else:
            cut = sum(self._cpu_params[k].numel() for k in names[: 2 * (self.L - 1)])  # routed convs first
            scale = grad_sync(buf[cut:])
            grad_sync(buf[:cut])
        flat = buf.float()
        o = 0
        for k in names:
            n = self._cpu_params[k].numel()
            self._cpu_params[k].grad = flat[o:o + n].view_as(self._cpu_params[k]).clone()
            o += n
        return 1.0 if scale is None else float(scale)

    def _cpu_apply(self, grad_scale=1.0):
        """optimizer step from p.grad (scaled by grad_scale), same update rule as tr_opt"""
        P = self._cpu_params
        with torch.no_grad():
            t = float(self.step_count)
            b1, b2 = self.betas
            for k, p in P.items():
                g = p.grad * grad_scale + self.wd * p
                m, v = self._cpu_m[k], self._cpu_v[k]
                if self.opt_name == "adam":
                    m.mul_(b1).add_(g, alpha=1 - b1)
                    v.mul_(b2).addcmul_(g, g, value=1 - b2)
                    p -= self.lr * (m / (1 - b1 ** t)) / (torch.sqrt(v / (1 - b2 ** t)) + self.eps)
                elif self.opt_name == "adagrad":
                    v.addcmul_(g, g)
                    p -= self.lr * g / (torch.sqrt(v) + self.eps)
                elif self.opt_name == "sgd":
                    p -= self.lr * g
                else:
                    m.mul_(b1).add_(g)
                    p -= self.lr * m

    def _cpu_step(self, grad_sync=None):
        loss = self._cpu_forward_backward()
        scale = self._cpu_grad_sync(grad_sync) if grad_sync is not None else 1.0
        self._cpu_apply(scale)
        self._cpu_loss = loss
        return self._cpu_loss
