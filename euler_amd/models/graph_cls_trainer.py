"""Fused device-path training step for the pooled graph-classification models whose
convolutions are a linear map of an aggregate: GIN and GraphGCN (``models/
graph_classification.py``), under ``GraphEstimator(device_graph=True)``.

Reference: ``examples/gin/gin.py`` / ``examples/graphgcn/graphgcn.py`` (sparse-feature
embedding bag, ``GNN(conv, 'full', dims)``, add pooling), ``tf_euler/python/convolution/
gin_conv.py:26-57`` (``mlp((1 + eps) x + sum_j x_j)``), ``convolution/graph_conv.py:26-46``
(``liner(x) + mean_j fc(x_j)``), ``mp_utils/base_graph.py:24-47`` (``out_fc``, sigmoid
cross-entropy), ``euler_estimator/python/graph_estimator.py:27-85`` (uniform graph draw).

The generic :class:`~euler_amd.models.graph_trainer.GraphTrainer` builds the batch's
induced blocks with :class:`~euler_amd.dataflow.device_flow.DeviceFullFlow` and runs the
model's own modules: ~60 launches per step for 5 layers.  Graphs are small (MUTAG: 10-28
nodes), so this trainer gives each drawn graph one workgroup that keeps all of its nodes in
LDS for the whole step (``csrc/hip/graph_cls.hip``): 2 launches per step; the graph is
densified in LDS (adjacency count matrix, feature bag matrix) so embedding, aggregation,
linear and their gradients are all fp32 MFMA GEMMs; every gradient is written once into a
per-graph slab row, and the slab reduction is fused with the flat optimizer on one process.
The graphs' adjacency (CSR with local node indices, per distinct edge-type mask), node
feature ids and labels are uploaded once.

The draw is the generic trainer's (the alias table on the graph RNG's Philox stream 3 at
the advanced counter), so both trainers see the same graphs from the same RNG state;
``tests/test_graph_cls_trainer.py`` pins the loss and every gradient against an fp32
torch oracle.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from euler_amd.models.graph_trainer import GraphTrainer
from euler_amd.ops._native import hip

__all__ = ["GraphClsTrainer"]

_MAX_ROWS, _MAX_WIDTH, _MAX_LABELS, _MAX_TABLE, _MAX_TABLE_ROWS, _MAX_LAYERS = 64, 128, 64, 8192, 64, 8


def _conv_kind(model):
    """0 (GIN, default mlp), 1 (GraphConv) or None for anything else"""
    from euler_amd.convolution.convs import GINConv, GraphConv
    from euler_amd.graph_pool import Pooling
    from euler_amd.mp_utils.models import BaseGNNNet
    from euler_amd.utils.layers import Dense, SparseEmbedding

    gnn = getattr(model, "gnn", None)
    if gnn is None or type(getattr(gnn, "encoder", None)) is not SparseEmbedding:
        return None
    if type(gnn).forward is not BaseGNNNet.forward or type(gnn).calculate_conv is not BaseGNNNet.calculate_conv:
        return None
    pool = getattr(model, "pool", None)
    if type(pool) is not Pooling or pool.aggr != "add":
        return None
    convs = list(gnn.convs)
    if not 1 <= len(convs) <= _MAX_LAYERS:
        return None
    dense = [gnn.fc, model.out_fc]
    if all(type(c) is GINConv for c in convs):
        if not all(type(c.mlp) is Dense and c.mlp.bias is None for c in convs):
            return None
        dense += [c.mlp for c in convs]
        kind = 0
    elif all(type(c) is GraphConv for c in convs):
        if not all(c.fc.bias is None and c.liner.bias is not None for c in convs):
            return None
        dense += [c.fc for c in convs] + [c.liner for c in convs]
        kind = 1
    else:
        return None
    if any(type(d) is not Dense or d.activation is not None for d in dense):
        return None
    if model.out_fc.bias is not None or gnn.fc.bias is None:
        return None
    return kind


class GraphClsTrainer(GraphTrainer):
    """:class:`GraphTrainer` with the fused two-launch step (same batches, same model)."""

    @staticmethod
    def supports(model) -> bool:
        if os.environ.get("EULER_AMD_GRAPH_FUSED", "1") == "0":
            return False
        return _conv_kind(model) is not None

    def __init__(self, model, graph, batch_size, label_feature, num_classes, optimizer="adam", learning_rate=0.01):
        if graph.device.type != "cuda":
            raise ValueError("the fused graph-classification step runs on the GPU (GraphTrainer covers the CPU)")
        self.kind = _conv_kind(model)
        if self.kind is None:
            raise ValueError("GraphClsTrainer trains GIN (default mlp) and GraphGCN models with add pooling")
        super().__init__(model, graph, batch_size, label_feature, num_classes, optimizer, learning_rate)
        self.plan = hip().GraphClsPlan(self._plan_dict())
        self._fused_opt = self._set_fused_optimizer()

    # ------------------------------------------------------------------ static inputs
    def _edge_pairs(self, mask, nodes):
        """every graph's edges t <- s under ``mask`` as (t << 8) | s in local node indices,
        graph by graph (the flow's full-neighbour expansion of t: its out-neighbour list,
        types in order, repeats kept), and each graph's [begin, end)"""
        g = self.graph
        T = g.num_types
        indptr = g.indptr.cpu().numpy()
        nbr = g.nbr.cpu().numpy()
        types = [t for t in range(T) if (mask >> t) & 1]
        pairs, spans = [], []
        for gi, rows in enumerate(nodes):
            local = {int(r): v for v, r in enumerate(rows)}
            e0 = len(pairs)
            for v, r in enumerate(rows):
                for t in types:
                    a, b = int(indptr[r * T + t]), int(indptr[r * T + t + 1])
                    for s in nbr[a:b]:
                        s = int(s)
                        if s not in local:
                            raise ValueError(f"graph {gi}: node row {r} has a neighbour outside its graph")
                        pairs.append((v << 8) | local[s])
            spans.append((e0, len(pairs)))
        return pairs, spans

    def _plan_dict(self):
        m, gnn = self.model, self.gnn
        convs = list(gnn.convs)
        L = len(convs)
        gmat = self.gnodes.cpu().numpy()
        nodes = [[int(r) for r in row if r >= 0] for row in gmat]
        if any(len(set(ns)) != len(ns) for ns in nodes):
            raise ValueError("a graph lists a node twice")
        counts = np.array([len(ns) for ns in nodes], np.int64)
        if counts.max() > _MAX_ROWS:
            raise ValueError(f"graphs of more than {_MAX_ROWS} nodes")
        # edge pairs of every distinct mask
        masks, adj_of, pairs, spans = [], [], [], []
        for mk in self._layer_masks():
            if mk not in masks:
                masks.append(mk)
                p, sp = self._edge_pairs(mk, nodes)
                pairs.append(p)
                spans.append(sp)
            adj_of.append(masks.index(mk))
        if len(masks) > 4:
            raise ValueError("more than 4 distinct edge-type masks")
        # feature occurrences (embedding-table rows, GraphTrainer.feat_ids) and bag weights
        enc = gnn.encoder
        fmat = self.feat_ids.cpu().numpy()
        fpair, fw, fspan = [], [], []
        for ns in nodes:
            f0 = len(fpair)
            for v, r in enumerate(ns):
                f = [int(x) for x in fmat[r] if x >= 0]
                fpair += [(v << 16) | x for x in f]
                fw += [1.0 / len(f) if enc.combiner == "mean" else 1.0] * len(f)
            fspan.append((f0, len(fpair)))
        rec = np.zeros((len(nodes), 12), np.int64)
        rec[:, 0] = counts
        rec[:, 1:3] = np.asarray(fspan, np.int64).reshape(-1, 2)
        for j, sp in enumerate(spans):
            rec[:, 3 + 2 * j:5 + 2 * j] = np.asarray(sp, np.int64).reshape(-1, 2)
        dev = self.graph.device
        i32 = lambda a: torch.as_tensor(np.asarray(a, np.int64).astype(np.int32), device=dev)
        D = [int(enc.weight.shape[1])]
        for c in convs:
            w = c.mlp.weight if self.kind == 0 else c.liner.weight
            D.append(int(w.shape[0]))
        E, C = int(gnn.fc.weight.shape[0]), int(m.out_fc.weight.shape[0])
        if any(d % 16 or d > _MAX_WIDTH for d in D) or E > _MAX_WIDTH or C > _MAX_LABELS:
            raise ValueError(f"widths must be multiples of 16 up to {_MAX_WIDTH} (labels <= {_MAX_LABELS})")
        if enc.weight.numel() > _MAX_TABLE or enc.weight.shape[0] > _MAX_TABLE_ROWS:
            raise ValueError(f"the embedding table exceeds {_MAX_TABLE_ROWS} rows / {_MAX_TABLE} elements")
        if int(gnn.fc.weight.shape[1]) != D[-1] or int(m.out_fc.weight.shape[1]) != E:
            raise ValueError("fc / out_fc widths do not chain")
        # flat offsets of every parameter
        where = {id(p): o for p, (o, n) in zip(self.flat.params, self.flat.offsets)}
        covered = []

        def off(p):
            o = where[id(p)]
            covered.append((o, p.numel()))
            return o

        W, Wf, bl, eps, oW, oWf, obl, oeps = [], [], [], [], [], [], [], []
        for c in convs:
            if self.kind == 0:
                W.append(c.mlp.weight.detach())
                oW.append(off(c.mlp.weight))
                e = c.eps
                eps.append(e.detach() if isinstance(e, torch.nn.Parameter) else e)
                oeps.append(off(e) if isinstance(e, torch.nn.Parameter) and e.requires_grad else -1)
                Wf.append(None)
                bl.append(None)
                oWf.append(-1)
                obl.append(-1)
            else:
                W.append(c.liner.weight.detach())
                Wf.append(c.fc.weight.detach())
                bl.append(c.liner.bias.detach())
                oW.append(off(c.liner.weight))
                oWf.append(off(c.fc.weight))
                obl.append(off(c.liner.bias))
                eps.append(None)
                oeps.append(-1)
        d = {"L": L, "B": self.B, "kind": self.kind, "self_loops": int(bool(gnn.sampler.add_self_loops)),
             "nmax": int(-(-counts.max() // 16) * 16), "D": D, "E": E, "C": C,
             "G": len(nodes), "tab_rows": int(enc.weight.shape[0]),
             "adj_pair": [i32(p if p else [0]) for p in pairs], "adj_of": adj_of, "rec": i32(rec),
             "fpair": i32(fpair if fpair else [0]),
             "fw": torch.tensor(fw if fw else [0.0], dtype=torch.float32, device=dev),
             "gprob": self.g_prob.float().contiguous(), "galias": self.g_alias.to(torch.int32).contiguous(),
             "rng": self.graph.rng,
             "onehot": self.onehot.float().contiguous(), "table": enc.weight.detach(),
             "W": W, "Wf": Wf, "bl": bl, "eps": eps, "o_W": oW, "o_Wf": oWf, "o_bl": obl, "o_eps": oeps,
             "Wfc": gnn.fc.weight.detach(), "bfc": gnn.fc.bias.detach(), "Wout": m.out_fc.weight.detach(),
             "o_fc": off(gnn.fc.weight), "o_bfc": off(gnn.fc.bias), "o_out": off(m.out_fc.weight),
             "o_tab": off(enc.weight), "S": int(self.flat.numel), "grad": self.flat.grad,
             "loss_out": self.loss_out, "right": self.right, "warm": self.flat.flat}
        if os.environ.get("EULER_AMD_GRAPH_MAX_LDS"):  # tests: force the recomputed-Z path
            d["max_lds"] = int(os.environ["EULER_AMD_GRAPH_MAX_LDS"])
        # every flat parameter gets its gradient from the slab (no other trainable tensor)
        cov = sorted(covered)
        pos = 0
        for o, n in cov:
            if o != pos:
                raise ValueError("the model has parameters the fused step does not train")
            pos = o + n
        if pos != self.flat.numel:
            raise ValueError("the model has parameters the fused step does not train")
        return d

    def _layer_masks(self):
        import euler_amd.ops.graph_api as ge

        out = []
        for mp in self.gnn.sampler.metapath:
            ids = None if mp is None else [int(t) for t in np.asarray(ge.get_edge_type_id(mp)).reshape(-1)]
            out.append(int(self.graph._mask(None if ids is None or any(t < 0 for t in ids) else ids)))
        return out

    def _set_fused_optimizer(self, grad_scale: float = 1.0) -> bool:
        from euler_amd.parallel.flat import _KINDS

        o = self.opt
        if o.decay_range[1] > o.decay_range[0]:
            return False
        return bool(self.plan.set_optimizer({
            "flat": self.flat.flat, "m": o.m, "v": o.v, "step": o.step_count, "kind": _KINDS[o.kind], "lr": o.lr,
            "b1": o.b1, "b2": o.b2, "eps": o.eps, "wd": o.wd, "grad_scale": float(grad_scale)}))

    def set_learning_rate(self, lr):
        super().set_learning_rate(lr)
        self._fused_opt = self._set_fused_optimizer()

    # ------------------------------------------------------------------ step
    def _step(self, grad_sync=None):
        if grad_sync is None and self._fused_opt:  # one process: the update rides the reduce
            self.plan.step(True)
            return self.loss_out
        self.plan.step()
        scale = 1.0
        if grad_sync is not None:
            s = grad_sync(self.flat.grad)
            scale = 1.0 if s is None else float(s)
        self.opt.step(scale)
        return self.loss_out

    def forward_backward_only(self):
        """the step without the optimizer (tests): loss_out and the flat gradient"""
        self.plan.step()
        return self.loss_out

    @property
    def launches_per_step(self) -> int:
        return 2 if self._fused_opt else 3

    def samples(self):
        return (self.plan.gidx(),)
