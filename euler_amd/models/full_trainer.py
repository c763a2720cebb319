"""Device-path training of the full-neighbourhood GNN zoo (GCN, APPNP, SGCN, TAGCN, AGNN,
ARMA, DNA, GAT — every ``SupervisedGNN`` whose flow is ``"full"``).

Reference: ``examples/gcn/gcn.py:52-58`` (``GNN('gcn', 'full', ...)``) over
``tf_euler/python/dataflow/gcn_dataflow.py:26-48``, ``convolution/gcn_conv.py:26-54``, the
supervised head of ``mp_utils/base.py:24-47`` and the estimator's ``sample_node`` roots
(``euler_estimator/python/node_estimator.py``).

The engine path samples every batch on the CPU graph engine (one GQL query per hop, a
``tf.unique`` per hop, dynamic shapes), then ships ids and features to the GPU: the GPU
waits on the host every step.  Here the whole step lives on the device:

* roots: the alias-table ``sample_node`` on the HBM graph (Philox stream 1 of the graph's
  (seed, counter));
* blocks: :class:`~euler_amd.dataflow.device_flow.DeviceFullFlow` (HIP full-neighbour
  expansion + hash unique, capacity-padded with ``-1``);
* the model: the user's own convolution modules, unchanged, on the padded blocks (every
  ``mp_ops`` kernel drops ``-1`` edges and reads ``-1`` rows as zeros), ``fc`` and
  ``out_fc``, sigmoid cross-entropy on the roots' dense labels;
* backward, the data-parallel all-reduce hook and one flat optimizer launch
  (``parallel/flat.py``, ``csrc/hip/optim.hip``) over the model's parameters re-homed into
  one buffer.

Every shape is fixed, so warm-up runs eagerly once and the step is captured into a
hipGraph (several steps per graph; ``replay_steps``), like ``SageTrainer``.  Checkpoints
hold the model's own parameter names (``state_dict``), the optimizer slots and the
graph's Philox (seed, counter).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist
import torch.nn.functional as F

from euler_amd.dataflow.device_flow import DeviceFullFlow
from euler_amd.models.captured import CapturedTrainer
from euler_amd.ops import gnn_ops, mp_ops

__all__ = ["FullFlowTrainer", "ShardedFlowTrainer", "full_flow_embed", "infer_flow"]


def full_flow_embed(gnn, flow, features, roots):
    """(gnn embedding [B, E], DataFlow) of ``roots`` through the model's convolutions on a
    device flow (ReLU after every conv, then ``gnn.fc``: BaseGNNNet.forward)"""
    df = flow.produce(roots)
    # a callable: rows -> feature rows (a row-sharded table's exchange, graph/sharded_graph.py)
    x = (features(df[0].n_id) if callable(features) else mp_ops.gather(features, df[0].n_id)).float()
    for conv, block in zip(gnn.convs, df):
        x_t = mp_ops.gather(x, block.res_n_id)
        x = F.relu(gnn.calculate_conv(conv, (x_t, x), block.edge_index, size=block.size))
    return gnn.fc(x), df


def infer_flow(owner, graph, masks, self_loops, n):
    """a cached exact-capacity DeviceFullFlow of ``n`` roots for inference batches (the
    last id-file batch is shorter; the GCN normalisation depends on the whole block, so
    a batch is never padded)"""
    cache = owner.__dict__.setdefault("_infer_flows", {})
    if n not in cache:
        cache[n] = DeviceFullFlow(graph, masks, n, self_loops, "exact")
    return cache[n]


class FullFlowTrainer(CapturedTrainer):
    metric_name = "f1"

    def __init__(self, model, graph, batch_size, masks, add_self_loops=True, features=None, labels=None,
                 optimizer="adam", learning_rate=0.01, caps=None, flow=None):
        self.gnn = getattr(model, "gnn", None)  # None: an encoder model (models/encoder_trainer.py)
        self.graph = graph
        self.B = int(batch_size)
        feats = features if features is not None else graph.features
        labs = labels if labels is not None else graph.labels
        if feats is None or labs is None:
            raise ValueError("the device graph needs dense features and labels (DeviceGraph.from_engine)")
        self.features = feats.to(graph.device)
        self.labels = labs.to(graph.device).float()
        # the full-neighbourhood flow by default; a given flow (DeviceSageFlow for models on
        # the sampled SageDataFlow whose convolutions are not the fused SAGE kernels)
        self.flow = flow if flow is not None else DeviceFullFlow(graph, masks, self.B, add_self_loops, caps)
        self.counts = torch.zeros(3, dtype=torch.int64, device=graph.device)
        super().__init__(model, graph, graph.device, optimizer, learning_rate)

    # ------------------------------------------------------------------ construction
    @classmethod
    def from_model(cls, model, graph, batch_size, optimizer="adam", learning_rate=0.01, **kw):
        """Trainer for a (materialised) full-flow ``SupervisedGNN``: metapath, self loops and
        the layers come from the model."""
        import euler_amd.ops.graph_api as ge
        from euler_amd.dataflow.dataflows import GCNDataFlow

        from euler_amd.dataflow.dataflows import SageDataFlow
        from euler_amd.dataflow.device_flow import DeviceSageFlow

        from euler_amd.dataflow.dataflows import FastGCNDataFlow, LayerwiseDataFlow
        from euler_amd.dataflow.device_flow import DeviceLayerFlow

        flow = getattr(model.gnn, "sampler", None)
        if not isinstance(flow, (GCNDataFlow, SageDataFlow, FastGCNDataFlow, LayerwiseDataFlow)):
            raise ValueError("FullFlowTrainer trains models on the full-neighbourhood flow (GCNDataFlow), the "
                             "sampled SageDataFlow or the layer-sampled FastGCN / AdaptiveGCN flows")
        ets = []
        for m in flow.metapath:
            ids = None if m is None else [int(t) for t in np.asarray(ge.get_edge_type_id(m)).reshape(-1)]
            ets.append(None if ids is None or any(t < 0 for t in ids) else ids)
        dflow = None
        if isinstance(flow, SageDataFlow):
            dflow = DeviceSageFlow(graph, ets, flow.fanouts, batch_size, bool(flow.add_self_loops))
        elif isinstance(flow, (FastGCNDataFlow, LayerwiseDataFlow)):
            fast = isinstance(flow, FastGCNDataFlow)
            samplers = [None] * len(ets)
            if fast:
                # FastGCN's layer: sample_node(total, metapath[h][0]) (fast_dataflow.py:44-46)
                import copy

                _, _, nw = ge.get_engine().export_nodes()
                for h, m in enumerate(flow.metapath[:-1]):
                    nt = m[0] if isinstance(m, (list, tuple)) else m
                    tid = int(np.asarray(ge.get_node_type_id(nt)).reshape(-1)[0])
                    samplers[h] = copy.copy(graph)
                    samplers[h].set_root_type(tid if tid >= 0 else -1, node_weights=np.asarray(nw))
            kinds = ["fast" if fast else "layer"] * (len(ets) - 1) + ["full"]
            dflow = DeviceLayerFlow(graph, [graph._mask(e) for e in ets], kinds, list(flow.fanouts)[:len(ets)],
                                    batch_size, bool(flow.add_self_loops), samplers=samplers)
        return cls(model, graph, batch_size, [graph._mask(e) for e in ets], add_self_loops=bool(flow.add_self_loops),
                   optimizer=optimizer, learning_rate=learning_rate, flow=dflow, **kw)

    def _materialize(self):
        """one no-grad pass so lazy layers get their shapes (they keep the values the
        model's own initialisation gives them)"""
        if not any(isinstance(p, torch.nn.parameter.UninitializedParameter) for p in self.model.parameters()):
            return
        state = self.graph.rng.clone()
        with torch.no_grad():
            self._forward(self.graph.sample_node(self.B).long())
        self.graph.rng.copy_(state)

    # ------------------------------------------------------------------ model
    def _forward(self, roots):
        """logits [B, label_dim] of the roots through the user's convolutions"""
        emb, df = full_flow_embed(self.gnn, self.flow, self.features, roots)
        return self.model.out_fc(emb).float(), df

    # ------------------------------------------------------------------ inference
    def _infer_flow(self, n):
        # exactly the full-neighbourhood flow: DeviceLayerFlow (FastGCN / AdaptiveGCN) subclasses
        # it but samples its layers, so those models infer on the engine path as the reference
        # does (fast_dataflow / LayerwiseDataFlow draws)
        if self.gnn is None or type(self.flow) is not DeviceFullFlow:
            return None  # sampled flows: the engine path infers (their draws are the engine's)
        return infer_flow(self, self.graph, self.flow.masks, self.flow.self_loops, n)

    @torch.no_grad()
    def infer_logits(self, ids):
        """(embeddings [n, E], logits [n, C], labels [n, C]) of raw node ids on the device,
        one full-neighbourhood block of exactly these roots (the engine path's batch)"""
        flow = self._infer_flow(int(torch.as_tensor(ids).numel()))
        if flow is None:
            raise NotImplementedError("device inference covers the full-neighbourhood flow")
        rows = self.graph.rows_of(ids).to(self.graph.device)
        self.model.eval()
        try:
            emb, _ = full_flow_embed(self.gnn, flow, self.features, rows)
            logits = self.model.out_fc(emb).float()
        finally:
            self.model.train()
        return emb.float(), logits, self.labels[rows.clamp(min=0)]

    def infer_embed(self, ids):
        return self.infer_logits(ids)[0]

    def _forward_loss(self):
        self._draw()
        roots = self.graph.sample_node(self.B, stream_id=1).long()
        logits, df = self._forward(roots)
        # sigmoid cross-entropy + the F1 counts in one kernel pair (gnn_ops.bce_f1_loss)
        loss = gnn_ops.bce_f1_loss(logits, self.labels, roots, self.counts)
        self._samples = roots
        return loss

    # ------------------------------------------------------------------ metric
    def metric(self) -> float:
        tp, fp, fn = self.counts.tolist()
        return 2.0 * tp / max(2.0 * tp + fp + fn, 1e-12)

    def reset_metric(self):
        self.counts.zero_()

    def samples(self):
        """roots of the last step"""
        return (self._samples,)

    # ------------------------------------------------------------------ oracle
    def reference_loss_and_grads(self, roots):
        """fp32 loss and parameter gradients of the model on ``roots`` through the engine
        path's own dataflow (``GCNDataFlow`` on the CPU graph engine, dynamic shapes) — the
        numerics oracle of the padded device step"""
        import euler_amd.ops.graph_api as ge

        raise_if = None  # noqa: F841
        ids = self.graph.ids
        raw = torch.as_tensor(np.asarray(ids)[roots.cpu().numpy()].astype(np.int64)) if ids is not None else \
            roots.cpu()
        params = {n: p for n, p in self.model.named_parameters()}
        saved = {n: p.grad for n, p in params.items()}
        for p in params.values():
            p.grad = None
        logits = self.model.embed(raw)
        logits = self.model.out_fc(logits).float()
        y = ge.get_dense_feature(raw, [self.model.label_idx], [self.model.label_dim])[0].to(logits.device).float()
        loss = F.binary_cross_entropy_with_logits(logits, y)
        loss.backward()
        grads = {n: p.grad.detach().clone() for n, p in params.items()}
        for n, p in params.items():
            p.grad = saved[n]
        self.flat.rebind_grads()
        return float(loss), grads


class ShardedFlowTrainer(FullFlowTrainer):
    """A sampled-``SageDataFlow`` model (any convolution) trained on a graph row-sharded over
    the data-parallel ranks (:class:`~euler_amd.graph.sharded_graph.ShardedDeviceGraph`):
    roots drawn with the global root weights, each hop's fixed-fanout draws answered by the
    rows' owners over the all-to-all, the input features and the roots' labels fetched from
    their owners; the model's own convolutions, loss, backward, gradient all-reduce and the
    flat optimizer run as in :class:`FullFlowTrainer`.  HBM per rank holds 1/W of the CSR,
    the features and the labels.  A ``GCNDataFlow`` model expands every hop through the
    rows' owners (``ShardedDeviceGraph.full_neighbors``).  Steps over RCCL capture into a
    hipGraph (fixed-size exchanges); gloo steps run eagerly (:meth:`capturable`)."""

    def __init__(self, model, graph, batch_size, flow, optimizer="adam", learning_rate=0.01):
        self.gnn = model.gnn
        self.graph = graph
        self.B = int(batch_size)
        if graph.features is None or graph.labels is None:
            raise ValueError("the sharded graph needs dense features and labels")
        self.features = graph.gather_features
        self.labels = None
        self.flow = flow
        self.counts = torch.zeros(3, dtype=torch.int64, device=graph.device)
        self._rows = torch.arange(self.B, device=graph.device)
        CapturedTrainer.__init__(self, model, graph, graph.device, optimizer, learning_rate)

    @classmethod
    def from_model(cls, model, graph, batch_size, optimizer="adam", learning_rate=0.01, caps="bounded", **kw):
        import euler_amd.ops.graph_api as ge
        from euler_amd.dataflow.dataflows import GCNDataFlow, SageDataFlow
        from euler_amd.dataflow.device_flow import DeviceFullFlow, DeviceSageFlow

        flow = getattr(model.gnn, "sampler", None)
        if not isinstance(flow, (SageDataFlow, GCNDataFlow)):
            raise ValueError("the sharded device graph trains models on the sampled SageDataFlow (fixed fanouts) "
                             "or the full-neighbourhood GCNDataFlow")
        ets = []
        for m in flow.metapath:
            ids = None if m is None else [int(t) for t in np.asarray(ge.get_edge_type_id(m)).reshape(-1)]
            ets.append(None if ids is None or any(t < 0 for t in ids) else ids)
        if isinstance(flow, SageDataFlow):
            dflow = DeviceSageFlow(graph, ets, flow.fanouts, batch_size, bool(flow.add_self_loops))
        else:
            # every hop expanded by the rows' owners (ShardedDeviceGraph.full_neighbors),
            # capacities from the degree statistics reduced over the ranks
            dflow = DeviceFullFlow(graph, [graph._mask(e) for e in ets], batch_size, bool(flow.add_self_loops), caps)
        return cls(model, graph, batch_size, dflow, optimizer=optimizer, learning_rate=learning_rate)

    def _forward_loss(self):
        self._draw()
        roots = self.graph.sample_node(self.B, stream_id=1).long()
        logits, df = self._forward(roots)
        y = self.graph.gather_labels(roots).float().contiguous()
        loss = gnn_ops.bce_f1_loss(logits, y, self._rows, self.counts)
        self._samples = roots
        return loss

    # evaluate / infer on the device, collectively: every rank calls with batches of the same
    # padded size in lockstep (estimator/base.py _lockstep_batches)
    collective_infer = True

    def _sharded_infer_flow(self, n):
        """the training flow's kind at ``n`` roots (cached): the sampled flow as trained, the
        full flow on degree-statistics caps grown on overflow (exact caps at hundreds of
        millions of rows would reach the whole edge set)"""
        from euler_amd.dataflow.device_flow import DeviceFullFlow, DeviceSageFlow

        cache = self.__dict__.setdefault("_infer_flows", {})
        if n not in cache:
            f = self.flow
            if isinstance(f, DeviceSageFlow):
                cache[n] = DeviceSageFlow(self.graph, f.edge_types, f.fanouts, n, f.self_loops)
            else:
                cache[n] = DeviceFullFlow(self.graph, f.masks, n, f.self_loops, "bounded")
        return cache[n]

    @torch.no_grad()
    def infer_logits(self, ids, pad_to=None):
        """(embeddings [n, E], logits [n, C], labels [n, C]) of raw node ids on the sharded
        graph: the rows' blocks built through the owners (sampled as in training, or full
        neighbourhoods), features and labels over the exchanges.  Collective: every rank
        calls it with the same ``pad_to`` (rows padded with -1, which touch nothing)."""
        g = self.graph
        rows = g.rows_of(ids).to(g.device).long().reshape(-1)
        n = rows.numel()
        B = max(n, int(pad_to or 0), 1)
        if B > n:
            rows = torch.cat([rows, torch.full((B - n,), -1, dtype=torch.long, device=rows.device)])
        flow = self._sharded_infer_flow(B)
        self.model.eval()
        try:
            while True:
                emb, _ = full_flow_embed(self.gnn, flow, g.gather_features, rows)
                if not callable(getattr(flow, "grow", None)):
                    break
                over = torch.tensor([int(flow.overflowed())], dtype=torch.int64)
                if g.comm:  # every rank regrows together
                    from euler_amd.parallel import comm

                    over = over.to(g.device)
                    comm.all_reduce(over, dist.ReduceOp.MAX, group=g.group)
                if not int(over.item()):
                    break
                flow.grow(2.0)
            logits = self.model.out_fc(emb).float()
        finally:
            self.model.train()
        g.advance()  # the next batch (and training) draw from fresh counters
        y = g.gather_labels(rows).float()
        return emb[:n].float(), logits[:n], y[:n]

    def infer_embed(self, ids, pad_to=None):
        return self.infer_logits(ids, pad_to)[0]

    def capturable(self) -> bool:
        """one rank without exchanges, or RCCL exchanges (every route, draw, expansion and
        feature row moves in fixed-capacity slots and captures like any kernel); gloo stages
        through host memory: those steps run eagerly"""
        g = self.graph
        if not g.comm:
            return True
        return self.on_gpu and dist.get_backend(g.group) != "gloo"

    def capture(self, grad_sync=None, warmup: int = 2, steps: int = 1, extra_sizes=()):
        if self.capturable():
            return super().capture(grad_sync, warmup, steps, extra_sizes)
        for _ in range(int(warmup)):  # host syncs in the step: eager
            self.step_count += 1
            self._step(grad_sync)
        self._grad_sync = grad_sync
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
            self._step(getattr(self, "_grad_sync", None))
        self.step_count += int(n)
        self.graph.check_overflow()
