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
import torch.nn.functional as F

from euler_amd.dataflow.device_flow import DeviceFullFlow
from euler_amd.ops import mp_ops
from euler_amd.parallel.flat import FlatOptimizer, FlatParams

__all__ = ["FullFlowTrainer"]


class FullFlowTrainer:
    metric_name = "f1"

    def __init__(self, model, graph, batch_size, masks, add_self_loops=True, features=None, labels=None,
                 optimizer="adam", learning_rate=0.01, caps=None):
        self.model = model
        self.gnn = model.gnn
        self.graph = graph
        self.device = graph.device
        self.on_gpu = self.device.type == "cuda"
        self.B = int(batch_size)
        feats = features if features is not None else graph.features
        labs = labels if labels is not None else graph.labels
        if feats is None or labs is None:
            raise ValueError("the device graph needs dense features and labels (DeviceGraph.from_engine)")
        self.features = feats.to(self.device)
        self.labels = labs.to(self.device).float()
        self.flow = DeviceFullFlow(graph, masks, self.B, add_self_loops, caps)
        model.to(self.device)
        self._materialize()
        self.flat = FlatParams([p for p in model.parameters() if p.requires_grad], self.device)
        self.opt = FlatOptimizer(self.flat, optimizer, learning_rate)
        self.loss_out = torch.zeros((), device=self.device)
        self.counts = torch.zeros(3, dtype=torch.int64, device=self.device)
        self.step_count = 0
        self._graphs = {}
        self._graph_exec = None
        self._samples = None

    # ------------------------------------------------------------------ construction
    @classmethod
    def from_model(cls, model, graph, batch_size, optimizer="adam", learning_rate=0.01, **kw):
        """Trainer for a (materialised) full-flow ``SupervisedGNN``: metapath, self loops and
        the layers come from the model."""
        import euler_amd.ops.graph_api as ge
        from euler_amd.dataflow.dataflows import GCNDataFlow

        flow = getattr(model.gnn, "sampler", None)
        if not isinstance(flow, GCNDataFlow):
            raise ValueError("FullFlowTrainer trains models on the full-neighbourhood flow (GCNDataFlow)")
        masks = []
        for m in flow.metapath:
            ids = None if m is None else [int(t) for t in np.asarray(ge.get_edge_type_id(m)).reshape(-1)]
            masks.append(graph._mask(None if ids is None or any(t < 0 for t in ids) else ids))
        return cls(model, graph, batch_size, masks, add_self_loops=bool(flow.add_self_loops), optimizer=optimizer,
                   learning_rate=learning_rate, **kw)

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
        df = self.flow.produce(roots)
        x = mp_ops.gather(self.features, df[0].n_id).float()
        for conv, block in zip(self.gnn.convs, df):
            x_t = mp_ops.gather(x, block.res_n_id)
            x = F.relu(self.gnn.calculate_conv(conv, (x_t, x), block.edge_index, size=block.size))
        emb = self.gnn.fc(x)
        return self.model.out_fc(emb).float(), df

    def _forward_loss(self):
        g = self.graph
        g.advance()
        if not self.on_gpu:
            g.reseed_cpu()
        roots = g.sample_node(self.B, stream_id=1).long()
        logits, df = self._forward(roots)
        y = mp_ops.gather(self.labels, roots)
        loss = F.binary_cross_entropy_with_logits(logits, y)
        with torch.no_grad():
            pred, pos = logits >= 0, y > 0.5
            self.counts += torch.stack([(pred & pos).sum(), (pred & ~pos).sum(), (~pred & pos).sum()])
        self._samples = roots
        return loss

    def _step(self, grad_sync=None):
        loss = self._forward_loss()
        self.opt.zero_grad()
        loss.backward()
        scale = 1.0
        if grad_sync is not None:
            s = grad_sync(self.flat.grad)
            scale = 1.0 if s is None else float(s)
        self.opt.step(scale)
        self.loss_out.copy_(loss.detach())
        return self.loss_out

    def step(self, grad_sync=None):
        """one training step (eager; after :meth:`capture`, a replay of the 1-step graph)"""
        self.step_count += 1
        if self._graph_exec is not None:
            self._graph_exec.replay()
            return self.loss_out
        return self._step(grad_sync)

    # ------------------------------------------------------------------ hipGraph
    def capture(self, grad_sync=None, warmup: int = 2, steps: int = 1, extra_sizes=()):
        """Record ``steps`` complete steps (sampling, blocks, model, backward, [all-reduce,]
        optimizer) into one hipGraph after ``warmup`` eager steps on a side stream; graphs of
        1 step and of each ``extra_sizes`` entry are kept too (:meth:`replay_steps`)."""
        if not self.on_gpu:
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
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, capture_error_mode="thread_local"):
                for _ in range(k):
                    self._step(grad_sync)
            self._graphs[k] = gr
        self._graph_exec = self._graphs[1]
        return self._graphs[int(steps)]

    def replay(self, n: int = 1):
        for _ in range(int(n)):
            self._graph_exec.replay()
        self.step_count += int(n)

    def replay_steps(self, n: int):
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

    # ------------------------------------------------------------------ state
    @property
    def loss(self):
        return self.loss_out

    def metric(self) -> float:
        tp, fp, fn = self.counts.tolist()
        return 2.0 * tp / max(2.0 * tp + fp + fn, 1e-12)

    def reset_metric(self):
        self.counts.zero_()

    def samples(self):
        """roots of the last step"""
        return (self._samples,)

    def state_dict(self):
        return {k: v.detach().cpu() for k, v in self.model.state_dict().items()}

    def logical_params(self):
        return {k: v.detach().clone() for k, v in self.model.state_dict().items()}

    def load_logical(self, sd):
        with torch.no_grad():
            own = self.model.state_dict()
            for k, v in sd.items():
                if k in own:
                    own[k].copy_(torch.as_tensor(v).to(own[k]))

    def write_to_model(self, model):
        if model is not self.model:
            model.load_state_dict(self.model.state_dict())

    def trainer_state(self):
        return {"m": self.opt.m.cpu().clone(), "v": self.opt.v.cpu().clone(),
                "step": int(self.opt.step_count.item()), "rng": self.graph.rng.detach().cpu().clone()}

    def load_trainer_state(self, st):
        self.opt.m.copy_(torch.as_tensor(st["m"]).to(self.opt.m))
        self.opt.v.copy_(torch.as_tensor(st["v"]).to(self.opt.v))
        self.opt.step_count.fill_(int(st["step"]))
        self.graph.rng.copy_(torch.as_tensor(st["rng"]).to(self.graph.rng))
        self.step_count = int(st["step"])

    def dp_state_tensors(self):
        return [self.flat.flat, self.opt.m, self.opt.v, self.opt.step_count]

    def set_learning_rate(self, lr):
        self.opt.lr = float(lr)

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
