"""Device-path training of models with historical-embedding encoders (ScalableSageEncoder /
ScalableGCNEncoder) under ``NodeEstimator(device_graph=True)``.

Reference: ``tf_euler/python/utils/encoders.py:294-408`` (ScalableGCNEncoder) and
``:629-748`` (ScalableSageEncoder) — SURVEY §5(d), the reference's answer to
neighbourhood explosion: each step computes only ONE fresh hop (the roots' sampled /
full neighbourhood) and reads every deeper layer's neighbour embeddings from per-layer
stores of stale embeddings; the fresh root embeddings are written back to the stores, and
the gradients that reach the stale neighbour rows are accumulated in gradient stores and
injected into those nodes' own embeddings the next time they are roots (``store_loss``).

Here the model runs ITS OWN forward (``SuperviseModel.forward`` -> ``embed`` -> the
encoder's training forward and store protocol) inside a
:func:`~euler_amd.graph.device_scope.device_graph_scope`: the roots are drawn by the
graph's alias table, the encoder's ``sample_fanout`` / ``get_multi_hop_neighbor`` and
every ``get_dense_feature`` (features, labels) are answered from the HBM graph, and the
stores are device buffers of the encoder (or its row-sharded stores over all-to-all when
world > 1, ``parallel/sharded_store.py``).  One step = draws, forward (+ store loss),
backward, the encoder's ``after_backward`` (store writes, gradient-store accumulation),
gradient sync, the flat optimizer.

ScalableSageEncoder steps have fixed shapes and no host read: on one GPU several are
captured per hipGraph like every other device trainer.  ScalableGCNEncoder's neighbour
sets have data-dependent sizes (and the multi-rank stores exchange variable-length rows),
so those steps run eagerly on the device.
"""
from __future__ import annotations

import torch

from euler_amd.graph.device_scope import DeviceGraphScope, device_graph_scope
from euler_amd.models.captured import CapturedTrainer

__all__ = ["ScalableTrainer", "store_encoder_of"]


def store_encoder_of(model):
    """the model's one historical-embedding encoder, or None"""
    from euler_amd.utils.encoders import _StoreMixin

    encs = [m for m in model.modules() if isinstance(m, _StoreMixin)]
    return encs[0] if len(encs) == 1 else None


class ScalableTrainer(CapturedTrainer):
    def __init__(self, model, graph, batch_size, feature_cols, label=None, optimizer="adam", learning_rate=0.01):
        from euler_amd.mp_utils.models import SuperviseModel
        from euler_amd.utils.encoders import ScalableSageEncoder

        enc = store_encoder_of(model)
        if enc is None or not isinstance(model, SuperviseModel):
            raise ValueError("ScalableTrainer trains SuperviseModels with one Scalable* encoder")
        ne = getattr(enc, "_node_encoder", None)
        if ne is None or ne.use_id or ne.use_sparse_feature:
            raise ValueError("the device path serves dense features only (no id / sparse-feature embeddings)")
        self.enc = enc
        self.graph = graph
        self.B = int(batch_size)
        self.scope = DeviceGraphScope(graph, feature_cols, label)
        self.metric_name = model.metric_name
        self._static = isinstance(enc, ScalableSageEncoder) and not getattr(enc, "_sharded", None)
        super().__init__(model, graph, graph.device, optimizer, learning_rate)
        import torch.distributed as dist

        self._multi = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1

    # ------------------------------------------------------------------ step
    def draw_roots(self):
        return self.scope.ids_of(self.graph.sample_node(self.B, stream_id=1).long())

    def _step(self, grad_sync=None):
        self._draw()
        roots = self.draw_roots()
        with device_graph_scope(self.scope):
            _, loss, _, _ = self.model(roots)
        extra = self.enc.store_loss
        obj = loss if extra is None else loss + extra
        self.opt.zero_grad()
        obj.backward()
        self.enc.after_backward()  # store writes + gradient-store accumulation
        scale = 1.0
        if grad_sync is not None:
            s = grad_sync(self.flat.grad)
            scale = 1.0 if s is None else float(s)
        self.opt.step(scale)
        self._samples = (roots,)
        self.loss_out.copy_(loss.detach())
        return self.loss_out

    # ------------------------------------------------------------------ hipGraph
    def capture(self, grad_sync=None, warmup: int = 2, steps: int = 1, extra_sizes=()):
        """ScalableSage on one GPU: captured like every device trainer; otherwise (data-
        dependent shapes, or variable-length store exchanges between ranks) eager steps"""
        if self._static and not self._multi:
            return super().capture(grad_sync, warmup, steps, extra_sizes)
        for _ in range(int(warmup)):
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

    # ------------------------------------------------------------------ metric / state
    def metric(self) -> float:
        m = self.model.metric
        acc = getattr(m, "acc", None)
        if acc is None:
            return 0.0
        if self.metric_name == "f1":
            tp, fp, fn = (float(v) for v in acc.tolist())
            eps = 1e-7
            p, r = tp / (eps + tp + fp), tp / (eps + tp + fn)
            return 2.0 * p * r / (p + r + eps)
        return float(acc[0]) / max(float(acc[1]), 1.0)

    def reset_metric(self):
        self.model.metric.reset()

    def dp_state_tensors(self):
        ts = list(super().dp_state_tensors())
        for i in range(self.enc._num_stores):
            if self.enc._sharded:
                ts += [st.local for st in self.enc._sharded[i]]
            else:
                ts += [self.enc.stores(i), self.enc.gradient_stores(i)]
        return ts

    def trainer_state(self):
        st = super().trainer_state()
        if not self.enc._sharded:
            st["stores"] = [self.enc.stores(i).detach().cpu().clone() for i in range(self.enc._num_stores)]
            st["gradient_stores"] = [self.enc.gradient_stores(i).detach().cpu().clone()
                                     for i in range(self.enc._num_stores)]
        return st

    def load_trainer_state(self, st):
        super().load_trainer_state(st)
        with torch.no_grad():
            for i, t in enumerate(st.get("stores") or []):
                self.enc.stores(i).copy_(torch.as_tensor(t).to(self.enc.stores(i)))
            for i, t in enumerate(st.get("gradient_stores") or []):
                self.enc.gradient_stores(i).copy_(torch.as_tensor(t).to(self.enc.gradient_stores(i)))
