"""Shared machinery of the device-path trainers whose step is the user's own torch model.

A subclass supplies :meth:`CapturedTrainer._forward_loss` — draw the step's batch on the
device (Philox counters of ``self.rng_source``: no host round trip), run the model, return
the loss and update device-resident metric accumulators.  This class adds the rest of the
estimator's device-path contract (``estimator/base.py`` ``_train_device_graph``):

* the model's parameters re-homed into one flat fp32 buffer (``parallel/flat.py``), one
  flat optimizer launch per step (``csrc/hip/optim.hip``) and an optional gradient sync
  (all-reduce of the flat gradient) between backward and update;
* warm-up eagerly on a side stream, then several complete steps captured per hipGraph
  (plus a 1-step graph and graphs of the log / checkpoint remainders), replayed greedily
  by :meth:`replay_steps`;
* checkpoints in the model's own parameter names, the optimizer slots and the sampler's
  (seed, counter).

``rng_source`` is any object with ``rng`` (int64 [2] device tensor: seed, counter),
``advance()`` and ``reseed_cpu()`` (DeviceGraph has them; so does
:class:`~euler_amd.models.kg_trainer.TripleTable`).
"""
from __future__ import annotations

import torch

from euler_amd.parallel.flat import FlatOptimizer, FlatParams

__all__ = ["CapturedTrainer", "new_graph", "graph_audit"]


def new_graph():
    """a torch CUDAGraph for a captured step; ``EULER_AMD_KEEP_GRAPHS=1`` keeps the
    underlying hipGraph (``raw_cuda_graph``) for :func:`graph_audit` (instantiated on the
    first replay)"""
    import os

    keep = os.environ.get("EULER_AMD_KEEP_GRAPHS", "0") == "1"
    return torch.cuda.CUDAGraph(keep_graph=True) if keep else torch.cuda.CUDAGraph()


def graph_audit(graphs):
    """node kinds of kept captured graphs (:func:`new_graph`): {steps: {kind: count}} plus
    the memset / memcpy / fill nodes by name — a captured step should hold kernels only
    (tests/test_graph_memset.py)"""
    from euler_amd.ops._native import hip

    out = {}
    for k, g in graphs.items():
        s = hip().graph_summary(g.raw_cuda_graph())
        kinds = {}
        for _, kind, _ in s["nodes"]:
            kinds[kind] = kinds.get(kind, 0) + 1
        preds, succs = {}, {}
        for a, b in s["edges"]:
            succs[a] = succs.get(a, 0) + 1
            preds[b] = preds.get(b, 0) + 1
        chain = len(s["edges"]) == len(s["nodes"]) - 1 and all(
            preds.get(i, 0) <= 1 and succs.get(i, 0) <= 1 for i, _, _ in s["nodes"])
        out[k] = {"kinds": kinds, "non_kernel": [(kind, d) for _, kind, d in s["nodes"] if kind != "kernel"],
                  "fills": [d for _, kind, d in s["nodes"] if kind == "kernel" and "rocclr" in d],
                  "linear_chain": chain}
    return out


class CapturedTrainer:
    metric_name = "loss"

    def __init__(self, model, rng_source, device, optimizer="adam", learning_rate=0.01):
        self.model = model
        self.rng_source = rng_source
        self.device = torch.device(device)
        self.on_gpu = self.device.type == "cuda"
        model.to(self.device)
        self._materialize()
        self.flat = FlatParams([p for p in model.parameters() if p.requires_grad], self.device)
        self.opt = FlatOptimizer(self.flat, optimizer, learning_rate)
        self.loss_out = torch.zeros((), device=self.device)
        self.step_count = 0
        self._graphs = {}
        self._graph_exec = None
        self._samples = None
        self.captures = 0  # hipGraph captures so far (graphs are released at the end of a run)

    # ------------------------------------------------------------------ subclass hooks
    def _materialize(self):
        """give lazy layers their shapes before the parameters are flattened"""

    def _forward_loss(self):
        raise NotImplementedError

    def metric(self) -> float:
        return float(self.loss_out.item())

    def reset_metric(self):
        pass

    # ------------------------------------------------------------------ step
    def _draw(self):
        """advance the sampler's Philox counter (and re-key the CPU twin's generator)"""
        src = self.rng_source
        src.advance()
        if not self.on_gpu:
            src.reseed_cpu()

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
        """Record ``steps`` complete steps (sampling, model, backward, [all-reduce,]
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
            gr = new_graph()
            with torch.cuda.graph(gr, capture_error_mode="thread_local"):
                for _ in range(k):
                    self._step(grad_sync)
            self._graphs[k] = gr
        self._graph_exec = self._graphs[1]
        self.captures += 1
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

    def samples(self):
        return self._samples

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
                "step": int(self.opt.step_count.item()), "rng": self.rng_source.rng.detach().cpu().clone()}

    def load_trainer_state(self, st):
        # slots saved before the flat buffers were padded to a multiple of 8 (or after):
        # the parameters' prefix is copied and the padding tail zeroed
        for name in ("m", "v"):
            dst, src = getattr(self.opt, name), torch.as_tensor(st[name]).reshape(-1)
            n = min(int(src.numel()), int(dst.numel()))
            if n < self.flat.numel:
                raise ValueError(f"checkpoint optimizer slot '{name}' has {src.numel()} elements for "
                                 f"{self.flat.numel} parameters")
            dst[:n].copy_(src[:n].to(dst))
            dst[n:].zero_()
        self.opt.step_count.fill_(int(st["step"]))
        self.rng_source.rng.copy_(torch.as_tensor(st["rng"]).to(self.rng_source.rng))
        self.step_count = int(st["step"])

    def dp_state_tensors(self):
        return [self.flat.flat, self.opt.m, self.opt.v, self.opt.step_count]

    def set_learning_rate(self, lr):
        self.opt.lr = float(lr)


class RowSparseTableMixin:
    """One id table of a CapturedTrainer held as a row-sharded, row-sparse
    :class:`~euler_amd.parallel.sparse_table.ShardedTable` (``self.id_table``) instead of
    in the flat buffer.  Row ``r`` lives on rank ``r % world`` (ShardedEmbedding's
    layout): a ``sharded=True`` model's shard, or any model's table on one rank, IS the
    trainer's table — the module's weight is rebound to it (no second copy) and leaves
    autograd and the flat buffer, so per-step work stays independent of |V|.  A dense
    model under 2+ ranks keeps its full table, written from the shards at the end.
    Checkpoints: per-rank shard files of the rows and their optimizer slots
    (parallel/shard_io.py), no all-gather."""

    def _adopt_table(self, model, mod, device, group, optimizer, learning_rate):
        from euler_amd.parallel.sparse_table import ShardedTable

        opt = optimizer if optimizer in ("adam", "adagrad", "sgd") else "adam"
        t = ShardedTable(int(mod.num), int(mod.dim), device, group, opt, learning_rate, init=None)
        w = mod.weight
        with torch.no_grad():
            if getattr(mod, "world", 1) > 1 or w.shape[0] == t.weight.shape[0]:
                t.weight.copy_(w.detach().to(t.weight))  # already this rank's rows
                w.data = t.weight
                self._table_bound = True
            else:
                t.weight.copy_(w.detach()[t.global_ids().to(w.device)].to(t.weight))
                self._table_bound = False
        w.requires_grad_(False)
        self.id_table, self._mod = t, mod
        # every state_dict key of the table (a table shared by two roles is listed twice)
        self._table_keys = [k for k, v in model.state_dict(keep_vars=True).items() if v is w]
        return t

    # ------------------------------------------------------------------ state
    def _full(self):
        return self.id_table.full()

    def logical_keys(self):
        return set(self.model.state_dict()) | set(self._table_keys)

    def state_dict(self):
        """model-named state with the WHOLE table (tests / export; a collective under 2+
        ranks — checkpoints use :meth:`checkpoint_shards`)"""
        sd = {k: v.detach().cpu() for k, v in self.model.state_dict().items()}
        full = self._full().cpu()
        for k in self._table_keys:
            sd[k] = full
        return sd

    def logical_params(self):
        return {k: v.to(self.device) for k, v in self.state_dict().items()}

    def checkpoint_model_state(self):
        return {k: v.detach().cpu() for k, v in self.model.state_dict().items() if k not in self._table_keys}

    def checkpoint_shards(self, ckpt_path):
        key = self._table_keys[0]
        meta = self.id_table.save_shard(ckpt_path, key)
        return {k: meta for k in self._table_keys}

    def load_shards(self, dirname, metas):
        for k in self._table_keys:
            if k in metas:
                self.id_table.load_shard(dirname, metas[k], name=k)
                return

    def load_logical(self, sd):
        with torch.no_grad():
            own = self.model.state_dict()
            for k, v in sd.items():
                if k in own and k not in self._table_keys:
                    own[k].copy_(torch.as_tensor(v).to(own[k]))
        for k in self._table_keys:
            if k in sd:
                self.id_table.load(sd[k])
                break

    def write_to_model(self, model):
        if not (self._table_bound and model is self.model):
            with torch.no_grad():
                w = self._mod.weight if model is self.model else model.state_dict()[self._table_keys[0]]
                t = self.id_table
                w.copy_((t.weight if w.shape[0] == t.weight.shape[0] else self._full()).to(w))
        if model is not self.model:
            model.load_state_dict(self.checkpoint_model_state(), strict=False)

    def finish(self):
        self.write_to_model(self.model)
        self._mod.weight.requires_grad_(True)

    def trainer_state(self):
        st = super().trainer_state()
        st["id_table_step"] = int(self.id_table.step.item())
        return st

    def load_trainer_state(self, st):
        super().load_trainer_state(st)
        if "id_table" in st:  # an older checkpoint: whole slot tensors of the same layout
            self.id_table.load_slot_state(st.get("id_table"))
        if "id_table_step" in st:
            self.id_table.step.fill_(int(st["id_table_step"]))

    def dp_state_tensors(self):
        return list(super().dp_state_tensors()) + self.id_table.state_tensors()
