"""Training loop (reference ``euler_estimator/python/base_estimator.py:28-188``).

``tf.estimator`` gave the reference: a model_fn per mode, a global step, optimizer
``minimize``, ``LoggingTensorHook`` every ``log_steps``, checkpoints under
``model_dir`` with auto-resume, and ``predict`` writing ``embedding_<worker>.npy`` /
``ids_<worker>.npy``.  This module provides the same contract on PyTorch-ROCm:

* ``train()``  — sample -> model -> loss -> backward -> (RCCL bucketed gradient
  all-reduce, overlapped with backward) -> optimizer; logs ``step/loss/<metric>`` and
  samples/s every ``log_steps``; checkpoints every ``save_checkpoints_steps`` and at
  the end (``model_dir/model.ckpt-<step>.pt`` + a ``checkpoint`` index file naming
  the latest, pruned to ``keep_checkpoint_max``); resumes from the latest checkpoint.
* ``evaluate()`` — streams the id file, logs loss + running metric per batch,
  returns the final values.
* ``infer()``  — streams the id file, writes ``embedding_<rank>.npy`` and
  ``ids_<rank>.npy`` into ``infer_dir``.

Parameters (``params`` dict, reference names): ``model_dir``, ``batch_size``,
``total_step``, ``optimizer``, ``learning_rate``, ``log_steps``, ``id_file``,
``infer_dir``; extras: ``device``, ``amp`` ("bf16" runs the model under bf16
autocast), ``save_checkpoints_steps``, ``keep_checkpoint_max``, ``seed``.
"""
from __future__ import annotations

import contextlib
import glob
import logging
import os
import re
import time

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn

from euler_amd.parallel import dp
from euler_amd.parallel.embedding import is_sharded, reshard_rows, sharded_param_names
from euler_amd.utils.prefetch import Prefetcher
from euler_amd.utils import trace
from euler_amd.utils.misc import get_optimizer

__all__ = ["BaseEstimator", "latest_checkpoint", "rank_checkpoint", "id_file_batches"]

log = logging.getLogger("euler_amd.estimator")


def latest_checkpoint(model_dir):
    idx = os.path.join(model_dir, "checkpoint")
    if os.path.exists(idx):
        with open(idx) as f:
            for line in f:
                m = re.match(r'model_checkpoint_path:\s*"?([^"\n]+)"?', line.strip())
                if m:
                    p = m.group(1)
                    p = p if os.path.isabs(p) else os.path.join(model_dir, p)
                    if os.path.exists(p):
                        return p
    # rank 0's files only: "model.ckpt-<step>.pt" (per-rank files carry a "-rank<r>" suffix)
    cks = [p for p in glob.glob(os.path.join(model_dir, "model.ckpt-*.pt"))
           if re.search(r"model\.ckpt-\d+\.pt$", p)]
    if not cks:
        return None
    return max(cks, key=lambda p: int(re.search(r"model\.ckpt-(\d+)\.pt$", p).group(1)))


def rank_checkpoint(path, rank):
    """Rank ``rank``'s file of the checkpoint whose rank-0 file is ``path``."""
    if rank == 0:
        return path
    # only the file name's ".pt" suffix: a model_dir such as "/runs/x.pt_exp/" stays intact
    return re.sub(r"\.pt$", "-rank%d.pt" % rank, path)


def id_file_batches(path, batch_size, parse=int, shard=(0, 1)):
    """Batches of parsed lines of a text file (reference ``TextLineDataset.batch``).

    ``shard=(rank, world)`` gives each data-parallel worker every world-th batch.
    """
    rk, ws = shard
    batch, bi = [], 0
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            batch.append(parse(line))
            if len(batch) == batch_size:
                if bi % ws == rk:
                    yield batch
                batch, bi = [], bi + 1
    if batch and bi % ws == rk:
        yield batch


def _memory_peaks(device):
    """peak HBM allocated by this process and its peak host resident set (VmHWM), GiB"""
    hbm = torch.cuda.max_memory_allocated(device) / 2 ** 30 if device.type == "cuda" else 0.0
    rss = 0.0
    try:
        with open("/proc/self/status") as f:
            for line in f:
                if line.startswith("VmHWM:"):
                    rss = int(line.split()[1]) / 2 ** 20
    except OSError:
        pass
    return {"peak_hbm_gib": round(hbm, 2), "peak_host_rss_gib": round(rss, 2)}


def dist_backend():
    import torch.distributed as dist

    return dist.get_backend() if dist.is_available() and dist.is_initialized() else None


def _first_name(x):
    return x[0] if isinstance(x, (list, tuple)) else x


class BaseEstimator:
    def __init__(self, model_fn, params, run_config=None, profiling=False):
        self.model = model_fn
        self.params = dict(params)
        self.run_config = dict(run_config or {})
        self.profiling = profiling
        self.evaluate_stop_onetime = False
        dev = self.params.get("device")
        if dev is None:
            dev = "cuda" if torch.cuda.is_available() else "cpu"
        self.device = torch.device(dev)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)))
        self.rank, self.world = dp.rank(), dp.world_size()
        self.global_step = 0
        self.optimizer = None
        self._sync = None

    # ------------------------------------------------------------------ hooks (reference names)
    def get_train_from_input(self, inputs, params):
        return inputs

    def get_evaluate_from_input(self, inputs, params):
        return inputs

    def get_infer_from_input(self, inputs, params):
        return inputs

    def transfer_embedding(self, source, emb):
        return source, emb

    def train_input_fn(self):
        raise NotImplementedError

    def evaluate_input_fn(self):
        raise NotImplementedError

    def infer_input_fn(self):
        return self.evaluate_input_fn()

    # ------------------------------------------------------------------ helpers
    @property
    def model_dir(self):
        return self.params.get("model_dir", "ckpt")

    def _autocast(self):
        amp = self.params.get("amp")
        if amp in ("bf16", "bfloat16") and self.device.type == "cuda":
            return torch.autocast("cuda", dtype=torch.bfloat16)
        return torch.autocast("cpu", enabled=False)

    def _run_model(self, source):
        with self._autocast():
            return self.model(source)

    def _extra_losses(self):
        total = None
        for m in self.model.modules():
            sl = getattr(m, "store_loss", None)
            if isinstance(sl, torch.Tensor):
                total = sl if total is None else total + sl
        return total

    def _after_backward(self):
        for m in self.model.modules():
            fn = getattr(m, "after_backward", None)
            if callable(fn) and m is not self.model:
                fn()

    def _prepare(self, source, build_optimizer=True):
        """Move the model, materialise lazy parameters with one no-grad pass,
        broadcast rank 0's initial weights, build the optimizer and gradient sync
        (``build_optimizer=False``: a device trainer runs its own optimizer — a torch
        Adagrad would allocate its accumulators for every parameter right here, 95 GiB for
        a 100M-node DeepWalk)."""
        self.model.to(self.device)
        if any(isinstance(p, nn.parameter.UninitializedParameter) for p in self.model.parameters()):
            was = self.model.training
            with torch.no_grad():
                self._run_model(source)
            self.model.train(was)
            for m in self.model.modules():
                if hasattr(m, "_pending"):
                    m._pending = None
            self.model.to(self.device)
        dp.broadcast_module(self.model)
        if self.params.get("historical_store", "replicated") == "sharded":
            # Scalable* encoders: row-sharded stale-embedding / gradient stores (parallel/sharded_store.py)
            for m in self.model.modules():
                if callable(getattr(m, "use_sharded_stores", None)) and not getattr(m, "_sharded", None):
                    m.use_sharded_stores()
        params = [p for p in self.model.parameters() if p.requires_grad]
        if not build_optimizer:
            self.optimizer, self._sync = None, None
            return
        name = self.params.get("optimizer", "adam")
        self.optimizer = get_optimizer(name)(params, self.params.get("learning_rate", 0.001))
        dense = [p for p in params if not is_sharded(p)]
        self._sync = dp.GradSync(dense, bucket_bytes=int(self.params.get("bucket_bytes", 32 << 20)))

    def save(self, step=None, extra=None, all_ranks=False, model_state=None, shards=None, commit=True):
        """Write ``model.ckpt-<step>.pt`` (rank 0) and, when some state differs per rank
        (sharded tables, or ``all_ranks``: e.g. the device path's per-rank sampler stream),
        ``model.ckpt-<step>-rank<r>.pt`` on every other rank (reference per-worker outputs,
        ``base_estimator.py:157-179``).  ``shards(path)``: writes this rank's rows of the
        row-sharded tables (and their optimizer slots) next to the file and returns their
        metadata (parallel/shard_io.py), kept under "shards".  ``commit``: rank 0 points
        the ``checkpoint`` index at the new step and keeps the newest
        ``keep_checkpoint_max`` steps (every rank's files of a step together); a caller
        whose ranks write concurrently commits after a barrier (:meth:`_commit`)."""
        step = self.global_step if step is None else step
        if self.rank != 0 and not all_ranks and not any(is_sharded(p) for p in self.model.parameters()):
            return None
        os.makedirs(self.model_dir, exist_ok=True)
        path = rank_checkpoint(os.path.join(self.model_dir, "model.ckpt-%d.pt" % step),
                               0 if self.world == 1 else self.rank)
        if model_state is None:
            model_state = {k: v for k, v in self.model.state_dict().items()
                           if not isinstance(v, nn.parameter.UninitializedParameter)}  # never-called lazy layers
        state = {"step": step, "model": model_state,
                 "optimizer": self.optimizer.state_dict() if self.optimizer is not None else None,
                 "world": self.world, "rank": self.rank, "torch_rng": torch.get_rng_state()}
        state.update(extra or {})
        if shards is not None:
            state["shards"] = shards(path)
        tmp = path + ".tmp"
        torch.save(state, tmp)
        os.replace(tmp, path)
        if commit and self.rank == 0:
            self._commit(step, path)
        return path

    def _commit(self, step, path):
        """rank 0: the ``checkpoint`` index names step ``step``; older steps beyond
        ``keep_checkpoint_max`` are deleted (every rank's file and shard files)"""
        from euler_amd.parallel.shard_io import sidecar_files

        with open(os.path.join(self.model_dir, "checkpoint"), "w") as f:
            f.write('model_checkpoint_path: "%s"\n' % os.path.basename(path))
        keep = int(self.run_config.get("keep_checkpoint_max", self.params.get("keep_checkpoint_max", 5)))
        cks = glob.glob(os.path.join(self.model_dir, "model.ckpt-*.pt"))
        step_of = {p: int(re.search(r"model\.ckpt-(\d+)", p).group(1)) for p in cks}
        steps = sorted(set(step_of.values()))
        drop = set(steps[:-keep]) - {step} if keep > 0 else set()
        for old in cks:
            if step_of[old] in drop:
                for f in [old] + sidecar_files(old):
                    try:
                        os.remove(f)
                    except FileNotFoundError:
                        pass

    def _shard_metas(self, path, saved_world, state=None):
        """table -> [per-rank shard metadata] of the checkpoint whose rank-0 file is ``path``
        (each rank's small .pt file holds its own; tables never leave the shard files)"""
        base = re.sub(r"-rank\d+\.pt$", ".pt", path)
        out = {}
        for r in range(int(saved_world)):
            f = rank_checkpoint(base, r) if saved_world > 1 else base
            st = state if state is not None and int(state.get("rank", 0)) == r and f == path else \
                torch.load(f, map_location="cpu", weights_only=True)
            for key, meta in (st.get("shards") or {}).items():
                out.setdefault(key, []).append(meta)
        return out

    def _load_model_shards(self, path, saved_world, state):
        """engine-path restore of tables kept in per-rank shard files: this rank's rows of a
        ShardedEmbedding, every row of a dense table; returns the keys filled"""
        from euler_amd.parallel.embedding import ShardedEmbedding
        from euler_amd.parallel.shard_io import read_rows

        metas = self._shard_metas(path, saved_world, state)
        mod_of = {id(p): m for m in self.model.modules() for p in m.parameters(recurse=False)}
        params = self.model.state_dict(keep_vars=True)  # a table shared by two roles: both names
        done, filled = set(), set()
        for key, ms in metas.items():
            p = params.get(key)
            if p is None:
                continue
            if id(p) not in filled:
                m = mod_of.get(id(p))
                rows = m.global_ids().cpu() if isinstance(m, ShardedEmbedding) else torch.arange(p.shape[0])
                with torch.no_grad():
                    read_rows(os.path.dirname(path), ms, "weight", rows, p.data)
                filled.add(id(p))
            done.add(key)
        return done

    def restore(self, path=None, strict=True):
        path = path or latest_checkpoint(self.model_dir)
        if path is None:
            return False
        if self.world > 1 and self.rank != 0:
            own = rank_checkpoint(path, self.rank)
            if os.path.exists(own):
                path = own
        state = torch.load(path, map_location=self.device, weights_only=True)
        saved_world = int(state.get("world", 1))
        names = sharded_param_names(self.model)
        if names and saved_world != self.world and not state.get("shards"):
            self._reshard(state, path, saved_world, names)
        from_shards = self._load_model_shards(path, saved_world, state) if state.get("shards") else set()
        missing, unexpected = self.model.load_state_dict(state["model"], strict=False)
        if strict and (set(missing) - from_shards or unexpected):
            raise RuntimeError(f"checkpoint {path}: missing keys {sorted(set(missing) - from_shards)}, "
                               f"unexpected keys {sorted(unexpected)}")
        if self.optimizer is not None and state.get("optimizer") is not None:
            self.optimizer.load_state_dict(state["optimizer"])
        self.global_step = int(state["step"])
        if state.get("torch_rng") is not None:
            torch.set_rng_state(state["torch_rng"].cpu())
        log.info("restored %s at step %d", path, self.global_step)
        return True

    def _reshard(self, state, path, saved_world, names):
        """Sharded embedding tables (and their optimizer slots) saved by ``saved_world``
        ranks, re-sharded for this run's world size: every rank reads all the shard files
        and keeps its ``mod`` rows."""
        base = re.sub(r"-rank\d+\.pt$", ".pt", path)
        files = [rank_checkpoint(base, r) for r in range(saved_world)]
        states = [torch.load(f, map_location="cpu", weights_only=True) for f in files]
        dev = self.device
        for n in names:
            state["model"][n] = reshard_rows([st["model"][n] for st in states], self.rank, self.world).to(dev)
        # optimizer slots of the sharded tables follow their rows (param order = optimizer order)
        opt = state.get("optimizer")
        if opt is None:
            return
        pnames = [n for n, p in self.model.named_parameters() if p.requires_grad]
        for i, n in enumerate(pnames):
            if n not in names or i not in opt["state"]:
                continue
            rows = [st["model"][n].shape[0] for st in states]
            for k, v in list(opt["state"][i].items()):
                if torch.is_tensor(v) and v.dim() > 0 and v.shape[0] == rows[0]:
                    parts = [st["optimizer"]["state"][i][k] for st in states]
                    opt["state"][i][k] = reshard_rows(parts, self.rank, self.world).to(dev)

    # ------------------------------------------------------------------ modes
    def train(self):
        if self.params.get("device_graph"):
            from euler_amd.estimator.device_trainers import NoDeviceTrainer, has_store_encoder

            try:
                return self._train_device_graph()
            except NoDeviceTrainer as e:
                if not has_store_encoder(self.model):
                    raise
                # historical-embedding encoders keep their stores' protocol on the engine
                # path rather than silently training as their plain parent encoder
                log.warning("device_graph=True: %s; training on the engine path", e)
        seed = self.params.get("seed")
        if seed is not None:
            torch.manual_seed(int(seed) + self.rank)
        total = self.params.get("total_step")
        total = int(total) if total is not None else 1
        log_steps = int(self.params.get("log_steps", 100))
        save_steps = int(self.run_config.get("save_checkpoints_steps", self.params.get("save_checkpoints_steps", 0))
                         or 0)
        inputs = self.train_input_fn()
        first = self.get_train_from_input(inputs, self.params)
        self.model.train()
        self._prepare(first)
        self.restore()
        if self.global_step >= total:
            log.info("already trained to step %d", self.global_step)
            return {}
        pending = first
        # asynchronous input pipeline: the next batches are sampled by the engine (which
        # releases the GIL) on a worker thread and copied to HBM on a side stream while
        # this thread runs the current step (utils/prefetch.py); params["prefetch"] = 0
        # turns it off
        prefetcher = self._native_pipeline()
        if prefetcher is not None:
            # every step's batch comes from the native pipeline (``first`` only materialised
            # the model): its keyed draws make the batch stream identical for an in-process
            # and a sharded remote graph
            pending = None
        eager_first = True
        depth = int(self.params.get("prefetch", 2 if self.device.type == "cuda" else 0))
        if prefetcher is None and depth > 0 and callable(getattr(self.model, "prepare", None)):
            prefetcher = Prefetcher(lambda: self.model.prepare(self.get_train_from_input(inputs, self.params)),
                                    self.device, depth=depth, workers=int(self.params.get("prefetch_workers", 1)))
        graphed = None
        if getattr(prefetcher, "static", False):
            from euler_amd.estimator.graph_step import GraphedTrainStep

            graphed = GraphedTrainStep(self, prefetcher)
        t0, n0 = time.time(), self.global_step
        last = {}
        prof = None
        if self.profiling:
            prof = torch.profiler.profile(schedule=torch.profiler.schedule(wait=5, warmup=5, active=20),
                                          on_trace_ready=torch.profiler.tensorboard_trace_handler("prof_dir"))
            prof.start()
        tracing = bool(self.params.get("trace")) or trace.enabled()
        rng = (lambda name: trace.trace_range(name)) if tracing else (lambda name: contextlib.nullcontext())
        while self.global_step < total:
            with rng("sample"):
                if pending is not None:
                    source = pending
                elif prefetcher is not None:
                    source = prefetcher.get()
                else:
                    source = self.get_train_from_input(inputs, self.params)
            if graphed is not None and not eager_first:
                # graph-captured step over the pipeline's static inputs (estimator/graph_step.py);
                # drop the eager step's autograd graph first
                _ = loss = obj = extra = metric = None
                with rng("graph_step"):
                    loss, metric_name, metric = graphed.step(source)
                self.global_step += 1
                if prof is not None:
                    prof.step()
                last, t0, n0 = self._log_step(total, log_steps, loss, metric_name, metric, t0, n0, tracing, last)
                if save_steps and self.global_step % save_steps == 0:
                    self.save()
                continue
            pending = None
            eager_first = False
            with rng("forward"):
                _, loss, metric_name, metric = self._run_model(source)
                extra = self._extra_losses()
                obj = loss if extra is None else loss + extra
            with rng("backward"):
                self.optimizer.zero_grad(set_to_none=True)
                obj.backward()
                self._after_backward()
            with rng("grad_sync"):
                self._sync.finish()
            with rng("optimizer"):
                self.optimizer.step()
            self.global_step += 1
            if prof is not None:
                prof.step()
            last, t0, n0 = self._log_step(total, log_steps, loss, metric_name, metric, t0, n0, tracing, last)
            if save_steps and self.global_step % save_steps == 0:
                self.save()
        if prefetcher is not None:
            prefetcher.close()
        if prof is not None:
            prof.stop()
        self.save()
        dp.barrier()
        return last

    def _log_step(self, total, log_steps, loss, metric_name, metric, t0, n0, tracing, last):
        if not (self.global_step % log_steps == 0 or self.global_step == total):
            return last, t0, n0
        dt = max(time.time() - t0, 1e-9)
        rate = (self.global_step - n0) * int(self.params.get("batch_size", 1)) / dt
        last = {"step": self.global_step, "loss": float(loss.detach()), metric_name: float(metric),
                "samples_per_sec": rate}
        if self.rank == 0:
            log.info("step = %d, loss = %.6f, %s = %.6f (%.1f samples/s)", self.global_step, last["loss"],
                     metric_name, last[metric_name], rate)
            if tracing:
                log.info("stage timings:\n%s\nengine: %s", trace.default_timer.report(), trace.engine_stats())
        return last, time.time(), self.global_step

    def _native_pipeline(self):
        """The C++ batch pipeline (dataflow/native_loader.py) for SupervisedGNN + SageDataFlow
        models on an in-process graph: params["native_pipeline"] = True / False / "auto"
        (default: on for GPU training), "pipeline_workers" worker threads."""
        mode = self.params.get("native_pipeline", "auto")
        if mode in (False, "0", "false", "off") or (mode == "auto" and self.device.type != "cuda"):
            return None
        from euler_amd.dataflow.native_loader import NativeSageLoader, native_spec
        from euler_amd.ops.base import get_engine

        spec = native_spec(self.model, self.params)
        if spec is None or get_engine().meta()["mode"] not in ("local", "remote", "local_sharded"):
            return None
        flow, names, dims, label, label_dim, node_type = spec
        seed = int(self.params.get("seed") or 0) * 1000003 + self.rank
        workers = int(self.params.get("pipeline_workers", 8))
        from euler_amd.estimator.graph_step import graph_step_blocker

        why = graph_step_blocker(self, sum(dims))
        log.info("native batch pipeline: %d workers; graph-captured step: %s", workers,
                 "yes" if why is None else "no (%s)" % why)
        return NativeSageLoader(flow, names, dims, label, label_dim, int(self.params["batch_size"]), node_type,
                                self.device, workers=workers, seed=seed, static=why is None)

    def _device_graph_trainer(self, first):
        """Upload the engine's graph (structure, the model's feature and label columns) to
        HBM and build the device trainer for ``self.model``: the first entry of
        ``estimator/device_trainers.py`` REGISTRY that accepts it (fused GraphSAGE, the
        full-neighbourhood zoo, TransX, DeepWalk / LINE, GAE, DGI, R-GCN, the solution API,
        graph classification, ...)."""
        from euler_amd.estimator.device_trainers import build_device_trainer

        return build_device_trainer(self, self.model, first)

    def _train_device_graph(self):
        """NodeEstimator.train() on the device path: the whole mini-batch pipeline
        (sample_node roots, SageDataFlow hops, feature / label lookup) and the model step
        run as captured gfx950 kernels on an HBM copy of the graph (models/sage_trainer.py);
        same params, logging, checkpoints (reference names + the device optimizer state
        and Philox counter under "device_trainer") and resume as :meth:`train`.

        Data parallel: every rank writes its own checkpoint file (same weights and
        optimizer slots, its own sampler stream), so a resumed job continues every rank's
        stream where it stopped; with a different world size each rank re-derives its key
        (``seed * 7919 + rank``) and keeps the saved counter.  A timed-out xGMI wait (lost
        peer) is checked at every log / checkpoint boundary: all ranks agree, drop the
        captured graphs, re-synchronise rank 0's parameters and continue over RCCL."""
        total = int(self.params.get("total_step") or 1)
        log_steps = int(self.params.get("log_steps", 100))
        save_steps = int(self.run_config.get("save_checkpoints_steps", self.params.get("save_checkpoints_steps", 0))
                         or 0)
        # a graph from params["device_graph_factory"] has no engine to draw a first batch from
        # (it only materialises lazy layers, which such models must not have)
        first = None if self.params.get("device_graph_factory") else \
            self.get_train_from_input(self.train_input_fn(), self.params)
        self.model.train()
        tr = self._device_graph_trainer(first)
        self.device_trainer = tr
        self._device_restore(tr)
        if self.global_step >= total:
            log.info("already trained to step %d", self.global_step)
            return {}
        grad_sync, xar, gbuf = None, None, None
        gbuf0 = self._device_grad_buffer(tr)
        empty = gbuf0 is not None and gbuf0.numel() == 0  # every parameter row-sparse: nothing dense to sum
        if self.world > 1 and not getattr(tr, "self_synced", False) and not empty:
            # xGMI two-shot peer-memory all-reduce or RCCL on GPUs, whichever the start-up
            # timing on this node finds faster (parallel/xgmi.py); gloo on CPUs
            from ..parallel.xgmi import make_grad_sync

            kind = "auto" if self.device.type == "cuda" else "rccl"
            gbuf = self._device_grad_buffer(tr)
            rebind = getattr(tr, "use_grad_buffer", None) if getattr(tr, "on_gpu", False) else None
            grad_sync, name, info = make_grad_sync(gbuf, str(self.params.get("grad_sync", kind)), rebind=rebind,
                                                   timeout_s=float(self.params.get("xgmi_timeout_s", 10.0)))
            xar = info.get("xar")
            log.info("device path gradient sync: %s all-reduce", name)

        use_graph = self.device.type == "cuda" and bool(self.params.get("hipgraph", True))
        multi = hasattr(tr, "replay_steps")
        # capacity-padded device flows (dataflow/device_flow.py): a batch beyond a cap sets
        # the flow's overflow flag; it is read at every boundary, and a chunk that overflowed
        # on any rank is rolled back (parameters, optimizer slots, sampler counter) and re-run
        # with grown caps and re-captured graphs, so no step trains on truncated blocks — the
        # capture's own eager warm-up steps included
        flow = getattr(tr, "flow", None)
        guard = flow is not None and callable(getattr(flow, "grow", None))
        self.flow_regrows = 0
        if use_graph:
            snap = self._device_snapshot(tr) if guard else None
            warm = self._device_capture(tr, grad_sync, total)
            if guard and self._flow_overflowed(flow):
                warm = self._regrow(tr, grad_sync, total, flow, snap, self.global_step + warm, use_graph)
            self.global_step += warm

        def run(n):
            if use_graph and multi:
                tr.replay_steps(n)
                return
            for _ in range(n):
                if use_graph:
                    tr.replay()
                else:
                    tr.step(grad_sync)

        bs = int(self.params["batch_size"])
        t0, n0 = time.time(), self.global_step
        tr.reset_metric()
        last = {}
        delay = self.params.get("debug_delay_rank")  # test hook: one rank arrives late
        while self.global_step < total:
            # run up to the next log / checkpoint boundary in one go
            nxt = min(total, (self.global_step // log_steps + 1) * log_steps)
            if save_steps:
                nxt = min(nxt, (self.global_step // save_steps + 1) * save_steps)
            if delay is not None and int(delay) == self.rank:
                time.sleep(float(self.params.get("debug_delay_s", 2.0)))
                delay = None
            snap = self._device_snapshot(tr) if guard else None
            run(nxt - self.global_step)
            if guard and self._flow_overflowed(flow):
                self.global_step += self._regrow(tr, grad_sync, total, flow, snap, nxt, use_graph)
                continue
            self.global_step = nxt
            if xar is not None and self._xgmi_failed(xar):
                # sums since the failed wait are partial: rank 0's state wins, RCCL from here
                from ..parallel.xgmi import make_grad_sync

                log.warning("rank %d: xGMI all-reduce wait timed out before step %d; re-synchronising rank 0's "
                            "parameters and continuing over RCCL", self.rank, self.global_step)
                self._device_release(tr)
                self._xar_failed = xar  # keeps the IPC region alive while tensors still view it
                xar = None
                self._device_resync(tr)
                grad_sync = make_grad_sync(gbuf, "rccl")[0]
                self.grad_sync_fallback = True
                if use_graph and dist_backend() == "gloo":
                    use_graph = False  # gloo collectives are not capturable
                if use_graph:
                    self.global_step += self._device_capture(tr, grad_sync, total)
            if self.global_step % log_steps == 0 or self.global_step == total:
                loss = float(tr.loss.item())  # syncs the stream
                dt = max(time.time() - t0, 1e-9)
                rate = (self.global_step - n0) * bs * self.world / dt
                mname = getattr(tr, "metric_name", "f1")
                last = {"step": self.global_step, "loss": loss, mname: tr.metric(), "samples_per_sec": rate}
                last.update(_memory_peaks(self.device))
                tr.reset_metric()
                if self.rank == 0:
                    log.info("step = %d, loss = %.6f, %s = %.6f (%.1f samples/s, device path; peak HBM %.1f GiB, "
                             "peak host RSS %.1f GiB)", self.global_step, loss, mname, last[mname], rate,
                             last["peak_hbm_gib"], last["peak_host_rss_gib"])
                t0, n0 = time.time(), self.global_step
            if save_steps and self.global_step % save_steps == 0 and self.global_step < total:
                self._device_save(tr)
        if self.params.get("save_final_checkpoint", True):
            self._device_save(tr)
        # graphs holding captured collectives keep the communicator busy: drop them before
        # the final barrier / process-group teardown
        self._device_release(tr)
        if callable(getattr(tr, "finish", None)):
            tr.finish()  # e.g. row-sparse tables back into the model's own modules
        dp.barrier()
        return last

    def _regrow(self, tr, grad_sync, total, flow, snap, nxt, use_graph):
        """roll the overflowed chunk back to ``snap``, grow the flow's caps and re-capture
        until the capture's own eager warm-up steps fit; returns the warm-up steps run"""
        while True:
            self._device_rollback(tr, snap)
            if self.flow_regrows >= int(self.params.get("max_flow_regrows", 8)):
                raise RuntimeError(f"device dataflow capacity exceeded {self.flow_regrows} times "
                                   f"(caps {flow.caps})")
            self.flow_regrows += 1
            old = list(flow.caps)
            self._device_release(tr)
            flow.grow(float(self.params.get("flow_grow_factor", 2.0)))
            log.warning("rank %d: a batch before step %d exceeded the device flow caps %s; rolled the "
                        "chunk back, caps now %s, re-capturing", self.rank, nxt, old, flow.caps)
            tr.reset_metric()
            if not use_graph:
                return 0
            warm = self._device_capture(tr, grad_sync, total)
            if not self._flow_overflowed(flow):  # the capture's own eager warm-up steps fit
                return warm

    def _flow_overflowed(self, flow) -> bool:
        """the flow's overflow flag, agreed over the process group (MAX)"""
        over = int(flow.overflowed())
        if self.world > 1:
            import torch.distributed as dist

            flag = torch.tensor([over], dtype=torch.int32)
            if dist_backend() == "nccl":
                flag = flag.to(self.device)
            dist.all_reduce(flag, op=dist.ReduceOp.MAX)
            over = int(flag.item())
        if over:
            flow.clear()
        return bool(over)

    @staticmethod
    def _device_snapshot(tr):
        """device copies of everything a chunk of steps changes: parameters, optimizer slots
        and step counter, the sampler's (seed, counter)"""
        ts = list(tr.dp_state_tensors())
        rng = getattr(getattr(tr, "rng_source", None), "rng", None)
        if rng is not None:
            ts.append(rng)
        return [(t, t.detach().clone()) for t in ts], getattr(tr, "step_count", None)

    @staticmethod
    def _device_rollback(tr, snap):
        pairs, step_count = snap
        with torch.no_grad():
            for t, saved in pairs:
                t.copy_(saved)
        if step_count is not None:
            tr.step_count = step_count
        if callable(getattr(tr, "refresh_shadows", None)):
            tr.refresh_shadows()

    @staticmethod
    def _device_grad_buffer(tr):
        """the buffer grad_sync receives: SageTrainer's flat grad (bf16 hand-off: grad16),
        UnsupSageTrainer's FlatParams grad"""
        gbuf = getattr(tr, "grad16", None)
        if gbuf is None:
            gbuf = getattr(tr, "grad", None)
        if gbuf is None and hasattr(tr, "flat"):
            gbuf = tr.flat.grad
        return gbuf

    def _device_capture(self, tr, grad_sync, total):
        """capture the step graph(s); returns the eager warm-up steps it ran"""
        warm = min(2, total - self.global_step)
        if hasattr(tr, "replay_steps"):
            # several complete steps per hipGraph replay (SageTrainer): the ~5 us gap between
            # replays is paid once per chunk instead of once per step
            spg = max(1, int(self.params.get("steps_per_graph", 8)))
            log_steps = int(self.params.get("log_steps", 100))
            save_steps = int(self.run_config.get("save_checkpoints_steps",
                                                 self.params.get("save_checkpoints_steps", 0)) or 0)
            # the remainders of the log / checkpoint chunks get graphs of their own
            tr.capture(grad_sync, warmup=warm, steps=spg, extra_sizes=(log_steps % spg, save_steps % spg))
        else:
            tr.capture(grad_sync, warmup=warm)
        return warm

    @staticmethod
    def _device_release(tr):
        if callable(getattr(tr, "release_graphs", None)):
            if getattr(tr, "on_gpu", False) or getattr(tr, "device", torch.device("cpu")).type == "cuda":
                torch.cuda.synchronize(tr.device)
            tr.release_graphs()
        else:
            tr._graph_exec = None

    def _xgmi_failed(self, xar) -> bool:
        """every rank's xGMI error word, agreed over the process group (MAX)"""
        import torch.distributed as dist

        err = int(xar.error())  # synchronises this rank's device
        flag = torch.tensor([err], dtype=torch.int32)
        if dist_backend() == "nccl":
            flag = flag.to(self.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        return int(flag.item()) != 0

    def _device_resync(self, tr):
        """broadcast rank 0's parameters and optimizer state to every rank (after a
        collective that may have left the ranks apart)"""
        import torch.distributed as dist

        for t in tr.dp_state_tensors():
            if dist_backend() == "gloo" and t.is_cuda:
                h = t.cpu()
                dist.broadcast(h, 0)
                t.copy_(h)
            else:
                dist.broadcast(t, 0)
        if callable(getattr(tr, "refresh_shadows", None)):
            tr.refresh_shadows()

    def _device_restore(self, tr):
        """resume from model_dir: weights + optimizer slots (rank 0's file, identical on every
        rank) and this rank's own sampler stream"""
        path = latest_checkpoint(self.model_dir)
        if path is None:
            return
        state = torch.load(path, map_location="cpu", weights_only=True)
        saved_world = int(state.get("world", 1))
        own = rank_checkpoint(path, self.rank)
        same_world = saved_world == self.world
        if self.rank != 0 and same_world and os.path.exists(own):
            state = torch.load(own, map_location="cpu", weights_only=True)
        elif self.rank != 0:
            same_world = False  # no file of this rank: derive its stream
        # the trainer's own parameter names (row-sharded trainers name them without assembling
        # any table); the tables themselves come from the per-rank shard files
        keys = tr.logical_keys() if callable(getattr(tr, "logical_keys", None)) else set(tr.state_dict())
        tr.load_logical({k: v for k, v in state["model"].items() if k in keys})
        if state.get("shards"):
            if not callable(getattr(tr, "load_shards", None)):
                raise RuntimeError(f"{path} keeps tables in per-rank shard files that this trainer cannot read")
            base = re.sub(r"-rank\d+\.pt$", ".pt", path)
            tr.load_shards(os.path.dirname(base), self._shard_metas(base, saved_world))
        st = state.get("device_trainer")
        if st is not None:
            st = dict(st)
            if not same_world:
                # a new rank layout: a per-rank key as at start-up, the saved counter (no
                # rank replays a stream another rank already consumed)
                rng = torch.as_tensor(st["rng"]).clone()
                rng[0] = int(self.params.get("seed") or 0) * 7919 + self.rank
                st["rng"] = rng
            tr.load_trainer_state(st)
        self.global_step = int(state["step"])
        tr.write_to_model(self.model)
        log.info("restored %s at step %d (device path, rank %d%s)", own if same_world else path, self.global_step,
                 self.rank, "" if same_world else ", re-derived sampler key")

    def _device_save(self, tr):
        """every rank writes its checkpoint file (its own Philox stream) — and, for a
        row-sharded trainer, its own rows of every table plus their optimizer slots
        (``checkpoint_shards``: no table is ever assembled); rank 0 commits the step after
        the barrier, once every rank's files exist.  The barrier also keeps the other ranks
        out of the next chunk's collectives until rank 0 has written (a rank spinning in an
        xGMI wait while rank 0 writes could time out)."""
        shards = getattr(tr, "checkpoint_shards", None)
        if not callable(shards):
            tr.write_to_model(self.model)
            shards = None
        # a trainer whose tables live outside the model's modules while it trains
        # (row-sparse tables) gives the checkpoint its own model-named state
        ms = tr.checkpoint_model_state() if callable(getattr(tr, "checkpoint_model_state", None)) else None
        path = self.save(extra={"device_trainer": tr.trainer_state(), "optimizer": None}, all_ranks=True,
                         model_state=ms, shards=shards, commit=False)
        dp.barrier()
        if self.rank == 0:
            self._commit(self.global_step, path)

    def _eval_batches(self):
        return self.evaluate_input_fn()

    # ------------------------------------------------------------------ device-path eval / infer
    def _device_inference_trainer(self):
        """the device trainer for evaluate / infer (``device_graph=True``): the live one
        after a device-path train, else one built on the HBM graph and restored from
        model_dir; None when its model has no device inference (``infer_logits``), which
        leaves evaluate / infer on the engine path (reference base_estimator.py:145-179:
        one model function for train, eval and predict)"""
        if not self.params.get("device_graph") or self.params.get("device_infer", True) is False:
            return None
        tr = getattr(self, "device_trainer", None)
        if tr is None:
            from euler_amd.estimator.device_trainers import device_infers

            if not device_infers(self.model):
                return None
            try:
                first = self.get_train_from_input(self.train_input_fn(), self.params)
                tr = self._device_graph_trainer(first)
            except (ValueError, NotImplementedError) as e:
                log.info("no device trainer for %s (%s): engine-path evaluate / infer", type(self.model).__name__, e)
                return None
            self._device_restore(tr)
            self.device_trainer = tr
        return tr if callable(getattr(tr, "infer_logits", None)) or callable(getattr(tr, "infer_embed", None)) \
            else None

    def _lockstep_batches(self, tr, batches, extract, first_only=False):
        """``(src, kwargs)`` per batch.  A trainer on a row-sharded graph answers inference
        collectively (``collective_infer``: every batch crosses the ranks' exchanges), so all
        ranks run the same number of batches of one padded size: the count is agreed over
        the group (MAX) and a rank out of ids runs empty batches, whose rows are all padding
        (``src`` None: nothing to record)."""
        if not getattr(tr, "collective_infer", False):
            for b in batches:
                yield extract(b), {}
            return
        srcs = [extract(b) for b in batches]
        n = torch.tensor([len(srcs)], dtype=torch.int64)
        if dp.is_distributed():
            n = n.to(self.device) if dist.get_backend() == "nccl" else n
            dist.all_reduce(n, op=dist.ReduceOp.MAX)
        pad = int(self.params["batch_size"])
        count = min(int(n.item()), 1) if first_only else int(n.item())  # the same on every rank
        for i in range(count):
            if i < len(srcs):
                yield srcs[i], {"pad_to": pad}
            else:
                yield None, {"pad_to": pad}

    def _device_evaluate(self, tr):
        """loss and the model's streaming metric over the eval id batches, every batch's
        block / tree built and run on the device"""
        import torch.nn.functional as F

        met = getattr(self.model, "metric", None)
        if met is not None and hasattr(met, "reset"):
            met.reset()
        name = getattr(self.model, "metric_name", getattr(tr, "metric_name", "f1"))
        losses, res, steps, n, t0 = [], {}, 0, 0, time.time()
        extract = lambda b: self.get_evaluate_from_input(b, self.params)  # noqa: E731
        for src, kw in self._lockstep_batches(tr, self._eval_batches(), extract, self.evaluate_stop_onetime):
            if src is None:  # a padding batch of the collective loop
                tr.infer_logits(torch.zeros(0, dtype=torch.int64), **kw)
                continue
            try:
                _, logits, y = tr.infer_logits(src, **kw)
            except NotImplementedError:
                return None
            losses.append(float(F.binary_cross_entropy_with_logits(logits, y.float())))
            value = met(y.detach(), torch.sigmoid(logits).detach()) if met is not None else float("nan")
            res = {"loss": float(np.mean(losses)), name: float(value)}
            steps += 1
            n += int(torch.as_tensor(src).numel())
            if self.evaluate_stop_onetime and not getattr(tr, "collective_infer", False):
                break
        if self.rank == 0:
            log.info("evaluate: %s over %d batches (device path, %.1f nodes/s)", res, steps,
                     n / max(time.time() - t0, 1e-9))
        return res

    def _device_infer(self, tr):
        ids_out, emb_out = [], []
        n, t0 = 0, time.time()
        extract = lambda b: self.get_infer_from_input(b, self.params)  # noqa: E731
        for src, kw in self._lockstep_batches(tr, self.infer_input_fn(), extract):
            if src is None:  # a padding batch of the collective loop
                tr.infer_embed(torch.zeros(0, dtype=torch.int64), **kw)
                continue
            try:
                emb = tr.infer_embed(src, **kw)
            except NotImplementedError:
                return None
            s, e = self.transfer_embedding(src, emb)
            ids_out.append(np.asarray(torch.as_tensor(s).detach().cpu()))
            emb_out.append(torch.as_tensor(e).detach().float().cpu().numpy())
            n += int(torch.as_tensor(src).numel())
        self.infer_rate = n / max(time.time() - t0, 1e-9)
        if self.rank == 0:
            log.info("infer: %d embeddings (device path, %.1f embeddings/s)", n, self.infer_rate)
        return self._write_infer(ids_out, emb_out)

    def _write_infer(self, ids_out, emb_out):
        out_dir = self.params.get("infer_dir", self.model_dir)
        os.makedirs(out_dir, exist_ok=True)
        ids = np.concatenate(ids_out, 0) if ids_out else np.zeros((0,), np.int64)
        embs = np.concatenate(emb_out, 0) if emb_out else np.zeros((0, 0), np.float32)
        np.save(os.path.join(out_dir, "embedding_%d.npy" % self.rank), embs)
        np.save(os.path.join(out_dir, "ids_%d.npy" % self.rank), ids)
        return ids, embs

    @torch.no_grad()
    def evaluate(self):
        tr = self._device_inference_trainer()
        if tr is not None and callable(getattr(tr, "infer_logits", None)):
            res = self._device_evaluate(tr)
            if res is not None:
                return res
        self.model.to(self.device)
        batches = iter(self._eval_batches())
        first = next(batches, None)
        if first is None:
            return {}
        src = self.get_evaluate_from_input(first, self.params)
        self.model.eval()
        if any(isinstance(p, nn.parameter.UninitializedParameter) for p in self.model.parameters()):
            self._run_model(src)
        self.restore(strict=False)
        for m in self.model.modules():
            met = getattr(m, "metric", None)
            if met is not None and hasattr(met, "reset"):
                met.reset()
        res = {}
        steps = 0
        losses = []
        while src is not None:
            _, loss, name, metric = self._run_model(src)
            losses.append(float(loss))
            res = {"loss": float(np.mean(losses)), name: float(metric)}
            steps += 1
            if self.evaluate_stop_onetime:
                break
            nxt = next(batches, None)
            src = None if nxt is None else self.get_evaluate_from_input(nxt, self.params)
        if self.rank == 0:
            log.info("evaluate: %s over %d batches", res, steps)
        return res

    @torch.no_grad()
    def infer(self):
        tr = self._device_inference_trainer()
        if tr is not None and callable(getattr(tr, "infer_embed", None)):
            out = self._device_infer(tr)
            if out is not None:
                return out
        self.model.to(self.device)
        self.model.eval()
        ids_out, emb_out = [], []
        restored = False
        for batch in self.infer_input_fn():
            src = self.get_infer_from_input(batch, self.params)
            if not restored:
                if any(isinstance(p, nn.parameter.UninitializedParameter) for p in self.model.parameters()):
                    self._run_model(src)
                self.restore(strict=False)
                restored = True
            emb, _, _, _ = self._run_model(src)
            s, e = self.transfer_embedding(src, emb)
            ids_out.append(np.asarray(torch.as_tensor(s).detach().cpu()))
            emb_out.append(torch.as_tensor(e).detach().float().cpu().numpy())
        return self._write_infer(ids_out, emb_out)

    def train_and_evaluate(self):
        res = self.train()
        ev = self.evaluate()
        return res, ev
