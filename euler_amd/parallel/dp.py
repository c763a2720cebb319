"""Data parallelism over RCCL (one process per GPU) — the replacement for the
reference's TF parameter-server between-graph replication (``dist_tf_euler.sh``,
``base_estimator.py:164``).

* :func:`init_distributed` reads ``RANK / LOCAL_RANK / WORLD_SIZE`` (torchrun), pins the
  process to ``cuda:LOCAL_RANK`` and initialises ``nccl`` (= RCCL on ROCm) on GPUs,
  ``gloo`` on CPU.
* :class:`GradSync` all-reduces gradients in a few large contiguous buckets, each
  launched asynchronously from a post-accumulate-grad hook as soon as every
  parameter in it has its gradient, so the ring all-reduce over xGMI overlaps the
  rest of backward.  With :class:`~euler_amd.parallel.flat.FlatParams` the buckets are
  zero-copy slices of the one flat gradient buffer; otherwise grads are copied into
  bucket buffers.  Buckets default to 32 MiB: large enough that per-link ring
  bandwidth (not launch latency) dominates, small enough to overlap.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

__all__ = ["init_distributed", "is_distributed", "rank", "world_size", "allreduce_flat", "broadcast_module",
           "GradSync", "barrier"]


def is_distributed() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else int(os.environ.get("RANK", 0))


def world_size() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else \
        int(os.environ.get("WORLD_SIZE", 1))


def init_distributed(backend: str | None = None, device: torch.device | None = None):
    """Initialise the default process group from torchrun-style env vars.

    Returns ``(rank, world_size, device)``; a no-op returning (0, 1, device) when
    ``WORLD_SIZE`` is unset or 1.
    """
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rk = int(os.environ.get("RANK", "0"))
    lr = int(os.environ.get("LOCAL_RANK", "0"))
    if device is None:
        device = torch.device("cuda", lr) if torch.cuda.is_available() else torch.device("cpu")
    if device.type == "cuda":
        torch.cuda.set_device(device)
    if ws <= 1:
        return 0, 1, device
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        if backend is None:
            backend = "nccl" if device.type == "cuda" else "gloo"
        kw = {"device_id": device} if backend == "nccl" else {}
        dist.init_process_group(backend, rank=rk, world_size=ws, **kw)
    return dist.get_rank(), dist.get_world_size(), device


def barrier():
    if is_distributed():
        dist.barrier()


def allreduce_flat(buf: torch.Tensor, average: bool = True, group=None):
    """One all-reduce of a flat buffer (sum, then scale by 1/world if ``average``)."""
    if not is_distributed():
        return buf
    dist.all_reduce(buf, group=group)
    if average:
        buf.mul_(1.0 / dist.get_world_size(group))
    return buf


@torch.no_grad()
def broadcast_module(module: torch.nn.Module, src: int = 0, group=None):
    """Make every rank start from rank ``src``'s parameters and buffers (one coalesced
    broadcast per dtype)."""
    if not is_distributed():
        return
    # row-sharded tables (ShardedEmbedding under 2+ ranks) hold different rows per rank
    tensors = [t for t in list(module.parameters()) + list(module.buffers())
               if not isinstance(t, torch.nn.parameter.UninitializedParameter)
               and not getattr(t, "_euler_sharded", False)]
    by_dtype = {}
    for t in tensors:
        by_dtype.setdefault((t.dtype, t.device), []).append(t)
    for (_, _), ts in by_dtype.items():
        flat = torch.cat([t.detach().reshape(-1) for t in ts])
        dist.broadcast(flat, src, group=group)
        o = 0
        for t in ts:
            n = t.numel()
            t.copy_(flat[o:o + n].view_as(t))
            o += n


class GradSync:
    """Bucketed, backward-overlapped gradient all-reduce.

    Usage::

        sync = GradSync(model.parameters())
        loss.backward()
        sync.finish()        # waits for the buckets, averages, writes p.grad
        opt.step()
    """

    def __init__(self, params, bucket_bytes: int = 32 << 20, group=None, flat=None):
        self.group = group
        self.enabled = is_distributed()
        self.flat = flat
        params = [p for p in params if p.requires_grad]
        self.params = params
        self._handles = {}
        self._hooks = []
        self._buckets = []  # list of dict(params, offsets, buffer, pending)
        if not self.enabled or not params:
            return
        # backward produces grads roughly in reverse parameter order
        order = list(reversed(params))
        cur, cur_bytes = [], 0
        for p in order:
            cur.append(p)
            cur_bytes += p.numel() * 4
            if cur_bytes >= bucket_bytes:
                self._buckets.append(cur)
                cur, cur_bytes = [], 0
        if cur:
            self._buckets.append(cur)
        self._bucket_of = {}
        self._state = []
        for bi, ps in enumerate(self._buckets):
            n = sum(p.numel() for p in ps)
            buf = None
            if flat is None:
                buf = torch.zeros(n, dtype=torch.float32, device=ps[0].device)
            self._state.append({"params": ps, "n": n, "buf": buf, "ready": 0})
            for p in ps:
                self._bucket_of[p] = bi
        for p in params:
            self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))

    def _flat_slice(self, bi):
        """For FlatParams-backed grads: the contiguous [lo, hi) range of the bucket."""
        st = self._state[bi]
        where = {id(q): i for i, q in enumerate(self.flat.params)}  # identity, not tensor ==
        ptrs = []
        for p in st["params"]:
            o, n = self.flat.offsets[where[id(p)]]
            ptrs.append((o, o + n))
        lo, hi = min(a for a, _ in ptrs), max(b for _, b in ptrs)
        if hi - lo != st["n"]:
            return None
        return self.flat.grad[lo:hi]

    def _launch(self, bi):
        st = self._state[bi]
        buf = self._flat_slice(bi) if self.flat is not None else None
        if buf is None:
            if st["buf"] is None:
                st["buf"] = torch.zeros(st["n"], dtype=torch.float32, device=st["params"][0].device)
            buf = st["buf"]
            o = 0
            for p in st["params"]:
                n = p.numel()
                if p.grad is None:
                    buf[o:o + n].zero_()
                else:
                    buf[o:o + n].copy_(p.grad.reshape(-1))
                o += n
            st["copy_back"] = True
        else:
            st["copy_back"] = False
        st["live"] = buf
        self._handles[bi] = dist.all_reduce(buf, group=self.group, async_op=True)

    def _on_grad(self, p):
        bi = self._bucket_of[p]
        st = self._state[bi]
        st["ready"] += 1
        if st["ready"] == len(st["params"]) and bi not in self._handles:
            self._launch(bi)

    def finish(self):
        if not self.enabled:
            return
        for bi in range(len(self._state)):
            if bi not in self._handles:
                self._launch(bi)
        inv = 1.0 / dist.get_world_size(self.group)
        for bi, h in self._handles.items():
            h.wait()
            st = self._state[bi]
            buf = st["live"]
            buf.mul_(inv)
            if st["copy_back"]:
                o = 0
                for p in st["params"]:
                    n = p.numel()
                    g = buf[o:o + n].view_as(p).to(p.dtype)
                    if p.grad is None:
                        p.grad = g.clone()
                    else:
                        p.grad.copy_(g)
                    o += n
        self._handles.clear()
        for st in self._state:
            st["ready"] = 0

    def remove(self):
        """detach the hooks and drop the bucket buffers (a trainer that syncs itself)"""
        for h in self._hooks:
            h.remove()
        self._hooks = []
        self._buckets, self._state, self.enabled = [], [], False
