"""Two-shot all-reduce over xGMI peer memory (``csrc/hip/xgmi_ar.hip``).

The data-parallel gradient of the headline step is ~1 MB, where a ring all-reduce is bound
by its 2 (W - 1) dependent hops, not by bytes.  MI355X's xGMI connects every GPU of a node
to each of its peers directly, so each rank maps its peers' buffers (HIP IPC handles
exchanged once over the process group) and reduces in two phases with one cross-GPU
barrier each: reduce-scatter (rank r sums shard r of every peer's staged input, reading all
7 links at once) and all-gather.  The kernel is capturable into the step's hipGraph like an
RCCL call, but it is one launch of a few dozen blocks with no proxy thread.

Usage (one process per GPU, after ``init_process_group``)::

    ar = XgmiAllReduce(capacity_bytes=grad.numel() * grad.element_size())
    if ar.self_test(): ar(grad)         # in place: grad <- sum over ranks

Every cross-GPU wait is bounded (``timeout_s``): a missing peer sets :meth:`error` instead of
hanging the GPU, and :meth:`self_test` agrees across ranks on whether the path works, so a
caller can fall back to RCCL.  Reference: the gradient sync of the reference's between-graph
data parallelism (tf_euler/scripts/dist_tf_euler.sh:1-49,
euler_estimator/python/base_estimator.py:164).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from ..ops._native import hip


def _blocks_for(numel: int, world: int, elem_bytes: int) -> int:
    # xar_vec_per_thread 16-byte vectors per thread per shard sweep, 256 threads per block
    # (EULER_AMD_XAR_BLOCKS overrides, for tuning)
    env = os.environ.get("EULER_AMD_XAR_BLOCKS")
    if env:
        return max(1, min(int(hip().xar_max_blocks), int(env)))
    # at least 16 blocks (two per XCD): the staging copy moves the WHOLE local tensor, not
    # one shard, and a few blocks cannot pull ~1 MB out of HBM quickly
    vec = 16 // elem_bytes
    shard_vecs = -(-numel // (vec * world))
    per_block = 256 * int(hip().xar_vec_per_thread)
    need = -(-shard_vecs // per_block)
    return max(1, min(int(hip().xar_max_blocks), max(need, min(16, -(-numel // (vec * 256))))))


class XgmiAllReduce:
    """In-place sum all-reduce of a GPU tensor (fp32 or bf16) across the ranks of ``group``
    (one process per GPU; ``group`` is only used to exchange handles at setup, so a gloo
    group works as well as an RCCL one)."""

    def __init__(self, capacity_bytes: int, group=None, timeout_s: float = 10.0):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if self.world > int(hip().xar_max_ranks):
            raise ValueError(f"xGMI all-reduce supports up to {hip().xar_max_ranks} ranks, got {self.world}")
        cap = -(-int(capacity_bytes) // 4096) * 4096
        # a rank that cannot allocate, export or map still takes part in every collective
        # below (no rank may hang in the exchange); self_test() then fails on every rank
        self.setup_error = None
        try:
            self._ar = hip().XgmiAr(cap, float(timeout_s))
            mine = self._ar.handle()
        except Exception as e:  # noqa: BLE001 - reported through self_test()
            self._ar, mine, self.setup_error = None, b"", repr(e)
        handles = [None] * self.world
        dist.all_gather_object(handles, mine, group=group)
        self.ok = self._ar is not None and all(len(h) > 0 for h in handles)
        if self.ok:
            try:
                self._ar.open(handles, self.rank)
            except Exception as e:  # noqa: BLE001
                self.ok, self.setup_error = False, repr(e)
        dist.barrier(group=group)  # every buffer zeroed and mapped before any flag is written

    @property
    def capacity(self) -> int:
        return int(self._ar.capacity()) if self._ar is not None else 0

    def __call__(self, t: torch.Tensor) -> torch.Tensor:
        if not self.ok:
            raise RuntimeError(f"xGMI all-reduce is not set up on this rank: {self.setup_error}")
        if t.numel() * t.element_size() > self.capacity:
            raise ValueError("tensor exceeds the xGMI all-reduce buffer")
        self._ar.run(t, _blocks_for(t.numel(), self.world, t.element_size()))
        return t

    def input_view(self, numel: int, dtype) -> torch.Tensor:
        """A tensor over this rank's IPC input region.  A producer that writes its gradient
        there (SageTrainer.use_grad_buffer) gets the all-reduce in place: no staging copy,
        one dependent memory round trip less per call.  Valid while this object lives; a
        call on any other tensor stages through the same region, so a caller that adopted
        the view reduces only the view (or slices of it, sliced alike on every rank)."""
        return self._ar.input_view(int(numel), dtype == torch.bfloat16)

    def error(self) -> int:
        """1 if a cross-GPU wait timed out on this rank since construction (synchronises)."""
        return int(self._ar.error()) if self._ar is not None else 1

    def self_test(self, numel: int | None = None, dtype=torch.float32, calls: int = 3,
                  in_place: bool = False) -> bool:
        """Eager check against an RCCL/gloo-free reference: in call c rank r contributes
        (r + 1) * 2^c * base with a rank-independent ``base``, so every element's sum is
        known in closed form and differs from call to call.  ``in_place``: the input is
        written into :meth:`input_view` first (the trainer's zero-copy mode).
        Returns the all-rank verdict (True only if every rank saw exact results)."""
        dev = torch.device("cuda", torch.cuda.current_device())
        # every rank must agree that every rank mapped its peers before any kernel runs
        # (a rank whose peers are not mapped would wait on flags nobody writes)
        flag = torch.tensor([0 if self.ok else 1], dtype=torch.int32)
        if dist.get_backend(self.group) == "nccl":
            flag = flag.to(dev)
        dist.all_reduce(flag, group=self.group)
        if int(flag.item()) != 0:
            return False
        esz = torch.empty((), dtype=dtype).element_size()
        vec = 16 // esz
        n = numel if numel is not None else self.capacity // esz
        n = max(vec, (min(n, self.capacity // esz) // vec) * vec)
        g = torch.Generator(device="cpu").manual_seed(1234)
        base = torch.randint(-8, 9, (n,), generator=g).to(dev, torch.float32)  # exact in bf16 sums
        want = base * (self.world * (self.world + 1) // 2)
        ok = True
        for c in range(calls):
            # a different sum every call (x 2^c keeps bf16 exact): a stale read of the
            # previous call's peer data cannot pass
            x = (base * ((self.rank + 1) * 2 ** c)).to(dtype)
            if in_place:  # written by a torch kernel into the IPC region, reduced there
                x = self.input_view(n, dtype).copy_(x)
            self(x)
            torch.cuda.synchronize()
            ok = ok and bool(torch.equal(x.float(), want * 2 ** c))
        ok = ok and self.error() == 0
        flag = torch.tensor([0 if ok else 1], dtype=torch.int32)
        if dist.get_backend(self.group) == "nccl":
            flag = flag.to(dev)
        dist.all_reduce(flag, group=self.group)
        return int(flag.item()) == 0


def _graph_call_us(fn, calls: int = 20, reps: int = 3, group=None) -> float:
    """Per-call time of ``fn`` replayed from a hipGraph of ``calls`` calls (best of ``reps``
    replays), the MAX over the ranks of ``group`` (every rank gets the same number)."""
    import time

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        for _ in range(calls):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        dist.barrier(group=group)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / calls * 1e6)
    del g
    t = torch.tensor([best], dtype=torch.float64)
    if dist.get_backend(group) == "nccl":
        t = t.cuda()
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def make_grad_sync(buf: torch.Tensor, kind: str = "auto", group=None, rebind=None, timeout_s: float = 10.0):
    """``grad_sync(g)`` for a data-parallel trainer step (SageTrainer / UnsupSageTrainer
    ``step(grad_sync)``): an in-place sum all-reduce of (slices of) ``buf`` returning the
    1 / world scale.  ``kind``: "xgmi" (this module's kernel), "rccl" (torch.distributed
    all_reduce), "auto": with 2+ ranks on GPUs, the xGMI kernel's self-test runs on every
    rank, then both all-reduces are timed on ``buf`` itself (hipGraph-replayed, max over
    ranks) and the faster one is kept — measured on the node the job runs on, not assumed —
    or "tune" (the same, also with one rank).
    ``rebind(view)``: with xGMI chosen, hand the producer a view of the IPC input region to
    write its gradient into (SageTrainer.use_grad_buffer), after an in-place self-test.
    ``timeout_s`` bounds every cross-GPU wait of the xGMI kernel.
    Returns ``(grad_sync, name, info)``; ``info`` holds the XgmiAllReduce (``xar``, None for
    RCCL, whose :meth:`~XgmiAllReduce.error` the caller checks after a run) and the timings."""
    world = dist.get_world_size(group)
    info = {"xar": None}
    xar = None
    world_ok = world > 1 or kind == "tune"  # "tune": "auto" also with one rank
    if kind == "tune":
        kind = "auto"
    if kind == "xgmi" or (kind == "auto" and world_ok and buf is not None and buf.is_cuda):
        xar = XgmiAllReduce(buf.numel() * buf.element_size(), group=group, timeout_s=timeout_s)
        if not xar.self_test(numel=buf.numel(), dtype=buf.dtype):
            if kind == "xgmi":
                raise RuntimeError("xGMI all-reduce self-test failed")
            info["xgmi_self_test"] = "failed"
            xar = None
    if xar is not None and kind == "auto" and dist.get_backend(group) == "nccl":
        scratch = torch.zeros_like(buf)
        t_x = _graph_call_us(lambda: xar(scratch), group=group)
        t_r = _graph_call_us(lambda: dist.all_reduce(scratch, group=group), group=group)
        info["us_per_call"] = {"xgmi": round(t_x, 2), "rccl": round(t_r, 2)}
        if xar.error() != 0 or t_r < t_x:
            xar = None
    if xar is not None and rebind is not None:
        # zero copy: the producer writes its gradient straight into the IPC input region
        if xar.self_test(numel=buf.numel(), dtype=buf.dtype, in_place=True):
            rebind(xar.input_view(buf.numel(), buf.dtype))
            info["in_place"] = True
        else:
            info["in_place"] = False
    if xar is not None:
        info["xar"] = xar

        def grad_sync(g):
            xar(g)
            return 1.0 / world

        return grad_sync, "xgmi", info

    if dist.get_backend(group) == "gloo":
        def grad_sync(g):  # gloo: through host memory (eager only, not capturable)
            if g.is_cuda:
                h = g.cpu()
                dist.all_reduce(h, group=group)
                g.copy_(h)
            else:
                dist.all_reduce(g, group=group)
            return 1.0 / world

        return grad_sync, "gloo", info

    def grad_sync(g):
        dist.all_reduce(g, group=group)
        return 1.0 / world

    return grad_sync, "rccl", info
