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

import torch
import torch.distributed as dist

from ..ops._native import hip


def _blocks_for(numel: int, world: int, elem_bytes: int) -> int:
    # one 16-byte vector per thread per shard sweep, 256 threads per block
    vec = 16 // elem_bytes
    shard_vecs = -(-numel // (vec * world))
    return max(1, min(int(hip().xar_max_blocks), -(-shard_vecs // 256)))


class XgmiAllReduce:
    """In-place sum all-reduce of a GPU tensor (fp32 or bf16) across the ranks of ``group``
    (one process per GPU; ``group`` is only used to exchange handles at setup, so a gloo
    group works as well as an RCCL one)."""

    def __init__(self, capacity_bytes: int, group=None, timeout_s: float = 2.0):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if self.world > int(hip().xar_max_ranks):
            raise ValueError(f"xGMI all-reduce supports up to {hip().xar_max_ranks} ranks, got {self.world}")
        cap = -(-int(capacity_bytes) // 4096) * 4096
        self._ar = hip().XgmiAr(cap, float(timeout_s))
        handles = [None] * self.world
        dist.all_gather_object(handles, self._ar.handle(), group=group)
        self._ar.open(handles, self.rank)
        dist.barrier(group=group)  # every buffer zeroed and mapped before any flag is written

    @property
    def capacity(self) -> int:
        return int(self._ar.capacity())

    def __call__(self, t: torch.Tensor) -> torch.Tensor:
        if t.numel() * t.element_size() > self.capacity:
            raise ValueError("tensor exceeds the xGMI all-reduce buffer")
        self._ar.run(t, _blocks_for(t.numel(), self.world, t.element_size()))
        return t

    def error(self) -> int:
        """1 if a cross-GPU wait timed out on this rank since construction (synchronises)."""
        return int(self._ar.error())

    def self_test(self, numel: int | None = None, dtype=torch.float32, calls: int = 3) -> bool:
        """Eager check against an RCCL/gloo-free reference: rank r contributes (r + 1) * base
        with a rank-independent ``base``, so every element's sum is known in closed form.
        Returns the all-rank verdict (True only if every rank saw exact results)."""
        dev = torch.device("cuda", torch.cuda.current_device())
        esz = torch.empty((), dtype=dtype).element_size()
        vec = 16 // esz
        n = numel if numel is not None else self.capacity // esz
        n = max(vec, (min(n, self.capacity // esz) // vec) * vec)
        g = torch.Generator(device="cpu").manual_seed(1234)
        base = torch.randint(-8, 9, (n,), generator=g).to(dev, torch.float32)  # exact in bf16 sums
        want = base * (self.world * (self.world + 1) // 2)
        ok = True
        for _ in range(calls):
            x = (base * (self.rank + 1)).to(dtype)
            self(x)
            torch.cuda.synchronize()
            ok = ok and bool(torch.equal(x.float(), want))
        ok = ok and self.error() == 0
        flag = torch.tensor([0 if ok else 1], dtype=torch.int32)
        if dist.get_backend(self.group) == "nccl":
            flag = flag.to(dev)
        dist.all_reduce(flag, group=self.group)
        return int(flag.item()) == 0
