"""Collectives that also run when several ranks share one GPU.

RCCL (``nccl``) needs one GPU per rank; the shared-GPU rehearsals of this repository run
their ranks on the box's single MI355X over ``gloo``, whose all-to-all takes host tensors
only.  :func:`all_to_all_single` is ``torch.distributed.all_to_all_single`` on RCCL (and on
host tensors) and stages device tensors through host memory on gloo — the same exchange,
so every sharded path (tables, graph, features, stores) runs its GPU kernels at W > 1 on a
one-GPU box.  The staged form is eager only (not hipGraph-capturable), like gloo itself.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

__all__ = ["all_reduce", "all_to_all_single"]


def all_to_all_single(output: torch.Tensor, input: torch.Tensor, output_split_sizes=None, input_split_sizes=None,
                      group=None):
    if (input.is_cuda or output.is_cuda) and dist.get_backend(group) == "gloo":
        host_out = torch.empty(output.shape, dtype=output.dtype)
        dist.all_to_all_single(host_out, input.detach().cpu().contiguous(), output_split_sizes, input_split_sizes,
                               group=group)
        output.copy_(host_out)
        return
    dist.all_to_all_single(output, input, output_split_sizes, input_split_sizes, group=group)


def all_reduce(t: torch.Tensor, op=dist.ReduceOp.SUM, group=None) -> torch.Tensor:
    """in-place ``all_reduce`` of ``t`` (device tensors staged through host on gloo)"""
    if t.is_cuda and dist.get_backend(group) == "gloo":
        host = t.detach().cpu()
        dist.all_reduce(host, op=op, group=group)
        t.copy_(host)
        return t
    dist.all_reduce(t, op=op, group=group)
    return t
