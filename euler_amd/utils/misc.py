"""Optimizers, embedding-store updates, hooks, flag defaults, dense adjacency helpers
(reference ``tf_euler/python/utils/{optimizers,embedding,hooks,flags,to_dense_adj,to_dense_batch}.py``)."""
from __future__ import annotations

import time

import torch

__all__ = ["get_optimizer", "optimizers", "embedding_update", "embedding_add", "SyncExitHook", "set_defaults",
           "to_dense_adj", "to_dense_batch", "FLAGS"]


# ----------------------------------------------------------------------------- optimizers
def _fused_ok(params):
    """GPU parameters: the single-kernel (fused) multi-tensor optimizer step"""
    params = list(params)
    return bool(params) and all(p.is_cuda and p.is_floating_point() for p in params), params


def _adam(params, lr):
    ok, params = _fused_ok(params)
    return torch.optim.Adam(params, lr=lr, fused=True) if ok else torch.optim.Adam(params, lr=lr)


def _sgd(momentum):
    def make(params, lr):
        ok, params = _fused_ok(params)
        return torch.optim.SGD(params, lr=lr, momentum=momentum, fused=True) if ok else \
            torch.optim.SGD(params, lr=lr, momentum=momentum)
    return make


optimizers = {
    "sgd": _sgd(0.0),
    "momentum": _sgd(0.9),
    "adagrad": lambda params, lr: torch.optim.Adagrad(params, lr=lr, initial_accumulator_value=0.1),
    "adam": _adam,
}


def get_optimizer(name):
    """``get(name)(params, lr)`` (reference optimizers.py:22-31 returned TF optimizer classes)."""
    return optimizers.get(name)


# ----------------------------------------------------------------------------- embedding stores
def embedding_update(params, ids, values, partition_strategy="mod", add=False):
    """Scatter-update (or add) rows of a (possibly 'mod'-partitioned list of) table(s)
    (reference embedding.py:24-68)."""
    if not isinstance(params, (list, tuple)):
        params = [params]
    ids = torch.as_tensor(ids, device=params[0].device).long()
    values = values.to(params[0].dtype)
    n = len(params)
    with torch.no_grad():
        if n == 1:
            (params[0].index_add_ if add else params[0].index_copy_)(0, ids, values)
            return
        if partition_strategy != "mod":
            raise ValueError("Unrecognized partition strategy: " + partition_strategy)
        part, local = ids % n, ids // n
        for p in range(n):
            sel = (part == p).nonzero(as_tuple=True)[0]
            if sel.numel():
                (params[p].index_add_ if add else params[p].index_copy_)(0, local[sel], values[sel])


def embedding_add(params, ids, values, partition_strategy="mod"):
    return embedding_update(params, ids, values, partition_strategy, add=True)


# ----------------------------------------------------------------------------- hooks
class SyncExitHook:
    """Wait until every worker finished (reference hooks.py:25-40): a barrier over the
    torch.distributed process group instead of a shared PS variable."""

    def __init__(self, num_workers):
        self.num_workers = num_workers

    def end(self, session=None):
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            dist.barrier()
        else:
            time.sleep(0)


# ----------------------------------------------------------------------------- flags
class _Flags(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e


FLAGS = _Flags()


def set_defaults(**kwargs):
    """Set default values of the example flags (reference flags.py:23-25)."""
    for k, v in kwargs.items():
        FLAGS.setdefault(k, v)


# ----------------------------------------------------------------------------- dense helpers
def to_dense_adj(edge_index, batch=None, edge_attr=None, max_num_nodes=None):
    """Dense adjacency [B, N, N] from an edge list (reference to_dense_adj.py)."""
    if batch is None:
        batch = torch.zeros(int(edge_index.max()) + 1 if edge_index.numel() else 0, dtype=torch.long,
                            device=edge_index.device)
    B = int(batch.max()) + 1 if batch.numel() else 1
    counts = torch.bincount(batch, minlength=B)
    cum = torch.cat([torch.zeros(1, dtype=torch.long, device=batch.device), counts.cumsum(0)[:-1]])
    N = int(counts.max()) if max_num_nodes is None else int(max_num_nodes)
    e_b = batch[edge_index[0]]
    i = edge_index[0] - cum[e_b]
    j = edge_index[1] - cum[e_b]
    val = torch.ones(edge_index.shape[1], device=edge_index.device) if edge_attr is None else edge_attr
    adj = torch.zeros((B, N, N) + tuple(val.shape[1:]), dtype=val.dtype, device=edge_index.device)
    adj.index_put_((e_b, i, j), val, accumulate=True)
    return adj


def to_dense_batch(x, batch=None, fill_value=0, max_num_nodes=None):
    """[N, D] + graph index -> ([B, Nmax, D], mask) (reference to_dense_batch.py)."""
    if batch is None:
        batch = torch.zeros(x.shape[0], dtype=torch.long, device=x.device)
    B = int(batch.max()) + 1 if batch.numel() else 1
    counts = torch.bincount(batch, minlength=B)
    cum = torch.cat([torch.zeros(1, dtype=torch.long, device=x.device), counts.cumsum(0)[:-1]])
    N = int(counts.max()) if max_num_nodes is None else int(max_num_nodes)
    pos = torch.arange(x.shape[0], device=x.device) - cum[batch]
    out = torch.full((B, N) + tuple(x.shape[1:]), fill_value, dtype=x.dtype, device=x.device)
    out[batch, pos] = x
    mask = torch.zeros(B, N, dtype=torch.bool, device=x.device)
    mask[batch, pos] = True
    return out, mask
