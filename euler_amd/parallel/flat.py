"""Flat parameter / gradient buffers and a one-launch optimizer.

GNN towers are small (10^4-10^6 parameters), so per-tensor optimizer launches and
per-tensor all-reduces are pure overhead.  ``FlatParams`` re-homes every parameter
of a module into ONE contiguous fp32 buffer (parameters become views) and gives
each parameter a ``.grad`` view into ONE flat gradient buffer, which autograd
accumulates into in place.  That makes

* the data-parallel gradient sync a single bucketed RCCL all-reduce
  (``parallel.dp.allreduce_flat``), and
* the optimizer a single gfx950 kernel over the whole model (``csrc/hip/optim.hip``),
  hipGraph-capturable because the Adam step count lives on the device.

Optimizer kinds mirror the reference's ``tf_euler/python/utils/optimizers.py:22-31``
(sgd, momentum, adagrad, adam).
"""
from __future__ import annotations

import torch

from euler_amd.ops._native import hip, use_hip

__all__ = ["FlatParams", "FlatOptimizer"]

_KINDS = {"adam": 0, "adagrad": 1, "sgd": 2, "momentum": 3}


class FlatParams:
    def __init__(self, params, device=None):
        self.params = [p for p in params if p.requires_grad]
        if device is None:
            device = self.params[0].device if self.params else torch.device("cpu")
        total = sum(p.numel() for p in self.params)
        self.numel = total  # parameter elements; the buffers are padded to a multiple of 8
        # (zeros that never get a gradient): the xGMI all-reduce moves 16-byte vectors of
        # fp32 or bf16 (parallel/xgmi.py), whatever the model's parameter count
        padded = total + (-total) % 8
        self.flat = torch.zeros(padded, dtype=torch.float32, device=device)
        self.grad = torch.zeros(padded, dtype=torch.float32, device=device)
        self.offsets = []
        o = 0
        for p in self.params:
            n = p.numel()
            self.flat[o:o + n].copy_(p.detach().reshape(-1).float())
            p.data = self.flat[o:o + n].view(p.shape)
            p.grad = self.grad[o:o + n].view(p.shape)
            self.offsets.append((o, n))
            o += n

    def zero_grad(self):
        if self.grad.numel() == 0:
            return
        if use_hip(self.grad):
            # one zero_kernel launch (a kernel node in captured steps; EULER_AMD_ZERO_MEMSET=1
            # makes it a hipMemsetAsync node instead: docs/DESIGN.md §9, tests/test_graph_memset.py)
            hip().zero_(self.grad)
        else:
            self.grad.zero_()

    def rebind_grads(self):
        """Re-attach the flat grad views (after something replaced ``p.grad``)."""
        for p, (o, n) in zip(self.params, self.offsets):
            if p.grad is None or p.grad.data_ptr() != self.grad[o:o + n].data_ptr():
                p.grad = self.grad[o:o + n].view(p.shape)


class FlatOptimizer:
    def __init__(self, flat: FlatParams, optimizer: str = "adam", learning_rate: float = 1e-3,
                 betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0, momentum: float = 0.9):
        if optimizer not in _KINDS:
            raise ValueError(f"unknown optimizer {optimizer!r}; expected one of {sorted(_KINDS)}")
        self.flat = flat
        self.kind = optimizer
        self.lr = float(learning_rate)
        self.b1, self.b2 = (float(momentum), 0.0) if optimizer == "momentum" else (float(betas[0]), float(betas[1]))
        self.eps = float(eps) if optimizer != "adagrad" else 1e-10
        self.wd = float(weight_decay)
        dev = flat.flat.device
        self.m = torch.zeros_like(flat.flat)
        self.v = torch.zeros_like(flat.flat)
        if optimizer == "adagrad":
            self.v.fill_(0.1)  # tf.train.AdagradOptimizer initial_accumulator_value
        self.step_count = torch.zeros(1, dtype=torch.int64, device=dev)
        # the last block of the update launch advances step_count (csrc/hip/optim.hip)
        self._ticket = torch.zeros(1, dtype=torch.int32, device=dev) if dev.type == "cuda" else None
        # (start, end, weight decay) replacing weight_decay on one element range of the flat
        # buffer (e.g. only an R-GCN's relation matrices): set_decay_range()
        self.decay_range = (0, 0, 0.0)

    def zero_grad(self):
        self.flat.zero_grad()

    def step(self, grad_scale: float = 1.0):
        f = self.flat
        if f.flat.numel() == 0:  # every parameter lives elsewhere (row-sparse tables)
            return
        w0, w1, wd2 = self.decay_range
        if use_hip(f.flat):
            hip().flat_optim_(f.flat, f.grad, self.m, self.v, self.step_count, self.lr, self.b1, self.b2,
                              self.eps, self.wd, float(grad_scale), _KINDS[self.kind], self._ticket, float(wd2),
                              int(w0), int(w1))
            return
        with torch.no_grad():
            self.step_count += 1
            wd = torch.full_like(f.flat, self.wd)
            wd[int(w0):int(w1)] = float(wd2)
            g = f.grad * grad_scale + wd * f.flat
            if self.kind == "adam":
                t = float(self.step_count.item())
                self.m.mul_(self.b1).add_(g, alpha=1 - self.b1)
                self.v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
                mh = self.m / (1 - self.b1 ** t)
                vh = self.v / (1 - self.b2 ** t)
                f.flat.sub_(self.lr * mh / (vh.sqrt() + self.eps))
            elif self.kind == "adagrad":
                self.v.addcmul_(g, g)
                f.flat.sub_(self.lr * g / (self.v.sqrt() + self.eps))
            elif self.kind == "sgd":
                f.flat.sub_(self.lr * g)
            else:
                self.m.mul_(self.b1).add_(g)
                f.flat.sub_(self.lr * self.m)

    def set_decay_range(self, start: int, end: int, weight_decay: float):
        """weight decay ``weight_decay`` instead of the optimizer's on flat elements
        [start, end) (one parameter group, e.g. a relation-matrix regulariser)"""
        self.decay_range = (int(start), int(end), float(weight_decay))

    def state_dict(self):
        return {"kind": self.kind, "lr": self.lr, "m": self.m, "v": self.v, "step": self.step_count}

    def load_state_dict(self, sd):
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        self.step_count.copy_(sd["step"])
