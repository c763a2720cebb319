"""Tracing and per-stage timing (SURVEY §5 "Tracing / profiling").

* :func:`trace_range` — a named range: a roctx range on ROCm GPUs (``torch.cuda.nvtx``
  is backed by roctx there, so ``rocprofv3 --marker-trace`` shows it next to the
  kernels) plus host wall time accumulated in a :class:`StageTimer`.
* :class:`StageTimer` — per-stage counts / total / mean milliseconds, ``report()``.
* :func:`engine_stats` — the C++ engine's process-wide counters (query compile /
  execute microseconds, DAG nodes, remote fan-out, RPC attempts / failures / bytes,
  server requests) from ``_engine.stats()``.

The reference had only an optional TF ``ProfilerHook`` (base_estimator.py:30-35) and
unused wall timers (euler/common/timmer.cc:21-33).
"""
from __future__ import annotations

import contextlib
import os
import time
from collections import defaultdict

import torch

__all__ = ["StageTimer", "trace_range", "default_timer", "engine_stats", "reset_engine_stats", "enabled"]


def enabled() -> bool:
    return os.environ.get("EULER_AMD_TRACE", "0") == "1"


class StageTimer:
    def __init__(self):
        self.total = defaultdict(float)
        self.count = defaultdict(int)

    def add(self, name, seconds):
        self.total[name] += seconds
        self.count[name] += 1

    def reset(self):
        self.total.clear()
        self.count.clear()

    def summary(self):
        return {k: {"count": self.count[k], "total_ms": 1e3 * self.total[k],
                    "mean_ms": 1e3 * self.total[k] / max(self.count[k], 1)} for k in self.total}

    def report(self) -> str:
        rows = sorted(self.summary().items(), key=lambda kv: -kv[1]["total_ms"])
        lines = ["%-24s %8s %12s %10s" % ("stage", "count", "total_ms", "mean_ms")]
        for k, v in rows:
            lines.append("%-24s %8d %12.3f %10.4f" % (k, v["count"], v["total_ms"], v["mean_ms"]))
        return "\n".join(lines)


default_timer = StageTimer()


@contextlib.contextmanager
def trace_range(name: str, timer: StageTimer | None = None, sync: bool = False):
    """roctx range + host timing.  ``sync=True`` synchronises the GPU at both ends so
    the host time covers the device work of the range (use for coarse stages only)."""
    timer = default_timer if timer is None else timer
    gpu = torch.cuda.is_available()
    if gpu:
        if sync:
            torch.cuda.synchronize()
        torch.cuda.nvtx.range_push(name)
    t0 = time.perf_counter()
    try:
        yield
    finally:
        if gpu:
            if sync:
                torch.cuda.synchronize()
            torch.cuda.nvtx.range_pop()
        timer.add(name, time.perf_counter() - t0)


def engine_stats() -> dict:
    from euler_amd.ops._native import engine

    return dict(engine().stats())


def reset_engine_stats():
    from euler_amd.ops._native import engine

    engine().reset_stats()
