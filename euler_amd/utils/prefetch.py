"""Asynchronous host -> HBM input pipeline for the CPU-engine training path.

The reference builds each mini-batch inside the TF graph, serially with the compute
(``tf_euler`` graph ops run as AsyncOpKernels of the same step).  Here the C++ engine
releases the GIL for every query, so batch ``t + 1`` is sampled on worker threads while
the GPU runs batch ``t``:

    worker thread(s):  produce() -> host tensors (engine sampling, feature fetch)
                       -> pinned copies -> non_blocking H2D on a dedicated side stream
                       -> event recorded on the side stream
    consumer:          get() -> current stream waits on the event (no host sync)

``produce`` returns any nesting of tensors / lists / tuples / dicts and objects with a
``to(device, non_blocking)`` method (e.g. :class:`~euler_amd.dataflow.dataflows.DataFlow`).
On CPU devices the pipeline still overlaps sampling with compute but skips the copies.
"""
from __future__ import annotations

import queue
import threading

import torch

__all__ = ["Prefetcher", "to_device"]

_STOP = object()


def _pin(obj):
    if isinstance(obj, torch.Tensor):
        return obj.pin_memory() if obj.device.type == "cpu" else obj
    if isinstance(obj, (list, tuple)):
        return type(obj)(_pin(o) for o in obj)
    if isinstance(obj, dict):
        return {k: _pin(v) for k, v in obj.items()}
    if hasattr(obj, "pin_memory"):
        return obj.pin_memory()
    return obj


def to_device(obj, device, non_blocking=True):
    """Recursively move tensors (and objects with ``.to``) to ``device``."""
    if isinstance(obj, torch.Tensor):
        return obj.to(device, non_blocking=non_blocking)
    if isinstance(obj, (list, tuple)):
        return type(obj)(to_device(o, device, non_blocking) for o in obj)
    if isinstance(obj, dict):
        return {k: to_device(v, device, non_blocking) for k, v in obj.items()}
    if hasattr(obj, "to") and callable(obj.to):
        return obj.to(device, non_blocking)
    return obj


class Prefetcher:
    def __init__(self, produce, device, depth: int = 2, workers: int = 1, pin: bool = True):
        self.produce = produce
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.pin = pin and self.cuda
        self.q: queue.Queue = queue.Queue(maxsize=max(1, int(depth)))
        self._stop = threading.Event()
        self._streams = [torch.cuda.Stream(device=self.device) for _ in range(workers)] if self.cuda else []
        self._threads = [threading.Thread(target=self._run, args=(i,), daemon=True, name="euler-prefetch-%d" % i)
                         for i in range(max(1, int(workers)))]
        for t in self._threads:
            t.start()

    def _run(self, wid):
        try:
            while not self._stop.is_set():
                host = self.produce()
                if host is None:
                    break
                ev = None
                dev_batch = host
                if self.cuda:
                    src = _pin(host) if self.pin else host
                    s = self._streams[wid]
                    with torch.cuda.stream(s):
                        dev_batch = to_device(src, self.device, True)
                        ev = torch.cuda.Event()
                        ev.record(s)
                while not self._stop.is_set():
                    try:
                        self.q.put((dev_batch, ev), timeout=0.1)
                        break
                    except queue.Full:
                        continue
        except BaseException as e:  # surfaced to the consumer
            self.q.put((_STOP, e))
            return
        self.q.put((_STOP, None))

    def get(self):
        """Next batch, already on the device; the current stream is ordered after its copy."""
        batch, ev = self.q.get()
        if batch is _STOP:
            self.q.put((_STOP, ev))  # keep reporting the end to later callers
            if isinstance(ev, BaseException):
                raise ev
            raise StopIteration
        if ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)
        return batch

    def __iter__(self):
        return self

    def __next__(self):
        return self.get()

    def close(self):
        self._stop.set()
        while True:
            try:
                self.q.get_nowait()
            except queue.Empty:
                break
        for t in self._threads:
            t.join(timeout=5)
