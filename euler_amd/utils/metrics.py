"""Streaming metrics (reference ``tf_euler/python/utils/metrics.py:23-98``).

TF's ``tf.metrics.*`` accumulate across ``session.run`` calls until the local
variables are reset; here every metric is an object with ``update(...) -> value``
(running value) and ``reset()``.  ``get(name)`` returns a *fresh* metric instance;
calling it like a function updates it.
"""
from __future__ import annotations

import torch

__all__ = ["Metric", "AccScore", "AucScore", "F1Score", "MrrScore", "HitKScore", "MrScore", "get", "metrics"]


class Lazy:
    """A metric value that stays on the device until read (``float(m)``): updates from
    GPU tensors never synchronise the stream."""

    __slots__ = ("fn",)

    def __init__(self, fn):
        self.fn = fn

    def __float__(self):
        return float(self.fn())

    def __repr__(self):
        return repr(float(self))

    def __format__(self, spec):
        return format(float(self), spec)

    # numeric protocol through the value (comparisons, arithmetic in user code / tests)
    def __eq__(self, o):
        return float(self) == o

    def __lt__(self, o):
        return float(self) < o

    def __le__(self, o):
        return float(self) <= o

    def __gt__(self, o):
        return float(self) > o

    def __ge__(self, o):
        return float(self) >= o

    def __add__(self, o):
        return float(self) + o

    __radd__ = __add__

    def __sub__(self, o):
        return float(self) - o

    def __rsub__(self, o):
        return o - float(self)

    def __mul__(self, o):
        return float(self) * o

    __rmul__ = __mul__

    def __truediv__(self, o):
        return float(self) / o

    def __abs__(self):
        return abs(float(self))

    def __round__(self, n=None):
        return round(float(self), n)

    __hash__ = None


class Metric:
    def __init__(self):
        self.reset()

    def reset(self):
        raise NotImplementedError

    def update(self, *args):
        raise NotImplementedError

    def __call__(self, *args):
        return self.update(*args)


def _accumulate(metric, parts):
    """Add the stacked per-batch counts into the metric's device accumulator IN PLACE, so
    a graph-captured step keeps accumulating on every replay (a rebinding ``a = a + v``
    would freeze the captured tensor)."""
    v = torch.stack([t.float() for t in parts])
    if metric.acc is None or metric.acc.device != v.device:
        metric.acc = torch.zeros_like(v)
    metric.acc.add_(v)
    return metric.acc


class AccScore(Metric):
    """accuracy of floor(p + 0.5) against labels (predict = probabilities)."""

    def reset(self):
        if getattr(self, "acc", None) is not None:
            self.acc.zero_()
        else:
            self.acc = None

    def update(self, labels, predict):
        labels = torch.as_tensor(labels).float()
        pred = torch.floor(torch.as_tensor(predict).float().to(labels.device) + 0.5)
        acc = _accumulate(self, [(pred == labels).float().sum(), labels.new_full((), float(labels.numel()))])
        return Lazy(lambda: float(acc[0]) / max(float(acc[1]), 1.0))

    @property
    def correct(self):
        return 0.0 if self.acc is None else float(self.acc[0])

    @property
    def total(self):
        return 0.0 if self.acc is None else float(self.acc[1])


class AucScore(Metric):
    """ROC AUC over sigmoid(predict) with ``num_thresholds`` buckets (tf.metrics.auc)."""

    def __init__(self, num_thresholds=5000):
        self.n = num_thresholds
        super().__init__()

    def reset(self):
        self.pos = torch.zeros(getattr(self, "n", 5000) + 1, dtype=torch.float64)
        self.neg = torch.zeros_like(self.pos)

    def update(self, labels, predict):
        p = torch.sigmoid(torch.as_tensor(predict).double()).reshape(-1).cpu()
        y = torch.as_tensor(labels).double().reshape(-1).cpu()
        b = torch.clamp((p * self.n).long(), 0, self.n)
        self.pos += torch.bincount(b, weights=y, minlength=self.n + 1)
        self.neg += torch.bincount(b, weights=1 - y, minlength=self.n + 1)
        # sweep thresholds from high to low
        tp = torch.flip(torch.cumsum(torch.flip(self.pos, [0]), 0), [0])
        fp = torch.flip(torch.cumsum(torch.flip(self.neg, [0]), 0), [0])
        P, N = self.pos.sum(), self.neg.sum()
        if P == 0 or N == 0:
            return 0.0
        tpr = torch.cat([tp / P, torch.zeros(1, dtype=torch.float64)])
        fpr = torch.cat([fp / N, torch.zeros(1, dtype=torch.float64)])
        return float(torch.sum((fpr[:-1] - fpr[1:]) * (tpr[:-1] + tpr[1:]) / 2))


class F1Score(Metric):
    def reset(self):
        if getattr(self, "acc", None) is not None:
            self.acc.zero_()
        else:
            self.acc = None

    def update(self, labels, predict):
        y = torch.as_tensor(labels).float()
        p = torch.floor(torch.as_tensor(predict).float().to(y.device) + 0.5)
        # device-resident accumulators [tp, fp, fn]: no host sync per step (read through Lazy)
        acc = _accumulate(self, [(p * y).sum(), (p * (1 - y)).sum(), ((1 - p) * y).sum()])

        def value():
            tp, fp, fn = (float(v) for v in acc.tolist())
            eps = 1e-7
            prec = tp / (eps + tp + fp)
            rec = tp / (eps + tp + fn)
            return 2.0 * prec * rec / (prec + rec + eps)

        return Lazy(value)


def _ranks(pos, neg):
    """rank (0 = best) of the positive among [neg, pos] on the last axis."""
    pos = torch.as_tensor(pos).float()
    neg = torch.as_tensor(neg).float()
    return (neg >= pos).sum(-1).float()  # ties count against the positive (top_k order)


class MrrScore(Metric):
    def reset(self):
        self.sum, self.n = 0.0, 0

    def update(self, logits, negative_logits):
        r = _ranks(logits, negative_logits)
        self.sum += float((1.0 / (r + 1)).sum())
        self.n += r.numel()
        return self.sum / max(self.n, 1)


class HitKScore(Metric):
    def __init__(self, k):
        self.k = k
        super().__init__()

    def reset(self):
        self.hit, self.n = 0.0, 0

    def update(self, pos, neg):
        r = _ranks(pos, neg)
        self.hit += float((r < self.k).float().sum())
        self.n += r.numel()
        return self.hit / max(self.n, 1)


class MrScore(Metric):
    def reset(self):
        self.sum, self.n = 0.0, 0

    def update(self, pos, neg):
        r = _ranks(pos, neg)
        self.sum += float(r.sum())
        self.n += r.numel()
        return self.sum / max(self.n, 1)


metrics = {
    "acc": AccScore,
    "auc": AucScore,
    "f1": F1Score,
    "mrr": MrrScore,
    "hit1": lambda: HitKScore(1),
    "hit3": lambda: HitKScore(3),
    "hit10": lambda: HitKScore(10),
    "mr": MrScore,
}


def get(name):
    f = metrics.get(name)
    return f() if f is not None else None
