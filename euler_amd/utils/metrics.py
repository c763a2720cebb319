"""Streaming metrics (reference ``tf_euler/python/utils/metrics.py:23-98``).

TF's ``tf.metrics.*`` accumulate across ``session.run`` calls until the local
variables are reset; here every metric is an object with ``update(...) -> value``
(running value) and ``reset()``.  ``get(name)`` returns a *fresh* metric instance;
calling it like a function updates it.
"""
from __future__ import annotations

import torch

__all__ = ["Metric", "AccScore", "AucScore", "F1Score", "MrrScore", "HitKScore", "MrScore", "get", "metrics"]


class Metric:
    def __init__(self):
        self.reset()

    def reset(self):
        raise NotImplementedError

    def update(self, *args):
        raise NotImplementedError

    def __call__(self, *args):
        return self.update(*args)


class AccScore(Metric):
    """accuracy of floor(p + 0.5) against labels (predict = probabilities)."""

    def reset(self):
        self.correct, self.total = 0.0, 0.0

    def update(self, labels, predict):
        labels = torch.as_tensor(labels).float()
        pred = torch.floor(torch.as_tensor(predict).float() + 0.5)
        self.correct += float((pred == labels).float().sum())
        self.total += float(labels.numel())
        return self.correct / max(self.total, 1.0)


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
        self.tp = self.fp = self.fn = 0.0

    def update(self, labels, predict):
        y = torch.as_tensor(labels).float()
        p = torch.floor(torch.as_tensor(predict).float() + 0.5)
        self.tp += float((p * y).sum())
        self.fp += float((p * (1 - y)).sum())
        self.fn += float(((1 - p) * y).sum())
        eps = 1e-7
        prec = self.tp / (eps + self.tp + self.fp)
        rec = self.tp / (eps + self.tp + self.fn)
        return 2.0 * prec * rec / (prec + rec + eps)


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
