"""Device-path training of Deep Graph Infomax (``models/unsupervised.py`` DGI) under
``NodeEstimator(device_graph=True)``.

Reference: ``examples/dgi/dgi.py:24-90`` (a ``ShuffleSageEncoder`` gives the real and the
corrupted embedding of every root, a bilinear discriminator scores both against the
sigmoid of the batch-mean readout, sigmoid cross-entropy), ``tf_euler/python/utils/
encoders.py:496-541`` (the corrupted view permutes the per-root positions of the whole
sample tree, one permutation shared by every root).

One step on the device: the roots and the fan-out tree drawn from the HBM graph (alias
tables, one Philox stream per hop), the dense features gathered once, the user's own
aggregators run on the real and the shuffled tree, the discriminator and the loss,
backward and one flat optimizer launch; several steps per hipGraph replay
(:class:`~euler_amd.models.captured.CapturedTrainer`).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from euler_amd.models.captured import CapturedTrainer
from euler_amd.models.gae_trainer import _type_ids
from euler_amd.ops import mp_ops

__all__ = ["DgiTrainer"]


class DgiTrainer(CapturedTrainer):
    metric_name = "acc"

    def __init__(self, model, graph, batch_size, optimizer="adam", learning_rate=0.01):
        from euler_amd.utils.encoders import ShuffleSageEncoder

        enc = getattr(model, "_target_encoder", None)
        ne = getattr(enc, "_node_encoder", None)
        if not isinstance(enc, ShuffleSageEncoder) or ne is None or ne.use_id or ne.use_sparse_feature or \
                not ne.use_feature:
            raise ValueError("DgiTrainer trains DGI over dense node features (no id / sparse-feature embeddings)")
        if graph.features is None:
            raise ValueError("the device graph needs the encoder's dense features (DeviceGraph.from_engine)")
        self.enc, self.graph = enc, graph
        self.B = int(batch_size)
        self.types = [_type_ids(m) for m in enc.metapath]
        self.fanouts = [int(f) for f in enc.fanouts]
        self.features = graph.features
        self.acc = torch.zeros(2, dtype=torch.float64, device=graph.device)  # correct, total
        super().__init__(model, graph, graph.device, optimizer, learning_rate)

    def _tree(self, roots):
        """node rows of every hop: [B], [B f0], [B f0 f1], ... (-1: no neighbour)"""
        hops = [roots]
        for i, (f, et) in enumerate(zip(self.fanouts, self.types)):
            hops.append(self.graph.sample_neighbor(hops[-1], f, edge_types=et, default=-1,
                                                   stream_id=4 + i).long().reshape(-1))
        return hops

    def _features(self, rows):
        x = mp_ops.gather(self.features, rows.clamp(min=0)).float()
        return x * (rows >= 0).unsqueeze(1).to(x.dtype)  # the reference's default node: zeros

    def _shuffle(self, hidden):
        """ShuffleSageEncoder.shuffle_tensors with the permutation drawn as an argsort of
        uniforms (capturable)"""
        b, d = hidden[0].shape[0], hidden[0].shape[-1]
        sizes = [h.shape[0] for h in hidden]
        cat = torch.cat([h.reshape(b, -1, d) for h in hidden], 1)
        perm = torch.rand(cat.shape[1], device=cat.device).argsort()
        cat = cat[:, perm].reshape(-1, d)
        return list(torch.split(cat, sizes))

    def _materialize(self):
        if not any(isinstance(p, torch.nn.parameter.UninitializedParameter) for p in self.model.parameters()):
            return
        state = self.graph.rng.clone()
        with torch.no_grad():
            self._logits(torch.zeros(self.B, dtype=torch.long, device=self.features.device))
        self.graph.rng.copy_(state)

    def _logits(self, roots):
        hidden = [self._features(h) for h in self._tree(roots)]
        emb = self.enc._aggregate(hidden)                    # [B, dim]
        emb_neg = self.enc._aggregate(self._shuffle(hidden))
        read = torch.sigmoid(emb.mean(0, keepdim=True))     # DGI.readout_func
        k = self.model.kernel
        return (k(emb) * read).sum(-1).float(), (k(emb_neg) * read).sum(-1).float()

    def _forward_loss(self):
        self._draw()
        roots = self.graph.sample_node(self.B, stream_id=1).long()
        logits, neg_logits = self._logits(roots)
        t = F.binary_cross_entropy_with_logits(logits, torch.ones_like(logits), reduction="sum")
        n = F.binary_cross_entropy_with_logits(neg_logits, torch.zeros_like(neg_logits), reduction="sum")
        loss = (t + n) / float(2 * self.B)
        with torch.no_grad():
            right = (logits >= 0).sum() + (neg_logits < 0).sum()
            self.acc += torch.stack([right.double(), torch.full_like(right.double(), float(2 * self.B))])
        self._samples = (roots,)
        return loss

    def metric(self) -> float:
        c, n = self.acc.tolist()
        return c / max(n, 1.0)

    def reset_metric(self):
        self.acc.zero_()
