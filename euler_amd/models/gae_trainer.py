"""Device-path training of the graph auto-encoder (``GraphAutoEncoder`` with a ``sage`` or
``gcn`` node encoder) under ``GaeEstimator(device_graph=True)``.

Reference: ``euler_estimator/python/gae_estimator.py:26-51`` (roots from ``sample_node``),
``tf_euler/python/mp_utils/base_gae.py:23-70`` (``num_negs`` positives from
``sample_neighbor`` and ``num_negs`` negatives from ``sample_node`` per root, dot-product
decoder, sigmoid cross-entropy over all of them, accuracy of the thresholded
probabilities).

One step on the device: the roots, their positives and negatives drawn from the HBM graph
(alias tables, Philox streams 1 / 4 / 5), the encoder's blocks for all
``B (1 + 2 num_negs)`` nodes built in fixed shapes (:class:`DeviceSageFlow` /
:class:`DeviceFullFlow`), the user's own convolutions and ``fc``, the decoder and the loss,
backward and one flat optimizer launch; several steps per hipGraph replay
(:class:`~euler_amd.models.captured.CapturedTrainer`).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from euler_amd.dataflow.device_flow import DeviceFullFlow, DeviceSageFlow
from euler_amd.models.captured import CapturedTrainer
from euler_amd.ops import mp_ops

__all__ = ["GaeTrainer", "VgaeTrainer"]


def _type_ids(edge_type):
    import euler_amd.ops.graph_api as ge

    if edge_type is None:
        return None
    ids = [int(t) for t in np.asarray(ge.get_edge_type_id(edge_type)).reshape(-1)]
    return None if any(t < 0 for t in ids) else ids


class GaeTrainer(CapturedTrainer):
    metric_name = "acc"

    def __init__(self, model, graph, batch_size, optimizer="adam", learning_rate=0.01):
        from euler_amd.dataflow.dataflows import GCNDataFlow, SageDataFlow

        gnn = getattr(model, "gnn", None)
        flow = getattr(gnn, "sampler", None)
        if gnn is None or not isinstance(flow, (SageDataFlow, GCNDataFlow)):
            raise ValueError("GaeTrainer trains GraphAutoEncoder with a sage or gcn node encoder")
        if graph.features is None:
            raise ValueError("the device graph needs the encoder's dense features (DeviceGraph.from_engine)")
        self.gnn = gnn
        self.graph = graph
        self.B = int(batch_size)
        self.K = int(model.num_negs)
        self.pos_types = _type_ids(model.edge_type)
        n = self.B * (1 + 2 * self.K)
        ets = [_type_ids(m) for m in flow.metapath]
        if isinstance(flow, SageDataFlow):
            self.flow = DeviceSageFlow(graph, ets, flow.fanouts, n, bool(flow.add_self_loops))
        else:
            self.flow = DeviceFullFlow(graph, [graph._mask(e) for e in ets], n, bool(flow.add_self_loops))
        self.features = graph.features
        self.acc = torch.zeros(2, dtype=torch.float64, device=graph.device)  # correct, total
        super().__init__(model, graph, graph.device, optimizer, learning_rate)

    def _embed(self, rows):
        """encoder output [n, dim] of node rows through the user's convolutions and fc"""
        df = self.flow.produce(rows)
        x = mp_ops.gather(self.features, df[0].n_id).float()
        for conv, block in zip(self.gnn.convs, df):
            x_t = mp_ops.gather(x, block.res_n_id)
            x = F.relu(self.gnn.calculate_conv(conv, (x_t, x), block.edge_index, size=block.size))
        return self.gnn.fc(x)

    def _forward_loss(self):
        self._draw()
        g = self.graph
        B, K = self.B, self.K
        src = g.sample_node(B, stream_id=1).long()
        pos = g.sample_neighbor(src, K, edge_types=self.pos_types, default=-1, stream_id=4).long().reshape(-1)
        neg = g.sample_node(B * K, stream_id=5).long()
        emb = self._embed(torch.cat([src, pos, neg]))
        d = emb.shape[-1]
        e_src = emb[:B].view(B, 1, d)
        e_pos = emb[B:B + B * K].view(B, K, d)
        e_neg = emb[B + B * K:].view(B, K, d)
        logits = torch.matmul(e_src, e_pos.transpose(1, 2)).float()
        neg_logits = torch.matmul(e_src, e_neg.transpose(1, 2)).float()
        t = F.binary_cross_entropy_with_logits(logits, torch.ones_like(logits), reduction="none")
        n = F.binary_cross_entropy_with_logits(neg_logits, torch.zeros_like(neg_logits), reduction="none")
        loss = torch.cat([t.reshape(-1), n.reshape(-1)]).mean()
        with torch.no_grad():
            right = (logits >= 0).sum() + (neg_logits < 0).sum()
            self.acc += torch.stack([right.double(), torch.full_like(right.double(), float(2 * B * K))])
        self._samples = (src, pos, neg)
        return loss

    def metric(self) -> float:
        c, n = self.acc.tolist()
        return c / max(n, 1.0)

    def reset_metric(self):
        self.acc.zero_()


class VgaeTrainer(GaeTrainer):
    """``VariationalGraphAutoEncoder`` on the device path (reference examples/gae/gae.py:94-153,
    this repo's ``models/unsupervised.py`` VariationalGraphAutoEncoder): the encoder gives
    mu, the model's id table ``log_var_encoder`` gives log sigma^2 of every node (graph row ->
    node id through ``graph.ids``; a ``-1`` sample is the model's out-of-range row, as on the
    engine path), the decoder reads ``mu + radius * eps * exp(log_var / 2)``, and the loss
    adds the mean KL over every root, positive and negative.  ``eps`` comes from torch's
    CUDA generator, which hipGraph replays advance like eager steps (the sampler's draws
    stay on the graph's Philox counter)."""

    def __init__(self, model, graph, batch_size, optimizer="adam", learning_rate=0.01):
        ids = graph.ids if graph.ids is not None else np.arange(graph.num_rows)
        self._ids = torch.as_tensor(np.asarray(ids).astype(np.int64), device=graph.device)
        self._pad_id = int(model.max_id) + 1
        self.radius = float(model.radius)
        super().__init__(model, graph, batch_size, optimizer, learning_rate)

    def _forward_loss(self):
        self._draw()
        g = self.graph
        B, K = self.B, self.K
        src = g.sample_node(B, stream_id=1).long()
        pos = g.sample_neighbor(src, K, edge_types=self.pos_types, default=-1, stream_id=4).long().reshape(-1)
        neg = g.sample_node(B * K, stream_id=5).long()
        rows = torch.cat([src, pos, neg])
        mu = self._embed(rows)
        node_ids = torch.where(rows >= 0, self._ids[rows.clamp(min=0)], torch.full_like(rows, self._pad_id))
        log_var = self.model.log_var_encoder(node_ids).reshape(mu.shape).to(mu.dtype)
        emb = mu + self.radius * torch.randn_like(log_var) * torch.exp(0.5 * log_var)
        d = emb.shape[-1]
        e_src = emb[:B].view(B, 1, d)
        e_pos = emb[B:B + B * K].view(B, K, d)
        e_neg = emb[B + B * K:].view(B, K, d)
        logits = torch.matmul(e_src, e_pos.transpose(1, 2)).float()
        neg_logits = torch.matmul(e_src, e_neg.transpose(1, 2)).float()
        t = F.binary_cross_entropy_with_logits(logits, torch.ones_like(logits), reduction="none")
        n = F.binary_cross_entropy_with_logits(neg_logits, torch.zeros_like(neg_logits), reduction="none")
        loss = torch.cat([t.reshape(-1), n.reshape(-1)]).mean()
        loss = loss + self.model.kl(mu, log_var).float().mean()
        with torch.no_grad():
            right = (logits >= 0).sum() + (neg_logits < 0).sum()
            self.acc += torch.stack([right.double(), torch.full_like(right.double(), float(2 * B * K))])
        self._samples = (src, pos, neg)
        return loss
