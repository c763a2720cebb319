"""Composable model templates (reference ``tf_euler/python/solution/*.py``).

Solutions are ``nn.Module``s so the encoders / logit layers they wrap register their
parameters; each returns ``(embedding, loss, metric_name, metric_value)`` like the
reference.  Metrics are streaming objects from :mod:`euler_amd.utils.metrics`.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

import euler_amd.ops.graph_api as ge
from euler_amd.utils import metrics as M
from euler_amd.utils.layers import Dense

__all__ = ["SuperviseSolution", "UnsuperviseSolution", "SuperviseSampleSolution", "UnsuperviseSampleSolution",
           "SampleNegWithTypes", "SamplePosWithTypes", "DenseLogits", "PosNegLogits", "CosineLogits",
           "sigmoid_loss", "xent_loss", "GetLabelFromFea"]


# ----------------------------------------------------------------------------- losses (losses.py:22-33)
def sigmoid_loss(labels, logits):
    return F.binary_cross_entropy_with_logits(logits.float(), labels.to(logits.device).float())


def xent_loss(logits, neg_logits):
    """mean over the concatenation of positive (label 1) and negative (label 0) BCE terms."""
    t = F.binary_cross_entropy_with_logits(logits.float(), torch.ones_like(logits, dtype=torch.float32),
                                           reduction="sum")
    n = F.binary_cross_entropy_with_logits(neg_logits.float(), torch.zeros_like(neg_logits, dtype=torch.float32),
                                           reduction="sum")
    return (t + n) / float(logits.numel() + neg_logits.numel())


# ----------------------------------------------------------------------------- logits (logits.py:23-42)
class DenseLogits(nn.Module):
    def __init__(self, logits_dim):
        super().__init__()
        self.out_fc = Dense(logits_dim, use_bias=False)

    def forward(self, inputs, **kwargs):
        return self.out_fc(inputs)


class PosNegLogits(nn.Module):
    def forward(self, emb, pos_emb, neg_emb):
        return torch.matmul(emb, pos_emb.transpose(-1, -2)), torch.matmul(emb, neg_emb.transpose(-1, -2))


class CosineLogits(nn.Module):
    def forward(self, target_emb, context_emb):
        x = F.normalize(target_emb, dim=-1)
        y = F.normalize(context_emb, dim=-1)
        return (x * y).sum(-1, keepdim=True) * 5.0


# ----------------------------------------------------------------------------- samplers (samplers.py:23-50)
class SampleNegWithTypes:
    def __init__(self, neg_type, num_negs=5):
        self.neg_type = neg_type if isinstance(neg_type, list) else [neg_type]
        self.num_negs = num_negs

    def __call__(self, inputs):
        b = torch.as_tensor(inputs).reshape(-1).numel()
        groups = [ge.sample_node(b * self.num_negs, t).reshape(b, self.num_negs) for t in self.neg_type]
        return groups[0] if len(groups) == 1 else groups


class SamplePosWithTypes:
    def __init__(self, edge_type, num_pos=1, max_id=-1):
        self.edge_type, self.num_pos, self.max_id = edge_type, num_pos, max_id

    def __call__(self, inputs):
        return ge.sample_neighbor(inputs, self.edge_type, self.num_pos, self.max_id + 1)[0]


class GetLabelFromFea:
    """dense feature ``label_idx`` as the label (utils.py:23-32)."""

    def __init__(self, label_idx, label_dim):
        self.label_idx, self.label_dim = label_idx, label_dim

    def __call__(self, inputs):
        return ge.get_dense_feature(torch.as_tensor(inputs).reshape(-1), [self.label_idx], [self.label_dim])[0]


def _as_module(fn):
    return fn if isinstance(fn, nn.Module) else None


class _FnHolder(nn.Module):
    """Register callables that are modules so their parameters are trained."""

    def _hold(self, name, fn):
        if isinstance(fn, nn.Module):
            self.add_module(name, fn)
        else:
            object.__setattr__(self, name, fn)


# ----------------------------------------------------------------------------- solutions
class SuperviseSolution(_FnHolder):
    """label -> encoder -> logits -> loss + metric (base_supervise.py:26-50)."""

    def __init__(self, get_label_fn, encoder_fn, logit_fn, metric_name="f1", loss_fn=sigmoid_loss):
        super().__init__()
        self.get_label_fn = get_label_fn
        self.metric_name = metric_name
        self.metric = M.get(metric_name)
        self._hold("encoder", encoder_fn)
        self._hold("logit_fn", logit_fn)
        self.loss_fn = loss_fn

    def embed(self, n_id):
        return self.encoder(n_id)

    def forward(self, inputs):
        label = self.get_label_fn(inputs)
        embedding = self.embed(inputs)
        logit = self.logit_fn(embedding)
        label = label.to(logit.device)
        loss = self.loss_fn(label, logit)
        metric = self.metric(label.detach().cpu(), torch.sigmoid(logit.float()).detach().cpu())
        return embedding, loss, self.metric_name, metric


class UnsuperviseSolution(_FnHolder):
    """target/context encoders + positive/negative samplers (base_unsupervise.py:27-73)."""

    def __init__(self, target_encoder_fn, context_encoder_fn, pos_sample_fn, neg_sample_fn, metric_name="mrr",
                 logit_fn=None, loss_fn=xent_loss):
        super().__init__()
        self.metric_name = metric_name
        self.metric = M.get(metric_name)
        self._hold("target_encoder", target_encoder_fn)
        self._hold("context_encoder", context_encoder_fn)
        self.pos_sample_fn, self.neg_sample_fn = pos_sample_fn, neg_sample_fn
        self._hold("logit_fn", logit_fn if logit_fn is not None else PosNegLogits())
        self.loss_fn = loss_fn

    @staticmethod
    def _embed3(encoder, n_id):
        n_id = torch.as_tensor(n_id)
        b = n_id.shape[0]
        emb = encoder(n_id.reshape(-1))
        return emb.reshape(b, -1, emb.shape[-1])

    def target_embed(self, n_id):
        return self._embed3(self.target_encoder, n_id)

    def context_embed(self, n_id):
        return self._embed3(self.context_encoder, n_id)

    def to_sample(self, inputs):
        inputs = torch.as_tensor(inputs).reshape(-1)
        pos, negs = self.pos_sample_fn(inputs), self.neg_sample_fn(inputs)
        assert pos.dim() == 2 and negs.dim() == 2
        return inputs.unsqueeze(-1), pos, negs

    def forward(self, inputs):
        src, pos, negs = self.to_sample(inputs)
        emb = self.target_embed(src)
        logits, neg_logits = self.logit_fn(emb, self.context_embed(pos), self.context_embed(negs))
        loss = self.loss_fn(logits, neg_logits)
        metric = self.metric(logits.detach().float().cpu(), neg_logits.detach().float().cpu())
        embedding = self.target_embed(torch.as_tensor(inputs).reshape(-1))
        return embedding, loss, self.metric_name, metric


class SuperviseSampleSolution(_FnHolder):
    """Supervised on explicit sample rows ``(label, node groups...)`` (base_sample.py:29-80).

    When ``neg_sample_fn`` is given, negatives are appended per node group with label 0
    (the reference concatenated the whole group lists instead of each pos/neg pair —
    SURVEY §2.10; fixed here).
    """

    def __init__(self, parse_input_fn, encoder_fn, parse_group_emb_fn, logit_fn=None, metric_name="auc",
                 neg_sample_fn=None, loss_fn=sigmoid_loss):
        super().__init__()
        self.metric_name = metric_name
        self.metric = M.get(metric_name)
        self.parse_input_fn, self.parse_group_emb_fn = parse_input_fn, parse_group_emb_fn
        self._hold("encoder", encoder_fn)
        self.neg_sample_fn = neg_sample_fn
        self._hold("logit_fn", logit_fn if logit_fn is not None else CosineLogits())
        self.loss_fn = loss_fn

    def embed(self, n_id):
        return self.encoder(n_id)

    def forward(self, inputs):
        parsed = self.parse_input_fn(inputs)
        label = torch.as_tensor(parsed[0]).float()
        groups = parsed[1] if len(parsed) == 2 else list(parsed[1:])
        if self.neg_sample_fn is not None:
            negs = self.neg_sample_fn(groups)
            label = torch.cat([label, torch.zeros(torch.as_tensor(negs[0]).shape[0], *label.shape[1:])], 0)
            groups = [torch.cat([torch.as_tensor(p), torch.as_tensor(n)], 0) for p, n in zip(groups, negs)]
        group_emb = self.embed(groups)
        target, context, output = self.parse_group_emb_fn(group_emb)
        logit = self.logit_fn(target, context_emb=context)
        label = label.to(logit.device).reshape(logit.shape)
        loss = self.loss_fn(label, logit)
        metric = self.metric(label.detach().cpu(), logit.detach().float().cpu())
        return output, loss, self.metric_name, metric


class UnsuperviseSampleSolution(_FnHolder):
    """Unsupervised on explicit sample rows ``(src, [neg], [pos])`` (base_sample.py:83-136)."""

    def __init__(self, parse_input_fn, target_encoder_fn, context_encoder_fn, pos_sample_fn, neg_sample_fn,
                 logit_fn=None, metric_name="auc", metric_fn=None, loss_fn=xent_loss):
        super().__init__()
        self.parse_input_fn = parse_input_fn
        self.metric_name = metric_name
        self.metric = metric_fn if metric_fn is not None else M.get(metric_name)
        self._hold("target_encoder", target_encoder_fn)
        self._hold("context_encoder", context_encoder_fn)
        self.pos_sample_fn, self.neg_sample_fn = pos_sample_fn, neg_sample_fn
        self._hold("logit_fn", logit_fn if logit_fn is not None else PosNegLogits())
        self.loss_fn = loss_fn

    def target_embed(self, n_id):
        return self.target_encoder(n_id)

    def context_embed(self, n_id):
        return self.context_encoder(n_id)

    def to_sample(self, inputs):
        parsed = self.parse_input_fn(inputs)
        neg, pos = [], []
        if len(parsed) == 2 and parsed[1] is not None:
            neg.append(torch.as_tensor(parsed[1]))
        if len(parsed) == 3:
            pos.append(torch.as_tensor(parsed[2]))
        if self.pos_sample_fn is not None:
            src, p = self.pos_sample_fn(parsed[0])
            pos.append(torch.as_tensor(p))
        else:
            src = parsed[0]
        if self.neg_sample_fn is not None:
            neg.append(torch.as_tensor(self.neg_sample_fn(parsed[0])))
        return src, torch.cat(pos, -1), torch.cat(neg, -1)

    def forward(self, inputs):
        src, pos, negs = self.to_sample(inputs)
        emb = self.target_embed(src)
        logits, neg_logits = self.logit_fn(emb, self.context_embed(pos), self.context_embed(negs))
        loss = self.loss_fn(logits, neg_logits)
        metric = self.metric(logits.detach().float().cpu(), neg_logits.detach().float().cpu())
        return emb, loss, self.metric_name, metric
