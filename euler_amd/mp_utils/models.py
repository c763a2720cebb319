"""GNN model skeletons (reference ``tf_euler/python/mp_utils/*.py``).

Every model keeps the reference's call contract::

    embedding, loss, metric_name, metric_value = model(inputs)

and is an ``nn.Module``.  Graph sampling / feature fetch run through the engine
(CPU or remote shards) and the resulting ids / features are moved to the model's
device; all message passing then runs on the GPU kernels.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

import euler_amd.ops.graph_api as ge
from euler_amd.convolution import convs as C
from euler_amd.dataflow import dataflows as D
from euler_amd.graph_pool.pools import Pooling
from euler_amd.ops import gnn_ops, mp_ops
from euler_amd.utils import metrics as M
from euler_amd.utils.layers import Dense

__all__ = ["conv_classes", "flow_classes", "get_conv_class", "get_flow_class", "BaseGNNNet", "JKGNNNet",
           "GraphGNNNet", "GroupGNNNet", "SharedGroupGNNNet", "SingleGNNNet", "SharedGNNNet", "SuperviseModel",
           "UnsuperviseModel", "BaseGraphAutoEncoder", "GraphModel", "model_device"]

conv_classes = {
    "sage": C.SAGEConv, "gcn": C.GCNConv, "gat": C.GATConv, "tag": C.TAGConv, "agnn": C.AGNNConv,
    "sgcn": C.SGCNConv, "graphgcn": C.GraphConv, "appnp": C.APPNPConv, "arma": C.ARMAConv, "dna": C.DNAConv,
    "gin": C.GINConv, "gated": C.GatedConv, "relation": C.RelationConv,
}


class WrappedGCNDataFlow(D.GCNDataFlow):
    def __init__(self, fanouts, metapath, add_self_loops=True, **kwargs):
        super().__init__(metapath, add_self_loops=add_self_loops, **kwargs)


class WrappedWholeDataFlow(D.WholeDataFlow):
    def __init__(self, fanouts, metapath, add_self_loops=True, **kwargs):
        super().__init__(metapath, add_self_loops=add_self_loops, **kwargs)


flow_classes = {
    "full": WrappedGCNDataFlow, "sage": D.SageDataFlow, "fast": D.FastGCNDataFlow, "adapt": D.LayerwiseDataFlow,
    "layerwise": D.LayerwiseEachDataFlow, "whole": WrappedWholeDataFlow, "relation": D.RelationDataFlow,
}


def get_conv_class(conv):
    return conv_classes.get(conv) if isinstance(conv, str) else conv


def get_flow_class(flow):
    return flow_classes.get(flow) if isinstance(flow, str) else flow


def model_device(m: nn.Module):
    for p in m.parameters():  # lazy (uninitialized) parameters carry their device too
        return p.device
    for b in m.buffers():
        return b.device
    return getattr(m, "_euler_device", torch.device("cpu"))


class Prepared:
    """Host-side inputs of one step built ahead of the compute (sampling, feature and
    label fetch); moved to the GPU by :class:`~euler_amd.utils.prefetch.Prefetcher`."""

    __slots__ = ("fields",)

    def __init__(self, **fields):
        self.fields = fields

    def __getattr__(self, k):
        try:
            return object.__getattribute__(self, "fields")[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def _map(self, fn):
        return Prepared(**{k: (v if v is None or isinstance(v, (int, float, str)) else fn(v))
                           for k, v in self.fields.items()})

    def to(self, device, non_blocking=True):
        from euler_amd.utils.prefetch import to_device

        return self._map(lambda v: to_device(v, device, non_blocking))

    def pin_memory(self):
        from euler_amd.utils.prefetch import _pin

        return self._map(_pin)


class _GNNBase(nn.Module):
    def to_x(self, n_id):
        raise NotImplementedError

    def to_edge(self, n_id_src, n_id_dst, e_id):
        return e_id

    def get_edge_attr(self, block):
        ids = block.n_id
        src = ids[block.res_n_id][block.edge_index[0]]
        dst = ids[block.edge_index[1]]
        return self.to_edge(src, dst, block.e_id)

    def calculate_conv(self, conv, inputs, edge_index, size=None, edge_attr=None):
        return conv(inputs, edge_index, size=size, edge_attr=edge_attr)

    def _dev(self):
        return model_device(self)


class BaseGNNNet(_GNNBase):
    """conv stack over a sampled DataFlow (reference base_gnn.py:27-92)."""

    def __init__(self, conv, flow, dims, fanouts, metapath, add_self_loops=True, max_id=-1, **kwargs):
        super().__init__()
        conv_class = get_conv_class(conv)
        flow_class = get_flow_class(flow)
        self.whole_graph = flow_class is WrappedWholeDataFlow
        self.convs = nn.ModuleList([self.get_conv(conv_class, d) for d in dims[:-1]])
        self.fc = Dense(dims[-1])
        self.sampler = flow_class(fanouts, metapath, add_self_loops, max_id=max_id)

    def get_conv(self, conv_class, dim):
        return conv_class(dim)

    def sample_inputs(self, n_id):
        """Host part of :meth:`forward` (dataflow sampling + input features) for the
        asynchronous input pipeline."""
        data_flow = self.sampler(n_id)
        return Prepared(flow=data_flow, x=self.to_x(data_flow[0].n_id))

    def _inputs(self, n_id):
        if isinstance(n_id, Prepared):
            return n_id.flow, n_id.x
        dev = self._dev()
        data_flow = self.sampler(n_id).to(dev)
        return data_flow, self.to_x(data_flow[0].n_id).to(dev)

    def forward(self, n_id):
        data_flow, x = self._inputs(n_id)
        for conv, block in zip(self.convs, data_flow):
            if not self.whole_graph and block.e_id is None and getattr(conv, "can_fuse", None) and \
                    conv.can_fuse(x, block):
                x = conv.fused_relu(x, block)  # fixed-fanout block: fused K3 kernel on the GPU
                continue
            edge_attr = None if block.e_id is None else self.get_edge_attr(block)
            x_src = mp_ops.gather(x, block.res_n_id)
            x_dst = None if self.whole_graph else x
            x = F.relu(self.calculate_conv(conv, (x_src, x_dst), block.edge_index, size=block.size,
                                           edge_attr=edge_attr))
        return self.fc(x)


class JKGNNNet(BaseGNNNet):
    """Jumping-knowledge variant (reference base_gnn.py:94-139)."""

    def __init__(self, conv, flow, dims, fanouts, metapath, add_self_loops=True, jk_mode="concat", max_id=-1,
                 **kwargs):
        super().__init__(conv, flow, dims, fanouts, metapath, add_self_loops, max_id, **kwargs)
        assert jk_mode in ("concat", "maxpool")
        self.jk_mode = jk_mode

    def forward(self, n_id):
        data_flow, x = self._inputs(n_id)
        hidden = []
        for i, (conv, block) in enumerate(zip(self.convs, data_flow)):
            edge_attr = None if block.e_id is None else self.get_edge_attr(block)
            x_src = mp_ops.gather(x, block.res_n_id)
            x = F.relu(self.calculate_conv(conv, (x_src, None if self.whole_graph else x), block.edge_index,
                                           size=block.size, edge_attr=edge_attr))
            hidden.append(x)
            for j in range(i):
                hidden[j] = mp_ops.gather(hidden[j], block.res_n_id)
        x = torch.cat(hidden, 1) if self.jk_mode == "concat" else torch.stack(hidden, 1).sum(1)
        return self.fc(x)


class GraphGNNNet(_GNNBase):
    """Whole-graph convs + graph pooling with JK over layers (reference graph_gnn.py:28-116)."""

    def __init__(self, conv, dims, fanouts, metapath, node_pool=None, graph_pool=Pooling, add_self_loops=True,
                 jk_mode="concat"):
        super().__init__()
        conv_class = get_conv_class(conv)
        self.convs = nn.ModuleList([conv_class(d) for d in dims[:-1]])
        self.fc = Dense(dims[-1])
        self.sampler = WrappedWholeDataFlow(fanouts, [metapath[0]], add_self_loops)
        assert jk_mode in ("concat", "maxpool")
        self.jk_mode = jk_mode
        self.graph_pool = graph_pool("add") if isinstance(graph_pool, type) else graph_pool

    def forward(self, n_id, graph_index):
        dev = self._dev()
        df = self.sampler(n_id).to(dev)
        x = self.to_x(df[0].n_id).to(dev)
        block = df[0]
        graph_index = torch.as_tensor(graph_index, device=dev).long()
        size = int(graph_index.max().item()) + 1 if graph_index.numel() else 0
        hidden = []
        for conv in self.convs:
            edge_attr = None if block.e_id is None else self.get_edge_attr(block)
            x = F.relu(self.calculate_conv(conv, (x, None), block.edge_index, size=block.size, edge_attr=edge_attr))
            hidden.append(self.graph_pool(x, graph_index, size))
        out = torch.cat(hidden, 1) if self.jk_mode == "concat" else torch.stack(hidden, 1).sum(1)
        return self.fc(out)


class GroupGNNNet(nn.Module):
    def __init__(self, gnns):
        super().__init__()
        self.group_gnn = nn.ModuleList(gnns)

    def forward(self, group_n_id):
        return [g(n) for n, g in zip(group_n_id, self.group_gnn)]


class SharedGroupGNNNet(_GNNBase):
    """One conv stack shared by several (flow, fanouts, metapath) groups (reference group_gnn.py)."""

    def __init__(self, conv, group_flow, dims, group_fanouts, group_metapath, add_self_loops=True, **kwargs):
        super().__init__()
        if "whole" in group_flow:
            raise ValueError("Group GNN does not support whole dataflow")
        conv_class = get_conv_class(conv)
        self.convs = nn.ModuleList([conv_class(d) for d in dims[:-1]])
        self.fc = Dense(dims[-1])
        self.group_sampler = [get_flow_class(f)(fo, mp, add_self_loops)
                              for f, fo, mp in zip(group_flow, group_fanouts, group_metapath)]

    def forward(self, group_n_id):
        dev = self._dev()
        outs = []
        for sampler, n_id in zip(self.group_sampler, group_n_id):
            df = sampler(n_id).to(dev)
            x = self.to_x(df[0].n_id).to(dev)
            for conv, block in zip(self.convs, df):
                edge_attr = None if block.e_id is None else self.get_edge_attr(block)
                x = F.relu(self.calculate_conv(conv, (mp_ops.gather(x, block.res_n_id), x), block.edge_index,
                                               size=block.size, edge_attr=edge_attr))
            outs.append(self.fc(x))
        return outs


class SingleGNNNet(BaseGNNNet):
    def __init__(self, conv, flow, dims, fanouts, metapath, encoder, add_self_loops=False):
        super().__init__(conv, flow, dims, fanouts, metapath, add_self_loops)
        self.encoder = encoder

    def to_x(self, n_id):
        return self.encoder(n_id)


class SharedGNNNet(SharedGroupGNNNet):
    def __init__(self, conv, group_flow, dims, group_fanouts, group_metapath, add_self_loops=True, **kwargs):
        super().__init__(conv, group_flow, dims, group_fanouts, group_metapath, add_self_loops)
        from euler_amd.utils.encoders import ShallowEncoder

        self.encoder = ShallowEncoder(**kwargs)

    def to_x(self, n_id):
        return self.encoder(n_id)


# ----------------------------------------------------------------------------- model heads
class SuperviseModel(nn.Module):
    """label from a dense feature, sigmoid CE, streaming metric (reference mp_utils/base.py:24-47)."""

    def __init__(self, label_idx, label_dim, metric_name="f1"):
        super().__init__()
        self.label_idx = label_idx
        self.label_dim = label_dim
        self.metric_name = metric_name
        self.metric = M.get(metric_name)
        self.out_fc = Dense(label_dim, use_bias=False)

    def embed(self, n_id):
        raise NotImplementedError

    def get_label(self, inputs):
        return ge.get_dense_feature(inputs, [self.label_idx], [self.label_dim])[0]

    def prepare_embed(self, inputs):
        """host-side inputs of :meth:`embed` (override to move sampling off the step)"""
        return inputs

    def prepare(self, inputs):
        """Everything of one step that only needs the graph engine (labels, sampled
        dataflow, input features), for :class:`~euler_amd.utils.prefetch.Prefetcher`."""
        return Prepared(inputs=inputs, label=self.get_label(inputs), embed_in=self.prepare_embed(inputs))

    def forward(self, inputs):
        if isinstance(inputs, Prepared):
            label, embedding = inputs.label, self.embed(inputs.embed_in)
        else:
            label = self.get_label(inputs)
            embedding = self.embed(inputs)
        label = label.to(embedding.device)
        logit = self.out_fc(embedding).float()
        loss = F.binary_cross_entropy_with_logits(logit, label.float())
        # streaming metric on the device (no per-step host sync; read at log steps)
        metric = self.metric(label.detach(), torch.sigmoid(logit).detach())
        return embedding, loss, self.metric_name, metric


class UnsuperviseModel(nn.Module):
    """positive = 1 sampled neighbor, negatives = sample_node, sigmoid CE (reference mp_utils/base.py:50-91)."""

    def __init__(self, node_type, edge_type, max_id, num_negs=20, metric_name="mrr"):
        super().__init__()
        self.node_type, self.edge_type, self.max_id = node_type, edge_type, max_id
        self.num_negs = num_negs
        self.metric_name = metric_name
        self.metric = M.get(metric_name)

    def embed(self, n_id):
        raise NotImplementedError

    def embed_context(self, n_id):
        raise NotImplementedError

    def to_sample(self, inputs):
        inputs = torch.as_tensor(inputs).reshape(-1)
        b = inputs.numel()
        src = inputs.unsqueeze(-1)
        pos = ge.sample_neighbor(inputs, self.edge_type, 1, self.max_id + 1)[0]
        negs = ge.sample_node(b * self.num_negs, self.node_type).reshape(b, self.num_negs)
        return src, pos, negs

    def forward(self, inputs):
        src, pos, negs = self.to_sample(inputs)
        emb = self.embed(src)
        emb_pos = self.embed_context(pos)
        emb_neg = self.embed_context(negs)
        # one fused kernel for the dot products, both sigmoid-CEs and the mean (embed.hip K11)
        b = emb.shape[0]
        loss, logits, neg_logits = gnn_ops.sgns_loss(emb.reshape(b, -1), emb_pos, emb_neg)
        logits, neg_logits = logits.float().view(b, 1, -1), neg_logits.float().view(b, 1, -1)
        metric = self.metric(logits.cpu(), neg_logits.cpu())
        embedding = self.embed(torch.as_tensor(inputs).reshape(-1))
        return embedding, loss, self.metric_name, metric


class BaseGraphAutoEncoder(nn.Module):
    """GAE skeleton (reference base_gae.py:23-70): num_negs positives + num_negs negatives."""

    def __init__(self, node_type, edge_type, max_id, num_negs=20):
        super().__init__()
        self.node_type, self.edge_type, self.max_id, self.num_negs = node_type, edge_type, max_id, num_negs
        self.metric = M.AccScore()

    def embed(self, n_id):
        raise NotImplementedError

    def to_sample(self, inputs):
        inputs = torch.as_tensor(inputs).reshape(-1)
        b = inputs.numel()
        pos = ge.sample_neighbor(inputs, self.edge_type, self.num_negs, self.max_id + 1)[0]
        negs = ge.sample_node(b * self.num_negs, self.node_type).reshape(b, self.num_negs)
        return inputs.unsqueeze(-1), pos, negs

    def forward(self, inputs):
        src, pos, negs = self.to_sample(inputs)
        emb, emb_pos, emb_neg = self.embed(src), self.embed(pos), self.embed(negs)
        logits = torch.matmul(emb, emb_pos.transpose(1, 2)).float()
        neg_logits = torch.matmul(emb, emb_neg.transpose(1, 2)).float()
        t = F.binary_cross_entropy_with_logits(logits, torch.ones_like(logits), reduction="none")
        n = F.binary_cross_entropy_with_logits(neg_logits, torch.zeros_like(neg_logits), reduction="none")
        loss = torch.cat([t.reshape(-1), n.reshape(-1)]).mean()
        pred = torch.cat([torch.sigmoid(logits), torch.sigmoid(neg_logits)], 2).detach().cpu()
        lab = torch.cat([torch.ones_like(logits), torch.zeros_like(neg_logits)], 2).cpu()
        acc = self.metric(lab, pred)
        return self.embed(torch.as_tensor(inputs).reshape(-1)), loss, "acc", acc


class GraphModel(nn.Module):
    """Graph classification head (reference base_graph.py:24-47)."""

    def __init__(self, label_dim):
        super().__init__()
        self.out_fc = Dense(label_dim, use_bias=False)
        self.metric = M.AccScore()

    def embed(self, n_id, graph_index):
        raise NotImplementedError

    def forward(self, inputs, label=None, graph_index=None):
        if isinstance(inputs, dict):
            label = inputs["graph_label"]
            graph_index = inputs["node_graph_idx"]
            inputs = inputs["node_idx"]
        assert label is not None or graph_index is not None
        embedding = self.embed(inputs, graph_index)
        logit = self.out_fc(embedding).float()
        label = torch.as_tensor(label, device=logit.device).float()
        loss = F.binary_cross_entropy_with_logits(logit, label)
        acc = self.metric(label.cpu(), torch.sigmoid(logit).detach().cpu())
        return embedding, loss, "accuracy", acc
