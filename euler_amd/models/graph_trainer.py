"""Device-path training of the graph-classification models (GIN, GraphGCN, GatedGraph,
Set2Set: ``models/graph_classification.py``) under ``GraphEstimator(device_graph=True)``.

Reference: ``euler_estimator/python/graph_estimator.py:27-85`` (``sample_graph_label`` ->
``get_graph_by_label`` -> node lists, the graph's label = the one-hot of its first node's
label feature), ``tf_euler/python/mp_utils/base_graph.py:24-47`` (node embeddings of the
induced full-neighbourhood subgraph, graph pooling, ``out_fc``, sigmoid cross-entropy).

Everything a step reads lives in HBM from the start: the graphs' node lists as one padded
``[G, max_nodes]`` row matrix, their one-hot labels, each node's sparse feature ids as a
padded ``[N, max_features]`` matrix.  A step draws B graphs (Philox, uniform, the device
graph's counter), lays their nodes out in ``B * max_nodes`` fixed slots (``-1`` padding),
builds the blocks with :class:`~euler_amd.dataflow.device_flow.DeviceFullFlow`, sums the
feature embeddings (the model's own ``SparseEmbedding`` table), runs the user's
convolutions and pooling (padding rows carry graph index ``-1``, which every segment op
drops) and the loss; several steps are captured per hipGraph
(:class:`~euler_amd.models.captured.CapturedTrainer`).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from euler_amd.dataflow.device_flow import DeviceFullFlow
from euler_amd.graph.device_graph import build_alias_table
from euler_amd.models.captured import CapturedTrainer
from euler_amd.ops import mp_ops
from euler_amd.ops._native import hip, use_hip

__all__ = ["GraphTrainer"]


class GraphTrainer(CapturedTrainer):
    metric_name = "accuracy"

    def __init__(self, model, graph, batch_size, label_feature, num_classes, optimizer="adam", learning_rate=0.01):
        import euler_amd.ops.graph_api as ge
        from euler_amd.dataflow.dataflows import GCNDataFlow
        from euler_amd.utils.layers import SparseEmbedding

        gnn = getattr(model, "gnn", None)
        enc = getattr(gnn, "encoder", None)
        if gnn is None or not isinstance(getattr(gnn, "sampler", None), GCNDataFlow) or \
                type(enc) is not SparseEmbedding or not hasattr(model, "pool"):
            raise ValueError("GraphTrainer trains the pooled graph-classification models (full flow, sparse-feature "
                             "embedding)")
        self.gnn, self.graph = gnn, graph
        self.B = int(batch_size)
        dev = graph.device
        meta = ge.get_engine().meta()
        labels = list(meta.get("graph_labels", []))
        if not labels:
            raise ValueError("the graph has no graph labels (get_graph_by_label)")
        sg = ge.get_graph_by_label(labels)
        ind = np.asarray(sg.indices).reshape(-1, 2)
        vals = np.asarray(sg.values).reshape(-1).astype(np.int64)
        G = len(labels)
        counts = np.bincount(ind[:, 0], minlength=G) if ind.size else np.zeros(G, np.int64)
        self.max_nodes = int(max(1, counts.max()))
        rows = graph.rows_of(vals).cpu().numpy().astype(np.int64)
        gmat = np.full((G, self.max_nodes), -1, np.int64)
        gmat[ind[:, 0], ind[:, 1]] = rows
        self.gnodes = torch.from_numpy(gmat).to(dev)
        # label of a graph: one-hot of its first node's label feature (graph_estimator.py:58-64)
        first = vals[np.searchsorted(ind[:, 0], np.arange(G))] if G else vals[:0]
        lab = np.asarray(ge.get_dense_feature(first, [label_feature], [1])[0]).reshape(-1).astype(np.int64)
        self.onehot = F.one_hot(torch.from_numpy(lab), int(num_classes)).float().to(dev)
        # sparse feature ids of every node row of the device graph, padded with -1
        sp = ge.get_sparse_feature(np.asarray(graph.ids, np.int64), gnn.feature_idx)[0]
        sidx = np.asarray(sp.indices).reshape(-1, 2)
        sval = enc._rows(torch.as_tensor(np.asarray(sp.values).astype(np.int64))).cpu().numpy()
        nf = np.bincount(sidx[:, 0], minlength=graph.num_rows) if sidx.size else np.zeros(graph.num_rows, np.int64)
        self.max_feats = int(max(1, nf.max()))
        fmat = np.full((graph.num_rows, self.max_feats), -1, np.int64)
        fmat[sidx[:, 0], sidx[:, 1]] = sval
        self.feat_ids = torch.from_numpy(fmat).to(dev)
        self.feat_n = torch.from_numpy(np.maximum(nf, 1).astype(np.float32)).to(dev).view(-1, 1)
        prob, alias = build_alias_table(np.ones(G))
        self.g_prob, self.g_alias = torch.from_numpy(prob).to(dev), torch.from_numpy(alias).to(dev)
        slot = torch.arange(self.B, device=dev).repeat_interleave(self.max_nodes)
        self.slot_graph = slot
        masks = []
        flow = gnn.sampler
        for mp in flow.metapath:
            ids = None if mp is None else [int(t) for t in np.asarray(ge.get_edge_type_id(mp)).reshape(-1)]
            masks.append(graph._mask(None if ids is None or any(t < 0 for t in ids) else ids))
        self.flow = DeviceFullFlow(graph, masks, self.B * self.max_nodes, bool(flow.add_self_loops))
        self.right = torch.zeros(2, dtype=torch.float64, device=dev)  # correct, total
        self._gidx = None
        super().__init__(model, graph, dev, optimizer, learning_rate)

    # ------------------------------------------------------------------ batch
    def sample_graphs(self) -> torch.Tensor:
        """B graph indices, uniform (reference sample_graph_label), stream 3 of the graph's
        Philox counter"""
        g = self.graph
        if use_hip(self.g_prob):
            return hip().alias_sample(self.g_prob, self.g_alias, None, self.B, g.rng, 3).long()
        n = self.g_prob.numel()
        k = torch.randint(0, n, (self.B,), generator=g._cpu_gen)
        u = torch.rand(self.B, generator=g._cpu_gen)
        return torch.where(u < self.g_prob[k], k, self.g_alias[k].long())

    def _embed_rows(self, rows):
        """SparseEmbedding (sum / mean) of the feature ids of node rows (-1: a zero row)"""
        enc = self.gnn.encoder
        r = rows.clamp(min=0)
        ids = torch.where((rows >= 0).view(-1, 1), self.feat_ids[r], torch.full_like(self.feat_ids[r], -1))
        e = mp_ops.gather(enc.weight, ids.reshape(-1)).view(rows.numel(), self.max_feats, -1).sum(1)
        if enc.combiner == "mean":
            e = e / self.feat_n[r]
        return e

    def _forward(self, gidx):
        roots = self.gnodes[gidx].reshape(-1)
        graph_of = torch.where(roots >= 0, self.slot_graph, torch.full_like(self.slot_graph, -1))
        df = self.flow.produce(roots)
        x = self._embed_rows(df[0].n_id)
        for conv, block in zip(self.gnn.convs, df):
            x_t = mp_ops.gather(x, block.res_n_id)
            x = F.relu(self.gnn.calculate_conv(conv, (x_t, x), block.edge_index, size=block.size))
        node_emb = self.gnn.fc(x)
        pooled = self.model.pool(node_emb, graph_of, self.B)
        return self.model.out_fc(pooled).float()

    def _materialize(self):
        if not any(isinstance(p, torch.nn.parameter.UninitializedParameter) for p in self.model.parameters()):
            return
        state = self.graph.rng.clone()
        with torch.no_grad():
            self._forward(torch.zeros(self.B, dtype=torch.long, device=self.gnodes.device))
        self.graph.rng.copy_(state)

    def _forward_loss(self):
        self._draw()
        gidx = self.sample_graphs()
        logits = self._forward(gidx)
        y = self.onehot[gidx]
        loss = F.binary_cross_entropy_with_logits(logits, y)
        with torch.no_grad():
            # accuracy of the arg-max class (reference metrics.acc_score on one-hot labels)
            ok = (logits.argmax(-1) == y.argmax(-1)).sum().double()
            self.right += torch.stack([ok, torch.full_like(ok, float(self.B))])
        self._gidx = gidx
        return loss

    def samples(self):
        return (self._gidx,)

    def metric(self) -> float:
        c, n = self.right.tolist()
        return c / max(n, 1.0)

    def reset_metric(self):
        self.right.zero_()

    # ------------------------------------------------------------------ oracle
    def graph_labels_of(self, gidx):
        """the engine-path labels (strings) of graph indices, for the estimator oracle"""
        import euler_amd.ops.graph_api as ge

        labels = list(ge.get_engine().meta().get("graph_labels", []))
        return [labels[int(i)] for i in torch.as_tensor(gidx).cpu().tolist()]
