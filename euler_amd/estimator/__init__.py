"""Estimators (reference ``euler_estimator/python/*.py``)."""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

import euler_amd.ops.graph_api as ge
from euler_amd.estimator.base import BaseEstimator, id_file_batches, latest_checkpoint

__all__ = ["BaseEstimator", "NodeEstimator", "EdgeEstimator", "GraphEstimator", "GaeEstimator", "SampleEstimator",
           "latest_checkpoint", "id_file_batches"]


def _shard(est):
    return (est.rank, est.world)


class NodeEstimator(BaseEstimator):
    """train: ``sample_node(batch_size, train_node_type)``; eval / infer: id file
    (reference node_estimator.py:26-51)."""

    def get_train_from_input(self, inputs, params):
        return ge.sample_node(inputs, params["train_node_type"])

    def train_input_fn(self):
        return self.params["batch_size"]

    def get_input_from_id_file(self):
        for b in id_file_batches(self.params["id_file"], self.params["batch_size"], int, _shard(self)):
            yield torch.tensor(b, dtype=torch.int64)

    def evaluate_input_fn(self):
        return self.get_input_from_id_file()

    def infer_input_fn(self):
        return self.get_input_from_id_file()


class GaeEstimator(NodeEstimator):
    """Same inputs as NodeEstimator (reference gae_estimator.py:26-51)."""


class EdgeEstimator(BaseEstimator):
    """train: ``sample_edge(batch_size, train_edge_type)`` -> [n, 3] (src, dst, type);
    eval / infer: "src dst type" lines; ``infer_type`` picks node_src / edge / node_dst
    embeddings (reference edge_estimator.py:27-72)."""

    def get_train_from_input(self, inputs, params):
        return ge.sample_edge(inputs, params["train_edge_type"])

    def train_input_fn(self):
        return self.params["batch_size"]

    def transfer_embedding(self, source, emb):
        t = self.params.get("infer_type", "node_src")
        source = torch.as_tensor(source)
        if t == "node_src":
            return source[:, 0], emb[0]
        if t == "edge":
            return source[:, :2], emb[1]
        if t == "node_dst":
            return source[:, 1], emb[2]
        raise ValueError("infer_type must be node_src/node_dst/edge.")

    def get_input_from_id_file(self):
        def parse(line):
            a = line.split()
            return [int(a[0]), int(a[1]), int(a[2])]

        for b in id_file_batches(self.params["id_file"], self.params["batch_size"], parse, _shard(self)):
            yield torch.tensor(b, dtype=torch.int64)

    def evaluate_input_fn(self):
        return self.get_input_from_id_file()

    def infer_input_fn(self):
        return self.get_input_from_id_file()


class GraphEstimator(BaseEstimator):
    """Graph classification: ``sample_graph_label`` -> ``get_graph_by_label`` ->
    {node_idx, graph_label (one-hot of the first node's label feature),
    node_graph_idx, graph_idx} (reference graph_estimator.py:27-85)."""

    def train_input_fn(self):
        return self.params["batch_size"]

    def get_graph_label(self, sample_graph):
        ind = torch.as_tensor(sample_graph.indices)
        vals = torch.as_tensor(sample_graph.values)
        first = vals[ind[:, 1] == 0]
        lab = ge.get_dense_feature(first, _as_list(self.params["label"]), [1])[0]
        lab = lab.reshape(-1).long()
        return F.one_hot(lab, int(self.params["num_classes"])).float()

    def _graph_inputs(self, labels):
        sg = ge.get_graph_by_label(labels)
        return {"node_idx": torch.as_tensor(sg.values), "graph_label": self.get_graph_label(sg),
                "node_graph_idx": torch.as_tensor(sg.indices)[:, 0], "graph_idx": labels}

    def get_train_from_input(self, inputs, params):
        return self._graph_inputs(ge.sample_graph_label(inputs))

    def get_input_from_id_file(self):
        for b in id_file_batches(self.params["id_file"], self.params["batch_size"], str, _shard(self)):
            yield b

    def get_evaluate_from_input(self, inputs, params):
        return self._graph_inputs(inputs)

    def get_infer_from_input(self, inputs, params):
        return self._graph_inputs(inputs)

    def transfer_embedding(self, source, emb):
        return np.asarray(source["graph_idx"]), emb

    def evaluate_input_fn(self):
        return self.get_input_from_id_file()

    def infer_input_fn(self):
        return self.get_input_from_id_file()


class SampleEstimator(BaseEstimator):
    """Explicit CSV sample rows, repeated ``epoch`` times for training
    (reference sample_estimator.py:25-53).  Each batch is a list of token lists."""

    def get_input_from_sample(self, epochs):
        for _ in range(int(epochs)):
            for b in id_file_batches(self.params["sample_dir"], self.params["batch_size"],
                                     lambda s: s.split(","), _shard(self)):
                yield b

    def train_input_fn(self):
        it = self.get_input_from_sample(self.params.get("epoch", 1))
        if self.params.get("total_step") is None:
            # one pass over the file defines the step count, like estimator.train(steps=None)
            batches = list(it)
            self.params["total_step"] = len(batches)
            it = iter(batches)
        return it

    def get_train_from_input(self, inputs, params):
        return next(inputs)

    def evaluate_input_fn(self):
        return self.get_input_from_sample(1)

    def infer_input_fn(self):
        return self.get_input_from_sample(1)

    def transfer_embedding(self, source, emb):
        # the target node is the second column of every row
        return np.asarray([int(r[1]) for r in source], dtype=np.int64).reshape(-1, 1), emb


def _as_list(x):
    return list(x) if isinstance(x, (list, tuple)) else [x]
