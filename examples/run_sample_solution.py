#!/usr/bin/env python3
"""Supervised training from an explicit sample file (reference
``examples/sample_solution/sample_solution_model.py``): a GraphSAGE ``BaseGNNNet`` encodes
the node in column 2 of each ``label,node`` row, ``SuperviseSampleSolution`` scores it with
``DenseLogits(1)`` and ``SampleEstimator`` repeats the file ``--epoch`` times.

    python examples/run_sample_solution.py --total_step 50
    python examples/run_sample_solution.py --sample_dir my_samples.csv --epoch 3

Without ``--sample_dir`` a ``label,node`` file is generated from the dataset's training
nodes (label = first label bit), since the reference's ``sample.txt`` is a 1-row stub.
"""
import argparse
import logging
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import euler_amd.ops.graph_api as ge  # noqa: E402
from euler_amd import solution as S  # noqa: E402
from euler_amd.dataset import get_dataset  # noqa: E402
from euler_amd.estimator import SampleEstimator  # noqa: E402
from euler_amd.mp_utils.models import BaseGNNNet  # noqa: E402


class GNN(BaseGNNNet):
    """``BaseGNNNet`` reading its inputs from a dense node feature (reference model file:37-60)."""

    def __init__(self, conv, flow, dims, fanouts, metapath, feature_idx, feature_dim, max_id=-1):
        super().__init__(conv=conv, flow=flow, dims=dims, fanouts=fanouts, metapath=metapath,
                         add_self_loops=False, max_id=max_id)
        self.feature_idx = feature_idx if isinstance(feature_idx, list) else [feature_idx]
        self.feature_dim = feature_dim if isinstance(feature_dim, list) else [feature_dim]

    def to_x(self, n_id):
        x, = ge.get_dense_feature(n_id, self.feature_idx, self.feature_dim)
        return x


def parse_rows(batch):
    """``label,node`` token rows -> (label [b,1] float, node ids [b])."""
    arr = np.asarray(batch, dtype=np.float64)
    return torch.tensor(arr[:, 0:1], dtype=torch.float32), torch.tensor(arr[:, 1].astype(np.int64))


def write_samples(ds, path, n, seed=0):
    """Sample ``n`` training nodes and label each with bit 0 of its label feature."""
    nodes = ge.sample_node(n, getattr(ds, "train_node_type", "train"))
    label, = ge.get_dense_feature(nodes, [ds.label_idx], [ds.label_dim])
    with open(path, "w") as f:
        for v, y in zip(nodes.tolist(), label[:, 0].tolist()):
            f.write("%d,%d\n" % (int(y > 0.5), v))
    return path


def main(argv=None):
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(message)s")
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--dataset", default="cora")
    p.add_argument("--data_dir", default=None)
    p.add_argument("--scale", type=float, default=1.0)
    p.add_argument("--sample_dir", default=None)
    p.add_argument("--num_samples", type=int, default=2048)
    p.add_argument("--fanouts", type=int, nargs="+", default=[5, 5])
    p.add_argument("--dim", type=int, default=32)
    p.add_argument("--batch_size", type=int, default=512)
    p.add_argument("--epoch", type=int, default=20)
    p.add_argument("--total_step", type=int, default=None)
    p.add_argument("--learning_rate", type=float, default=0.001)
    p.add_argument("--model_dir", default="ckpt")
    p.add_argument("--log_steps", type=int, default=20)
    a = p.parse_args(argv)

    ds = get_dataset(a.dataset, data_dir=a.data_dir, scale=a.scale)
    ds.load_graph()
    os.makedirs(a.model_dir, exist_ok=True)
    sample_dir = a.sample_dir or write_samples(ds, os.path.join(a.model_dir, "sample.txt"), a.num_samples)

    metapath = [["train"]] * len(a.fanouts)
    enc = GNN("sage", "sage", [a.dim] * (len(a.fanouts) + 1), a.fanouts, metapath,
              ds.feature_idx, ds.feature_dim, max_id=ds.max_node_id)
    model = S.SuperviseSampleSolution(parse_rows, enc, lambda emb: (emb, None, emb),
                                      logit_fn=S.DenseLogits(1))
    params = {"batch_size": a.batch_size, "optimizer": "adam", "learning_rate": a.learning_rate,
              "log_steps": a.log_steps, "model_dir": a.model_dir, "sample_dir": sample_dir,
              "infer_dir": a.model_dir, "epoch": a.epoch, "total_step": a.total_step}
    return SampleEstimator(model, params).train()


if __name__ == "__main__":
    print(main())
