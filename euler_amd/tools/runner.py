"""Model-zoo runner: the ``examples/*/run_*.py`` entry points of the reference
(e.g. ``examples/graphsage/run_graphsage.py:30-43``) as one registry.

``python -m euler_amd.tools.runner --model graphsage --dataset cora --run_mode train``
or the thin per-model scripts under ``examples/``.  Flags keep the reference names
(``dataset, hidden_dim, layers, fanouts, batch_size, num_epochs, log_steps, model_dir,
id_file, infer_dir, optimizer, learning_rate, run_mode``); ``total_step`` defaults to
``num_epochs * total_size / batch_size`` like the reference runners.  Data parallelism:
``--gpus N`` starts N ranks on this node (parallel/launch.py maybe_spawn), or launch under
torchrun (``WORLD_SIZE`` > 1 initialises RCCL/gloo automatically); reference launcher
``tf_euler/scripts/dist_tf_euler.sh:1-49``.
"""
from __future__ import annotations

import argparse
import logging
import os
import sys

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL, before torch loads HIP

import torch  # noqa: E402

__all__ = ["MODELS", "build", "main", "parse_args"]


def _node(ds, a):
    return {"train_node_type": _first(ds.train_node_type), "id_file": ds.id_file}


def _first(x):
    return x[0] if isinstance(x, (list, tuple)) else x


def _hidden(a, out):
    return [a.hidden_dim] * a.layers + [out]


def _mp(a, n=None):
    """metapath: the training edges for run_mode train, every edge type otherwise (the
    reference's run_graphsage.py:53-57 — evaluation reaches the held-out nodes, whose
    edges are not training edges)"""
    ds = a._ds
    et = ds.train_edge_type
    if a.run_mode != "train" and getattr(ds, "all_edge_type", None) not in (None, -1):
        et = ds.all_edge_type
    et = list(et) if isinstance(et, (list, tuple)) else [et]
    return [et] * (n or a.layers)


# name -> (default dataset, estimator kind, builder(args, ds))
def _models():
    from euler_amd import models as Z

    F = lambda ds: ds.feature_dim  # noqa: E731
    return {
        # reference run_graphsage.py:48: dims = [hidden_dim] * (layers + 1)
        "graphsage": ("cora", "node", lambda a, ds: Z.SupervisedGraphSage(
            _hidden(a, a.hidden_dim), a.fanouts, _mp(a), ds.feature_idx, F(ds), ds.label_idx, ds.label_dim,
            max_id=ds.max_node_id)),
        "graphsage_unsup": ("cora", "node", lambda a, ds: Z.UnsupervisedGraphSage(
            _hidden(a, a.dim), a.fanouts, _mp(a), ds.feature_idx, F(ds), _first(ds.train_node_type),
            _first(ds.train_edge_type), ds.max_node_id, num_negs=a.num_negs)),
        "gcn": ("cora", "node", lambda a, ds: Z.SupervisedGCN(_hidden(a, ds.label_dim), _mp(a), ds.feature_idx,
                                                              F(ds), ds.label_idx, ds.label_dim)),
        "gat": ("cora", "node", lambda a, ds: Z.GAT(_hidden(a, ds.label_dim), _mp(a), ds.feature_idx, F(ds),
                                                    ds.label_idx, ds.label_dim, head_num=a.head_num)),
        "fastgcn": ("cora", "node", lambda a, ds: Z.FastGCN(_hidden(a, ds.label_dim), a.fanouts, _mp(a),
                                                            ds.feature_idx, F(ds), ds.label_idx, ds.label_dim)),
        "adaptivegcn": ("cora", "node", lambda a, ds: Z.AdaptiveGCN(_hidden(a, ds.label_dim), a.fanouts, _mp(a),
                                                                    ds.feature_idx, F(ds), ds.label_idx,
                                                                    ds.label_dim)),
        "agnn": ("cora", "node", lambda a, ds: Z.AGNN("f1", _hidden(a, ds.label_dim), _mp(a), ds.feature_idx, F(ds),
                                                      ds.label_idx, ds.label_dim)),
        "appnp": ("cora", "node", lambda a, ds: Z.APPNP(_hidden(a, ds.label_dim), _mp(a), ds.feature_idx, F(ds),
                                                        ds.label_idx, ds.label_dim, K=a.K, alpha=a.alpha)),
        "arma": ("cora", "node", lambda a, ds: Z.ARMA(_hidden(a, ds.label_dim), _mp(a), ds.feature_idx, F(ds),
                                                      ds.label_idx, ds.label_dim, K=a.K)),
        "dna": ("cora", "node", lambda a, ds: Z.DNA(_hidden(a, ds.label_dim), _mp(a), ds.feature_idx, F(ds),
                                                    ds.label_idx, ds.label_dim, head_num=a.head_num)),
        "sgcn": ("cora", "node", lambda a, ds: Z.SGCN(_hidden(a, ds.label_dim), _mp(a), ds.feature_idx, F(ds),
                                                      ds.label_idx, ds.label_dim, K=a.K)),
        "tagcn": ("cora", "node", lambda a, ds: Z.TAGCN(_hidden(a, ds.label_dim), _mp(a), ds.feature_idx, F(ds),
                                                        ds.label_idx, ds.label_dim, K=a.K)),
        "geniepath": ("cora", "node", lambda a, ds: Z.GeniePath(a.hidden_dim, _mp(a), ds.label_idx, ds.label_dim,
                                                                feature_idx=ds.feature_idx, feature_dim=F(ds),
                                                                head_num=a.head_num)),
        "lgcn": ("cora", "node", lambda a, ds: Z.LGCN(a.hidden_dim, [_first(ds.train_edge_type)], ds.label_idx,
                                                      ds.label_dim, feature_idx=ds.feature_idx, feature_dim=F(ds))),
        "deepwalk": ("cora", "node", lambda a, ds: Z.DeepWalk(_first(ds.train_node_type), _first(ds.train_edge_type),
                                                              ds.max_node_id, a.dim, walk_len=a.walk_len,
                                                              num_negs=a.num_negs, sharded=a.sharded)),
        "node2vec": ("cora", "node", lambda a, ds: Z.Node2Vec(_first(ds.train_node_type), _first(ds.train_edge_type),
                                                              ds.max_node_id, a.dim, walk_len=a.walk_len,
                                                              walk_p=a.walk_p, walk_q=a.walk_q, num_negs=a.num_negs,
                                                              sharded=a.sharded)),
        "line": ("cora", "node", lambda a, ds: Z.Line(_first(ds.train_node_type), _first(ds.train_edge_type),
                                                      ds.max_node_id, a.dim, num_negs=a.num_negs, order=a.order,
                                                      sharded=a.sharded)),
        "dgi": ("cora", "node", lambda a, ds: Z.DGI(_first(ds.train_node_type), _first(ds.train_edge_type),
                                                    ds.max_node_id, _mp(a), a.fanouts, a.dim,
                                                    feature_idx=ds.feature_idx, feature_dim=F(ds))),
        "gae": ("cora", "node", lambda a, ds: Z.GraphAutoEncoder("gcn" if a.gae_encoder == "gcn" else "sage",
                                                                 _hidden(a, a.dim)[1:], a.fanouts[:a.layers - 1] or
                                                                 a.fanouts, _mp(a, a.layers - 1 or 1),
                                                                 ds.feature_idx, F(ds), _first(ds.train_node_type),
                                                                 _first(ds.train_edge_type), ds.max_node_id,
                                                                 num_negs=a.num_negs)),
        "vgae": ("cora", "node", lambda a, ds: Z.VariationalGraphAutoEncoder(
            0.1, "gcn" if a.gae_encoder == "gcn" else "sage", _hidden(a, a.dim)[1:],
            a.fanouts[:a.layers - 1] or a.fanouts, _mp(a, a.layers - 1 or 1), ds.feature_idx, F(ds),
            _first(ds.train_node_type), _first(ds.train_edge_type), ds.max_node_id, num_negs=a.num_negs)),
        "rgcn": ("wn18", "node", lambda a, ds: Z.UnsupervisedRGCN(
            _first(ds.train_node_type), _first(ds.train_edge_type), ds.max_node_id, _hidden(a, a.dim),
            [[_first(ds.train_edge_type)]] * a.layers, ds.max_edge_id + 1, "id", 1, a.dim, num_negs=a.num_negs)),
        "transe": ("fb15k", "edge", lambda a, ds: Z.TransE(_first(ds.train_node_type), _first(ds.train_edge_type),
                                                          ds.max_node_id, ds.max_edge_id, a.dim, a.dim,
                                                          num_negs=a.num_negs, margin=a.margin, sharded=a.sharded)),
        "transh": ("fb15k", "edge", lambda a, ds: Z.TransH(_first(ds.train_node_type), _first(ds.train_edge_type),
                                                          ds.max_node_id, ds.max_edge_id, a.dim, a.dim,
                                                          num_negs=a.num_negs, margin=a.margin)),
        "transr": ("fb15k", "edge", lambda a, ds: Z.TransR(_first(ds.train_node_type), _first(ds.train_edge_type),
                                                          ds.max_node_id, ds.max_edge_id, a.dim, a.dim,
                                                          num_negs=a.num_negs, margin=a.margin)),
        "transd": ("fb15k", "edge", lambda a, ds: Z.TransD(_first(ds.train_node_type), _first(ds.train_edge_type),
                                                          ds.max_node_id, ds.max_edge_id, a.dim, a.dim,
                                                          num_negs=a.num_negs, margin=a.margin)),
        "distmult": ("fb15k", "edge", lambda a, ds: Z.DistMult(_first(ds.train_node_type),
                                                              _first(ds.train_edge_type), ds.max_node_id,
                                                              ds.max_edge_id, a.dim, a.dim, num_negs=a.num_negs)),
        "gin": ("mutag", "graph", lambda a, ds: Z.GIN(_hidden(a, a.hidden_dim), _mp(a), ds.num_classes,
                                                      ds.sparse_fea_idx, ds.sparse_fea_max_id)),
        "gated_graph": ("mutag", "graph", lambda a, ds: Z.GatedGraph(_hidden(a, a.hidden_dim), _mp(a),
                                                                     ds.num_classes, ds.sparse_fea_idx,
                                                                     ds.sparse_fea_max_id)),
        "graphgcn": ("mutag", "graph", lambda a, ds: Z.GraphGCN(_hidden(a, a.hidden_dim), _mp(a), ds.num_classes,
                                                                ds.sparse_fea_idx, ds.sparse_fea_max_id)),
        "set2set": ("mutag", "graph", lambda a, ds: Z.Set2SetModel(_hidden(a, a.hidden_dim), _mp(a),
                                                                   ds.num_classes, ds.sparse_fea_idx,
                                                                   ds.sparse_fea_max_id)),
        "solution": ("cora", "node", _solution),
        "scalable_sage": ("ppi", "node", lambda a, ds: Z.ScalableSage(_mp(a, 1)[0], a.fanouts[0], a.layers,
                                                                      a.hidden_dim, ds.label_idx, ds.label_dim,
                                                                      ds.feature_idx, F(ds), ds.max_node_id)),
        "scalable_gcn": ("ppi", "node", lambda a, ds: Z.ScalableGCN(_mp(a, 1)[0], a.layers, a.hidden_dim,
                                                                    ds.label_idx, ds.label_dim, ds.feature_idx,
                                                                    F(ds), ds.max_node_id)),
    }


def _solution(a, ds):
    """examples/solution/run_solution.py: SuperviseSolution over a SageEncoder."""
    from euler_amd import solution as S
    from euler_amd.utils import encoders as E

    enc = E.SageEncoder(_mp(a), a.fanouts, a.hidden_dim, feature_idx=ds.feature_idx, feature_dim=ds.feature_dim,
                        max_id=ds.max_node_id)
    return S.SuperviseSolution(S.GetLabelFromFea(ds.label_idx, ds.label_dim), enc, S.DenseLogits(ds.label_dim))


MODELS = None


def parse_args(argv=None, model=None):
    p = argparse.ArgumentParser(description="euler_amd model-zoo runner")
    p.add_argument("--model", default=model, required=model is None)
    p.add_argument("--gpus", type=int, default=None, help="data-parallel ranks on this node, one per GPU "
                   "(self-spawned; default: WORLD_SIZE or 1)")
    p.add_argument("--dataset", default=None)
    p.add_argument("--data_dir", default=None)
    p.add_argument("--scale", type=float, default=1.0, help="synthetic-dataset scale when no raw files exist")
    p.add_argument("--hidden_dim", type=int, default=32)
    p.add_argument("--dim", type=int, default=32, help="embedding dim (unsupervised / KG models)")
    p.add_argument("--layers", type=int, default=2)
    p.add_argument("--fanouts", type=int, nargs="+", default=[10, 10])
    p.add_argument("--batch_size", type=int, default=32)
    p.add_argument("--num_epochs", type=int, default=10)
    p.add_argument("--total_step", type=int, default=None)
    p.add_argument("--log_steps", type=int, default=20)
    p.add_argument("--model_dir", default="ckpt")
    p.add_argument("--infer_dir", default="infer")
    p.add_argument("--id_file", default=None)
    p.add_argument("--optimizer", default="adam")
    p.add_argument("--learning_rate", type=float, default=0.01)
    p.add_argument("--run_mode", default="train", choices=["train", "evaluate", "infer", "train_and_evaluate"])
    p.add_argument("--num_negs", type=int, default=5)
    p.add_argument("--walk_len", type=int, default=3)
    p.add_argument("--walk_p", type=float, default=1.0)
    p.add_argument("--walk_q", type=float, default=1.0)
    p.add_argument("--order", type=int, default=1)
    p.add_argument("--head_num", type=int, default=1)
    p.add_argument("--K", type=int, default=3)
    p.add_argument("--alpha", type=float, default=0.1)
    p.add_argument("--margin", type=float, default=1.0)
    p.add_argument("--gae_encoder", default="gcn")
    p.add_argument("--infer_type", default="node_src")
    p.add_argument("--sharded", action="store_true", help="row-shard id embeddings over the process group")
    p.add_argument("--row_sparse_tables", default="auto", choices=["auto", "on", "off"],
                   help="device path: id tables trained row-sparse (ShardedTable + sparse optimizer); auto = "
                        "for sharded models and tables of >= 2^20 rows")
    p.add_argument("--device", default=None)
    p.add_argument("--amp", default=None, help="bf16 for bf16 autocast on the GPU")
    p.add_argument("--device_graph", action="store_true",
                   help="graphsage / graphsage_unsup: train on an HBM copy of the graph with the fused "
                        "gfx950 step (models/sage_trainer.py, models/sage_tower.py) instead of the "
                        "CPU-engine input pipeline")
    p.add_argument("--device_graph_sharded", action="store_true",
                   help="with --device_graph: row-shard the graph (CSR, features, labels) over the ranks, "
                        "neighbour draws and features over all-to-all (graph/sharded_graph.py; supervised "
                        "SageDataFlow models)")
    p.add_argument("--engine_shards", action="store_true",
                   help="with --device_graph_sharded: every rank's engine loads only its partitions "
                        "(shard_idx = rank): host memory per rank is 1/W of the graph (training only: "
                        "an engine-path evaluate would see one shard)")
    p.add_argument("--device_feature_dtype", default="bf16", choices=["bf16", "fp32"])
    p.add_argument("--cuda_graph", default="auto", choices=["auto", "off"],
                   help="capture the engine-path training step in a hipGraph when eligible")
    p.add_argument("--native_pipeline", default="auto", choices=["auto", "on", "off"],
                   help="engine path: C++ batch pipeline (sampling + features into pinned slots) for "
                        "SupervisedGNN + SageDataFlow models; auto = on for GPU training")
    p.add_argument("--pipeline_workers", type=int, default=8)
    p.add_argument("--seed", type=int, default=None)
    return p.parse_args(argv)


def build(a):
    """(model, estimator) for parsed args; loads (or synthesises) the dataset."""
    global MODELS
    from euler_amd.dataset import get_dataset
    from euler_amd.estimator import EdgeEstimator, GraphEstimator, NodeEstimator
    from euler_amd.parallel import dp

    dp.init_distributed()
    MODELS = MODELS or _models()
    if a.model not in MODELS:
        raise SystemExit("unknown model %r; choose from %s" % (a.model, sorted(MODELS)))
    ds_name, kind, builder = MODELS[a.model]
    ds = get_dataset(a.dataset or ds_name, data_dir=a.data_dir, scale=a.scale)
    if getattr(a, "engine_shards", False):
        import torch.distributed as dist

        from euler_amd.ops.base import initialize_graph

        on = dist.is_available() and dist.is_initialized()
        initialize_graph({"mode": "local", "data_path": ds.get_data_dir(), "data_type": ds.data_type,
                          "shard_idx": dist.get_rank() if on else 0, "shard_num": dist.get_world_size() if on else 1})
    else:
        ds.load_graph()
    a._ds = ds
    model = builder(a, ds)
    total = a.total_step or max(1, int(a.num_epochs * ds.total_size / max(a.batch_size, 1)))
    params = {"model_dir": a.model_dir, "infer_dir": a.infer_dir, "batch_size": a.batch_size, "total_step": total,
              "log_steps": a.log_steps, "optimizer": a.optimizer, "learning_rate": a.learning_rate,
              "device": a.device, "amp": a.amp, "device_graph": a.device_graph or a.device_graph_sharded,
              "device_graph_sharded": ("engine_shards" if a.engine_shards else True) if a.device_graph_sharded
              else False,
              "device_feature_dtype": a.device_feature_dtype, "seed": a.seed,
              "native_pipeline": {"auto": "auto", "on": True, "off": False}[a.native_pipeline],
              "cuda_graph": a.cuda_graph if a.cuda_graph == "auto" else False,
              "pipeline_workers": a.pipeline_workers,
              "row_sparse_tables": {"auto": "auto", "on": True, "off": False}[a.row_sparse_tables]}
    if kind == "node":
        params.update(train_node_type=_first(ds.train_node_type), id_file=a.id_file or ds.id_file)
        est = NodeEstimator(model, params)
    elif kind == "edge":
        params.update(train_edge_type=_first(ds.train_edge_type), id_file=a.id_file or ds.edge_id_file,
                      infer_type=a.infer_type)
        est = EdgeEstimator(model, params)
    else:
        params.update(label=[ds.label_idx], num_classes=ds.num_classes, id_file=a.id_file or ds.id_file)
        est = GraphEstimator(model, params)
    return model, est


def main(argv=None, model=None):
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(message)s")
    a = parse_args(argv, model)
    if argv is None:  # a command line (not a library call): --gpus N starts the ranks here
        from euler_amd.parallel.launch import maybe_spawn

        rc = maybe_spawn(a.gpus, sys.argv[1:], sys.argv[0])
        if rc is not None:
            raise SystemExit(rc)
    _, est = build(a)
    if a.run_mode == "train":
        return est.train()
    if a.run_mode == "evaluate":
        return est.evaluate()
    if a.run_mode == "infer":
        return est.infer()
    return est.train_and_evaluate()


if __name__ == "__main__":
    main()
