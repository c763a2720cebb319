"""Which device-path trainer trains an estimator's model (``params["device_graph"] = True``).

The reference runs one ``model_fn`` per mode through ``tf.estimator``
(``euler_estimator/python/base_estimator.py:102-179``); here every model family has a
trainer that draws its batches on an HBM copy of the graph and captures whole steps in
hipGraphs.  :data:`REGISTRY` is an ordered list of ``(name, predicate, builder)``; the
first entry whose predicate accepts the model builds its trainer.  Every builder gets a
:class:`Ctx` — the estimator's parameters plus one graph-upload helper
(:meth:`Ctx.upload`), so node-type resolution, the feature dtype and the per-rank sampler
key (``seed * 7919 + rank``) are decided in one place.

Before a builder runs, the estimator materialises the model, broadcasts rank 0's weights
(``BaseEstimator._prepare``) and removes its autograd gradient-sync hooks: every device
trainer all-reduces its own flat gradient (or runs a row-sparse update) itself.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Callable, List, Tuple

import numpy as np
import torch

__all__ = ["Ctx", "REGISTRY", "build_device_trainer", "build_sharded_trainer", "register", "device_infers",
           "has_store_encoder", "NoDeviceTrainer", "sharded_supported"]


class NoDeviceTrainer(ValueError):
    """no device-path trainer accepts the model (the estimator may fall back to the engine path)"""


@dataclass
class Ctx:
    est: Any   # the BaseEstimator
    model: Any

    @property
    def params(self):
        return self.est.params

    @property
    def seed(self) -> int:
        return int(self.params.get("seed") or 0)

    @property
    def batch(self) -> int:
        return int(self.params["batch_size"])

    def opt_kw(self) -> dict:
        return {"optimizer": self.params.get("optimizer", "adam"),
                "learning_rate": float(self.params.get("learning_rate", 0.001))}

    def node_type(self, default=-1) -> int:
        """``train_node_type`` (or the model's default) as a type id; -1 = every type"""
        import euler_amd.ops.graph_api as ge

        nt = self.params.get("train_node_type", default)
        return -1 if nt in (None, -1, "-1") else int(np.asarray(ge.get_node_type_id(nt)).reshape(-1)[0])

    def feature_dtype(self):
        return torch.float32 if self.params.get("device_feature_dtype", "bf16") == "fp32" else torch.bfloat16

    def upload(self, default_node_type=-1, features=(), feature_dims=(), label=None, label_dim=None, node_type=None):
        """the engine's graph (structure + the named dense feature / label columns) in HBM;
        ``params["device_graph_factory"](rank, device)`` supplies it instead (e.g. a
        ``DeviceGraph.synthetic`` 100M-node graph generated straight in HBM, no engine)"""
        from euler_amd.graph.device_graph import DeviceGraph

        factory = self.params.get("device_graph_factory")
        if callable(factory):
            g = factory(self.est.rank, self.est.device)
            g.manual_seed(self.seed * 7919 + self.est.rank)
            return g

        kw = {}
        if label is not None:
            kw.update(label=label, label_dim=label_dim)
        nt = self.node_type(default_node_type) if node_type is None else node_type
        # every rank uploads together: with 2+ ranks on a node the export happens once
        # (local rank 0 into /dev/shm, the others map it: graph/device_graph.py shared_export)
        return DeviceGraph.from_engine(node_type=nt, features=features, feature_dims=feature_dims,
                                       feature_dtype=self.feature_dtype(), seed=self.seed * 7919 + self.est.rank,
                                       device=self.est.device, share=self.est.world > 1, **kw)


Builder = Callable[[Ctx], Any]
REGISTRY: List[Tuple[str, Callable[[Any], bool], Builder]] = []


def register(name: str, predicate: Callable[[Any], bool]):
    def deco(fn: Builder) -> Builder:
        REGISTRY.append((name, predicate, fn))
        return fn
    return deco


def has_store_encoder(model) -> bool:
    """True when ``model`` holds a historical-embedding encoder (ScalableGCNEncoder /
    ScalableSageEncoder: stale per-layer stores + gradient stores, reference
    tf_euler/python/utils/encoders.py:294-408, 629-748)"""
    from euler_amd.utils.encoders import _StoreMixin

    return any(isinstance(m, _StoreMixin) for m in model.modules())


# trainers that run a store encoder's own protocol (stores read / written inside the step)
STORE_AWARE = {"scalable"}


def device_infers(model) -> bool:
    """False for models whose evaluate / infer must stay on the engine path whatever the
    trainer: layer-sampled GCNs (FastGCN / AdaptiveGCN draw their layers, reference
    fast_dataflow.py / layerwise_dataflow.py) — building a device trainer only to learn
    that would also consume the engine's sampler stream before the engine-path eval."""
    from euler_amd.dataflow import dataflows as D

    sampler = getattr(getattr(model, "gnn", None), "sampler", None)
    return not isinstance(sampler, (D.FastGCNDataFlow, D.LayerwiseDataFlow))


def build_device_trainer(est, model, first):
    """the first registered trainer that accepts ``model`` (NoDeviceTrainer if none does).
    A model with a historical-embedding encoder is only taken by a store-aware trainer:
    any other trainer would train it as its plain parent encoder without stores.
    ``params["device_graph_sharded"]``: the graph is row-sharded over the ranks
    (:func:`build_sharded_trainer`)."""
    if est.params.get("device_graph_sharded"):
        return build_sharded_trainer(est, model, first)
    stores = has_store_encoder(model)
    for name, pred, builder in REGISTRY:
        if stores and name not in STORE_AWARE:
            continue
        if pred(model):
            # materialise lazy layers, broadcast rank 0's weights; no torch optimizer and no
            # autograd gradient sync: every device trainer runs its own update and sync
            est._prepare(first, build_optimizer=False)
            tr = builder(Ctx(est, model))
            tr.device_trainer_kind = name
            return tr
    if stores:
        raise NoDeviceTrainer(f"{type(model).__name__} holds a historical-embedding (Scalable*) encoder that no "
                              "device trainer accepts")
    raise NoDeviceTrainer("device_graph=True trains: " + ", ".join(n for n, _, _ in REGISTRY) +
                          f"; {type(model).__name__} is none of them")


def _sharded_unsup(model) -> bool:
    """UnsupervisedGraphSage: two 2-hop SAGEConv towers on SageDataFlow"""
    from euler_amd.convolution.convs import SAGEConv
    from euler_amd.dataflow import dataflows as D

    gnn = getattr(model, "gnn", None)
    return (_is_unsup_gnn(model) and isinstance(getattr(gnn, "sampler", None), D.SageDataFlow)
            and len(gnn.convs) == 2 and all(isinstance(c, SAGEConv) for c in gnn.convs))


def sharded_supported(model) -> bool:
    """supervised models on the sampled ``SageDataFlow`` or the full-neighbourhood
    ``GCNDataFlow`` (any convolution, no stores), and the unsupervised 2-hop GraphSAGE"""
    from euler_amd.dataflow import dataflows as D

    gnn = getattr(model, "gnn", None)
    if _sharded_unsup(model):
        return True
    return (gnn is not None and hasattr(gnn, "feature_idx") and hasattr(model, "label_idx")
            and not hasattr(model, "context_gnn") and not has_store_encoder(model)
            and isinstance(getattr(gnn, "sampler", None), (D.SageDataFlow, D.GCNDataFlow)))


def build_sharded_trainer(est, model, first):
    """a graph larger than one GPU's HBM: every rank uploads only its rows (r % W) of the
    CSR, features and labels (graph/sharded_graph.py) and the neighbour draws, features and
    labels cross the ranks over all-to-all (models/full_trainer.py ShardedFlowTrainer)"""
    from euler_amd.graph.sharded_graph import ShardedDeviceGraph
    from euler_amd.models.full_trainer import ShardedFlowTrainer

    if not sharded_supported(model):
        raise NoDeviceTrainer("device_graph_sharded=True trains supervised models on the sampled SageDataFlow or "
                              "the full-neighbourhood GCNDataFlow, and the unsupervised GraphSAGE; "
                              f"{type(model).__name__} is not one")
    est._prepare(first, build_optimizer=False)
    c = Ctx(est, model)
    gnn = model.gnn
    # "engine_shards": every rank's engine holds only its partitions (initialize_graph with
    # shard_idx = rank, shard_num = W): host memory per rank is 1/W of the graph
    build = ShardedDeviceGraph.from_engine_shard if est.params.get("device_graph_sharded") == "engine_shards" \
        else ShardedDeviceGraph.from_engine
    if _sharded_unsup(model):
        # UnsupervisedGraphSage: both towers' trees, the positives and the negatives drawn
        # through the owners (models/sharded_unsup.py); one rank without collectives: the
        # whole-graph fused trainer
        from euler_amd.models.sage_tower import UnsupSageTrainer
        from euler_amd.models.sharded_unsup import ShardedUnsupSageTrainer

        g = build(node_type=c.node_type(-1), features=gnn.feature_idx, feature_dims=gnn.feature_dim,
                  feature_dtype=c.feature_dtype(), seed=c.seed * 7919 + est.rank, device=est.device)
        if not g.comm:
            tr = UnsupSageTrainer.from_model(model, g.local, c.batch, **c.opt_kw())
            tr.device_trainer_kind = "unsupervised_graphsage"
            return tr
        tr = ShardedUnsupSageTrainer.from_model(model, g, c.batch, **c.opt_kw())
        tr.device_trainer_kind = "sharded_unsupervised_graphsage"
        return tr
    g = build(node_type=c.node_type(-1), features=gnn.feature_idx, feature_dims=gnn.feature_dim,
              label=model.label_idx, label_dim=model.label_dim, feature_dtype=c.feature_dtype(),
              seed=c.seed * 7919 + est.rank, device=est.device)
    from euler_amd.convolution.convs import SAGEConv

    from euler_amd.dataflow import dataflows as D

    if isinstance(gnn.sampler, D.GCNDataFlow):
        # GCN / APPNP / TAGCN / ...: full-neighbourhood blocks expanded by the rows' owners;
        # one rank holds the whole graph: the whole-graph trainers (fused GCN step, captured)
        caps = c.params.get("device_flow_caps", "bounded")
        if not g.comm:
            from euler_amd.models.full_trainer import FullFlowTrainer
            from euler_amd.models.gcn_trainer import GcnTrainer

            if c.params.get("gcn_fused", True) and GcnTrainer.supports(model, g.local, c.batch):
                tr = GcnTrainer.from_model(model, g.local, c.batch, caps=caps, **c.opt_kw())
            else:
                tr = FullFlowTrainer.from_model(model, g.local, c.batch, **c.opt_kw(), caps=caps)
            tr.device_trainer_kind = "full_flow"
            return tr
        tr = ShardedFlowTrainer.from_model(model, g, c.batch, caps=caps, **c.opt_kw())
        tr.device_trainer_kind = "sharded_full_flow"
        return tr
    if all(isinstance(cv, SAGEConv) for cv in gnn.convs) and c.params.get("sharded_fused", True):
        # SupervisedGraphSage: the fused tree-step kernels on trees drawn across the ranks;
        # one rank holds the whole graph: the whole-graph trainer (its sampler runs inside
        # the head launch)
        from euler_amd.models.sharded_sage import ShardedSageTrainer

        if not g.comm:
            from euler_amd.models.sage_trainer import SageTrainer

            tr = SageTrainer.from_model(model, g.local, c.batch, keep_samples=False, **c.opt_kw())
            tr.device_trainer_kind = "graphsage"
            return tr

        tr = ShardedSageTrainer.from_model(model, g, c.batch, keep_samples=False, **c.opt_kw())
        tr.device_trainer_kind = "sharded_graphsage"
        return tr
    tr = ShardedFlowTrainer.from_model(model, g, c.batch, **c.opt_kw())
    tr.device_trainer_kind = "sharded_sage_flow"
    return tr


# ----------------------------------------------------------------------------------- predicates
def _cls(*names):
    """isinstance against classes resolved lazily (the model modules import torch layers)"""
    def pred(model):
        import euler_amd.models.unsupervised as U
        from euler_amd import solution as S

        space = {**vars(U), **vars(S)}
        return isinstance(model, tuple(space[n] for n in names))
    return pred


def _encoder(kind):
    def pred(model):
        from euler_amd.utils import encoders as enc

        return isinstance(getattr(model, "_encoder", None), getattr(enc, kind)) and hasattr(model, "label_idx")
    return pred


def _gnn_flow(*flows, sage_only=None):
    """supervised GNN models over one of ``flows`` (sage_only: True = every conv is SAGEConv,
    False = at least one is not, None = either)"""
    def pred(model):
        from euler_amd.convolution.convs import SAGEConv
        from euler_amd.dataflow import dataflows as D

        gnn = getattr(model, "gnn", None)
        if gnn is None or not hasattr(gnn, "feature_idx") or hasattr(model, "context_gnn"):
            return False
        if not hasattr(model, "label_idx") or not isinstance(getattr(gnn, "sampler", None),
                                                              tuple(getattr(D, f) for f in flows)):
            return False
        all_sage = all(isinstance(c, SAGEConv) for c in gnn.convs)
        return sage_only is None or all_sage == sage_only
    return pred


def _is_kg(model):
    return hasattr(model, "loss_scores")


def _is_graph_model(model):
    from euler_amd.mp_utils.models import GraphModel

    return isinstance(model, GraphModel) and hasattr(model, "pool") and hasattr(getattr(model, "gnn", None),
                                                                                 "encoder")


def _is_line1(model):
    from euler_amd.models.unsupervised import Line

    return isinstance(model, Line) and model._target_encoder is model._context_encoder


def _is_unsup_gnn(model):
    gnn = getattr(model, "gnn", None)
    return hasattr(model, "context_gnn") and gnn is not None and hasattr(gnn, "feature_idx")


ROW_SPARSE_AUTO_ROWS = 1 << 20


def row_sparse(c: Ctx, rows: int, sharded: bool = False) -> bool:
    """an id table trained row-sparse (ShardedTable + sparse optimizer) instead of in the
    dense flat buffer: ``row_sparse_tables`` True / False decides; "auto" (default) picks
    row-sparse for a sharded model or a table of >= 2^20 rows (per-step work then stays
    independent of |V|)"""
    v = c.params.get("row_sparse_tables", "auto")
    if isinstance(v, bool):
        return v
    return bool(sharded) or int(rows) >= ROW_SPARSE_AUTO_ROWS


# ----------------------------------------------------------------------------------- builders
@register("knowledge_graph", _is_kg)
def _kg(c: Ctx):
    # TransE / TransH / TransR / TransD / DistMult (EdgeEstimator): the triple table and the
    # corruption sampler in HBM, the model's own scores (models/kg_trainer.py)
    # row-sharded, row-sparse entity tables (RowSparseKGTrainer) for sharded models or on
    # request (``row_sparse_tables``): per-step work independent of |V|
    from euler_amd.models.kg_trainer import KGTrainer, RowSparseKGTrainer
    from euler_amd.parallel.embedding import ShardedEmbedding

    m = c.model
    edge_type = c.params.get("train_edge_type", getattr(m, "edge_type", -1))
    sharded = isinstance(m.entity_encoder, ShardedEmbedding)
    sparse = row_sparse(c, getattr(m.entity_encoder, "num", 0), sharded)
    if sparse and getattr(m, "l2_regular", False):
        # DistMult(l2_regular=True) regularises every entity row each step: only the dense
        # trainer computes that term; a sharded table or an explicit request cannot
        if sharded or c.params.get("row_sparse_tables", "auto") is True:
            raise ValueError("DistMult(l2_regular=True) needs the whole entity table every step: train it with "
                             "a dense (sharded=False) table and row_sparse_tables=False")
        import logging

        logging.getLogger(__name__).info("DistMult(l2_regular=True): dense KGTrainer (the L2 term spans every row)")
        sparse = False
    cls = RowSparseKGTrainer if sparse else KGTrainer
    return cls.from_model(m, c.batch, edge_type, seed=c.seed * 7919 + c.est.rank, device=c.est.device,
                          **c.opt_kw())


@register("graph_classification", _is_graph_model)
def _graph(c: Ctx):
    # GraphEstimator: graphs' node lists, labels and sparse feature ids in HBM, induced
    # blocks built on the device (models/graph_trainer.py)
    from euler_amd.models.graph_cls_trainer import GraphClsTrainer
    from euler_amd.models.graph_trainer import GraphTrainer

    p = c.params
    label = p["label"][0] if isinstance(p["label"], (list, tuple)) else p["label"]
    g = c.upload(node_type=-1)
    cls = GraphTrainer
    if p.get("graph_fused", True) and g.device.type == "cuda" and GraphClsTrainer.supports(c.model):
        # GIN / GraphGCN: one workgroup per graph, the whole step in two launches
        # (models/graph_cls_trainer.py); graphs beyond its limits take the generic step
        cls = GraphClsTrainer
    try:
        return cls(c.model, g, c.batch, label, int(p["num_classes"]), **c.opt_kw())
    except ValueError as e:
        if cls is GraphTrainer:
            raise
        import logging

        logging.getLogger(__name__).warning("fused graph-classification step not applicable (%s): generic step", e)
        return GraphTrainer(c.model, g, c.batch, label, int(p["num_classes"]), **c.opt_kw())


@register("graph_autoencoder", _cls("GraphAutoEncoder", "VariationalGraphAutoEncoder"))
def _gae(c: Ctx):
    # GAE / VGAE (sage / gcn encoder): roots, positives, negatives and the encoder's blocks
    # on the HBM graph (models/gae_trainer.py)
    from euler_amd.models.gae_trainer import GaeTrainer, VgaeTrainer
    from euler_amd.models.unsupervised import VariationalGraphAutoEncoder

    gnn = c.model.gnn
    g = c.upload(c.model.node_type, features=gnn.feature_idx, feature_dims=gnn.feature_dim)
    cls = VgaeTrainer if isinstance(c.model, VariationalGraphAutoEncoder) else GaeTrainer
    return cls(c.model, g, c.batch, **c.opt_kw())


@register("line_first_order", _is_line1)
def _line1(c: Ctx):
    # first-order LINE: one id table in both roles, autograd over the model's own lookups;
    # row-sharded / row-sparse (RowSparseIdPairTrainer) for a sharded table or on request
    from euler_amd.models.line_trainer import IdPairTrainer, RowSparseIdPairTrainer

    enc = c.model._target_encoder
    sharded = getattr(enc, "table", None) is not None
    rows = getattr(getattr(enc, "embedding", None), "num", 0)
    cls = RowSparseIdPairTrainer if row_sparse(c, rows, sharded) else IdPairTrainer
    return cls(c.model, c.upload(c.model.node_type), c.batch, **c.opt_kw())


@register("skipgram_walks", _cls("BaseNode2Vec", "Line"))
def _walks(c: Ctx):
    # DeepWalk / Node2Vec / LINE (second order): walks, pairs, negatives and the row-sparse
    # SGNS update on the HBM graph; with 2+ ranks the id tables are row-sharded (owner =
    # id % world) and every step's rows travel over fixed-capacity all-to-alls
    from euler_amd.models.deepwalk_step import DeepWalkEstimatorTrainer

    return DeepWalkEstimatorTrainer(c.model, c.upload(c.model.node_type), c.batch, seed=c.seed, **c.opt_kw())


@register("dgi", _cls("DGI"))
def _dgi(c: Ctx):
    # Deep Graph Infomax: roots, the fan-out tree and its shuffled view on the HBM graph
    from euler_amd.models.dgi_trainer import DgiTrainer

    ne = c.model._target_encoder._node_encoder
    g = c.upload(c.model.node_type, features=ne.feature_idx if ne.use_feature else (),
                 feature_dims=ne.feature_dim if ne.use_feature else ())
    return DgiTrainer(c.model, g, c.batch, **c.opt_kw())


@register("unsupervised_rgcn", _cls("UnsupervisedRGCN"))
def _urgcn(c: Ctx):
    # R-GCN over id embeddings: relation blocks and the model's own layers on the HBM graph;
    # the id table row-sparse (RowSparseRgcnTrainer) when large or on request
    from euler_amd.models.rgcn_trainer import RowSparseRgcnTrainer, UnsupRgcnTrainer

    emb = getattr(c.model.gnn._encoder, "embedding", None)
    cls = RowSparseRgcnTrainer if row_sparse(c, getattr(emb, "num", 0)) else UnsupRgcnTrainer
    return cls(c.model, c.upload(c.model.node_type), c.batch, **c.opt_kw())


@register("unsupervise_solution", _cls("UnsuperviseSolution"))
def _usol(c: Ctx):
    from euler_amd.models.encoder_trainer import UnsupSolutionTrainer

    ne = getattr(c.model.target_encoder, "_node_encoder", None)
    if ne is None or not getattr(ne, "use_feature", False):
        raise ValueError("device_graph=True trains UnsuperviseSolution over dense-feature SageEncoders")
    g = c.upload(features=ne.feature_idx, feature_dims=ne.feature_dim)
    return UnsupSolutionTrainer(c.model, g, c.batch, **c.opt_kw())


@register("supervise_solution", _cls("SuperviseSolution"))
def _sol(c: Ctx):
    # the solution API over a SageEncoder: tree draws, features and the encoder's
    # aggregators on the HBM graph (models/encoder_trainer.py SolutionTrainer)
    from euler_amd.models.encoder_trainer import SolutionTrainer

    ne = getattr(c.model.encoder, "_node_encoder", None)
    lab = c.model.get_label_fn
    if ne is None or not getattr(ne, "use_feature", False) or not hasattr(lab, "label_idx"):
        raise ValueError("device_graph=True trains SuperviseSolution over a dense-feature SageEncoder "
                         "with GetLabelFromFea labels")
    g = c.upload(features=ne.feature_idx, feature_dims=ne.feature_dim, label=lab.label_idx, label_dim=lab.label_dim)
    return SolutionTrainer.from_model(c.model, g, c.batch, **c.opt_kw())


@register("lgcn", _encoder("LGCEncoder"))
def _lgcn(c: Ctx):
    from euler_amd.models.encoder_trainer import LgcnTrainer

    enc = c.model._encoder
    g = c.upload(features=[enc.feature_idx], feature_dims=[enc.feature_dim], label=c.model.label_idx,
                 label_dim=c.model.label_dim)
    return LgcnTrainer.from_model(c.model, g, c.batch, **c.opt_kw())


def _is_scalable(model):
    from euler_amd.models.scalable_trainer import store_encoder_of
    from euler_amd.mp_utils.models import SuperviseModel

    return isinstance(model, SuperviseModel) and store_encoder_of(model) is not None


@register("scalable", _is_scalable)
def _scalable(c: Ctx):
    # ScalableSageEncoder / ScalableGCNEncoder (historical embeddings): the model's own
    # forward and store protocol with every graph query answered from HBM
    # (graph/device_scope.py, models/scalable_trainer.py)
    from euler_amd.models.scalable_trainer import ScalableTrainer, store_encoder_of

    m = c.model
    ne = store_encoder_of(m)._node_encoder
    names = [str(n) for n in ne.feature_idx] if ne.use_feature else []
    dims = [int(d) for d in ne.feature_dim] if ne.use_feature else []
    g = c.upload(features=names, feature_dims=dims, label=m.label_idx, label_dim=m.label_dim)
    cols, off = {}, 0
    for n, d in zip(names, dims):
        cols[n] = (off, d)
        off += d
    return ScalableTrainer(m, g, c.batch, cols, label=(m.label_idx, m.label_dim), **c.opt_kw())


@register("encoder_flow", _encoder("GCNEncoder"))
def _enc(c: Ctx):
    # GeniePath and other full-neighbour encoder models: hop sets and adjacencies built on
    # the device, the model's own encode (models/encoder_trainer.py)
    from euler_amd.models.encoder_trainer import EncoderFlowTrainer

    ne = c.model._encoder._node_encoder
    g = c.upload(features=ne.feature_idx if ne.use_feature else (), feature_dims=ne.feature_dim if ne.use_feature
                 else (), label=c.model.label_idx, label_dim=c.model.label_dim)
    return EncoderFlowTrainer.from_model(c.model, g, c.batch, **c.opt_kw())


def _supervised_upload(c: Ctx):
    gnn = c.model.gnn
    return c.upload(features=gnn.feature_idx, feature_dims=gnn.feature_dim, label=c.model.label_idx,
                    label_dim=c.model.label_dim)


@register("full_flow", _gnn_flow("GCNDataFlow", "FastGCNDataFlow", "LayerwiseDataFlow"))
def _full(c: Ctx):
    # GCN / APPNP / SGCN / TAGCN / ... : full-neighbourhood (or layer-sampled) blocks built on
    # the device; bounded capacities by default, grown and re-captured on overflow
    from euler_amd.models.full_trainer import FullFlowTrainer
    from euler_amd.models.gcn_trainer import GcnTrainer

    g = _supervised_upload(c)
    caps = c.params.get("device_flow_caps", "bounded")
    if c.params.get("gcn_fused", True) and GcnTrainer.supports(c.model, g, c.batch):
        # SupervisedGCN-shaped: the fused hand-written step (models/gcn_trainer.py)
        return GcnTrainer.from_model(c.model, g, c.batch, caps=caps, **c.opt_kw())
    return FullFlowTrainer.from_model(c.model, g, c.batch, **c.opt_kw(), caps=caps)


@register("sampled_flow_other_conv", _gnn_flow("SageDataFlow", sage_only=False))
def _sampled_other(c: Ctx):
    # other convolutions on the sampled SageDataFlow: fixed-fanout blocks on the device
    from euler_amd.models.full_trainer import FullFlowTrainer

    return FullFlowTrainer.from_model(c.model, _supervised_upload(c), c.batch, **c.opt_kw())


@register("unsupervised_graphsage", _is_unsup_gnn)
def _unsup_sage(c: Ctx):
    from euler_amd.models.sage_tower import UnsupSageTrainer

    gnn = c.model.gnn
    g = c.upload(features=gnn.feature_idx, feature_dims=gnn.feature_dim)
    return UnsupSageTrainer.from_model(c.model, g, c.batch, **c.opt_kw())


@register("graphsage", _gnn_flow("SageDataFlow", sage_only=True))
def _sage(c: Ctx):
    # SupervisedGraphSage: the fused tree-step kernels (models/sage_trainer.py)
    from euler_amd.models.sage_trainer import SageTrainer

    return SageTrainer.from_model(c.model, _supervised_upload(c), c.batch, keep_samples=False, **c.opt_kw())
