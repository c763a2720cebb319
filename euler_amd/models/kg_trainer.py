"""Device-path training of the knowledge-graph embedding models (TransE / TransH / TransR /
TransD / DistMult) under ``EdgeEstimator(device_graph=True)``.

Reference: ``euler_estimator/python/edge_estimator.py:27-72`` (``sample_edge(batch,
train_edge_type)`` batches), ``examples/TransX/transX.py:63-145`` (relation id = the dense
edge feature ``id``, ``num_negs`` corruptions from ``sample_node(node_type)``, margin loss
against the mean corrupted score).

The engine path draws every batch on the CPU engine (two GQL queries and a feature lookup
per step) and copies it to the GPU.  Here the triple table lives in HBM and the step is
device-only:

* :class:`TripleTable` — every edge of the training edge type (src id, dst id, relation
  id from the edge feature) plus two Walker alias tables: edges by edge weight (the
  reference ``sample_edge``) and candidate corruptions by node weight over the model's
  ``node_type`` (the reference ``sample_node``); draws are the ``alias_sample`` kernel on
  Philox streams (seed, counter, stream) — stream 1 triples, stream 2 corruptions;
* the model's own ``loss_scores`` (the fused ``kg_score`` kernels for TransE / DistMult,
  the torch compositions for the projected variants), the metric (MRR / MR / hit@10 of the
  positive among its corruptions) accumulated on the device;
* one flat optimizer launch over every table and parameter (``models/captured.py``),
  several steps per hipGraph replay.
"""
from __future__ import annotations

import numpy as np
import torch

from euler_amd.graph.device_graph import build_alias_table
from euler_amd.models.captured import CapturedTrainer
from euler_amd.ops._native import hip, use_hip

__all__ = ["TripleTable", "KGTrainer", "RowSparseKGTrainer"]


class _Alias:
    def __init__(self, weights, device):
        w = np.asarray(weights, np.float64)
        if w.size == 0 or not (w > 0).any():
            raise ValueError("nothing to sample (empty set or all weights zero)")
        prob, alias = build_alias_table(w)
        self.prob = torch.from_numpy(prob).to(device)
        self.alias = torch.from_numpy(alias).to(device)


class TripleTable:
    """Training triples + the edge / corruption samplers in HBM, keyed by a device
    (seed, counter) pair."""

    def __init__(self, src, dst, rel, edge_weights, cand_ids, cand_weights, seed=0, device="cuda"):
        self.device = torch.device(device)
        self.src = torch.as_tensor(np.asarray(src, np.int64)).to(self.device)
        self.dst = torch.as_tensor(np.asarray(dst, np.int64)).to(self.device)
        self.rel = torch.as_tensor(np.asarray(rel, np.int64)).to(self.device)
        self.edges = _Alias(edge_weights, self.device)
        self.cand = torch.as_tensor(np.asarray(cand_ids, np.int64)).to(self.device)
        self.negs = _Alias(cand_weights, self.device)
        self.rng = torch.tensor([int(seed), 0], dtype=torch.int64, device=self.device)
        self._cpu_gen = torch.Generator(device="cpu")
        self._cpu_gen.manual_seed(int(seed))

    @classmethod
    def from_engine(cls, edge_type, node_type=-1, relation_feature="id", engine=None, seed=0, device="cuda"):
        """every edge of ``edge_type`` of the engine's local graph; relation ids from the dense
        edge feature ``relation_feature``; corruption candidates = nodes of ``node_type``"""
        import euler_amd.ops.graph_api as ge
        from euler_amd.ops import base

        eng = engine if engine is not None else base.get_engine()
        et = -1 if edge_type in (None, -1, "-1") else int(np.asarray(ge.get_edge_type_id(edge_type)).reshape(-1)[0])
        src, dst, w, feat = eng.export_edges(et, "dense_" + str(relation_feature), 1)
        ids, types, nw = eng.export_nodes()
        nt = -1 if node_type in (None, -1, "-1") else int(np.asarray(ge.get_node_type_id(node_type)).reshape(-1)[0])
        keep = np.ones(len(ids), bool) if nt < 0 else np.asarray(types) == nt
        rel = np.asarray(feat).reshape(-1).astype(np.int64)
        return cls(np.asarray(src).astype(np.int64), np.asarray(dst).astype(np.int64), rel, np.asarray(w),
                   np.asarray(ids)[keep].astype(np.int64), np.asarray(nw)[keep], seed=seed, device=device)

    # ------------------------------------------------------------------ randomness
    def advance(self, inc: int = 1):
        if use_hip(self.rng):
            hip().rng_advance(self.rng, int(inc))
        else:
            self.rng[1] += inc

    def reseed_cpu(self):
        self._cpu_gen.manual_seed((int(self.rng[0]) * 1000003 + int(self.rng[1])) % (1 << 63))

    def _draw(self, a: _Alias, count: int, stream: int) -> torch.Tensor:
        if use_hip(a.prob):
            return hip().alias_sample(a.prob, a.alias, None, int(count), self.rng, int(stream)).long()
        n = a.prob.numel()
        k = torch.randint(0, n, (count,), generator=self._cpu_gen)
        u = torch.rand(count, generator=self._cpu_gen)
        return torch.where(u < a.prob[k], k, a.alias[k].long())

    def sample_triples(self, count: int):
        """(src, rel, dst) [count] by edge weight (reference sample_edge)"""
        e = self._draw(self.edges, count, 1)
        return self.src[e], self.rel[e], self.dst[e]

    def sample_corruptions(self, count: int) -> torch.Tensor:
        """[count] node ids of the candidate type by node weight (reference sample_node)"""
        return self.cand[self._draw(self.negs, count, 2)]


class KGTrainer(CapturedTrainer):
    def __init__(self, model, table: TripleTable, batch_size, optimizer="adam", learning_rate=0.01):
        if not hasattr(model, "loss_scores"):
            raise ValueError("KGTrainer trains the TransX family (models/knowledge_graph.py)")
        from euler_amd.utils.layers import Embedding

        if not isinstance(model.entity_encoder, Embedding):
            raise ValueError("device_graph=True needs the dense (non-sharded) entity table")
        self.table = table
        self.B = int(batch_size)
        self.metric_name = model.metric_name
        self.msum = torch.zeros(2, dtype=torch.float64, device=table.device)  # metric sum, count
        super().__init__(model, table, table.device, optimizer, learning_rate)

    @classmethod
    def from_model(cls, model, batch_size, edge_type, seed=0, device="cuda", optimizer="adam", learning_rate=0.01):
        table = TripleTable.from_engine(edge_type, node_type=model.node_type, seed=seed, device=device)
        return cls(model, table, batch_size, optimizer=optimizer, learning_rate=learning_rate)

    def _forward_loss(self):
        self._draw()
        t = self.table
        src, rel, dst = t.sample_triples(self.B)
        neg = t.sample_corruptions(self.B * self.model.num_negs).view(self.B, self.model.num_negs)
        src, rel, dst = src.view(-1, 1), rel.view(-1, 1), dst.view(-1, 1)
        loss, pos, neg_s = self.model.loss_scores(src, dst, neg, rel)
        with torch.no_grad():
            r = (neg_s >= pos).sum(-1).double()  # 0 = best (utils/metrics.py _ranks)
            if self.metric_name == "mrr":
                v = (1.0 / (r + 1)).sum()
            elif self.metric_name == "mr":
                v = (r + 1).sum()
            else:  # hit10
                v = (r < 10).double().sum()
            self.msum += torch.stack([v, torch.full_like(v, float(r.numel()))])
        self._samples = (src, rel, dst, neg)
        return loss

    def metric(self) -> float:
        s, n = self.msum.tolist()
        return s / max(n, 1.0)

    def reset_metric(self):
        self.msum.zero_()


# ---------------------------------------------------------------------------- row-sparse tables
class RowSparseKGTrainer(KGTrainer):
    """KGTrainer with the per-entity tables (``entity_encoder``, TransD's
    ``entity_transfer``) held as row-sharded, row-sparse :class:`ShardedTable` s instead of
    FlatParams: per step only the touched rows (the batch's src, dst and corruptions,
    de-duplicated on the device) are gathered — from their owner ranks over one fixed-
    capacity all-to-all when world > 1 — and updated by the row-sparse Adam / Adagrad /
    SGD kernel (optim.hip sparse_optim).  Per-step work is independent of |V|; the
    relation tables and projections stay in the flat buffer (dense, all-reduced).

    The model scores the step on the gathered rows: the trainer passes them with src /
    dst / corruption POSITIONS into them (``loss_scores(..., rows=)``), so TransE /
    DistMult run the fused kg_fwd / kg_bwd kernels straight on the gathered rows and the
    row gradients come out per gathered row, ready for the owners' update; the projected
    variants run their torch compositions on the same rows.

    Table ownership: row ``r`` lives on rank ``r % world`` (ShardedEmbedding's layout), so
    a ``sharded=True`` model's shard — or any model's table on one rank — IS the trainer's
    table (the module's weight is rebound to it: no second copy).  A dense model under 2+
    ranks keeps its full table, written from the shards when training ends.  Checkpoints
    are per-rank shard files of the rows and their optimizer slots (parallel/shard_io.py).

    Reference: tf_euler/python/utils/embedding.py:24-68 (mod-partitioned embedding
    variables, sparse updates), examples/TransX/transX.py:63-145."""

    TABLES = ("entity_encoder", "entity_transfer")

    def __init__(self, model, table, batch_size, optimizer="adam", learning_rate=0.01, group=None):
        from euler_amd.parallel.sparse_table import ShardedTable

        if not hasattr(model, "loss_scores"):
            raise ValueError("RowSparseKGTrainer trains the TransX family (models/knowledge_graph.py)")
        if getattr(model, "l2_regular", False):
            # DistMult's L2 term covers the WHOLE entity table every step (distmult.py): a
            # row-sparse step touches only the batch's rows and cannot compute it
            raise ValueError("row-sparse entity tables cannot train DistMult(l2_regular=True): its L2 term spans "
                             "every entity row; use the dense KGTrainer (row_sparse_tables=False)")
        self.table = table
        self.B = int(batch_size)
        self.metric_name = model.metric_name
        self.msum = torch.zeros(2, dtype=torch.float64, device=table.device)
        self.tables, self._mods, self._bound = {}, {}, {}
        opt = optimizer if optimizer in ("adam", "adagrad", "sgd") else "adam"
        names = {id(p): k for k, p in model.named_parameters()}
        self._keys = {}
        for name in self.TABLES:
            mod = getattr(model, name, None)
            if mod is None:
                continue
            num, dim = int(mod.num), int(mod.dim)
            t = ShardedTable(num, dim, table.device, group, opt, learning_rate, init=None)
            w = mod.weight
            self._keys[name] = names[id(w)]
            with torch.no_grad():
                if getattr(mod, "world", 1) > 1 or w.shape[0] == t.weight.shape[0]:
                    t.weight.copy_(w.detach().to(t.weight))  # already this rank's rows (r % world == rank)
                    w.data = t.weight                       # the module's table IS the trainer's shard
                    self._bound[name] = True
                else:
                    t.weight.copy_(w.detach()[t.global_ids().to(w.device)].to(t.weight))
                    self._bound[name] = False
            w.requires_grad_(False)  # row-sparse: never in the flat buffer, no autograd into it
            self.tables[name] = t
            self._mods[name] = mod
        if "entity_encoder" not in self.tables:
            raise ValueError("the model has no entity_encoder table")
        CapturedTrainer.__init__(self, model, table, table.device, optimizer, learning_rate)
        self.world = self.tables["entity_encoder"].world

    @classmethod
    def from_model(cls, model, batch_size, edge_type, seed=0, device="cuda", optimizer="adam", learning_rate=0.01):
        table = TripleTable.from_engine(edge_type, node_type=model.node_type, seed=seed, device=device)
        return cls(model, table, batch_size, optimizer=optimizer, learning_rate=learning_rate)

    # ------------------------------------------------------------------ step
    def _step(self, grad_sync=None):
        from euler_amd.ops.gnn_ops import unique_first_padded

        self._draw()
        t = self.table
        K = self.model.num_negs
        src, rel, dst = t.sample_triples(self.B)
        neg = t.sample_corruptions(self.B * K)
        num = self.tables["entity_encoder"].num_rows
        ids = torch.cat([src, dst, neg])
        ids = torch.where((ids < 0) | (ids >= num), torch.full_like(ids, num - 1), ids)
        uids, inv, _ = unique_first_padded(ids)
        rows, handles = {}, {}
        for name, tab in self.tables.items():
            r, h = tab.lookup_static(uids, trash_row=True)
            leaf = r.detach().requires_grad_(True)
            rows[name] = leaf
            handles[name] = (tab, h, leaf)
        # every table shares one id set: the positions of the step's ids in the gathered rows
        p = handles["entity_encoder"][1].pos[inv]
        ps, pd, pn = p[: self.B].view(-1, 1), p[self.B: 2 * self.B].view(-1, 1), p[2 * self.B:].view(self.B, K)
        self.opt.zero_grad()
        loss, pos, neg_s = self.model.loss_scores(ps, pd, pn, rel.view(-1, 1), rows=rows)
        loss.backward()
        with torch.no_grad():
            r = (neg_s >= pos).sum(-1).double()
            v = {"mrr": (1.0 / (r + 1)).sum(), "mr": (r + 1).sum()}.get(self.metric_name, (r < 10).double().sum())
            self.msum += torch.stack([v, torch.full_like(v, float(r.numel()))])
        scale = 1.0
        if grad_sync is not None:
            s = grad_sync(self.flat.grad)
            scale = 1.0 if s is None else float(s)
        self.opt.step(scale)
        for tab, h, leaf in handles.values():
            g = leaf.grad
            if g is None:
                g = torch.zeros_like(leaf)
            n = g.shape[0] - 1  # the trash row (ids a capacity overflow dropped) is not applied
            # the dense buffer's all-reduce averages over ranks; the owners sum the ranks'
            # row gradients, so they are scaled to the same mean here
            tab.apply_static(h, g[:n] / self.world if self.world > 1 else g[:n])
        self._samples = (src.view(-1, 1), rel.view(-1, 1), dst.view(-1, 1), neg.view(self.B, K))
        self.loss_out.copy_(loss.detach())
        return self.loss_out

    # ------------------------------------------------------------------ state
    def _full_table(self, tab):
        return tab.full()

    def logical_keys(self):
        return set(self.model.state_dict())

    def state_dict(self):
        """model-named state with the WHOLE tables (tests / export; a collective under 2+
        ranks — checkpoints use :meth:`checkpoint_shards` instead)"""
        sd = {k: v.detach().cpu() for k, v in self.model.state_dict().items()}
        for name, tab in self.tables.items():
            sd[self._keys[name]] = self._full_table(tab).cpu()
        return sd

    def checkpoint_model_state(self):
        """the model's state without the row-sharded tables (those go to the shard files)"""
        skip = set(self._keys.values())
        return {k: v.detach().cpu() for k, v in self.model.state_dict().items() if k not in skip}

    def checkpoint_shards(self, ckpt_path):
        return {self._keys[name]: tab.save_shard(ckpt_path, self._keys[name]) for name, tab in self.tables.items()}

    def load_shards(self, dirname, metas):
        for name, tab in self.tables.items():
            key = self._keys[name]
            if key in metas:
                tab.load_shard(dirname, metas[key], name=key)

    def logical_params(self):
        sd = {k: v.detach().clone() for k, v in self.model.state_dict().items()}
        for name, tab in self.tables.items():
            sd[self._keys[name]] = self._full_table(tab)
        return sd

    def load_logical(self, sd):
        with torch.no_grad():
            own = self.model.state_dict()
            tab_keys = {self._keys[n]: n for n in self.tables}
            for k, v in sd.items():
                if k in own and k not in tab_keys:
                    own[k].copy_(torch.as_tensor(v).to(own[k]))
            for key, name in tab_keys.items():
                if key in sd:
                    self.tables[name].load(sd[key])

    def write_to_model(self, model):
        """bound tables are the model's own; a dense model under 2+ ranks gets the gathered
        tables (a collective)"""
        for name, tab in self.tables.items():
            if self._bound[name] and model is self.model:
                continue
            mod = self._mods[name]
            with torch.no_grad():
                w = mod.weight if model is self.model else model.state_dict()[self._keys[name]]
                w.copy_((tab.weight if w.shape[0] == tab.weight.shape[0] else self._full_table(tab)).to(w))
        if model is not self.model:
            skip = set(self._keys.values())
            model.load_state_dict({k: v for k, v in self.model.state_dict().items() if k not in skip}, strict=False)

    def finish(self):
        """end of training: every table in the model's own modules (engine-path evaluate /
        infer and the user's model see them), trainable again"""
        self.write_to_model(self.model)
        for mod in self._mods.values():
            mod.weight.requires_grad_(True)

    def trainer_state(self):
        """flat-buffer slots, step and sampler counter (the tables' rows and slots are in
        the shard files)"""
        st = super().trainer_state()
        st["table_steps"] = {name: int(tab.step.item()) for name, tab in self.tables.items()}
        return st

    def load_trainer_state(self, st):
        super().load_trainer_state(st)
        for name, tab in self.tables.items():
            if name in st:  # an older checkpoint: whole slot tensors of the same layout
                tab.load_slot_state(st.get(name))
            stp = (st.get("table_steps") or {}).get(name)
            if stp is not None:
                tab.step.fill_(int(stp))

    def dp_state_tensors(self):
        ts = list(super().dp_state_tensors())
        for tab in self.tables.values():
            ts += tab.state_tensors()
        return ts
