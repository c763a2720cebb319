"""Node encoders (reference ``tf_euler/python/utils/encoders.py:32-922``).

Every encoder maps a 1-D batch of node ids to embeddings.  Graph access (sampling,
feature fetch) goes through :mod:`euler_amd.ops.graph_api` -- the C++ engine, local or
sharded/remote -- and the dense math runs wherever the module's parameters live
(``model.to('cuda')`` puts it on the MI355X; gathers/segment reductions then run on the
gfx950 kernels of :mod:`euler_amd.ops.mp_ops`).

Store-based encoders (``ScalableGCNEncoder`` / ``ScalableSageEncoder``) keep per-layer
embedding stores and gradient stores as device buffers.  TF wired the store update /
gradient accumulation through extra session ops; here the training loop calls
``encoder.after_backward()`` after ``loss.backward()`` (the estimators do this for every
sub-module that defines it), and the store loss is returned as ``encoder.store_loss``
to be added to the objective (the reference minimised it with a second Adam; adding
it to the main loss drives the same gradients through the shared optimizer).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from euler_amd.ops import graph_api as G
from euler_amd.parallel.replicated import apply_replicated, sync_group
from euler_amd.utils import aggregators as dense_aggs
from euler_amd.utils import sparse_aggregators
from euler_amd.utils.layers import (AttLayer, Dense, Embedding, HashEmbedding, HashSparseEmbedding, SparseEmbedding)

__all__ = ["ShallowEncoder", "GCNEncoder", "GenieEncoder", "ScalableGCNEncoder", "SageEncoder",
           "ShuffleSageEncoder", "SageEncoderNew", "ScalableSageEncoder", "LayerEncoder", "SparseSageEncoder",
           "LGCEncoder", "module_device"]


def module_device(m: nn.Module) -> torch.device:
    for b in m.buffers():
        return b.device
    for p in m.parameters():
        return p.device
    return getattr(m, "_device_hint", torch.device("cpu"))


def _shaped(inputs, out):
    """reshape [n, d] -> inputs.shape + [d] (the reference's output_shape idiom)."""
    shape = tuple(torch.as_tensor(inputs).shape)
    return out.reshape(*shape, out.shape[-1])


def _as_list(x, n=None):
    if isinstance(x, (list, tuple)):
        return list(x)
    return [x] * (n if n is not None else 1)


class ShallowEncoder(nn.Module):
    """id embedding (+) dense features (+) sparse-feature embedding bags
    (reference encoders.py:32-171)."""

    def __init__(self, dim=None, feature_idx="f1", feature_dim=0, max_id=-1, sparse_feature_idx=-1,
                 sparse_feature_max_id=-1, embedding_dim=16, use_hash_embedding=False, combiner="concat", **kwargs):
        super().__init__()
        if combiner not in ("add", "concat"):
            raise ValueError("combiner must be 'add' or 'concat'.")
        if combiner == "add" and dim is None:
            raise ValueError("add must be used with dim provided.")
        use_feature = feature_idx != -1
        use_id = max_id != -1
        use_sparse = sparse_feature_idx != -1
        if use_feature:
            feature_idx = _as_list(feature_idx)
            feature_dim = _as_list(feature_dim)
            if len(feature_idx) != len(feature_dim):
                raise ValueError("feature_dim must be the same length as feature_idx. idx:%s, dim:%s"
                                 % (feature_idx, feature_dim))
        if use_sparse:
            sparse_feature_idx = _as_list(sparse_feature_idx)
            sparse_feature_max_id = _as_list(sparse_feature_max_id)
            if len(sparse_feature_idx) != len(sparse_feature_max_id):
                raise ValueError("sparse_feature_idx must be the same length as sparse_feature_max_id.")
        n_emb = (1 if use_id else 0) + (len(sparse_feature_idx) if use_sparse else 0)
        if combiner == "add":
            embedding_dim = dim
        if n_emb:
            embedding_dim = _as_list(embedding_dim, n_emb)
            use_hash_embedding = _as_list(use_hash_embedding, n_emb)
            if len(embedding_dim) != n_emb:
                raise ValueError("length of embedding_dim must be int(use_id) + len(sparse_feature_idx)")
            if len(use_hash_embedding) != n_emb:
                raise ValueError("length of use_hash_embedding must be int(use_id) + len(sparse_feature_idx)")
        self.dim, self.use_id, self.use_feature, self.use_sparse_feature = dim, use_id, use_feature, use_sparse
        self.combiner = combiner
        self.feature_idx, self.feature_dim = feature_idx, feature_dim
        self.sparse_feature_idx, self.sparse_feature_max_id = sparse_feature_idx, sparse_feature_max_id
        self.embedding_dim = embedding_dim
        # follows .to(device) even when the encoder has no parameters (features only)
        self.register_buffer("_device_anchor", torch.empty(0), persistent=False)
        if dim and (combiner == "concat" or use_feature):  # only when forward() uses it
            self.dense = Dense(dim, use_bias=False)
        ed, uh = (list(embedding_dim), list(use_hash_embedding)) if n_emb else ([], [])
        if use_id:
            self.embedding = (HashEmbedding if uh[0] else Embedding)(max_id + 1, ed[0])
            ed, uh = ed[1:], uh[1:]
        if use_sparse:
            self.sparse_embeddings = nn.ModuleList([
                (HashSparseEmbedding if h else SparseEmbedding)(m + 1, d)
                for m, d, h in zip(sparse_feature_max_id, ed, uh)])

    @property
    def output_dim(self):
        if self.dim is not None:
            return self.dim
        out = 0
        if self.use_feature:
            out += sum(self.feature_dim)
        if self.use_id or self.use_sparse_feature:
            out += sum(self.embedding_dim)
        return out

    def forward(self, inputs):
        shape = tuple(torch.as_tensor(inputs).shape)
        ids = torch.as_tensor(inputs).reshape(-1)
        dev = module_device(self)
        embs = []
        if self.use_id:
            embs.append(self.embedding(ids))
        if self.use_feature:
            # a device-graph scope answers from HBM with device ids (no host round trip)
            q = ids if G.device_scope_active() else ids.cpu()
            feats = torch.cat(G.get_dense_feature(q, self.feature_idx, self.feature_dim), -1).to(dev)
            if self.combiner == "add":
                feats = self.dense(feats)
            embs.append(feats)
        if self.use_sparse_feature:
            defaults = [m + 1 for m in self.sparse_feature_max_id]
            sps = G.get_sparse_feature(ids.cpu(), self.sparse_feature_idx, default_values=defaults)
            embs.extend(e(sp) for e, sp in zip(self.sparse_embeddings, sps))
        if self.combiner == "add":
            emb = embs[0]
            for e in embs[1:]:
                emb = emb + e
        else:
            emb = torch.cat(embs, -1)
            if self.dim:
                emb = self.dense(emb)
        return emb.reshape(*shape, self.output_dim)


class GCNEncoder(nn.Module):
    """Full-neighbour multi-hop GCN with sparse aggregators (reference encoders.py:174-235)."""

    def __init__(self, metapath, dim, aggregator="mean", feature_idx=-1, feature_dim=0, max_id=-1, use_id=False,
                 sparse_feature_idx=-1, sparse_feature_max_id=-1, embedding_dim=16, use_hash_embedding=False,
                 use_residual=False, head_num=4, **kwargs):
        super().__init__()
        self.metapath = metapath
        self.num_layers = len(metapath)
        if isinstance(head_num, int):
            self.head_num = [head_num] * self.num_layers
        elif isinstance(head_num, list):
            assert len(head_num) == self.num_layers
            self.head_num = head_num
        else:
            raise ValueError("head_num error: expect int or list, got {}".format(head_num))
        self.use_residual = use_residual
        self._node_encoder = ShallowEncoder(
            dim=dim if use_residual else None, feature_idx=feature_idx, feature_dim=feature_dim,
            max_id=max_id if use_id else -1, sparse_feature_idx=sparse_feature_idx,
            sparse_feature_max_id=sparse_feature_max_id, embedding_dim=embedding_dim,
            use_hash_embedding=use_hash_embedding, combiner="add" if use_residual else "concat")
        cls = sparse_aggregators.get(aggregator)
        self.aggregators = nn.ModuleList([
            cls(dim, activation=torch.relu if layer < self.num_layers - 1 else None, head_num=self.head_num[layer])
            for layer in range(self.num_layers)])

    def node_encoder(self, inputs):
        return self._node_encoder(inputs)

    def _propagate(self, hidden, adjs):
        for layer in range(self.num_layers):
            agg = self.aggregators[layer]
            nxt = []
            for hop in range(self.num_layers - layer):
                h = agg((hidden[hop], hidden[hop + 1], adjs[hop]))
                nxt.append(hidden[hop] + h if self.use_residual else h)
            hidden = nxt
        return hidden

    def encode(self, hidden, adjs):
        """root embeddings from the per-hop node embeddings and the hop adjacencies (the
        device path passes -1-padded sets and adjacencies: models/encoder_trainer.py)"""
        return self._propagate(hidden, adjs)[0]

    def forward(self, inputs):
        nodes, adjs = G.get_multi_hop_neighbor(inputs, self.metapath)
        return _shaped(inputs, self.encode([self.node_encoder(n) for n in nodes], adjs))


class GenieEncoder(GCNEncoder):
    """GeniePath: per-depth projections fed through an LSTM over depth
    (reference encoders.py:238-291)."""

    def __init__(self, metapath, dim, aggregator="attention", *args, **kwargs):
        super().__init__(metapath, dim, aggregator, *args, **kwargs)
        self.dim = dim
        self.depth_fc = nn.ModuleList([Dense(dim) for _ in range(self.num_layers + 1)])
        self.lstm = nn.LSTM(dim, dim, batch_first=True)

    def forward(self, inputs):
        nodes, adjs = G.get_multi_hop_neighbor(inputs, self.metapath)
        return _shaped(inputs, self.encode([self.node_encoder(n) for n in nodes], adjs))

    def encode(self, hidden, adjs):
        h_t = [self.depth_fc[0](hidden[0])]
        for layer in range(self.num_layers):
            agg = self.aggregators[layer]
            nxt = []
            for hop in range(self.num_layers - layer):
                h = agg((hidden[hop], hidden[hop + 1], adjs[hop]))
                nxt.append(hidden[hop] + h if self.use_residual else h)
            hidden = nxt
            h_t.append(self.depth_fc[layer + 1](hidden[0]))
        seq = torch.stack(h_t, 1)  # [B, L+1, dim]
        out, _ = self.lstm(seq)
        return out[:, 0, :]


class _StoreMixin:
    """Stale-embedding stores + gradient stores (reference encoders.py:313-408, 657-748).

    Data parallel: by default every rank keeps a full replica and applies every rank's
    writes (parallel/replicated.py); :meth:`use_sharded_stores` switches to row-sharded
    stores (parallel/sharded_store.py: row r on rank r % world, reads and writes over
    all-to-all) when a replica per rank is too large."""

    def _build_stores(self, dims, max_id, init_maxval):
        g = torch.Generator().manual_seed(1)
        for i, d in enumerate(dims, 1):
            self.register_buffer("store_layer_%d" % i, torch.rand(max_id + 2, d, generator=g) * init_maxval,
                                 persistent=False)
            self.register_buffer("gradient_store_layer_%d" % i, torch.zeros(max_id + 2, d), persistent=False)
        self._num_stores = len(dims)
        self._n_store_rows = max_id + 2
        self._sharded = None  # [(store, gradient store)] when row-sharded
        self._pending = None
        self.store_loss = None

    def stores(self, i):
        return getattr(self, "store_layer_%d" % (i + 1))

    def gradient_stores(self, i):
        return getattr(self, "gradient_store_layer_%d" % (i + 1))

    def use_sharded_stores(self, group=None):
        """Replace the replicated stores by row-sharded ones (every rank must call this;
        the initial rows are taken from this rank's replica, which starts identical on
        every rank)."""
        from euler_amd.parallel.sharded_store import ShardedRowStore

        shards = []
        for i in range(self._num_stores):
            full, gfull = self.stores(i), self.gradient_stores(i)
            n, d = full.shape
            st = ShardedRowStore(n, d, full.device, group, init=lambda ids, f=full: f[ids])
            gs = ShardedRowStore(n, d, full.device, group, init=lambda ids, f=gfull: f[ids])
            shards.append((st, gs))
            # drop the replicas (keep empty placeholders so .to() / state handling still work)
            setattr(self, "store_layer_%d" % (i + 1), torch.empty(0, d, device=full.device))
            setattr(self, "gradient_store_layer_%d" % (i + 1), torch.empty(0, d, device=full.device))
        self._sharded = shards
        self.store_group = group
        return self

    def _store_device(self):
        return self._sharded[0][0].device if self._sharded else self.stores(0).device

    def _rows(self, ids):
        ids = torch.as_tensor(ids).to(self._store_device()).long()
        n = self._n_store_rows
        return torch.where((ids < 0) | (ids >= n), torch.full_like(ids, n - 1), ids)

    def _read(self, i, rows, grad=False):
        if self._sharded:
            return self._sharded[i][1 if grad else 0].read(rows)
        return (self.gradient_stores(i) if grad else self.stores(i))[rows]

    def _lookup_neighbors(self, layer, neighbor):
        rows = self._rows(neighbor)
        leaf = self._read(layer, rows.reshape(-1)).reshape(tuple(rows.shape) + (-1,))
        return leaf.detach().requires_grad_(self.training)

    def _finish_training_forward(self, node, node_embeddings, neighbor, neigh_leaves):
        rows = self._rows(node)
        losses = []
        for i in range(self._num_stores):
            g = self._read(i, rows.reshape(-1), grad=True).reshape(tuple(rows.shape) + (-1,)).clone()
            if not self._sharded:
                # the other ranks zero these rows in after_backward (sharded: the owner does)
                self.gradient_stores(i).index_fill_(0, rows.reshape(-1), 0.0)
            losses.append((node_embeddings[i] * g.to(node_embeddings[i].dtype)).sum())
        self.store_loss = sum(losses) if losses else torch.zeros((), device=rows.device)
        self._pending = (rows, [e.detach() for e in node_embeddings[:self._num_stores]], self._rows(neighbor),
                         neigh_leaves)

    @torch.no_grad()
    def after_backward(self):
        """Write fresh node embeddings into the stores and accumulate neighbour grads."""
        if self._pending is None:
            return
        rows, embs, nrows, leaves = self._pending
        if self._sharded:
            for i, (st, gs) in enumerate(self._sharded):
                gs.write(rows, None, "zero")
                st.write(rows, embs[i], "copy")
            for i, leaf in enumerate(leaves):
                grad = leaf.grad if leaf.grad is not None else torch.zeros_like(leaf)
                self._sharded[i][1].write(nrows, grad.reshape(nrows.numel(), -1).float(), "add")
            self._pending = None
            return
        # data parallel: every rank applies every rank's writes (parallel/replicated.py), so
        # the replicas behave like the reference's shared PS stores
        group = getattr(self, "store_group", None)
        synced = sync_group(group) is not None
        for i in range(self._num_stores):
            if synced:
                apply_replicated(self.gradient_stores(i), rows, None, "zero", group)
            apply_replicated(self.stores(i), rows, embs[i], "copy", group)
        for i, leaf in enumerate(leaves):
            grad = leaf.grad if leaf.grad is not None else torch.zeros_like(leaf)
            if leaf.grad is not None or synced:  # ranks must join the same collectives
                apply_replicated(self.gradient_stores(i), nrows, grad.reshape(nrows.numel(), -1).float(), "add",
                                 group)
        self._pending = None


class ScalableGCNEncoder(_StoreMixin, GCNEncoder):
    def __init__(self, edge_type, num_layers, dim, aggregator="mean", feature_idx=-1, feature_dim=0, max_id=-1,
                 use_id=False, sparse_feature_idx=-1, sparse_feature_max_id=-1, embedding_dim=16,
                 use_hash_embedding=False, use_residual=False, store_learning_rate=0.001, store_init_maxval=0.05,
                 **kwargs):
        super().__init__([edge_type] * num_layers, dim, aggregator, feature_idx, feature_dim, max_id, use_id,
                         sparse_feature_idx, sparse_feature_max_id, embedding_dim, use_hash_embedding, use_residual)
        self.dim, self.edge_type, self.max_id = dim, edge_type, max_id
        self.store_learning_rate = store_learning_rate
        self._build_stores([dim] * (num_layers - 1), max_id, store_init_maxval)

    def forward(self, inputs):
        if not self.training:
            return GCNEncoder.forward(self, inputs)
        (node, neighbor), (adj,) = G.get_multi_hop_neighbor(inputs, [self.edge_type])
        node_emb = self.node_encoder(node)
        neigh_emb = self.node_encoder(neighbor)
        node_embs, leaves = [], []
        for layer in range(self.num_layers):
            h = self.aggregators[layer]((node_emb, neigh_emb, adj))
            node_emb = node_emb + h if self.use_residual else h
            node_embs.append(node_emb)
            if layer < self.num_layers - 1:
                neigh_emb = self._lookup_neighbors(layer, neighbor)
                leaves.append(neigh_emb)
        self._finish_training_forward(node, node_embs, neighbor, leaves)
        return _shaped(inputs, node_emb)


class SageEncoder(nn.Module):
    """GraphSAGE over fixed fan-out samples (reference encoders.py:411-493)."""

    @staticmethod
    def create_aggregators(dim, num_layers, aggregator, **kwargs):
        cls = dense_aggs.get(aggregator)
        return nn.ModuleList([cls(dim, activation=torch.relu if layer < num_layers - 1 else None, **kwargs)
                              for layer in range(num_layers)])

    def __init__(self, metapath, fanouts, dim, aggregator="mean", concat=False, shared_aggregators=None,
                 feature_idx=-1, feature_dim=0, max_id=-1, use_feature=None, use_id=None, sparse_feature_idx=-1,
                 sparse_feature_max_id=-1, embedding_dim=16, use_hash_embedding=False, use_residual=False,
                 shared_node_encoder=None, **kwargs):
        super().__init__()
        if len(metapath) != len(fanouts):
            raise ValueError("Len of metapath must be the same as fanouts.")
        self.metapath, self.fanouts = metapath, list(fanouts)
        self.num_layers = len(metapath)
        self.concat = concat
        self.feature_dim = feature_dim
        self.sparse_feature_idx, self.sparse_feature_max_id = sparse_feature_idx, sparse_feature_max_id
        self.use_hash_embedding, self.embedding_dim = use_hash_embedding, embedding_dim
        if shared_node_encoder is not None:
            self._node_encoder = shared_node_encoder
        else:
            self._node_encoder = ShallowEncoder(
                feature_idx=feature_idx, feature_dim=feature_dim, max_id=max_id if use_id else -1,
                sparse_feature_idx=sparse_feature_idx, sparse_feature_max_id=sparse_feature_max_id,
                embedding_dim=embedding_dim, use_hash_embedding=use_hash_embedding)
        self.dims = [self._node_encoder.output_dim] + [dim] * self.num_layers
        self.aggregators = shared_aggregators if shared_aggregators is not None else \
            self.create_aggregators(dim, self.num_layers, aggregator, concat=concat)
        self._max_id = max_id

    def node_encoder(self, inputs):
        return self._node_encoder(inputs)

    def _sample(self, inputs):
        return G.sample_fanout(inputs, self.metapath, self.fanouts, default_node=self._max_id + 1)[0]

    def _aggregate(self, hidden):
        for layer in range(self.num_layers):
            agg = self.aggregators[layer]
            hidden = [agg((hidden[hop], hidden[hop + 1].reshape(-1, self.fanouts[hop], hidden[hop + 1].shape[-1])))
                      for hop in range(self.num_layers - layer)]
        return hidden[0]

    def forward(self, inputs):
        return _shaped(inputs, self._aggregate([self.node_encoder(s) for s in self._sample(inputs)]))


class ShuffleSageEncoder(SageEncoder):
    """Returns ``[h, h_corrupted]`` where the corrupted view permutes node features
    within each root's sample tree (DGI; reference encoders.py:496-541)."""

    @staticmethod
    def shuffle_tensors(hidden):
        b, d = hidden[0].shape[0], hidden[0].shape[-1]
        sizes = [h.shape[0] for h in hidden]
        cat = torch.cat([h.reshape(b, -1, d) for h in hidden], 1)  # [b, total/b, d]
        # tf.random_shuffle on the transposed [L, b, d] tensor: one permutation of the
        # per-root position axis shared by every root
        perm = torch.randperm(cat.shape[1], device=cat.device)
        cat = cat[:, perm].reshape(-1, d)
        out, off = [], 0
        # the reference splits the permuted [b*, d] flat buffer by the original hop sizes
        for s in sizes:
            out.append(cat[off:off + s])
            off += s
        return out

    def agg(self, samples, shuffle):
        hidden = [self.node_encoder(s) for s in samples]
        if shuffle:
            hidden = self.shuffle_tensors(hidden)
        return self._aggregate(hidden)

    def forward(self, inputs):
        samples = self._sample(inputs)
        return [_shaped(inputs, self.agg(samples, False)), _shaped(inputs, self.agg(samples, True))]


class SageEncoderNew(SageEncoder):
    """Sparse-feature-only SAGE with shared embedding layers, sampling features
    together with the fan-out (reference encoders.py:544-626)."""

    def __init__(self, metapath, fanouts, dim, aggregator="mean", concat=False, shared_aggregators=None,
                 feature_idx=-1, feature_dim=0, max_id=-1, use_feature=None, use_id=None, sparse_feature_idx=-1,
                 sparse_feature_max_id=-1, embedding_dim=16, use_hash_embedding=False, shared_node_encoder=None,
                 use_residual=False, shared_embedding_layers=None, **kwargs):
        super().__init__(metapath, fanouts, dim, aggregator, concat, shared_aggregators, feature_idx, feature_dim,
                         max_id, use_feature, use_id, sparse_feature_idx, sparse_feature_max_id, embedding_dim,
                         use_hash_embedding, use_residual, shared_node_encoder)
        self.sparse_embeddings = shared_embedding_layers
        if self.sparse_embeddings is None:
            self.sparse_embeddings = nn.ModuleList([SparseEmbedding(m + 1, embedding_dim)
                                                    for m in _as_list(sparse_feature_max_id)])
        self.dims[0] = embedding_dim * len(_as_list(sparse_feature_idx))

    def forward(self, inputs):
        names = _as_list(self.sparse_feature_idx)
        defaults = [m + 1 for m in _as_list(self.sparse_feature_max_id)]
        samples, _, _, _, feats = G.sample_fanout_with_feature(
            inputs, self.metapath, self.fanouts, self._max_id + 1, [], [], names, defaults)
        f = len(names)
        hidden = []
        for layer in range(self.num_layers + 1):
            embs = [e(sp) for e, sp in zip(self.sparse_embeddings, feats[layer * f:(layer + 1) * f])]
            hidden.append(torch.cat(embs, -1).reshape(-1, self.embedding_dim * f))
        return _shaped(inputs, self._aggregate(hidden))


class ScalableSageEncoder(_StoreMixin, SageEncoder):
    """SAGE with one sampled hop per step + stale stores for deeper layers
    (reference encoders.py:629-748)."""

    def __init__(self, edge_type, fanout, num_layers, dim, aggregator="mean", concat=False,
                 shared_aggregators=None, feature_idx=-1, feature_dim=0, max_id=-1, use_feature=True,
                 use_id=False, sparse_feature_idx=-1, sparse_feature_max_id=-1, embedding_dim=16,
                 use_hash_embedding=False, shared_node_encoder=None, use_residual=False, store_learning_rate=0.001,
                 store_init_maxval=0.05, **kwargs):
        super().__init__([edge_type] * num_layers, [fanout] * num_layers, dim, aggregator, concat,
                         shared_aggregators, feature_idx, feature_dim, max_id, use_feature, use_id,
                         sparse_feature_idx, sparse_feature_max_id, embedding_dim, use_hash_embedding, use_residual,
                         shared_node_encoder)
        self.edge_type, self.fanout, self.max_id = edge_type, fanout, max_id
        self.store_learning_rate = store_learning_rate
        self._build_stores(self.dims[1:-1], max_id, store_init_maxval)

    def forward(self, inputs):
        if not self.training:
            return SageEncoder.forward(self, inputs)
        node, neighbor = G.sample_fanout(inputs, [self.edge_type], [self.fanout], default_node=self.max_id + 1)[0]
        node_emb, neigh_emb = self.node_encoder(node), self.node_encoder(neighbor)
        node_embs, leaves = [], []
        for layer in range(self.num_layers):
            node_emb = self.aggregators[layer]((node_emb, neigh_emb.reshape(-1, self.fanout, self.dims[layer])))
            node_embs.append(node_emb)
            if layer < self.num_layers - 1:
                neigh_emb = self._lookup_neighbors(layer, neighbor)
                leaves.append(neigh_emb)
        self._finish_training_forward(node, node_embs, neighbor, leaves)
        return _shaped(inputs, node_emb)


class LayerEncoder(SageEncoder):
    """Layer-wise attention pooling of each hop + FM-style cross terms
    (reference encoders.py:751-826)."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.hop_att = nn.ModuleList([AttLayer(self.feature_dim, hidden_dim=[128], head_num=[2, 2])
                                      for _ in range(self.num_layers)])
        self.out_fc = Dense(self.dims[-1], activation="relu", use_bias=True)

    def _sample(self, inputs):
        return G.sample_fanout(inputs, self.metapath, self.fanouts, default_node=0)[0]

    def layerwise_embed(self, hidden):
        span = [self.fanouts[0]]
        for f in self.fanouts[1:]:
            span.append(span[-1] * f)
        out = [hidden[0]]
        for i in range(1, len(hidden)):
            out.append(self.hop_att[i - 1](hidden[i].reshape(-1, span[i - 1], self.feature_dim)))
        return out

    def fm(self, hidden):
        hidden = list(hidden) + [hidden[0] * h for h in hidden[1:]]
        return self.out_fc(torch.cat(hidden, 1))

    def forward(self, inputs):
        hidden = [self.node_encoder(s) for s in self._sample(inputs)]
        return _shaped(inputs, self.fm(self.layerwise_embed(hidden)))


class SparseSageEncoder(SageEncoder):
    """SAGE whose node features are bags of sparse-feature embeddings
    (reference encoders.py:829-869)."""

    @staticmethod
    def create_sparse_embeddings(feature_dims):
        return nn.ModuleList([SparseEmbedding(d + 1, 16) for d in feature_dims])

    def __init__(self, metapath, fanouts, dim, feature_ixs, feature_dims, shared_embeddings=None, aggregator="mean",
                 concat=False, shared_aggregators=None, **kwargs):
        super().__init__(metapath, fanouts, dim, aggregator=aggregator, concat=concat,
                         shared_aggregators=shared_aggregators)
        self.feature_ixs, self.feature_dims = feature_ixs, feature_dims
        self.dims[0] = 16 * len(feature_ixs)
        self.sparse_embeddings = shared_embeddings if shared_embeddings is not None else \
            self.create_sparse_embeddings(feature_dims)

    def node_encoder(self, inputs):
        defaults = [d + 1 for d in self.feature_dims]
        feats = G.get_sparse_feature(torch.as_tensor(inputs).reshape(-1), self.feature_ixs, defaults)
        return torch.cat([e(f) for e, f in zip(self.sparse_embeddings, feats)], 1)


class LGCEncoder(nn.Module):
    """Learnable GCN: per-channel top-k over neighbour features, then two 1-D convs
    (reference encoders.py:872-922)."""

    def __init__(self, edge_type=(0,), feature_idx=-1, feature_dim=0, k=3, hidden_dim=128, nb_num=10, out_dim=64,
                 **kwargs):
        super().__init__()
        self.edge_type, self.feature_idx, self.feature_dim = list(edge_type), feature_idx, feature_dim
        self.k, self.hidden_dim, self.out_dim, self.nb_num = k, hidden_dim, out_dim, nb_num
        ks = k // 2 + 1
        self.conv1 = nn.Conv1d(feature_dim, hidden_dim, ks)
        self.conv2 = nn.Conv1d(hidden_dim, out_dim, ks)

    def forward(self, inputs):
        ids = torch.as_tensor(inputs).reshape(-1)
        b = ids.numel()
        dev = self.conv1.weight.device
        nbrs = G.sample_neighbor(ids, self.edge_type, self.nb_num)[0]
        node_f = G.get_dense_feature(ids, [self.feature_idx], [self.feature_dim])[0].to(dev)
        nb_f = G.get_dense_feature(nbrs.reshape(-1), [self.feature_idx], [self.feature_dim])[0].to(dev)
        return self.encode(node_f, nb_f.reshape(b, self.nb_num, self.feature_dim))

    def encode(self, node_f, nb_f):
        """node features [b, D] and sampled-neighbour features [b, nb_num, D] -> [b, out_dim]
        (the device path passes features gathered in HBM: models/encoder_trainer.py)"""
        topk = torch.topk(nb_f.transpose(1, 2), self.k, dim=-1).values  # [b, D, k]
        seq = torch.cat([node_f.unsqueeze(-1), topk], -1)  # [b, D, k+1] (channels-first)
        out = self.conv2(self.conv1(seq))
        return out[:, :, 0]
