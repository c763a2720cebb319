"""tf_euler-compatible graph query API on torch tensors.

Names, arguments and return structures follow the reference's Python ops
(``tf_euler/python/euler_ops/{sample_ops,neighbor_ops,feature_ops,walk_ops,type_ops,
util_ops}.py``); every call builds the same GQL the reference's TF kernels issue
 and runs it through the C++ engine, so local, in-process
sharded and remote (RPC) graphs behave identically.  ``tf.SparseTensor`` results
are returned as :class:`SparseTensor` (indices [nnz, rank], values, dense_shape).

Ids are int64 torch tensors (uint64 on the engine side; ``-1`` maps to the
reference's DEFAULT_UINT64 padding id).
"""
from __future__ import annotations

from collections import namedtuple

import numpy as np
import torch

from euler_amd.ops.base import get_engine

__all__ = [
    "SparseTensor", "ALL_NODE_TYPE", "get_node_type_id", "get_edge_type_id", "get_node_type",
    "sample_node", "sample_edge", "sample_node_with_src", "sample_n_with_types", "sample_graph_label",
    "get_graph_by_label", "sample_neighbor", "sage_flow", "get_top_k_neighbor", "get_full_neighbor",
    "get_sorted_full_neighbor", "get_in_neighbor", "sample_fanout", "sample_fanout_with_feature",
    "sample_neighbor_layerwise", "sample_fanout_layerwise", "sample_fanout_layerwise_each_node",
    "get_multi_hop_neighbor", "sparse_get_adj", "get_dense_feature", "get_sparse_feature",
    "get_binary_feature", "get_edge_dense_feature", "get_edge_sparse_feature", "get_edge_binary_feature",
    "random_walk", "gen_pair", "inflate_idx", "sparse_gather", "run_gql", "explain_gql",
]

ALL_NODE_TYPE = -1


class SparseTensor(namedtuple("SparseTensor", ["indices", "values", "dense_shape"])):
    """Minimal stand-in for ``tf.SparseTensor`` (COO, row-major)."""

    def to_dense(self, default_value=0):
        shape = [int(x) for x in self.dense_shape]
        out = torch.full(shape, default_value, dtype=self.values.dtype)
        if self.indices.numel():
            out[tuple(self.indices.t().long())] = self.values
        return out

    def to_torch(self):
        return torch.sparse_coo_tensor(self.indices.t().long(), self.values, [int(x) for x in self.dense_shape])


# ----------------------------------------------------------------------------- plumbing
_SCOPE_MOD = [None]


def _scope():
    """the active device-graph scope (graph/device_scope.py): queries answered from HBM"""
    m = _SCOPE_MOD[0]
    if m is None:
        from euler_amd.graph import device_scope as m

        _SCOPE_MOD[0] = m
    return m.active_scope()


def device_scope_active() -> bool:
    return _scope() is not None


def _u64(x) -> np.ndarray:
    if isinstance(x, torch.Tensor):
        x = x.detach().cpu().numpy()
    a = np.asarray(x)
    if a.dtype.kind == "f":
        a = a.astype(np.int64)
    return a.reshape(-1).astype(np.int64).view(np.uint64) if a.dtype != np.uint64 else a.reshape(-1)


def _edges(x) -> np.ndarray:
    if isinstance(x, torch.Tensor):
        x = x.detach().cpu().numpy()
    a = np.asarray(x).astype(np.int64).reshape(-1, 3)
    return a.view(np.uint64)


def _i64(a) -> torch.Tensor:
    a = np.asarray(a)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    return torch.from_numpy(np.ascontiguousarray(a))


def _t(a) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(np.asarray(a)))


def run_gql(gql: str, inputs: dict, outputs):
    """Run any GQL query (reference ``QueryProxy::RunGremlin``) and return numpy arrays."""
    return get_engine().run(gql, inputs, list(outputs))


def explain_gql(gql: str) -> str:
    """Physical DAG the engine compiled for a query (local or distribute mode)."""
    return get_engine().explain(gql)


def _meta():
    return get_engine().meta()


def _type_ids(values, table, what):
    if isinstance(values, torch.Tensor):
        values = values.tolist()
    if isinstance(values, (int, np.integer)):
        values = [int(values)]
    if isinstance(values, (str, bytes)):
        values = [values]
    out = []
    for v in values:
        if isinstance(v, bytes):
            v = v.decode()
        if isinstance(v, str):
            if v == "-1":
                out.append(-1)
                continue
            if v not in table:
                raise ValueError("unknown %s type name %r (known: %s)" % (what, v, sorted(table)))
            out.append(int(table[v]))
        else:
            out.append(int(v))
    return np.asarray(out, dtype=np.int32)


def get_node_type_id(type_id_or_names):
    """Names -> ids (ids pass through), reference ``type_ops.get_node_type_id``."""
    return _t(_type_ids(type_id_or_names, _meta()["node_types"], "node"))


def get_edge_type_id(type_id_or_names):
    return _t(_type_ids(type_id_or_names, _meta()["edge_types"], "edge"))


def _et(edge_types):
    if edge_types is None:
        return np.asarray([-1], dtype=np.int32)
    return _type_ids(edge_types, _meta()["edge_types"], "edge")


def _has(condition: str) -> str:
    """Condition -> GQL suffix.  Accepts GQL (``has(price gt 3)``, ``hasLabel(x)``,
    ``order_by``/``limit``) or the reference's plain DNF text (``price gt 3 and att lt 2``),
    which its TF kernels wrapped in ``has(...)``."""
    import re

    c = (condition or "").strip()
    if not c:
        return ""
    if c.startswith("."):
        return c
    if re.match(r"^(has|hasLabel|hasKey|order_by|limit)\s*\(", c):
        return "." + c
    disj = []
    for d in re.split(r"\s+or\s+", c):
        disj.append(".and.".join("has(%s)" % t.strip() for t in re.split(r"\s+and\s+", d)))
    return "." + ".or.".join(disj)


# ----------------------------------------------------------------------------- sampling
def sample_node(count, node_type, condition=""):
    """``sampleN(node_type, count)[.has(cond)]`` (reference sample_node_op.cc:60-76)."""
    sc = _scope()
    if sc is not None and not condition:
        return sc.sample_node(count, node_type)
    t = -1 if (isinstance(node_type, str) and node_type == "-1") else int(_type_ids(node_type, _meta()["node_types"], "node")[0])
    r = run_gql("sampleN(node_type, count)%s.as(id)" % _has(condition),
                {"node_type": np.asarray([t], np.int32), "count": np.asarray([int(count)], np.int64)}, ["id:0"])
    return _i64(r[0])


def sample_edge(count, edge_type="-1"):
    t = -1 if (edge_type is None or (isinstance(edge_type, str) and edge_type == "-1")) else int(_et(edge_type)[0])
    r = run_gql("sampleE(edge_type, count).as(eid)",
                {"edge_type": np.asarray([t], np.int32), "count": np.asarray([int(count)], np.int64)}, ["eid:0"])
    return _i64(r[0]).reshape(-1, 3)


def sample_n_with_types(count, types):
    """``count`` nodes per type in ``types`` -> [len(types), count]."""
    ty = _type_ids(types, _meta()["node_types"], "node")
    r = run_gql("sampleNWithTypes(types, counts).as(n)",
                {"types": ty, "counts": np.full(len(ty), int(count), np.int32)}, ["n:0", "n:1"])
    idx, ids = r[0], r[1]
    out = np.zeros((len(ty), int(count)), dtype=np.uint64)
    for i in range(len(ty)):
        seg = ids[idx[i, 0]:idx[i, 1]]
        out[i, :len(seg)] = seg[:int(count)]
    return _i64(out)


def sample_node_with_src(src_nodes, count):
    """For each source node sample ``count`` nodes of the same type (reference sample_ops.py:75-87)."""
    types = get_node_type(src_nodes).numpy()
    out = np.zeros((len(types), int(count)), dtype=np.int64)
    uniq = np.unique(types)
    for t in uniq:
        rows = np.nonzero(types == t)[0]
        s = sample_node(int(count) * len(rows), int(t)).numpy()
        if s.size == int(count) * len(rows):
            out[rows] = s.reshape(len(rows), int(count))
    return torch.from_numpy(out)


def sample_graph_label(count):
    """Uniformly sampled graph labels (reference single-op API_SAMPLE_GRAPH_LABEL)."""
    r = get_engine().run_op("API_SAMPLE_GRAPH_LABEL", {}, [], [str(int(count))], 1)
    return list(r[0])


def get_graph_by_label(labels):
    """Node lists of the given graph labels as a SparseTensor [len(labels), max_nodes]
    (reference single-op API_GET_GRAPH_BY_LABEL)."""
    labs = [l if isinstance(l, bytes) else str(l).encode() for l in labels]
    r = get_engine().run_op("API_GET_GRAPH_BY_LABEL", {"labels": labs}, ["labels"], [], 2)
    return _ragged_to_sparse(r[0], r[1])


def get_node_type(nodes):
    r = run_gql("v(nodes).label().as(l)", {"nodes": _u64(nodes)}, ["l:0"])
    return _t(r[0].astype(np.int32))


# ----------------------------------------------------------------------------- neighbors
def _ragged_slots(idx, k):
    """(row, slot, source position) of the first k entries of every ragged row"""
    idx = np.asarray(idx).reshape(-1, 2)
    b = idx[:, 0].astype(np.int64)
    m = np.clip(idx[:, 1].astype(np.int64) - b, 0, int(k))
    rows = np.repeat(np.arange(len(b)), m)
    slot = np.arange(int(m.sum())) - np.repeat(np.cumsum(m) - m, m)
    return rows, slot, np.repeat(b, m) + slot


def _dense_rows(idx, ids, w, t, n, k, default_node):
    if _uniform_rows(np.asarray(idx).reshape(-1, 2)[:n], k) and len(ids) >= n * k:
        return (_i64(np.asarray(ids, dtype=np.uint64)[: n * k].reshape(n, k)),
                _t(np.asarray(w, dtype=np.float32)[: n * k].reshape(n, k)),
                _t(np.asarray(t, dtype=np.int32)[: n * k].reshape(n, k)))
    out_id = np.full((n, k), np.uint64(default_node & 0xFFFFFFFFFFFFFFFF), dtype=np.uint64)
    out_w = np.zeros((n, k), np.float32)
    out_t = np.full((n, k), -1, np.int32)
    rows, slot, src = _ragged_slots(idx[:n], k)
    out_id[rows, slot] = np.asarray(ids)[src]
    out_w[rows, slot] = np.asarray(w)[src]
    out_t[rows, slot] = np.asarray(t)[src]
    return _i64(out_id), _t(out_w), _t(out_t)


def sample_neighbor(nodes, edge_types, count, default_node=-1, condition=""):
    """Weighted with-replacement sampling -> (ids, weights, types), each [n, count]."""
    sc = _scope()
    if sc is not None and not condition:
        return sc.sample_neighbor(nodes, edge_types, count, default_node)
    ids = _u64(nodes)
    et = _et(edge_types)
    eng = get_engine()
    if not condition and _meta()["mode"] == "local":
        o_id, o_w, o_t = eng.sample_neighbor(ids, [int(x) for x in et if x >= 0], int(count),
                                             int(np.int64(default_node).astype(np.uint64)))
        return _i64(o_id), _t(o_w), _t(o_t)
    r = eng.run("v(nodes).sampleNB(edge_types, nb_count, %d)%s.as(nb)" % (int(default_node), _has(condition)),
                {"nodes": ids, "edge_types": et, "nb_count": np.asarray([int(count)])},
                ["nb:0", "nb:1", "nb:2", "nb:3"])
    return _dense_rows(r[0], r[1], r[2], r[3], len(ids), int(count), int(default_node))


def sage_flow(roots, metapath, fanouts, default_node=-1, self_loops=True):
    """Native SageDataFlow (``_engine.sage_flow``, GIL released): per hop fixed-fanout
    sampling + first-occurrence unique + edge index, innermost hop first, as
    ``[(n_id, res_n_id, edge_index [2, E])]`` int64 tensors.  Returns None when the graph
    is not in-process (remote / sharded mode: the GQL path is used instead)."""
    if _meta()["mode"] != "local":
        return None
    ets = [[int(x) for x in _et(et) if x >= 0] for et in metapath]
    hops = get_engine().sage_flow(np.ascontiguousarray(_u64(roots).view(np.int64)), ets,
                                  [int(c) for c in fanouts], int(default_node), bool(self_loops))
    return [(torch.from_numpy(a), torch.from_numpy(b), torch.from_numpy(c)) for a, b, c in hops]


def get_top_k_neighbor(nodes, edge_types, k, default_node=-1, condition=""):
    ids = _u64(nodes)
    r = run_gql("v(nodes).outV(edge_types)%s.order_by(weight, desc).limit(%d).as(nb)" % (_has(condition), int(k)),
                {"nodes": ids, "edge_types": _et(edge_types)}, ["nb:0", "nb:1", "nb:2", "nb:3"])
    return _dense_rows(r[0], r[1], r[2], r[3], len(ids), int(k), int(default_node))


def _ragged_to_sparse(idx, vals, values_cast=None):
    idx = np.asarray(idx).reshape(-1, 2)
    n = idx.shape[0]
    lens = (idx[:, 1] - idx[:, 0]).astype(np.int64)
    rows = np.repeat(np.arange(n, dtype=np.int64), lens)
    # position inside each row and source index, vectorised (no per-row Python loop)
    out_off = np.cumsum(lens) - lens
    cols = np.arange(int(lens.sum()), dtype=np.int64) - np.repeat(out_off, lens)
    sel = np.repeat(idx[:, 0].astype(np.int64), lens) + cols
    v = np.asarray(vals)[sel.astype(np.int64)] if len(sel) else np.asarray(vals)[:0]
    if values_cast is not None:
        v = v.astype(values_cast)
    shape = torch.tensor([n, int(lens.max()) if n and lens.size else 0], dtype=torch.int64)
    vt = _i64(v) if v.dtype == np.uint64 else _t(v)
    return SparseTensor(torch.from_numpy(np.stack([rows, cols], 1) if n else np.zeros((0, 2), np.int64)), vt, shape)


def get_full_neighbor(nodes, edge_types, condition=""):
    """All out-neighbors -> (ids, weights, types) SparseTensors [n, max_degree]."""
    r = run_gql("v(nodes).outV(edge_types)%s.as(nb)" % _has(condition),
                {"nodes": _u64(nodes), "edge_types": _et(edge_types)}, ["nb:0", "nb:1", "nb:2", "nb:3"])
    return _ragged_to_sparse(r[0], r[1]), _ragged_to_sparse(r[0], r[2]), _ragged_to_sparse(r[0], r[3])


def get_sorted_full_neighbor(nodes, edge_types, condition=""):
    r = run_gql("v(nodes).outV(edge_types)%s.order_by(id, asc).as(nb)" % _has(condition),
                {"nodes": _u64(nodes), "edge_types": _et(edge_types)}, ["nb:0", "nb:1", "nb:2", "nb:3"])
    return _ragged_to_sparse(r[0], r[1]), _ragged_to_sparse(r[0], r[2]), _ragged_to_sparse(r[0], r[3])


def get_in_neighbor(nodes, edge_types, condition=""):
    """In-neighbors (``inV``; the reference translated it but had no kernel)."""
    r = run_gql("v(nodes).inV(edge_types)%s.as(nb)" % _has(condition),
                {"nodes": _u64(nodes), "edge_types": _et(edge_types)}, ["nb:0", "nb:1", "nb:2", "nb:3"])
    return _ragged_to_sparse(r[0], r[1]), _ragged_to_sparse(r[0], r[2]), _ragged_to_sparse(r[0], r[3])


def sample_fanout(nodes, edge_types, counts, default_node=-1):
    """Multi-hop sampling: ([n, n*c0, n*c0*c1, ...], weights, types) (reference neighbor_ops.py)."""
    sc = _scope()
    if sc is not None:
        return sc.sample_fanout(nodes, edge_types, counts, default_node)
    nb = [torch.as_tensor(_u64(nodes).view(np.int64))]
    ws, ts = [], []
    for et, c in zip(edge_types, counts):
        i, w, t = sample_neighbor(nb[-1], et, int(c), default_node)
        nb.append(i.reshape(-1))
        ws.append(w.reshape(-1))
        ts.append(t.reshape(-1))
    return nb, ws, ts


def sample_fanout_with_feature(nodes, edge_types, count, default_node, dense_feature_names, dense_dimensions,
                               sparse_feature_names, sparse_default_values):
    """Multi-hop sampling plus the features of every hop's nodes as ONE GQL query (the
    reference's ``v(nodes).as(nb_0).sampleNB(...).as(nb_1)... .v_select(nb_i).values(...)``,
    sample_fanout_with_feature_op.cc:43-69).  In remote mode the compiler fuses each hop's
    sampleNB with the values() of the same frontier into one REMOTE per shard, so the
    query costs one RPC per shard per hop (+1 for the leaf features)."""
    dense_feature_names = list(dense_feature_names or [])
    sparse_feature_names = list(sparse_feature_names or [])
    names = ["dense_" + str(n) for n in dense_feature_names] + ["sparse_" + str(n) for n in sparse_feature_names]
    ids = _u64(nodes)
    L = len(count)
    q = "v(nodes).as(nb_0)"
    inputs = {"nodes": ids}
    outs = []
    for i in range(1, L + 1):
        q += ".sampleNB(et_%d, c_%d, %d).as(nb_%d)" % (i, i, int(default_node), i)
        inputs["et_%d" % i] = _et(edge_types[i - 1])
        inputs["c_%d" % i] = np.asarray([int(count[i - 1])])
        outs += ["nb_%d:%d" % (i, k) for k in range(4)]
    if names:
        keys = ["__f%d" % j for j in range(len(names))]
        for k, nm in zip(keys, names):
            inputs[k] = nm
        for i in range(L + 1):
            q += ".v_select(nb_%d).values(%s).as(fea_%d)" % (i, ", ".join(keys), i)
            outs += ["fea_%d:%d" % (i, k) for k in range(2 * len(names))]
    r = run_gql(q, inputs, outs)
    neighbors = [torch.as_tensor(ids.view(np.int64))]
    weights, types = [], []
    n = len(ids)
    for i in range(L):
        c = int(count[i])
        nb, w, t = _dense_rows(r[4 * i], r[4 * i + 1], r[4 * i + 2], r[4 * i + 3], n, c, int(default_node))
        neighbors.append(nb.reshape(-1))
        weights.append(w.reshape(-1))
        types.append(t.reshape(-1))
        n *= c
    dense, sparse = [], []
    base = 4 * L
    nd = len(dense_feature_names)
    for i in range(L + 1 if names else 0):
        res = [(r[base + 2 * j], r[base + 2 * j + 1]) for j in range(len(names))]
        base += 2 * len(names)
        dense.extend(_dense_from_ragged(idx, vals, d) for (idx, vals), d in zip(res[:nd], dense_dimensions))
        if sparse_feature_names:
            sparse.extend(_sparse_list(res[nd:], sparse_default_values))
    return neighbors, weights, types, dense, sparse


def sample_neighbor_layerwise(nodes, edge_types, count, default_node=-1, weight_func=""):
    """Layer-wise sampling (FastGCN / AdaptiveGCN): nodes [b, n] -> (neighbors [b, count], adj [b, n, count])."""
    nodes_t = torch.as_tensor(nodes)
    if nodes_t.dim() == 1:
        nodes_t = nodes_t.view(1, -1)
    b, n = nodes_t.shape
    wf = (weight_func + ", ") if weight_func else ""
    r = run_gql("v(nodes).sampleLNB(edge_types, n, m, %s%d).as(layer)" % (wf, int(default_node)),
                {"nodes": _u64(nodes_t), "edge_types": _et(edge_types), "n": np.asarray([int(n)]),
                 "m": np.asarray([int(count)])}, ["layer:0", "layer:1", "layer:2"])
    adj_idx, adj_col, layer = r[0], r[1].astype(np.int64), r[2]
    rows, bi, li, ci = [], [], [], []
    for i in range(adj_idx.shape[0]):
        bb, ee = adj_idx[i]
        for k in range(bb, ee):
            c = adj_col[k]
            bi.append(i // n)
            li.append(i % n)
            ci.append(c - (i // n) * int(count))
    idx = np.stack([np.asarray(bi, np.int64), np.asarray(li, np.int64), np.asarray(ci, np.int64)], 1) \
        if bi else np.zeros((0, 3), np.int64)
    adj = SparseTensor(torch.from_numpy(idx), torch.ones(len(bi), dtype=torch.float32),
                       torch.tensor([b, n, int(count)], dtype=torch.int64))
    return _i64(layer).reshape(b, int(count)), adj


def sample_fanout_layerwise_each_node(nodes, edge_types, counts, default_node=-1):
    neighbors_list = [torch.as_tensor(_u64(nodes).view(np.int64))]
    adj_list = []
    last_count = None
    for hop_edge_types, count in zip(edge_types, counts):
        if len(neighbors_list) == 1:
            nb, _, _ = sample_neighbor(neighbors_list[-1], hop_edge_types, count, default_node)
            neighbors_list.append(nb.reshape(-1))
        else:
            nb, adj = sample_neighbor_layerwise(neighbors_list[-1].reshape(-1, last_count), hop_edge_types, count,
                                                default_node)
            neighbors_list.append(nb.reshape(-1))
            adj_list.append(adj)
        last_count = count
    return neighbors_list, adj_list


def sample_fanout_layerwise(nodes, edge_types, counts, default_node=-1, weight_func=""):
    neighbors_list = [torch.as_tensor(_u64(nodes).view(np.int64))]
    adj_list = []
    last_count = neighbors_list[0].numel()
    for hop_edge_types, count in zip(edge_types, counts):
        nb, adj = sample_neighbor_layerwise(neighbors_list[-1].reshape(-1, last_count), hop_edge_types, count,
                                            default_node, weight_func)
        neighbors_list.append(nb.reshape(-1))
        adj_list.append(adj)
        last_count = count
    return neighbors_list, adj_list


def get_multi_hop_neighbor(nodes, edge_types):
    """Unique node set per hop + sparse adjacency between hops (reference neighbor_ops.py)."""
    sc = _scope()
    if sc is not None:
        return sc.get_multi_hop_neighbor(nodes, edge_types)
    cur = torch.as_tensor(_u64(nodes).view(np.int64))
    nodes_list, adj_list = [cur], []
    for et in edge_types:
        nb, w, _ = get_full_neighbor(cur, et)
        uniq, inv = np.unique(nb.values.numpy(), return_inverse=True)
        # keep first-occurrence order like tf.unique
        first = {}
        order = []
        for v in nb.values.numpy().tolist():
            if v not in first:
                first[v] = len(order)
                order.append(v)
        next_nodes = torch.tensor(order, dtype=torch.int64)
        next_idx = torch.tensor([first[v] for v in nb.values.numpy().tolist()], dtype=torch.int64)
        ind = torch.stack([nb.indices[:, 0], next_idx], 1) if next_idx.numel() else torch.zeros((0, 2), dtype=torch.int64)
        adj = SparseTensor(ind, w.values, torch.tensor([cur.numel(), next_nodes.numel()], dtype=torch.int64))
        nodes_list.append(next_nodes)
        adj_list.append(adj)
        cur = next_nodes
    return nodes_list, adj_list


def sparse_get_adj(nodes, nb_nodes, edge_types, n=-1, m=-1):
    """Adjacency between ``nodes`` and ``nb_nodes`` as a SparseTensor [len(nodes), len(nb_nodes)]."""
    attrs = ["edge_types", str(int(n))] + ([str(int(m))] if int(m) > 0 else [])
    r = get_engine().run_op("API_SPARSE_GET_ADJ",
                            {"nodes": _u64(nodes), "nb_nodes": _u64(nb_nodes), "edge_types": _et(edge_types)},
                            ["nodes", "nb_nodes"], attrs, 2)
    idx, col = r[0], r[1]
    N, M = len(_u64(nodes)), len(_u64(nb_nodes))
    lens = idx[:, 1] - idx[:, 0]
    rows = np.repeat(np.arange(N, dtype=np.int64), lens)
    ind = np.stack([rows, col.astype(np.int64)], 1) if len(col) else np.zeros((0, 2), np.int64)
    return SparseTensor(torch.from_numpy(ind), torch.ones(len(col), dtype=torch.float32),
                        torch.tensor([N, M], dtype=torch.int64))


# ----------------------------------------------------------------------------- features
def _feature_query(root, ids_key, ids, prefix, names):
    keys = ["__f%d" % i for i in range(len(names))]
    inputs = {ids_key: ids}
    for k, nm in zip(keys, names):
        inputs[k] = prefix + str(nm)
    outs = []
    for i in range(len(names)):
        outs += ["fea:%d" % (2 * i), "fea:%d" % (2 * i + 1)]
    r = run_gql("%s(%s).values(%s).as(fea)" % (root, ids_key, ", ".join(keys)), inputs, outs)
    return [(r[2 * i], r[2 * i + 1]) for i in range(len(names))]


def _uniform_rows(idx, k):
    """True when ragged row i is exactly [i*k, (i+1)*k) (the common full-row case)"""
    idx = np.asarray(idx).reshape(-1, 2)
    n = idx.shape[0]
    if n == 0:
        return True
    b, e = idx[:, 0].astype(np.int64), idx[:, 1].astype(np.int64)
    return bool(b[0] == 0 and (e - b == k).all() and (n == 1 or (b[1:] == e[:-1]).all()))


def _dense_from_ragged(idx, vals, dim):
    n = idx.shape[0]
    if _uniform_rows(idx, int(dim)):  # every row present and full: a reshape
        return _t(np.asarray(vals, dtype=np.float32)[: n * int(dim)].reshape(n, int(dim)))
    out = np.zeros((n, int(dim)), np.float32)
    rows, slot, src = _ragged_slots(idx, dim)
    out[rows, slot] = np.asarray(vals)[src]
    return _t(out)


def get_dense_feature(nodes, feature_names, dimensions, thread_num=1):
    """Dense node features -> list of float32 [n, dim] (missing = 0)."""
    sc = _scope()
    if sc is not None:
        return sc.get_dense_feature(nodes, feature_names, dimensions)
    ids = _u64(nodes)
    eng = get_engine()
    if _meta()["mode"] == "local":
        return [_t(eng.dense_feature(ids, "dense_" + str(nm), int(d))) for nm, d in zip(feature_names, dimensions)]
    res = _feature_query("v", "nodes", ids, "dense_", list(feature_names))
    return [_dense_from_ragged(idx, vals, d) for (idx, vals), d in zip(res, dimensions)]


def _sparse_list(res, default_values):
    out = []
    for i, (idx, vals) in enumerate(res):
        idx = idx.copy()
        vals = vals.astype(np.uint64) if vals.dtype != np.uint64 else vals
        dv = (default_values[i] if default_values is not None else 0)
        # empty rows get the default value (reference fills default_values)
        lens = idx[:, 1] - idx[:, 0]
        if (lens == 0).any():
            new_vals, new_idx, acc = [], [], 0
            for r, (b, e) in enumerate(idx):
                seg = vals[b:e] if e > b else np.asarray([dv], np.uint64)
                new_vals.append(seg)
                new_idx.append((acc, acc + len(seg)))
                acc += len(seg)
            vals = np.concatenate(new_vals) if new_vals else vals
            idx = np.asarray(new_idx, np.int64).reshape(-1, 2)
        out.append(_ragged_to_sparse(idx, vals))
    return out


def get_sparse_feature(nodes, feature_names, default_values=None, thread_num=1):
    return _sparse_list(_feature_query("v", "nodes", _u64(nodes), "sparse_", list(feature_names)), default_values)


def get_binary_feature(nodes, feature_names, thread_num=1):
    res = _feature_query("v", "nodes", _u64(nodes), "binary_", list(feature_names))
    out = []
    for idx, vals in res:
        out.append([vals[b] if e > b else b"" for b, e in idx])
    return out


def get_edge_dense_feature(edges, feature_names, dimensions, thread_num=1):
    res = _feature_query("e", "edges", _edges(edges), "dense_", list(feature_names))
    return [_dense_from_ragged(idx, vals, d) for (idx, vals), d in zip(res, dimensions)]


def get_edge_sparse_feature(edges, feature_names, default_values=None, thread_num=1):
    return _sparse_list(_feature_query("e", "edges", _edges(edges), "sparse_", list(feature_names)), default_values)


def get_edge_binary_feature(edges, feature_names, thread_num=1):
    res = _feature_query("e", "edges", _edges(edges), "binary_", list(feature_names))
    return [[vals[b] if e > b else b"" for b, e in idx] for idx, vals in res]


# ----------------------------------------------------------------------------- walks
def random_walk(nodes, edge_types, p=1.0, q=1.0, default_node=-1, seed=None):
    """Random walks [n, len(edge_types) + 1] (``edge_types[s]`` = the edge types of step
    s); node2vec bias when p or q != 1 (reference random_walk_op.cc:70-188: 1/p back to
    the previous node, 1 to common neighbours of the previous node, 1/q otherwise).

    Local graph: one GIL-free native call (``Engine.random_walk``, csrc/graph/walk.cc),
    each walk on its own Philox stream.  ``seed`` None draws the next seed of
    :func:`euler_amd.set_seed`'s sequence, so results are reproducible per global seed.
    Remote shards: one full-neighbour query per step and a vectorised numpy draw with the
    same bias, seeded the same way."""
    from euler_amd.ops import base as _base

    if float(p) <= 0.0 or float(q) <= 0.0:
        raise ValueError("random_walk: p and q must be positive")
    seed = _base.next_walk_seed() if seed is None else int(seed)
    ids = _u64(nodes)
    steps = [[int(x) for x in _et(et) if x >= 0] for et in edge_types]
    eng = get_engine()
    if _meta()["mode"] == "local":
        return torch.as_tensor(eng.random_walk(ids, steps, float(p), float(q), int(default_node), seed))
    return _random_walk_remote(ids, edge_types, float(p), float(q), int(default_node), seed)


def _pair_keys(rows, ids):
    """(row, id) pairs as 16-byte void scalars, for exact vectorised set membership"""
    a = np.ascontiguousarray(np.stack([np.asarray(rows, np.uint64), np.asarray(ids, np.uint64)], 1))
    return a.view(np.dtype((np.void, 16))).reshape(-1)


def _random_walk_remote(ids, edge_types, p, q, default_node, seed):
    rng = np.random.default_rng(seed)
    n = len(ids)
    cur = ids.astype(np.int64)
    prev, prev_keys = cur.copy(), None  # step 0: the previous node is the start, no neighbour set
    cols = [cur.copy()]
    biased = p != 1.0 or q != 1.0
    for et in edge_types:
        nb, w, _ = get_full_neighbor(cur, et)
        ind = nb.indices.numpy()
        r, c = ind[:, 0], nb.values.numpy().astype(np.int64)
        wt = w.values.numpy().astype(np.float64)
        if biased and len(r):
            bias = np.full(len(r), 1.0 / q)
            if prev_keys is not None:
                bias[np.isin(_pair_keys(r, c.view(np.uint64)), prev_keys)] = 1.0
            bias[c == prev[r]] = 1.0 / p
            wt = wt * bias
        nxt = np.full(n, int(default_node), dtype=np.int64)
        if len(r):
            order = np.argsort(r, kind="stable")
            r, c, wt = r[order], c[order], wt[order]
            cum = np.cumsum(wt)
            starts = np.searchsorted(r, np.arange(n), "left")
            ends = np.searchsorted(r, np.arange(n), "right")
            has = ends > starts
            base = np.where(starts > 0, cum[np.maximum(starts - 1, 0)], 0.0)
            tot = np.where(has, cum[np.maximum(ends - 1, 0)] - base, 0.0)
            u = base + rng.random(n) * tot
            pick = np.minimum(np.searchsorted(cum, u, "right"), np.maximum(ends - 1, 0))
            ok = has & (tot > 0)
            nxt[ok] = c[pick[ok]]
        prev_keys = _pair_keys(r, c.view(np.uint64)) if biased else None
        prev = cur
        cur = nxt
        cols.append(cur.copy())
    return torch.as_tensor(np.stack(cols, 1))


def gen_pair(paths, left_win_size, right_win_size):
    """Skip-gram pairs [b, P, 2] from walks [b, L] (reference gen_pair_op.cc:60-92)."""
    paths = torch.as_tensor(paths)
    b, L = paths.shape
    pairs = []
    for j in range(L):
        k = 0
        while j - k - 1 >= 0 and k < left_win_size:
            pairs.append((j, j - k - 1))
            k += 1
        k = 0
        while j + k + 1 < L and k < right_win_size:
            pairs.append((j, j + k + 1))
            k += 1
    if not pairs:
        return torch.zeros((b, 0, 2), dtype=paths.dtype)
    src = torch.tensor([a for a, _ in pairs])
    dst = torch.tensor([c for _, c in pairs])
    return torch.stack([paths[:, src], paths[:, dst]], 2)


# ----------------------------------------------------------------------------- utils
def inflate_idx(idx):
    """Make ``tf.unique``-style indices unique per occurrence (reference inflate_idx_op.cc:32-66)."""
    idx = torch.as_tensor(idx).reshape(-1).long()
    if idx.numel() == 0:
        return idx.int()
    counts = torch.bincount(idx)
    offsets = torch.cumsum(counts, 0) - counts
    # rank of each occurrence among equal values, in input order (stable sort)
    order = torch.argsort(idx, stable=True)
    pos_in_sorted = torch.empty_like(idx)
    pos_in_sorted[order] = torch.arange(idx.numel())
    return (pos_in_sorted).int()  # = offsets[idx] + occurrence rank


def sparse_gather(gather_idx, sp: SparseTensor):
    """Row gather on a SparseTensor (reference sparse_gather_op.cc)."""
    gather_idx = torch.as_tensor(gather_idx).reshape(-1).long()
    rows = sp.indices[:, 0]
    new_ind, new_val = [], []
    for new_r, r in enumerate(gather_idx.tolist()):
        sel = rows == r
        k = int(sel.sum())
        if k:
            cols = sp.indices[sel, 1:]
            new_ind.append(torch.cat([torch.full((k, 1), new_r, dtype=torch.int64), cols], 1))
            new_val.append(sp.values[sel])
    ind = torch.cat(new_ind) if new_ind else torch.zeros((0, sp.indices.shape[1]), dtype=torch.int64)
    val = torch.cat(new_val) if new_val else sp.values[:0]
    shape = sp.dense_shape.clone()
    shape[0] = gather_idx.numel()
    return SparseTensor(ind, val, shape)
