"""C++ graph engine + tf_euler-style API on the reference's test fixture
(tools/test_data/graph.json: 6 nodes, 2 node types, 2 edge types; converted with
2 partitions like the reference's build.sh test mode).  Expected values are the
ones the reference asserts in tf_euler/python/euler_ops/*_test.py."""
import os
import tempfile

import numpy as np
import pytest
import torch

import euler_amd as ea
from euler_amd.tools.converter import convert_json

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def data_dir():
    d = tempfile.mkdtemp(prefix="euler_amd_test_")
    convert_json(os.path.join(HERE, "data", "graph.json"), d, 2, os.path.join(HERE, "data", "index_meta.json"))
    return d


@pytest.fixture(params=["local", "local_sharded"])
def graph(request, data_dir):
    if request.param == "local":
        ea.initialize_embedded_graph(data_dir)
    else:
        ea.initialize_graph({"mode": "local_sharded", "data_path": data_dir, "shard_num": 2})
    ea.set_seed(1234)
    return request.param


def test_layout(data_dir):
    assert sorted(os.listdir(data_dir)) == ["Edge", "Index", "Node", "euler.meta"]
    assert sorted(os.listdir(os.path.join(data_dir, "Node"))) == ["graph_0.dat", "graph_1.dat"]


def test_full_neighbor(graph):
    ids, w, t = ea.get_full_neighbor([1, 2], ["0", "1"])
    assert ids.to_dense().tolist() == [[2, 4, 3], [3, 5, 0]]
    assert np.allclose(w.to_dense().numpy(), [[2.0, 4.0, 3.0], [3.0, 5.0, 0.0]])
    assert t.to_dense().tolist() == [[0, 0, 1], [1, 1, 0]]


def test_full_neighbor_with_condition(graph):
    ids, w, t = ea.get_full_neighbor([1, 2, 3, 4], ["0", "1"], "price gt 3")
    assert ids.to_dense().tolist() == [[4, 3], [3, 5], [4, 0], [5, 0]]
    assert t.to_dense().tolist() == [[0, 1], [1, 1], [0, 0], [1, 0]]


def test_sorted_full_neighbor(graph):
    ids, w, t = ea.get_sorted_full_neighbor([1, 2], ["0", "1"])
    assert ids.to_dense().tolist() == [[2, 3, 4], [3, 5, 0]]
    assert t.to_dense().tolist() == [[0, 1, 0], [1, 1, 0]]
    ids, _, _ = ea.get_sorted_full_neighbor([1, 2, 3, 4], ["0", "1"], "price gt 3")
    assert ids.to_dense().tolist() == [[3, 4], [3, 5], [4, 0], [5, 0]]


def test_top_k(graph):
    ids, w, t = ea.get_top_k_neighbor([1, 2], ["0", "1"], 2)
    assert ids.tolist() == [[4, 3], [5, 3]]
    assert t.tolist() == [[0, 1], [1, 1]]
    ids, w, t = ea.get_top_k_neighbor([1, 2], ["0", "1"], 2, condition="price gt 4")
    assert ids.tolist() == [[4, -1], [5, -1]]
    assert t.tolist() == [[0, -1], [1, -1]]


def test_sample_neighbor(graph):
    ids, w, t = ea.sample_neighbor([1, 2], ["0", "1"], 10)
    assert ids.shape == (2, 10)
    assert set(ids[0].tolist()) <= {2, 3, 4}
    assert set(ids[1].tolist()) <= {3, 5}
    assert set(int(x) for x in w[0].tolist()) <= {2, 3, 4}
    # empty neighborhood -> default node
    ids, w, t = ea.sample_neighbor([1], ["1"], 3, default_node=-1, condition="price gt 100")
    assert ids.tolist() == [[-1, -1, -1]]


def test_sampling_distribution(graph):
    """Statistical ratios (reference end2end_local_test.cc:66-72 style): node 1 ->
    {2 (w2), 4 (w4)} over edge type 0, so 4 must be drawn ~2x as often as 2."""
    ids, _, _ = ea.sample_neighbor([1] * 2000, ["0"], 10)
    c = np.bincount(ids.numpy().reshape(-1), minlength=5)
    assert 1.85 < c[4] / c[2] < 2.15


def test_sample_node_weights(graph):
    """Global node sampling is node-weight proportional (weights are 1..6)."""
    s = ea.sample_node(60000, "-1").numpy()
    c = np.bincount(s, minlength=7).astype(float)
    assert 1.85 < c[4] / c[2] < 2.15 and 2.8 < c[6] / c[2] < 3.2
    typed = ea.sample_node(1000, "0").numpy()
    assert set(typed.tolist()) <= {2, 4, 6}


def test_sample_node_with_condition(graph):
    s = ea.sample_node(200, "0", "price gt 3").numpy()
    assert set(s.tolist()) <= {4, 6}


def test_sample_edge_and_features(graph):
    e = ea.sample_edge(50, "0")
    assert e.shape == (50, 3)
    assert (e[:, 2] == 0).all()
    f = ea.get_edge_dense_feature([[1, 2, 0], [5, 6, 0]], ["f3"], [2])[0]
    assert np.allclose(f.numpy(), [[12.1, 12.2], [56.1, 56.2]])


def test_dense_sparse_binary_features(graph):
    f3, f4 = ea.get_dense_feature([1, 2, 7], ["f3", "f4"], [2, 3])
    assert np.allclose(f3.numpy(), [[1.1, 1.2], [2.1, 2.2], [0, 0]])
    assert np.allclose(f4.numpy(), [[1.3, 1.4, 1.5], [2.3, 2.4, 2.5], [0, 0, 0]])
    sp = ea.get_sparse_feature([1, 2], ["f1"])[0]
    assert sp.to_dense().tolist() == [[11, 12], [21, 22]]
    assert ea.get_binary_feature([1, 2], ["f5"])[0] == [b"1a", b"2a"]


def test_node_types(graph):
    assert ea.get_node_type([1, 2, 3]).tolist() == [0, 1, 0]
    assert ea.get_node_type_id(["1", "0"]).tolist() == [0, 1]
    assert ea.get_edge_type_id(["0", "1"]).tolist() == [0, 1]


def test_neighbor_index_condition(graph):
    ids, _, _ = ea.get_full_neighbor([1, 2, 3], ["0", "1"], "att gt 4")
    assert ids.to_dense().tolist() == [[4], [5], [4]]


def test_in_neighbors(graph):
    ids, _, _ = ea.get_in_neighbor([2, 3], ["0", "1"])
    assert ids.to_dense().tolist() == [[1, 5, 0], [1, 2, 6]]


def test_random_walk_and_pairs(graph):
    w = ea.random_walk([1, 2], [["0", "1"]] * 3)
    assert w.shape == (2, 4)
    assert w[:, 0].tolist() == [1, 2]
    w2 = ea.random_walk([1, 2], [["0", "1"]] * 3, p=0.5, q=2.0)
    assert w2.shape == (2, 4)
    pairs = ea.gen_pair(torch.tensor([[1, 2, 3]]), 1, 1)
    assert pairs.tolist() == [[[1, 2], [2, 1], [2, 3], [3, 2]]]


def test_graph_labels(graph):
    g = ea.get_graph_by_label(["1", "2"]).to_dense()
    assert g.tolist() == [[1], [2]]
    labs = ea.sample_graph_label(5)
    assert len(labs) == 5 and all(l in [b"1", b"2", b"3", b"4", b"5", b"6"] for l in labs)


def test_sparse_get_adj(graph):
    adj = ea.sparse_get_adj([1, 2], [2, 3, 4, 5], ["0", "1"]).to_dense()
    assert adj.tolist() == [[1, 1, 1, 0], [0, 1, 0, 1]]


def test_layerwise(graph):
    nb, adj = ea.sample_neighbor_layerwise(torch.tensor([[1, 2, 3], [4, 5, 6]]), ["0", "1"], 3)
    assert nb.shape == (2, 3)
    assert adj.dense_shape.tolist() == [2, 3, 3]
    # every adjacency entry is a real edge
    full = {1: {2, 3, 4}, 2: {3, 5}, 3: {4}, 4: {5}, 5: {2, 6}, 6: {1, 3, 5}}
    roots = [[1, 2, 3], [4, 5, 6]]
    for b, i, j in adj.indices.tolist():
        assert int(nb[b, j]) in full[roots[b][i]]
    nb2, _ = ea.sample_neighbor_layerwise(torch.tensor([[1, 2, 3]]), ["0", "1"], 4, weight_func="sqrt")
    assert set(nb2.reshape(-1).tolist()) <= {2, 3, 4, 5}


def test_multi_hop(graph):
    nodes, adjs = ea.get_multi_hop_neighbor([1], [["0", "1"], ["0", "1"]])
    assert nodes[1].tolist() == [2, 4, 3]
    assert adjs[0].dense_shape.tolist() == [1, 3]


def test_util_ops():
    assert ea.inflate_idx(torch.tensor([0, 1, 0, 2, 1])).tolist() == [0, 2, 1, 4, 3]
    sp = ea.SparseTensor(torch.tensor([[0, 0], [1, 0], [1, 1]]), torch.tensor([5, 6, 7]), torch.tensor([2, 2]))
    g = ea.sparse_gather(torch.tensor([1, 1, 0]), sp)
    assert g.to_dense().tolist() == [[6, 7], [6, 7], [5, 0]]


def test_gql_parse_corpus():
    """Every query shape of SURVEY Appendix A parses and compiles (local + distribute)."""
    import euler_amd._engine as E

    corpus = [
        "sampleN(node_type, count).as(id)",
        "sampleN(node_type, cnt).has(p0 eq 23)",
        "sampleNWithTypes(types, counts).as(n)",
        "sampleE(edge_type, count).as(eid)",
        "v(nodes).label().as(l)",
        "v(nodes).values(__f1,__f2).as(fea)",
        "e(edges).values(fid).as(e_feature)",
        "e(edges).values(fid1, fid2).max(fid2).as(e_feature)",
        "e(edges).values(fid3).mean(fid3).as(e_feature)",
        "v(nodes).outV(edge_types).as(nb)",
        "v(nodes).outV(edge_types).has(price gt 2).order_by(id, asc).limit(2).as(nb)",
        "v(nodes).outV(edge_types).order_by(id,asc).as(nb)",
        "v(nodes).outV(edge_types).order_by(weight, desc).limit(k).as(nb)",
        "v(nodes).outE(edge_types).has(p gt 3).as(oe)",
        "v(nodes).inV().has(p gt 2).as(l)",
        "v(nodes).sampleNB(edge_types, nb_count, -1).as(nb)",
        "v(nodes).sampleNB(edge_types, n, 0).limit(5).as(nb)",
        "v(nodes).sampleNB(et_0,nb_count_0,d).as(nb_0).sampleNB(et_1,nb_count_1,d).as(nb_1)",
        "v(nodes).as(nb_0).sampleNB(et_1, c1, d).as(nb_1).v_select(nb_0).values(__f0).as(fea_0)",
        "sampleN(node_type, count).as(node).sampleNB(edge_types, count, 0).as(nb)",
        "sampleN(node_type, count).as(node_id).values(fid).as(p3)",
        "sampleN(node_type, n_count).as(node_id).outV(edge_types).order_by(id, asc).limit(2).as(nb)"
        ".values(fid).as(nb_feature).v_select(node_id).values(fid).as(n_feature)",
        "sampleN(node_type, n_count).as(node_id).select(node_id).outV(edge_types).order_by(id, asc)"
        ".limit(3).as(nb).values(fid).as(nb_feature).v_select(node_id).values(fid).as(n_feature)",
        "v(nodes).sampleNB(edge_types, n, 0).as(n1).sampleNB(edge_types, n, 0).as(n2).v_select(n1)"
        ".values(fid).as(n1_f)",
        "v(nodes).sampleLNB(edge_types, n, m, 0).as(layer)",
        "v(nodes).sampleLNB(edge_types, n, m, sqrt, 0).as(layer)",
    ]
    for q in corpus:
        E.parse_gql(q)
        local = E.compile_gql(q, "local", 1, [])
        dist = E.compile_gql(q, "distribute", 3, ["att"])
        assert local and dist
    with pytest.raises(RuntimeError):
        E.parse_gql("outV(x)")  # syntax errors raise, they never exit() the process


def test_distribute_plan_shapes():
    """Rule table of the distribute optimizer (reference compiler.cc:37-573)."""
    import euler_amd._engine as E

    ops = [n["op"] for n in E.compile_gql("v(nodes).sampleNB(et, c, 0).as(nb)", "distribute", 2, [])]
    assert ops.count("ID_SPLIT") == 1 and ops.count("REMOTE") == 2
    assert ops.count("IDX_MERGE") == 1 and ops.count("DATA_MERGE") == 3
    ops = [n["op"] for n in E.compile_gql("sampleN(t, c).as(n)", "distribute", 3, [])]
    assert ops[:1] == ["SAMPLE_NODE_SPLIT"] and ops.count("REMOTE") == 3 and "APPEND_MERGE" in ops
    ops = [n["op"] for n in E.compile_gql("v(nodes).values(f).as(x)", "distribute", 2, [])]
    assert "ID_UNIQUE" in ops and "IDX_GATHER" in ops and "DATA_GATHER" in ops
    ops = [n["op"] for n in E.compile_gql("v(nodes).outV(et).has(price gt 1).as(nb)", "distribute", 2, [])]
    assert "API_GET_NB_FILTER" in ops  # attribute index in distribute mode -> client filter
    ops = [n["op"] for n in E.compile_gql("v(nodes).outV(et).has(att gt 1).as(nb)", "distribute", 2, ["att"])]
    assert "API_GET_NB_FILTER" not in ops  # neighbor index filters on the shard


def test_builder_and_synthetic():
    b = ea.GraphBuilder()
    b.add_nodes(np.array([10, 11, 12], np.uint64), np.array([0, 0, 1], np.int32), np.array([1, 1, 1], np.float32))
    b.add_edges(np.array([10, 10, 11], np.uint64), np.array([11, 12, 12], np.uint64), np.array([0, 0, 0], np.int32),
                np.array([1, 3, 1], np.float32))
    b.derive_in_from_edges(True)
    eng = ea.use_graph(b.finish())
    ids, w, _ = ea.get_full_neighbor([10, 12], [0])
    assert ids.to_dense().tolist() == [[11, 12], [0, 0]]
    ids, _, _ = ea.get_in_neighbor([12], [0])
    assert ids.to_dense().tolist() == [[10, 11]]
    s = ea.synthetic_graph(2000, 8.0, 64, 2, 2, 8, 4, seed=3)
    assert "nodes=2000" in s.summary()
    f = ea.get_dense_feature([0, 1], ["feature"], [8])[0]
    assert f.shape == (2, 8)


def test_plumbing_ops_via_run_op(graph):
    """Engine ops of the graph-partition / adjacency plumbing: GP_* merges,
    GP_UNIQUE_MERGE (row-level, no text-key collisions), API_SPARSE_GEN_ADJ,
    API_GATHER_RESULT, API_RESHAPE."""
    eng = ea.get_engine()
    u64 = lambda *v: np.asarray(v, dtype=np.uint64)  # noqa: E731
    # rows {1, 23} and {12, 3} are distinct (decimal-concatenation keys would merge them)
    a = u64(1, 23, 5, 6).reshape(2, 2)
    b = u64(12, 3, 1, 23).reshape(2, 2)
    out = eng.run_op("GP_UNIQUE_MERGE", {"a": a, "m0": np.zeros(2, np.int32), "b": b, "m1": np.zeros(2, np.int32)},
                     ["a", "m0", "b", "m1"], [], 3)
    assert out[0].reshape(-1, 2).tolist() == [[1, 23], [5, 6], [12, 3]]
    assert out[1].tolist() == [0, 1] and out[2].tolist() == [2, 0]
    # GP_APPEND_MERGE = APPEND_MERGE
    out = eng.run_op("GP_APPEND_MERGE", {"a": u64(1, 2), "b": u64(3)}, ["a", "b"], [], 1)
    assert out[0].tolist() == [1, 2, 3]
    # (root, batch) pairs; l_nb passed through
    out = eng.run_op("API_SPARSE_GEN_ADJ", {"r": u64(10, 11, 12, 13), "l": u64(7, 8), "n": np.asarray([2], np.int32)},
                     ["r", "l", "n"], [], 2)
    assert out[0].reshape(-1, 2).tolist() == [[10, 0], [11, 0], [12, 1], [13, 1]]
    assert out[1].tolist() == [7, 8]
    out = eng.run_op("API_GATHER_RESULT", {"x": u64(1), "y": np.asarray([2.5], np.float32), "z": u64(3)},
                     ["x", "y", "z"], [], 3)
    assert [o.tolist() for o in out] == [[1], [2.5], [3]]
    out = eng.run_op("API_RESHAPE", {"x": np.arange(6, dtype=np.int32)}, ["x"], ["?,3"], 1)
    assert out[0].shape == (2, 3) and out[0].tolist() == [[0, 1, 2], [3, 4, 5]]
    with pytest.raises(Exception):
        eng.run_op("API_RESHAPE", {"x": np.arange(6, dtype=np.int32)}, ["x"], ["4,?"], 1)


def _udf_queries():
    n = {"nodes": np.array([1, 2, 3], dtype=np.uint64)}
    top2 = ea.run_gql("v(nodes).values(dense_f3, dense_f4).udf_topk(dense_f4)[2].as(x)", n,
                      ["x:0", "x:1", "x:2", "x:3"])
    smax = ea.run_gql("v(nodes).values(sparse_f1, dense_f4).max(sparse_f1).as(x)", n, ["x:0", "x:1", "x:2", "x:3"])
    mean = ea.run_gql("v(nodes).values(dense_f4).mean(dense_f4).as(x)", n, ["x:0", "x:1"])
    return top2, smax, mean


def check_udfs(top2, smax, mean):
    # f3 untouched, topk(f4)[2] = the two largest values per node, descending
    assert top2[0].tolist() == [[0, 2], [2, 4], [4, 6]]
    np.testing.assert_allclose(top2[1], [1.1, 1.2, 2.1, 2.2, 3.1, 3.2], rtol=1e-6)
    assert top2[2].tolist() == [[0, 2], [2, 4], [4, 6]]
    np.testing.assert_allclose(top2[3], [1.5, 1.4, 2.5, 2.4, 3.5, 3.4], rtol=1e-6)
    # sparse max (reference end2end_local_test.cc:146-174 style), dense column passes through
    assert smax[0].tolist() == [[0, 1], [1, 2], [2, 3]] and smax[1].tolist() == [12, 22, 32]
    assert smax[2].tolist() == [[0, 3], [3, 6], [6, 9]]
    np.testing.assert_allclose(mean[1], [1.4, 2.4, 3.4], rtol=1e-6)


def test_udf_registry(graph):
    """REGISTER_UDF registry (framework/udf.h): built-ins and a numeric-parameter UDF
    (udf_topk [k]) through local and local-sharded mode; remote mode: test_rpc.py."""
    import euler_amd._engine as E

    assert {"udf_mean", "udf_min", "udf_max", "udf_sum", "udf_topk"} <= set(E.registered_udfs())
    check_udfs(*_udf_queries())
    with pytest.raises(RuntimeError, match="unknown udf"):
        ea.run_gql("v(nodes).values(dense_f4).udf_nope(dense_f4).as(x)", {"nodes": np.array([1], np.uint64)},
                   ["x:0"])


def test_graph_partition_plan_shape():
    """mode graph_partition: an id-routed op's ids go through one ownership round (ID_SRC,
    a REMOTE API_GET_NODE_T per shard) and GP_ID_SPLIT instead of the hash ID_SPLIT, once
    per distinct routed input of the query"""
    import euler_amd._engine as E

    q = "v(nodes).as(n0).sampleNB(et, n, -1).as(nb).v_select(n0).values(fid).as(f)"
    plan = E.compile_gql(q, "graph_partition", 2, [], False)
    ops = [n["op"] for n in plan]
    # two distinct routed inputs: the raw ids (sampleNB) and their unique set (values)
    assert "ID_SPLIT" not in ops and ops.count("ID_SRC") == 2 and ops.count("GP_ID_SPLIT") == 2
    owner = [n for n in plan if n["op"] == "REMOTE" and n["inner"] == ["API_GET_NODE_T"]]
    assert sorted(n["shard"] for n in owner) == [0, 0, 1, 1]
    hash_plan = [n["op"] for n in E.compile_gql(q, "distribute", 2, [], False)]
    assert "ID_SPLIT" in hash_plan and "GP_ID_SPLIT" not in hash_plan


def test_engine_save_round_trips_the_on_disk_format(tmp_path):
    """engine.save writes the Euler on-disk format natively (euler.meta + Node / Edge
    partitions, reference tools/json2partdat.py layout); loading it back gives the same
    graph: CSR, node table, dense feature columns, edges (weights to the float precision of
    the format's prefix sums)"""
    import numpy as np

    import euler_amd as ea
    from euler_amd.ops import base

    e = ea.synthetic_graph(20000, 8.0, 64, node_types=2, edge_types=2, feature_dim=16, label_dim=4, seed=5,
                           make_current=False)
    e.save(str(tmp_path), partitions=3, threads=4)
    assert sorted(p.name for p in (tmp_path / "Node").iterdir()) == ["graph_0.dat", "graph_1.dat", "graph_2.dat"]
    ea.initialize_embedded_graph(str(tmp_path))
    e2 = base.get_engine()
    a, b = e.export_csr(), e2.export_csr()
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[3] == b[3]
    np.testing.assert_allclose(a[2], b[2], rtol=1e-5, atol=1e-5)
    for x, y in zip(e.export_nodes(), e2.export_nodes()):
        assert np.array_equal(np.asarray(x), np.asarray(y))
    ids = np.asarray(e.export_nodes()[0])
    for nm, d in (("dense_feature", 16), ("dense_label", 4)):
        assert np.array_equal(np.asarray(e.dense_feature(ids, nm, d)), np.asarray(e2.dense_feature(ids, nm, d)))
    s1, d1, w1, _ = e.export_edges(-1, "", 0)
    s2, d2, w2, _ = e2.export_edges(-1, "", 0)
    o1, o2 = np.lexsort((d1, s1)), np.lexsort((d2, s2))
    assert np.array_equal(np.asarray(s1)[o1], np.asarray(s2)[o2]) and np.array_equal(np.asarray(d1)[o1],
                                                                                       np.asarray(d2)[o2])

