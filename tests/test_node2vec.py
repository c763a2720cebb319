"""node2vec-biased random walks (reference tf_euler/kernels/random_walk_op.cc:70-188):
transition ratios 1/p : 1 : 1/q on a fixture graph, in the C++ engine, in the vectorised
remote-mode path and in the HIP kernel on a DeviceGraph; reproducibility per seed.

Fixture: node 0 -> {1 (weight 1e6), 2 (1e-6)}, so the first step lands on 1 almost surely.
From 1 the candidates are 0 (the previous node: 1/p), 2 (a neighbour of 0: 1) and 3
(1/q), all with weight 1.
"""
import numpy as np
import pytest
import torch

import euler_amd as ea

P, Q = 2.0, 0.5
WANT = np.array([1 / P, 1.0, 1 / Q]) / (1 / P + 1.0 + 1 / Q)  # shares of 0, 2, 3


def _edges():
    src = np.array([0, 0, 1, 1, 1, 2, 3], np.uint64)
    dst = np.array([1, 2, 0, 2, 3, 1, 1], np.uint64)
    w = np.array([1e6, 1e-6, 1, 1, 1, 1, 1], np.float32)
    return src, dst, w


def _engine():
    b = ea.GraphBuilder()
    b.add_nodes(np.arange(4, dtype=np.uint64), np.zeros(4, np.int32), np.ones(4, np.float32))
    s, d, w = _edges()
    b.add_edges(s, d, np.zeros(len(s), np.int32), w)
    b.derive_in_from_edges(True)
    return ea.use_graph(b.finish())


def _shares(walks):
    second = np.asarray(walks)[:, 2]
    return np.array([(second == k).mean() for k in (0, 2, 3)])


def test_engine_node2vec_ratios_and_seed():
    _engine()
    n = 60000
    w1 = ea.random_walk(np.zeros(n, np.int64), [[0], [0]], p=P, q=Q, seed=7)
    assert w1.shape == (n, 3)
    assert (w1[:, 1] == 1).float().mean() > 0.999
    np.testing.assert_allclose(_shares(w1), WANT, atol=0.01)
    w2 = ea.random_walk(np.zeros(n, np.int64), [[0], [0]], p=P, q=Q, seed=7)
    assert torch.equal(w1, w2), "same seed must give the same walks"
    w3 = ea.random_walk(np.zeros(n, np.int64), [[0], [0]], p=P, q=Q, seed=8)
    assert not torch.equal(w1, w3)
    # global seed sequence: reproducible after set_seed
    ea.set_seed(11)
    a = ea.random_walk(np.zeros(64, np.int64), [[0]] * 4, p=P, q=Q)
    ea.set_seed(11)
    b = ea.random_walk(np.zeros(64, np.int64), [[0]] * 4, p=P, q=Q)
    assert torch.equal(a, b)
    # p = q = 1 is the plain weighted walk: uniform over 1's three neighbours
    u = ea.random_walk(np.zeros(n, np.int64), [[0], [0]], seed=3)
    np.testing.assert_allclose(_shares(u), [1 / 3] * 3, atol=0.01)
    # dead ends fill the default node
    dead = ea.random_walk(np.array([99], np.int64), [[0], [0]], p=P, q=Q, default_node=-1, seed=1)
    assert dead.tolist() == [[99, -1, -1]]


def test_remote_path_node2vec_ratios(monkeypatch):
    """the sharded-mode fallback (per-step full-neighbour queries, vectorised draw)"""
    from euler_amd.ops import graph_api

    _engine()
    w = graph_api._random_walk_remote(np.zeros(30000, np.uint64), [[0], [0]], P, Q, -1, seed=5)
    np.testing.assert_allclose(_shares(w), WANT, atol=0.012)


def _device_graph(device):
    from euler_amd.graph.device_graph import DeviceGraph

    s, d, w = _edges()
    indptr = np.zeros(5, np.int64)
    np.add.at(indptr, s.astype(np.int64) + 1, 1)
    indptr = np.cumsum(indptr)
    return DeviceGraph.from_csr(indptr, d.astype(np.int32), w, seed=3, device=device)


def test_device_graph_node2vec_cpu():
    g = _device_graph("cpu")
    walks = g.random_walk(torch.zeros(40000, dtype=torch.int32), 2, p=P, q=Q)
    np.testing.assert_allclose(_shares(walks), WANT, atol=0.012)


@pytest.mark.gpu
def test_device_graph_node2vec_gpu(cuda):
    g = _device_graph(cuda)
    g.manual_seed(5)
    walks = g.random_walk(torch.zeros(200000, dtype=torch.int32, device=cuda), 2, p=P, q=Q).cpu()
    np.testing.assert_allclose(_shares(walks), WANT, atol=0.008)
    g.manual_seed(5)
    again = g.random_walk(torch.zeros(200000, dtype=torch.int32, device=cuda), 2, p=P, q=Q).cpu()
    assert torch.equal(walks, again)
    plain = g.random_walk(torch.zeros(200000, dtype=torch.int32, device=cuda), 2).cpu()
    np.testing.assert_allclose(_shares(plain), [1 / 3] * 3, atol=0.008)
