"""kNN retrieval tool and the graph console (reference knn/knn.py, euler/tools/remote_console)."""
import io
import os
import tempfile
from contextlib import redirect_stdout

import numpy as np
import pytest

import euler_amd as ea
from euler_amd.tools import console, knn
from euler_amd.tools.converter import convert_json

HERE = os.path.dirname(os.path.abspath(__file__))


def test_flat_index_exact():
    rng = np.random.default_rng(0)
    x = rng.normal(size=(500, 16)).astype(np.float32)
    idx = knn.FlatIndex(16, device="cpu")
    idx.add(x)
    D, I = idx.search(x[:7], 5)
    ref = ((x[:7, None, :] - x[None, :, :]) ** 2).sum(-1)
    assert (I[:, 0] == np.arange(7)).all()
    assert np.allclose(np.sort(ref, 1)[:, :5], D, atol=1e-3)


def test_ivfflat_recall():
    rng = np.random.default_rng(1)
    centers = rng.normal(size=(20, 8)) * 10
    x = (centers[rng.integers(0, 20, 4000)] + rng.normal(size=(4000, 8))).astype(np.float32)
    ivf = knn.build_index(x, "ivfflat", device="cpu")
    flat = knn.build_index(x, "flat", device="cpu")
    _, I = ivf.search(x[:50], 10)
    _, J = flat.search(x[:50], 10)
    recall = np.mean([len(set(a) & set(b)) / 10.0 for a, b in zip(I, J)])
    assert recall > 0.9, recall


def test_knn_cli(tmp_path):
    rng = np.random.default_rng(2)
    emb = rng.normal(size=(200, 4)).astype(np.float32)
    ids = np.arange(1000, 1200)
    np.save(tmp_path / "e.npy", emb)
    np.save(tmp_path / "i.npy", ids)
    D, I = knn.main(["--embedding_file", str(tmp_path / "e.npy"), "--id_file", str(tmp_path / "i.npy"),
                     "--index_type", "flat", "--k", "3", "--out", str(tmp_path / "r.npz"), "--device", "cpu"])
    assert (I[:, 0] == ids[:25]).all()
    r = np.load(tmp_path / "r.npz")
    assert r["idx"].shape == (25, 3)


@pytest.fixture(scope="module")
def fixture_graph():
    d = tempfile.mkdtemp(prefix="euler_amd_console_")
    convert_json(os.path.join(HERE, "data", "graph.json"), d, 2, os.path.join(HERE, "data", "index_meta.json"))
    return d


def test_console_commands(fixture_graph):
    ea.initialize_embedded_graph(fixture_graph)
    buf = io.StringIO()
    with redirect_stdout(buf):
        assert console.handle("query_nb 1 0")
        assert console.handle("query_sp_fea 1 f1")
        assert console.handle("query_dense_fea 1 f4 2")
        assert console.handle("gql v(nodes).outV(et).as(nb) -- nodes=1 et=0")
        assert console.handle("stats")
        assert console.handle("bogus")
        assert not console.handle("quit")
    text = buf.getvalue()
    assert "nb: 2 4" in text
    assert "feature: 11 12" in text
    assert "unknown command" in text


def test_cpu_baseline_runs(tmp_path):
    """reference-equivalent CPU path on a small graph: loss drops"""
    import json

    from euler_amd.tools import cpu_baseline

    out = tmp_path / "b.json"
    res = cpu_baseline.main(["--num-nodes", "20000", "--batch-size", "64", "--fanouts", "5,3", "--feature-dim", "32",
                             "--hidden-dim", "32", "--label-dim", "8", "--steps", "30", "--warmup", "1",
                             "--threads", "2", "--out", str(out)])
    assert res["value"] > 0
    first, last = res["config"]["loss_first_last"]
    assert last < first
    assert json.loads(out.read_text())["value"] == res["value"]


def test_engine_out_only_synthetic():
    import numpy as np

    from euler_amd.ops import base

    e = base.synthetic_graph(5000, 6.0, 64, 1, 1, 8, 4, 3, make_current=False, out_only=True)
    nb, w, t = e.sample_neighbor(np.arange(10, dtype=np.uint64), [], 4, np.uint64(5000))
    assert nb.shape == (10, 4) and (nb < 5000).all()
    f = e.dense_feature(np.arange(3, dtype=np.uint64), "dense_feature", 8)
    lab = e.dense_feature(np.arange(3, dtype=np.uint64), "dense_label", 4)
    assert (lab.argmax(1) == f[:, :4].argmax(1)).all()
