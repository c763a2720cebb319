"""Raw-file converters of the dataset registry (euler_amd/dataset/base.py) on small
fixtures in the release formats (no network: the real files cannot be fetched; the
fixtures follow the formats the reference's converters parse)."""
import json
import os

import numpy as np

from euler_amd.dataset.base import Cora, Pubmed

_NODE_TAB = """NODE\tpaper
cat=1,2,3:label\tnumeric:w-rat:0.0\tnumeric:w-insulin:0.0\tnumeric:w-cell:0.0\tstring:summary
12187484\tlabel=1\tw-rat=0.09\tw-cell=0.03\tsummary=w-rat,w-cell
2344352\tlabel=3\tw-insulin=0.2\tsummary=w-insulin
14654069\tlabel=2\tw-rat=0.1\tw-insulin=0.1\tw-cell=0.1\tsummary=w-rat,w-insulin,w-cell
999\tlabel=2\tw-cell=0.5\tsummary=w-cell
"""
_CITES_TAB = """DIRECTED\tcites
NO_FEATURES
33824\tpaper:2344352\t|\tpaper:12187484
33825\tpaper:14654069\t|\tpaper:2344352
33826\tpaper:14654069\t|\tpaper:12187484
"""


def _write(d, name, text):
    p = os.path.join(d, name)
    os.makedirs(os.path.dirname(p), exist_ok=True)
    with open(p, "w") as f:
        f.write(text)


def test_pubmed_tab_converter(tmp_path):
    d = str(tmp_path)
    _write(d, "data/Pubmed-Diabetes.NODE.paper.tab", _NODE_TAB)
    _write(d, "data/Pubmed-Diabetes.DIRECTED.cites.tab", _CITES_TAB)
    ds = Pubmed(data_dir=d)
    ds.test_start_num = 1  # ids 2.. are test nodes in this 4-paper fixture
    assert ds.raw_present()
    data = ds.convert2json(d)
    # ids: first appearance in the citation file (2344352, 12187484, 14654069), then the
    # uncited paper 999
    by_id = {n["id"]: n for n in data["nodes"]}
    assert sorted(by_id) == [0, 1, 2, 3]
    feat = lambda i: np.asarray(by_id[i]["features"][1]["value"])  # noqa: E731
    lab = lambda i: by_id[i]["features"][0]["value"]  # noqa: E731
    # 12187484 -> id 1: rat 0.09, cell 0.03, normalised to sum 1, label 1 -> [1, 0, 0]
    np.testing.assert_allclose(feat(1), np.array([0.09, 0.0, 0.03]) / (0.12 + 1e-7))
    assert lab(1) == [1.0, 0.0, 0.0] and lab(0) == [0.0, 0.0, 1.0] and lab(2) == [0.0, 1.0, 0.0]
    np.testing.assert_allclose(feat(3), [0.0, 0.0, 1.0], rtol=1e-6)
    assert [by_id[i]["type"] for i in range(4)] == ["train", "train", "test", "test"]
    # one directed edge per citation; an end past test_start_num -> train_removed
    got = [(e["src"], e["dst"], e["type"]) for e in data["edges"]]
    assert got == [(0, 1, "train"), (2, 0, "train_removed"), (2, 1, "train_removed")]
    with open(ds.id_file) as f:
        assert [int(x) for x in f.read().split()] == [2, 3]


def test_pubmed_raw_files_load_into_the_engine(tmp_path):
    d = str(tmp_path)
    _write(d, "data/Pubmed-Diabetes.NODE.paper.tab", _NODE_TAB)
    _write(d, "data/Pubmed-Diabetes.DIRECTED.cites.tab", _CITES_TAB)
    ds = Pubmed(data_dir=d)
    ds.load_graph()
    assert not ds.synthetic
    import euler_amd.ops.graph_api as ge

    f = np.asarray(ge.get_dense_feature(np.array([1, 3]), ["feature"], [3])[0])
    np.testing.assert_allclose(f[0], np.array([0.09, 0.0, 0.03]) / (0.12 + 1e-7), rtol=1e-5)
    np.testing.assert_allclose(f[1], [0.0, 0.0, 1.0], rtol=1e-5)


def test_cora_planetoid_converter(tmp_path):
    d = str(tmp_path)
    _write(d, "cora.content", "31336\t0\t1\t1\tNeural_Networks\n1061127\t1\t0\t0\tRule_Learning\n"
                              "1106406\t0\t0\t1\tNeural_Networks\n")
    _write(d, "cora.cites", "31336\t1061127\n1106406\t31336\n")
    ds = Cora(data_dir=d)
    ds.test_start_num = 2
    data = ds.convert2json(d)
    assert [n["type"] for n in data["nodes"]] == ["train", "train", "test"]
    np.testing.assert_allclose(data["nodes"][0]["features"][1]["value"], [0.0, 0.5, 0.5], rtol=1e-6)
    # undirected: both directions of each citation (cited <- citing)
    got = sorted((e["src"], e["dst"], e["type"]) for e in data["edges"])
    assert got == [(0, 1, "train"), (0, 2, "train_removed"), (1, 0, "train"), (2, 0, "train_removed")]
    json.dumps(data)
