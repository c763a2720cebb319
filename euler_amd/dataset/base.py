"""Dataset registry, raw-file converters and same-schema synthetic generators
(reference ``tf_euler/python/dataset/{base_dataset,utils,cora,citeseer,pubmed,ppi,reddit,
fb15k,fb15k237,wn18,mutag,ml_1m,test_data}.py``)."""
from __future__ import annotations

import json
import os
import shutil

import numpy as np

__all__ = ["DataSet", "get_dataset", "dataset_names", "Cora", "Citeseer", "Pubmed", "PPI", "Reddit", "FB15K",
           "FB15K237", "WN18", "Mutag", "MovieLens1M", "TestData", "Community"]

_HOME = os.environ.get("EULER_AMD_DATA", os.path.join(os.path.expanduser("~"), ".euler_amd", "data"))


def _node(i, t, feats, w=1.0):
    return {"id": int(i), "type": t, "weight": float(w), "features": feats}


def _edge(s, d, t, feats=None, w=1.0):
    return {"src": int(s), "dst": int(d), "type": t, "weight": float(w), "features": feats or []}


class DataSet:
    """Base: ``load_graph()`` = (raw -> json | synthetic json) -> Euler binary ->
    ``initialize_embedded_graph`` (base_dataset.py:38-118)."""

    name = "base"
    partition_num = 1

    def __init__(self, data_dir=None, data_type="all", scale=1.0, seed=0, synthetic=None):
        self.data_dir = data_dir or os.path.join(_HOME, self.name)
        self.data_type = data_type
        self.scale = float(scale)
        self.seed = int(seed)
        self.force_synthetic = synthetic
        self.synthetic = False
        self.meta_file = None
        self.origin_files = []
        self.id_file = os.path.join(self.data_dir, "%s_test.id" % self.name)

    # ------------------------------------------------------------------ pipeline
    def raw_present(self):
        return bool(self.origin_files) and all(os.path.exists(os.path.join(self.data_dir, f))
                                               for f in self.origin_files)

    def get_data_dir(self):
        """Prepare ``<data_dir>/euler``.  Under torch.distributed rank 0 prepares while
        the other ranks wait at a barrier, then everyone reads the same files."""
        from euler_amd.parallel import dp

        if not dp.is_distributed():
            return self._prepare()
        if dp.rank() == 0:
            try:
                return self._prepare()
            finally:
                dp.barrier()
        dp.barrier()
        return self._prepare()

    def _prepare(self):
        os.makedirs(self.data_dir, exist_ok=True)
        out = os.path.join(self.data_dir, "euler")
        stamp = os.path.join(out, "euler.meta")
        if os.path.exists(stamp):
            self.synthetic = os.path.exists(os.path.join(self.data_dir, "SYNTHETIC"))
            return out
        use_raw = self.raw_present() and self.force_synthetic is not True
        if use_raw:
            data = self.convert2json(self.data_dir)
        else:
            if self.force_synthetic is False:
                raise FileNotFoundError("raw files %s not found under %s (no network to download them)"
                                        % (self.origin_files, self.data_dir))
            data = self.synthesize(np.random.default_rng(self.seed))
            self.synthetic = True
            with open(os.path.join(self.data_dir, "SYNTHETIC"), "w") as f:
                f.write("synthetic graph of the %s schema (scale %.4g)\n" % (self.name, self.scale))
        self.convert2euler(data, out)
        return out

    def load_graph(self):
        from euler_amd.ops.base import initialize_embedded_graph

        d = self.get_data_dir()
        if not initialize_embedded_graph(d, data_type=self.data_type):
            raise RuntimeError("Failed to initialize graph.")
        return d

    def convert2euler(self, data, out_dir):
        from euler_amd.tools.converter import EulerGenerator

        if os.path.isdir(out_dir):
            shutil.rmtree(out_dir)
        meta = None
        if self.meta_file and os.path.exists(self.meta_file):
            meta = self.meta_file
        EulerGenerator(data, meta, out_dir, self.partition_num).do()

    def convert2json(self, origin_dir):
        raise NotImplementedError("raw conversion for %s" % self.name)

    def synthesize(self, rng):
        raise NotImplementedError

    def remove_data(self):
        shutil.rmtree(self.data_dir, ignore_errors=True)

    def _n(self, full):
        return max(8, int(round(full * self.scale)))

    def _write_ids(self, ids, path=None):
        with open(path or self.id_file, "w") as f:
            for i in ids:
                f.write("%s\n" % (i,))


# ============================================================================ node classification
class _Citation(DataSet):
    """Homophilous citation-style graph: bag-of-words features, one-hot labels,
    ``train`` / ``test`` node types, ``train`` / ``train_removed`` edges (gcn_utils.py)."""

    num_nodes = 0
    feature_dim = 0
    label_dim = 0
    test_start_num = 0
    multilabel = False
    avg_degree = 4.0
    words_per_node = 18

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.max_node_id = self._n(self.num_nodes) if self.scale != 1.0 else self.num_nodes
        self.total_size = self.max_node_id
        self.train_node_type = ["train"]
        self.train_edge_type = ["train"]
        self.all_node_type = -1
        self.all_edge_type = ["train", "train_removed"]
        self.feature_idx, self.label_idx = "feature", "label"
        self.num_classes = self.label_dim if not self.multilabel or self.label_dim > 1 else self.label_dim

    def _split_start(self, n):
        return int(round(self.test_start_num * n / max(self.num_nodes, 1)))

    def synthesize(self, rng):
        n, F, L = self.total_size, self.feature_dim, self.label_dim
        cls = rng.integers(0, max(L, 1), n)
        start = self._split_start(n)
        # class-specific vocabularies make the labels learnable from features
        vocab = rng.integers(0, F, (max(L, 1), max(F // max(L, 1), 4)))
        nodes = []
        for i in range(n):
            words = np.concatenate([rng.choice(vocab[cls[i]], self.words_per_node // 2),
                                    rng.integers(0, F, self.words_per_node - self.words_per_node // 2)])
            feat = np.bincount(words, minlength=F).astype(np.float64)
            feat /= feat.sum() + 1e-7
            if self.multilabel:
                lab = (rng.random(L) < 0.15).astype(np.float64)
                lab[cls[i] % L] = 1.0
            elif L == 1:
                lab = np.asarray([float(cls[i])])
            else:
                lab = np.eye(L)[cls[i]]
            t = "train" if i < start else "test"
            nodes.append(_node(i, t, [{"name": "label", "type": "dense", "value": lab.tolist()},
                                      {"name": "feature", "type": "dense", "value": feat.tolist()}]))
        m = int(n * self.avg_degree / 2)
        src = rng.integers(0, n, m)
        same = rng.random(m) < 0.8
        by_cls = [np.flatnonzero(cls == c) for c in range(max(L, 1))]
        dst = np.where(same, [rng.choice(by_cls[cls[s]]) if len(by_cls[cls[s]]) else s for s in src],
                       rng.integers(0, n, m))
        edges = []
        for s, d in zip(src.tolist(), dst.tolist()):
            if s == d:
                continue
            t = "train" if s < start and d < start else "train_removed"
            edges.append(_edge(s, d, t))
            edges.append(_edge(d, s, t))
        self._write_ids(range(start, n))
        return {"nodes": nodes, "edges": edges}


class Community(_Citation):
    """Planted-community node classification (no reference counterpart: a learnable
    synthetic task for the supervised GraphSAGE paths).  Node i is in community i % 64
    (dataset/synthetic.py community_graph: 90 % of edges inside the community, both
    directions stored), its label is its community mod 16 (10 % flipped,
    community_labels, one-hot), its features a weak noisy community cue
    (community_features) — the neighbourhood mean carries the signal, so aggregation
    must beat a feature-only classifier.  Test nodes are the last 20 %."""

    name, num_nodes, feature_dim, label_dim, test_start_num = "community", 20000, 64, 16, 16000
    num_comm = 64
    avg_degree = 10.0

    def synthesize(self, rng):
        from euler_amd.dataset.synthetic import community_features, community_graph, community_labels

        n, L = self.total_size, self.label_dim
        seed = int(rng.integers(0, 2 ** 31))
        src, dst, comm = community_graph(n, self.num_comm, self.avg_degree / 2, seed=seed)
        x = community_features(comm, self.feature_dim, signal=0.5, seed=seed).numpy()
        y = community_labels(comm, L, noise=0.1, seed=seed).numpy()
        start = self._split_start(n)
        eye = np.eye(L)
        nodes = [_node(i, "train" if i < start else "test",
                       [{"name": "label", "type": "dense", "value": eye[y[i]].tolist()},
                        {"name": "feature", "type": "dense", "value": x[i].tolist()}]) for i in range(n)]
        edges = []
        for s, d in zip(src.tolist(), dst.tolist()):
            if s == d:
                continue
            t = "train" if s < start and d < start else "train_removed"
            edges.append(_edge(s, d, t))
            edges.append(_edge(d, s, t))
        self._write_ids(range(start, n))
        return {"nodes": nodes, "edges": edges}


class Cora(_Citation):
    name, num_nodes, feature_dim, label_dim, test_start_num = "cora", 2708, 1433, 7, 1708

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.origin_files = ["cora.cites", "cora.content"]

    def convert2json(self, d):
        return _planetoid_like(self, os.path.join(d, "cora.content"), os.path.join(d, "cora.cites"))


class Citeseer(_Citation):
    name, num_nodes, feature_dim, label_dim, test_start_num = "citeseer", 3327, 3703, 6, 2312

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.origin_files = ["citeseer.cites", "citeseer.content"]

    def convert2json(self, d):
        return _planetoid_like(self, os.path.join(d, "citeseer.content"), os.path.join(d, "citeseer.cites"))


class Pubmed(_Citation):
    name, num_nodes, feature_dim, label_dim, test_start_num = "pubmed", 19717, 500, 3, 18717
    words_per_node = 50

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.origin_files = ["data/Pubmed-Diabetes.NODE.paper.tab", "data/Pubmed-Diabetes.DIRECTED.cites.tab"]

    def convert2json(self, d):
        return _pubmed_tab(self, os.path.join(d, self.origin_files[0]), os.path.join(d, self.origin_files[1]))


class PPI(_Citation):
    name, num_nodes, feature_dim, label_dim, test_start_num = "ppi", 56944, 50, 121, 51420
    multilabel = True
    avg_degree = 28.0

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.origin_files = ["ppi-G.json", "ppi-feats.npy", "ppi-class_map.json", "ppi-id_map.json"]

    def convert2json(self, d):
        return _graphsage_format(self, d, "ppi")


class Reddit(_Citation):
    name, num_nodes, feature_dim, label_dim, test_start_num = "reddit", 231443, 602, 1, 176000
    avg_degree = 50.0

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.num_classes = 41
        self.max_node_id = 240000 if self.scale == 1.0 else self.total_size
        self.origin_files = ["reddit-G.json", "reddit-feats.npy", "reddit-class_map.json", "reddit-id_map.json"]

    def synthesize(self, rng):
        # one label column holding the class id (label_dim 1, 41 classes)
        L = self.label_dim
        self.label_dim = self.num_classes
        try:
            data = super().synthesize(rng)
        finally:
            self.label_dim = L
        for nd in data["nodes"]:
            lab = nd["features"][0]["value"]
            nd["features"][0]["value"] = [float(int(np.argmax(lab)))]
        return data

    def convert2json(self, d):
        return _graphsage_format(self, d, "reddit")


def _planetoid_like(ds, content, cites):
    """``<paper> <w_1..w_F> <label>`` + ``<cited> <citing>`` files (gcn_utils.parse_graph_file)."""
    ids, feats, labels = [], [], []
    with open(content) as f:
        for line in f:
            a = line.strip().split()
            if len(a) < 3:
                continue
            ids.append(a[0])
            feats.append(np.asarray(a[1:-1], np.float64))
            labels.append(a[-1])
    classes = sorted(set(labels))
    idmap = {p: i for i, p in enumerate(ids)}
    nodes = []
    start = ds.test_start_num
    for i, (fv, lab) in enumerate(zip(feats, labels)):
        fv = fv / (fv.sum() + 1e-7)
        one = np.eye(len(classes))[classes.index(lab)]
        nodes.append(_node(i, "train" if i < start else "test",
                           [{"name": "label", "type": "dense", "value": one.tolist()},
                            {"name": "feature", "type": "dense", "value": fv.tolist()}]))
    edges = []
    with open(cites) as f:
        for line in f:
            a = line.strip().split()
            if len(a) != 2 or a[0] not in idmap or a[1] not in idmap:
                continue
            s, d = idmap[a[1]], idmap[a[0]]
            t = "train" if s < start and d < start else "train_removed"
            edges += [_edge(s, d, t), _edge(d, s, t)]
    ds._write_ids(range(start, len(ids)))
    return {"nodes": nodes, "edges": edges}


def _pubmed_tab(ds, node_tab, cites_tab):
    """Pubmed-Diabetes release (reference pubmed.py:38-41 + pubmed_utils.py): node ids in
    order of first appearance in the DIRECTED citation file (papers that are never cited and
    cite nothing follow, in node-file order); one directed edge per citation, ``train_removed``
    when an end is past ``test_start_num``; TF-IDF features in the header's word order,
    normalised to sum 1; one-hot labels of ``label=1..3``; ``test`` nodes past
    ``test_start_num`` (the reference's ``id > train_num``), their ids in the id file."""
    node_map, cites = {}, []
    with open(cites_tab) as f:
        for line in f:
            a = line.strip().split("\t")
            if len(a) != 4:
                continue
            s, t = a[1].split(":", 1)[1], a[3].split(":", 1)[1]
            for p in (s, t):
                if p not in node_map:
                    node_map[p] = len(node_map)
            cites.append((node_map[s], node_map[t]))
    words, rows = None, []
    with open(node_tab) as f:
        for line in f:
            a = line.rstrip("\n").split("\t")
            if len(a) <= 2:
                continue
            if a[0].startswith("cat="):  # header: cat=1,2,3:label, numeric:<word>:0.0, ..., string:summary
                words = {fld.split(":")[-2]: i for i, fld in enumerate(a[1:-1])}
                continue
            rows.append(a)
    if words is None:
        raise ValueError("%s: no feature header line" % node_tab)
    start = ds.test_start_num
    nodes, test_ids = [], []
    for a in rows:
        if a[0] not in node_map:
            node_map[a[0]] = len(node_map)
        i = node_map[a[0]]
        one = np.zeros(ds.label_dim)
        one[int(a[1].split("=")[1]) - 1] = 1.0
        fv = np.zeros(len(words))
        for fld in a[2:-1]:
            k, v = fld.split("=")
            fv[words[k]] = float(v)
        fv = fv / (fv.sum() + 1e-7)
        t = "test" if i > start else "train"
        if t == "test":
            test_ids.append(i)
        nodes.append(_node(i, t, [{"name": "label", "type": "dense", "value": one.tolist()},
                                  {"name": "feature", "type": "dense", "value": fv.tolist()}]))
    edges = [_edge(s, t, "train_removed" if s > start or t > start else "train") for s, t in cites]
    ds._write_ids(test_ids)
    return {"nodes": nodes, "edges": edges}


def _graphsage_format(ds, d, prefix):
    """GraphSAGE release format: -G.json (networkx node-link), -feats.npy,
    -class_map.json, -id_map.json (ppi.py / reddit.py)."""
    with open(os.path.join(d, prefix + "-G.json")) as f:
        g = json.load(f)
    feats = np.load(os.path.join(d, prefix + "-feats.npy"), allow_pickle=False)
    with open(os.path.join(d, prefix + "-class_map.json")) as f:
        cmap = json.load(f)
    with open(os.path.join(d, prefix + "-id_map.json")) as f:
        imap = json.load(f)
    nodes, test = [], []
    for nd in g["nodes"]:
        key = str(nd["id"])
        i = int(imap[key])
        lab = cmap[key]
        lab = lab if isinstance(lab, list) else [float(lab)]
        t = "test" if nd.get("test") else ("val" if nd.get("val") else "train")
        if t == "test":
            test.append(i)
        nodes.append(_node(i, t, [{"name": "label", "type": "dense", "value": [float(x) for x in lab]},
                                  {"name": "feature", "type": "dense", "value": feats[i].astype(float).tolist()}]))
    types = {int(imap[str(n["id"])]): n for n in g["nodes"]}
    edges = []
    for lk in g["links"]:
        s, t = int(imap[str(lk["source"])]), int(imap[str(lk["target"])])
        rm = types[s].get("test") or types[t].get("test") or types[s].get("val") or types[t].get("val")
        et = "train_removed" if rm else "train"
        edges += [_edge(s, t, et), _edge(t, s, et)]
    ds._write_ids(test)
    return {"nodes": nodes, "edges": edges}


# ============================================================================ knowledge graphs
class _KG(DataSet):
    """Entities are nodes (type ``train``); each triple is an edge whose type is the
    split (train / valid / test) and whose dense feature ``id`` is the relation
    (fb15k.py:44-82)."""

    num_entities = 0
    num_relations = 0
    num_triples = 0
    raw_names = ("train.txt", "valid.txt", "test.txt")

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.max_node_id = self._n(self.num_entities) if self.scale != 1.0 else self.num_entities
        self.max_edge_id = self.num_relations
        self.train_node_type = ["train"]
        self.train_edge_type = ["train"]
        self.total_size = self._n(self.num_triples) if self.scale != 1.0 else self.num_triples
        self.all_node_type = -1
        self.all_edge_type = ["train", "valid", "test"]
        self.edge_id_idx, self.edge_id_dim = "id", 1
        self.edge_id_file = os.path.join(self.data_dir, "%s_test.edgeid" % self.name)
        self.node_id_file = os.path.join(self.data_dir, "%s_test.nodeid" % self.name)
        self.id_file = self.edge_id_file
        self.origin_files = list(self.raw_names)

    def _emit(self, triples_by_split, n_ent):
        nodes = [_node(i, "train", []) for i in range(n_ent)]
        edges, test_edges = [], []
        for split, triples in triples_by_split.items():
            for h, t, r in triples:
                edges.append(_edge(h, t, split, [{"name": "id", "type": "dense", "value": [float(r)]}]))
                if split == "test":
                    test_edges.append((h, t))
        # test edge ids: "src dst type" with type = the test split's edge type id (2)
        self._write_ids(["%d %d 2" % e for e in test_edges], self.edge_id_file)
        self._write_ids(sorted({h for h, _ in test_edges}), self.node_id_file)
        return {"nodes": nodes, "edges": edges}

    def synthesize(self, rng):
        n, R, m = self.max_node_id, max(self.num_relations, 1), self.total_size
        # latent translation model: t ~ h + r in a 1-D ring, so TransE can fit it
        h = rng.integers(0, n, m)
        r = rng.integers(0, R, m)
        shift = (np.arange(R) * 7919 + 13) % n
        t = (h + shift[r] + rng.integers(-2, 3, m)) % n
        split = rng.random(m)
        sp = {"train": [], "valid": [], "test": []}
        for i in range(m):
            k = "train" if split[i] < 0.9 else ("valid" if split[i] < 0.95 else "test")
            if h[i] != t[i]:
                sp[k].append((int(h[i]), int(t[i]), int(r[i])))
        return self._emit(sp, n)

    def convert2json(self, d):
        ent, rel = {}, {}
        sp = {}
        for split, fn in zip(("train", "valid", "test"), self.raw_names):
            rows = []
            with open(os.path.join(d, fn)) as f:
                for line in f:
                    a = line.strip().split("\t") if "\t" in line else line.strip().split()
                    if len(a) != 3:
                        continue
                    h, r, t = a
                    hi = ent.setdefault(h, len(ent))
                    ti = ent.setdefault(t, len(ent))
                    ri = rel.setdefault(r, len(rel))
                    rows.append((hi, ti, ri))
            sp[split] = rows
        self.max_node_id, self.max_edge_id = len(ent), len(rel)
        return self._emit(sp, len(ent))


class FB15K(_KG):
    name, num_entities, num_relations, num_triples = "fb15k", 14951, 1345, 592213
    raw_names = ("freebase_mtr100_mte100-train.txt", "freebase_mtr100_mte100-valid.txt",
                 "freebase_mtr100_mte100-test.txt")


class FB15K237(_KG):
    name, num_entities, num_relations, num_triples = "fb15k-237", 14541, 237, 310116
    raw_names = ("Release/train.txt", "Release/valid.txt", "Release/test.txt")


class WN18(_KG):
    name, num_entities, num_relations, num_triples = "wn18", 40943, 18, 151442
    raw_names = ("wordnet-mlj12/wordnet-mlj12-train.txt", "wordnet-mlj12/wordnet-mlj12-valid.txt",
                 "wordnet-mlj12/wordnet-mlj12-test.txt")


# ============================================================================ graph classification
class Mutag(DataSet):
    """188 molecule graphs; node sparse feature ``f1`` (atom type < 7), dense ``label``
    = graph class, binary ``graph_label`` = graph id, hash index on graph_label (mutag.py)."""

    name = "mutag"
    partition_num = 3

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.max_graph_id = self._n(188) if self.scale != 1.0 else 188
        self.total_size = self.max_graph_id
        self.max_node_id = 3371
        self.max_edge_id = 7442
        self.train_node_type = -1
        self.train_edge_type = ["0"]
        self.all_node_type = -1
        self.all_edge_type = ["0"]
        self.train_rate = 0.9
        self.sparse_fea_idx = "f1"
        self.sparse_fea_max_id = 7
        self.num_classes = 2
        self.label_idx, self.label_dim = "label", 1
        self.meta_file = os.path.join(self.data_dir, "mutag_meta.json")
        self.origin_files = ["MUTAG_A.txt", "MUTAG_graph_indicator.txt", "MUTAG_graph_labels.txt",
                             "MUTAG_node_labels.txt"]

    def _index_meta(self):
        os.makedirs(self.data_dir, exist_ok=True)
        with open(self.meta_file, "w") as f:
            json.dump({"node": {"features": {"graph_label": "graph_label:string:uint64_t:hash_index"}},
                       "edge": {}}, f)

    def _emit(self, edges, indicator, glabels, nlabels):
        nodes = []
        for i, (g, nl) in enumerate(zip(indicator, nlabels)):
            nodes.append(_node(i, int(nl), [{"name": "f1", "type": "sparse", "value": [int(nl)]},
                                            {"name": "label", "type": "dense", "value": [float(glabels[g])]},
                                            {"name": "graph_label", "type": "binary", "value": str(g)}]))
        es = [_edge(s, d, 0) for s, d in edges]
        self._index_meta()
        G = len(glabels)
        self._write_ids(range(int(G * self.train_rate), G))
        return {"nodes": nodes, "edges": es}

    def synthesize(self, rng):
        G = self.max_graph_id
        glabels = rng.integers(0, 2, G)
        indicator, nlabels, edges = [], [], []
        nid = 0
        for g in range(G):
            size = int(rng.integers(10, 28))
            # class 1 molecules carry more atoms of types 4..6
            p = np.full(7, 1.0)
            p[4:] += 3.0 * glabels[g]
            p /= p.sum()
            atoms = rng.choice(7, size, p=p)
            base = nid
            for a in atoms:
                indicator.append(g)
                nlabels.append(int(a))
                nid += 1
            for k in range(1, size):  # a chain plus a few rings
                j = base + int(rng.integers(0, k))
                edges += [(base + k, j), (j, base + k)]
        self.max_node_id = nid
        return self._emit(edges, indicator, glabels, nlabels)

    def convert2json(self, d):
        def ints(fn):
            with open(os.path.join(d, fn)) as f:
                return [int(x.strip()) for x in f if x.strip()]

        with open(os.path.join(d, "MUTAG_A.txt")) as f:
            edges = [tuple(int(v) - 1 for v in line.replace(",", " ").split()) for line in f if line.strip()]
        indicator = [g - 1 for g in ints("MUTAG_graph_indicator.txt")]
        glabels = [max(v, 0) for v in ints("MUTAG_graph_labels.txt")]
        return self._emit(edges, indicator, glabels, ints("MUTAG_node_labels.txt"))


# ============================================================================ recommendation
class MovieLens1M(DataSet):
    """Users and movies as nodes, ratings as ``train`` edges; user/movie sparse
    features (gender, age, occupation / genres) (ml_1m.py)."""

    name = "movielens-1m"

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.movie_len = self._n(3952) if self.scale != 1.0 else 3952
        self.num_users = self._n(6040) if self.scale != 1.0 else 6040
        self.max_node_id = self.movie_len + self.num_users
        self.total_size = self.max_node_id
        self.train_node_type = ["train"]
        self.train_edge_type = ["train"]
        self.all_node_type = -1
        self.all_edge_type = ["train", "train_removed"]
        self.origin_files = ["ml-1m/movies.dat", "ml-1m/users.dat", "ml-1m/ratings.dat"]

    def synthesize(self, rng):
        M, U = self.movie_len, self.num_users
        nodes = [_node(i, "train", [{"name": "genre", "type": "sparse",
                                     "value": sorted(set(rng.integers(0, 18, 2).tolist()))}]) for i in range(M)]
        nodes += [_node(M + u, "train", [{"name": "user", "type": "sparse",
                                          "value": [int(rng.integers(0, 2)), 2 + int(rng.integers(0, 7)),
                                                    9 + int(rng.integers(0, 21))]}]) for u in range(U)]
        edges = []
        for u in range(U):
            for m in rng.integers(0, M, 20):
                t = "train" if rng.random() < 0.9 else "train_removed"
                r = float(rng.integers(1, 6))
                edges += [_edge(M + u, m, t, w=r), _edge(m, M + u, t, w=r)]
        self._write_ids(range(M, M + U))
        return {"nodes": nodes, "edges": edges}

    def convert2json(self, d):
        genre = ["Action", "Adventure", "Animation", "Children's", "Comedy", "Crime", "Documentary", "Drama",
                 "Fantasy", "Film-Noir", "Horror", "Musical", "Mystery", "Romance", "Sci-Fi", "Thriller", "War",
                 "Western"]
        gmap = {g: i for i, g in enumerate(genre)}
        age = {"1": 0, "18": 1, "25": 2, "35": 3, "45": 4, "50": 5, "56": 6}
        nodes, edges = [], []
        M = 3952
        with open(os.path.join(d, "ml-1m/movies.dat"), encoding="latin-1") as f:
            for line in f:
                a = line.strip().split("::")
                if len(a) == 3:
                    nodes.append(_node(int(a[0]) - 1, "train", [{"name": "genre", "type": "sparse",
                                                                 "value": [gmap[g] for g in a[2].split("|")
                                                                           if g in gmap]}]))
        with open(os.path.join(d, "ml-1m/users.dat"), encoding="latin-1") as f:
            for line in f:
                a = line.strip().split("::")
                if len(a) >= 4:
                    nodes.append(_node(M + int(a[0]) - 1, "train", [{"name": "user", "type": "sparse",
                                                                     "value": [0 if a[1] == "M" else 1,
                                                                               2 + age.get(a[2], 0),
                                                                               9 + int(a[3])]}]))
        with open(os.path.join(d, "ml-1m/ratings.dat"), encoding="latin-1") as f:
            for line in f:
                a = line.strip().split("::")
                if len(a) >= 3:
                    u, m, r = M + int(a[0]) - 1, int(a[1]) - 1, float(a[2])
                    edges += [_edge(u, m, "train", w=r), _edge(m, u, "train", w=r)]
        self._write_ids(sorted({n["id"] for n in nodes if n["id"] >= M}))
        return {"nodes": nodes, "edges": edges}


# ============================================================================ test fixture
class TestData(DataSet):
    """The 6-node fixture of the reference's tests (tools/test_data/graph.json)."""

    name = "test_data"
    partition_num = 2

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.max_node_id = 6
        self.train_node_type = [0, 1]
        self.train_edge_type = [0, 1]
        self.total_size = 6
        self.all_node_type = -1
        self.all_edge_type = [0, 1]
        self.id_file = ""
        here = os.path.dirname(os.path.abspath(__file__))
        self._fixture = os.path.join(here, "test_data", "graph.json")
        self.meta_file = os.path.join(here, "test_data", "index_meta.json")
        self.origin_files = []

    def raw_present(self):
        return os.path.exists(self._fixture)

    def convert2json(self, d):
        with open(self._fixture) as f:
            return json.load(f)


_REGISTRY = {
    "cora": Cora, "citeseer": Citeseer, "pubmed": Pubmed, "ppi": PPI, "reddit": Reddit, "fb15k": FB15K,
    "fb15k-237": FB15K237, "wn18": WN18, "mutag": Mutag, "movielens-1m": MovieLens1M, "test_data": TestData,
    "community": Community,
}


def dataset_names():
    return sorted(_REGISTRY)


def get_dataset(data_name, **kwargs):
    """``get_dataset(name)`` (dataset/utils.py:33-71); kwargs: data_dir, scale, seed, synthetic."""
    key = data_name.lower()
    if key not in _REGISTRY:
        raise RuntimeError("Failed to get dataset. Dataset name must be one of %s" % dataset_names())
    return _REGISTRY[key](**kwargs)
