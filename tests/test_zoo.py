"""Model zoo smoke-training through the estimators on same-schema synthetic datasets
(reference strategy: every example runner trains for N steps)."""
import os

import numpy as np
import pytest
import torch

import euler_amd as ea
from euler_amd import models as Z
from euler_amd.dataset import get_dataset
from euler_amd.estimator import EdgeEstimator, GraphEstimator, NodeEstimator, latest_checkpoint


@pytest.fixture(scope="module")
def _cora(tmp_path_factory):
    ds = get_dataset("cora", data_dir=str(tmp_path_factory.mktemp("cora")), scale=0.08)
    ds.get_data_dir()
    return ds


@pytest.fixture
def cora(_cora):
    # the engine graph is process-global: (re)activate this dataset for every test
    _cora.load_graph()
    ea.set_seed(3)
    return _cora


def _params(ds, tmp, **kw):
    tnt = ds.train_node_type[0] if isinstance(ds.train_node_type, list) else ds.train_node_type
    p = {"model_dir": str(tmp / "ckpt"), "batch_size": 16, "total_step": 3, "optimizer": "adam",
         "learning_rate": 0.01, "log_steps": 1, "train_node_type": tnt, "id_file": ds.id_file,
         "infer_dir": str(tmp / "infer"), "device": "cpu"}
    p.update(kw)
    return p


F = 1433


def _node_models(ds):
    fi, li, ld = "feature", "label", ds.label_dim
    et = ["train"]
    return {
        "graphsage": lambda: Z.SupervisedGraphSage([16, 16, ld], [3, 3], [et, et], fi, F, li, ld, max_id=ds.max_node_id),
        "gcn": lambda: Z.SupervisedGCN([16, 16, ld], [et, et], fi, F, li, ld),
        "gat": lambda: Z.GAT([16, 16, ld], [et, et], fi, F, li, ld, head_num=2),
        "fastgcn": lambda: Z.FastGCN([16, 16, ld], [8, 8], [et, et], fi, F, li, ld),
        "adaptivegcn": lambda: Z.AdaptiveGCN([16, 16, ld], [8, 8], [et, et], fi, F, li, ld),
        "agnn": lambda: Z.AGNN("f1", [16, 16, ld], [et, et], fi, F, li, ld),
        "appnp": lambda: Z.APPNP([16, 16, ld], [et, et], fi, F, li, ld, K=3),
        "arma": lambda: Z.ARMA([16, 16, ld], [et, et], fi, F, li, ld, K=2, num_layers=2),
        "dna": lambda: Z.DNA([16, 16, ld], [et, et], fi, F, li, ld, head_num=2, group_num=2),
        "sgcn": lambda: Z.SGCN([16, 16, ld], [et, et], fi, F, li, ld, K=2),
        "tagcn": lambda: Z.TAGCN([16, 16, ld], [et, et], fi, F, li, ld, K=2),
        "geniepath": lambda: Z.GeniePath(16, [et, et], li, ld, feature_idx=fi, feature_dim=F, head_num=2),
        "lgcn": lambda: Z.LGCN(16, et, li, ld, feature_idx=fi, feature_dim=F, k=3, nb_num=4, out_dim=8),
    }


@pytest.mark.parametrize("name", ["graphsage", "gcn", "gat", "fastgcn", "adaptivegcn", "agnn", "appnp", "arma",
                                  "dna", "sgcn", "tagcn", "geniepath", "lgcn"])
def test_node_classification_zoo(cora, tmp_path, name):
    torch.manual_seed(0)
    model = _node_models(cora)[name]()
    est = NodeEstimator(model, _params(cora, tmp_path))
    res = est.train()
    assert np.isfinite(res["loss"])
    assert latest_checkpoint(str(tmp_path / "ckpt")).endswith("model.ckpt-3.pt")


def test_estimator_resume_eval_infer(cora, tmp_path):
    torch.manual_seed(0)
    mk = _node_models(cora)["graphsage"]
    NodeEstimator(mk(), _params(cora, tmp_path, total_step=4, save_checkpoints_steps=2)).train()
    # resume continues from step 4 to 6
    est = NodeEstimator(mk(), _params(cora, tmp_path, total_step=6))
    est.train()
    assert est.global_step == 6
    with open(os.path.join(str(tmp_path / "ckpt"), "checkpoint")) as f:
        assert "model.ckpt-6.pt" in f.read()
    ev = NodeEstimator(mk(), _params(cora, tmp_path)).evaluate()
    assert "loss" in ev and "f1" in ev
    ids, embs = NodeEstimator(mk(), _params(cora, tmp_path)).infer()
    n_test = sum(1 for _ in open(cora.id_file))
    assert ids.shape[0] == n_test and embs.shape == (n_test, cora.label_dim)
    assert os.path.exists(str(tmp_path / "infer" / "embedding_0.npy"))
    assert os.path.exists(str(tmp_path / "infer" / "ids_0.npy"))


@pytest.mark.parametrize("name", ["sage_unsup", "deepwalk", "node2vec", "line1", "line2", "dgi", "gae", "vgae"])
def test_unsupervised_zoo(cora, tmp_path, name):
    torch.manual_seed(0)
    mid, et = cora.max_node_id, "train"
    mk = {
        "sage_unsup": lambda: Z.UnsupervisedGraphSage([16, 16, 8], [3, 3], [[et], [et]], "feature", F, "train", et,
                                                      mid, num_negs=3),
        "deepwalk": lambda: Z.DeepWalk("train", et, mid, 8, walk_len=3, num_negs=3),
        "node2vec": lambda: Z.Node2Vec("train", et, mid, 8, walk_len=3, walk_p=0.5, walk_q=2.0, num_negs=3),
        "line1": lambda: Z.Line("train", et, mid, 8, order=1),
        "line2": lambda: Z.Line("train", et, mid, 8, order=2),
        "dgi": lambda: Z.DGI("train", et, mid, [[et], [et]], [3, 3], 8, feature_idx="feature", feature_dim=F),
        "gae": lambda: Z.GraphAutoEncoder("sage", [16, 8], [3], [[et]], "feature", F, "train", et, mid, num_negs=3),
        "vgae": lambda: Z.VariationalGraphAutoEncoder(0.1, "sage", [16, 8], [3], [[et]], "feature", F, "train", et,
                                                      mid, num_negs=3),
    }[name]
    est = NodeEstimator(mk(), _params(cora, tmp_path))
    res = est.train()
    assert np.isfinite(res["loss"])


@pytest.fixture(scope="module")
def _fb(tmp_path_factory):
    ds = get_dataset("fb15k", data_dir=str(tmp_path_factory.mktemp("fb")), scale=0.01)
    ds.get_data_dir()
    return ds


@pytest.fixture
def fb(_fb):
    _fb.load_graph()
    ea.set_seed(5)
    return _fb


@pytest.mark.parametrize("name", ["transe", "transh", "transr", "transd", "distmult"])
def test_kg_zoo(fb, tmp_path, name):
    torch.manual_seed(0)
    args = ("train", "train", fb.max_node_id, fb.max_edge_id, 8, 8)
    model = {"transe": lambda: Z.TransE(*args, num_negs=3), "transh": lambda: Z.TransH(*args, num_negs=3),
             "transr": lambda: Z.TransR(*args[:-1], 6, num_negs=3), "transd": lambda: Z.TransD(*args, num_negs=3),
             "distmult": lambda: Z.DistMult(*args, num_negs=3, l2_regular=True)}[name]()
    p = _params(fb, tmp_path, train_edge_type="train", id_file=fb.edge_id_file, infer_type="node_src",
                batch_size=32, total_step=5)
    est = EdgeEstimator(model, p)
    res = est.train()
    assert np.isfinite(res["loss"])
    ids, embs = EdgeEstimator(model, p).infer()
    assert ids.shape[0] == embs.shape[0] > 0


def test_transe_learns(fb, tmp_path):
    torch.manual_seed(0)
    model = Z.TransE("train", "train", fb.max_node_id, fb.max_edge_id, 16, 16, num_negs=4)
    est = EdgeEstimator(model, _params(fb, tmp_path, train_edge_type="train", batch_size=64, total_step=60,
                                       log_steps=60, learning_rate=0.02))
    first = None
    losses = []
    model.to("cpu")
    est._prepare(est.get_train_from_input(64, est.params))
    for _ in range(60):
        _, loss, _, _ = model(est.get_train_from_input(64, est.params))
        est.optimizer.zero_grad()
        loss.backward()
        est.optimizer.step()
        losses.append(float(loss))
    assert np.mean(losses[-10:]) < np.mean(losses[:10])


@pytest.fixture(scope="module")
def _mutag(tmp_path_factory):
    ds = get_dataset("mutag", data_dir=str(tmp_path_factory.mktemp("mutag")), scale=0.25)
    ds.get_data_dir()
    return ds


@pytest.fixture
def mutag(_mutag):
    _mutag.load_graph()
    ea.set_seed(9)
    return _mutag


@pytest.mark.parametrize("name", ["gin", "gated", "graphgcn", "set2set"])
def test_graph_classification_zoo(mutag, tmp_path, name):
    torch.manual_seed(0)
    fi, fm = mutag.sparse_fea_idx, mutag.sparse_fea_max_id
    model = {"gin": lambda: Z.GIN([8, 8, 8], [["0"], ["0"]], 2, fi, fm),
             "gated": lambda: Z.GatedGraph([8, 8], [["0"]], 2, fi, fm, processing_steps=2),
             "graphgcn": lambda: Z.GraphGCN([8, 8], [["0"]], 2, fi, fm),
             "set2set": lambda: Z.Set2SetModel([8, 8], [["0"]], 2, fi, fm, processing_steps=2)}[name]()
    p = _params(mutag, tmp_path, label=["label"], num_classes=2, batch_size=4)
    est = GraphEstimator(model, p)
    res = est.train()
    assert np.isfinite(res["loss"])
    ev = GraphEstimator(model, p).evaluate()
    assert "accuracy" in ev


def test_rgcn(fb, tmp_path):
    torch.manual_seed(0)
    model = Z.UnsupervisedRGCN("train", "train", fb.max_node_id, [8, 8], [["train"]], fb.max_edge_id + 1, "id", 1,
                               8, num_negs=3)
    res = NodeEstimator(model, _params(fb, tmp_path, batch_size=8)).train()
    assert np.isfinite(res["loss"])


def test_solutions_and_sample_estimator(cora, tmp_path):
    from euler_amd import solution as S
    from euler_amd.estimator import SampleEstimator
    from euler_amd.utils import encoders as E

    torch.manual_seed(0)
    enc = E.SageEncoder([["train"], ["train"]], [3, 3], 16, feature_idx="feature", feature_dim=F,
                        max_id=cora.max_node_id)
    sup = S.SuperviseSolution(S.GetLabelFromFea("label", cora.label_dim), enc, S.DenseLogits(cora.label_dim))
    assert np.isfinite(NodeEstimator(sup, _params(cora, tmp_path)).train()["loss"])

    tgt = E.ShallowEncoder(dim=8, feature_idx=-1, max_id=cora.max_node_id, combiner="add")
    ctx = E.ShallowEncoder(dim=8, feature_idx=-1, max_id=cora.max_node_id, combiner="add")
    uns = S.UnsuperviseSolution(tgt, ctx, S.SamplePosWithTypes("train", 1, cora.max_node_id),
                                S.SampleNegWithTypes("train", 4))
    assert np.isfinite(NodeEstimator(uns, _params(cora, tmp_path / "u")).train()["loss"])

    # explicit sample file: "label,src,dst" rows
    rows = tmp_path / "samples.csv"
    rng = np.random.default_rng(0)
    with open(rows, "w") as f:
        for _ in range(40):
            a, b = rng.integers(0, cora.max_node_id, 2)
            f.write("%d,%d,%d\n" % (int(rng.integers(0, 2)), a, b))

    def parse(batch):
        arr = np.asarray(batch, dtype=np.int64)
        return torch.tensor(arr[:, 0:1], dtype=torch.float32), torch.tensor(arr[:, 1]), torch.tensor(arr[:, 2])

    shared = E.ShallowEncoder(dim=8, feature_idx=-1, max_id=cora.max_node_id, combiner="add")

    class GroupEnc(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.enc = shared

        def forward(self, groups):
            return [self.enc(g) for g in groups]

    sss = S.SuperviseSampleSolution(parse, GroupEnc(), lambda e: (e[0], e[1], e[0]), metric_name="auc")
    p = _params(cora, tmp_path / "s", sample_dir=str(rows), batch_size=8, epoch=2, total_step=None)
    res = SampleEstimator(sss, p).train()
    assert np.isfinite(res["loss"])
    ids, embs = SampleEstimator(sss, _params(cora, tmp_path / "s", sample_dir=str(rows), batch_size=8)).infer()
    assert ids.shape == (40, 1) and embs.shape == (40, 8)


def test_scalable_encoder_through_estimator(cora, tmp_path):
    from euler_amd.mp_utils.models import SuperviseModel
    from euler_amd.utils import encoders as E

    class M(SuperviseModel):
        def __init__(self):
            super().__init__("label", cora.label_dim)
            self.enc = E.ScalableSageEncoder(["train"], 3, 2, 16, feature_idx="feature", feature_dim=F,
                                             max_id=cora.max_node_id)

        def embed(self, n_id):
            return self.enc(n_id)

    m = M()
    res = NodeEstimator(m, _params(cora, tmp_path, total_step=4)).train()
    assert np.isfinite(res["loss"])
    assert float(m.enc.stores(0).abs().sum()) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["graphsage", "gat", "gcn", "dna"])
def test_node_zoo_gpu(cora, tmp_path, name):
    from euler_amd.ops import _native

    assert _native.hip() is not None
    torch.manual_seed(0)
    model = _node_models(cora)[name]()
    res = NodeEstimator(model, _params(cora, tmp_path, device="cuda", total_step=5)).train()
    assert np.isfinite(res["loss"])
    assert next(model.parameters()).is_cuda


@pytest.mark.gpu
def test_kg_zoo_gpu(fb, tmp_path):
    torch.manual_seed(0)
    model = Z.TransE("train", "train", fb.max_node_id, fb.max_edge_id, 16, 16, num_negs=4)
    p = _params(fb, tmp_path, train_edge_type="train", batch_size=64, total_step=5, device="cuda", amp="bf16")
    res = EdgeEstimator(model, p).train()
    assert np.isfinite(res["loss"])


def test_prefetcher_order_and_errors():
    from euler_amd.utils.prefetch import Prefetcher

    it = iter(range(5))
    pf = Prefetcher(lambda: next(it, None), "cpu", depth=2)
    assert [pf.get() for _ in range(5)] == [0, 1, 2, 3, 4]
    with pytest.raises(StopIteration):
        pf.get()
    pf.close()

    def boom():
        raise ValueError("sampler failed")

    pf = Prefetcher(boom, "cpu")
    with pytest.raises(ValueError):
        pf.get()
    pf.close()


@pytest.mark.parametrize("name", ["graphsage", "gat"])
def test_estimator_async_input_pipeline(cora, tmp_path, name):
    """prefetch > 0: engine sampling of the next batches runs on a worker thread"""
    torch.manual_seed(0)
    est = NodeEstimator(_node_models(cora)[name](), _params(cora, tmp_path, total_step=6, prefetch=2))
    res = est.train()
    assert np.isfinite(res["loss"]) and est.global_step == 6


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["graphsage", "gcn", "gat"])
def test_estimator_gpu_prefetch(cora, tmp_path, name):
    """CPU engine sampling -> pinned -> side-stream H2D -> gfx950 kernels, through the estimator"""
    torch.manual_seed(0)
    est = NodeEstimator(_node_models(cora)[name](), _params(cora, tmp_path, total_step=8, device="cuda"))
    res = est.train()
    assert np.isfinite(res["loss"]) and est.global_step == 8
