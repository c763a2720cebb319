"""NodeEstimator(device_graph=True) for Deep Graph Infomax (models/dgi_trainer.py;
reference examples/dgi/dgi.py:24-90, encoders.py:496-541 ShuffleSageEncoder)."""
import numpy as np
import pytest
import torch

import euler_amd as ea
from euler_amd import models as Z
from euler_amd.dataset import get_dataset
from euler_amd.estimator import NodeEstimator

F = 1433


@pytest.fixture(scope="module")
def _cora(tmp_path_factory):
    ds = get_dataset("cora", data_dir=str(tmp_path_factory.mktemp("cora")), scale=0.08)
    ds.get_data_dir()
    return ds


@pytest.fixture
def cora(_cora):
    _cora.load_graph()
    ea.set_seed(3)
    return _cora


def _params(ds, tmp, device, **kw):
    tnt = ds.train_node_type[0] if isinstance(ds.train_node_type, list) else ds.train_node_type
    p = {"model_dir": str(tmp / "ckpt"), "batch_size": 16, "total_step": 24, "optimizer": "adam",
         "learning_rate": 0.01, "log_steps": 8, "train_node_type": tnt, "device": device, "device_graph": True,
         "seed": 5, "device_feature_dtype": "fp32"}
    p.update(kw)
    return p


def _dgi(ds, agg="mean"):
    torch.manual_seed(0)
    return Z.DGI("train", ["train"], ds.max_node_id, [["train"], ["train"]], [3, 2], 8, aggregator=agg,
                 feature_idx="feature", feature_dim=F)


@pytest.mark.parametrize("agg", ["mean", "gcn"])
def test_dgi_device_path_cpu(cora, tmp_path, agg):
    m = _dgi(cora, agg)
    est = NodeEstimator(m, _params(cora, tmp_path, "cpu"))
    res = est.train()
    assert res["step"] == 24 and np.isfinite(res["loss"]) and 0.0 <= res["acc"] <= 1.0
    # resume continues the sampler's counter
    ctr = int(est.device_trainer.graph.rng[1])
    est2 = NodeEstimator(_dgi(cora, agg), _params(cora, tmp_path, "cpu", total_step=32))
    assert est2.train()["step"] == 32
    assert int(est2.device_trainer.graph.rng[1]) == ctr + 8


def test_dgi_device_tree_and_real_view_match_engine_encoder(cora, tmp_path):
    """the real view of the device step = the model's own SageEncoder aggregation over the
    same sampled tree's features read from the engine (default node: zero features)"""
    import euler_amd.ops.graph_api as ge

    m = _dgi(cora)
    est = NodeEstimator(m, _params(cora, tmp_path, "cpu", total_step=4))
    est.train()
    tr = est.device_trainer
    roots = tr.graph.sample_node(4, stream_id=1).long()
    hops = tr._tree(roots)
    assert [h.numel() for h in hops] == [4, 12, 24]
    ids = np.asarray(tr.graph.ids).astype(np.int64)
    feats = []
    for h in hops:
        x = torch.as_tensor(np.asarray(ge.get_dense_feature(ids[h.clamp(min=0).numpy()], ["feature"], [F])[0]))
        feats.append(x.float().reshape(h.numel(), F) * (h >= 0).unsqueeze(1))
    with torch.no_grad():
        want = m._target_encoder._aggregate(feats)
        got = m._target_encoder._aggregate([tr._features(h) for h in hops])
    assert torch.allclose(got, want, atol=1e-5)
    # the shuffled view is a permutation of per-root positions shared by every root
    sh = tr._shuffle([torch.arange(4.0).view(4, 1), torch.arange(4.0, 16).view(12, 1)])
    flat = torch.cat(sh).view(4, -1)
    orig = torch.cat([torch.arange(4.0).view(4, 1), torch.arange(4.0, 16).view(4, 3)], 1)
    perm = [int((orig[0] == v).nonzero()) for v in flat[0]]
    assert sorted(perm) == [0, 1, 2, 3] and torch.equal(flat, orig[:, perm])


@pytest.mark.gpu
def test_dgi_device_path_gpu_captured(cora, tmp_path, cuda):
    m = _dgi(cora)
    est = NodeEstimator(m, _params(cora, tmp_path, "cuda", total_step=64, log_steps=32, steps_per_graph=8))
    res = est.train()
    assert res["step"] == 64 and np.isfinite(res["loss"]) and est.device_trainer.captures >= 1


def _unsup_solution(ds):
    from euler_amd import solution as S
    from euler_amd.utils import encoders as E

    torch.manual_seed(0)
    mk = lambda: E.SageEncoder([["train"], ["train"]], [3, 2], 8, feature_idx="feature", feature_dim=F,  # noqa
                               max_id=ds.max_node_id)
    return S.UnsuperviseSolution(mk(), mk(), S.SamplePosWithTypes(["train"], 1, ds.max_node_id),
                                 S.SampleNegWithTypes("train", 3))


def test_unsupervise_solution_device_path_cpu(cora, tmp_path):
    """solution.UnsuperviseSolution (base_unsupervise.py:27-73) on the device path"""
    m = _unsup_solution(cora)
    est = NodeEstimator(m, _params(cora, tmp_path, "cpu"))
    res = est.train()
    assert res["step"] == 24 and np.isfinite(res["loss"]) and 0.0 < res["mrr"] <= 1.0
    assert type(est.device_trainer).__name__ == "UnsupSolutionTrainer"


@pytest.mark.gpu
def test_unsupervise_solution_device_path_gpu_captured(cora, tmp_path, cuda):
    m = _unsup_solution(cora)
    est = NodeEstimator(m, _params(cora, tmp_path, "cuda", total_step=64, log_steps=32, steps_per_graph=8))
    res = est.train()
    assert res["step"] == 64 and np.isfinite(res["loss"]) and est.device_trainer.captures >= 1
