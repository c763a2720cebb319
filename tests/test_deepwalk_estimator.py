"""NodeEstimator(device_graph=True) for DeepWalk / Node2Vec (models/deepwalk_step.py
DeepWalkEstimatorTrainer; reference examples/deepwalk/deepwalk.py:27-99): walks, skip-gram
pairs, negatives and the row-sparse SGNS update on the HBM graph; the model's two id
tables are the trainer's table halves."""
import numpy as np
import pytest
import torch

import euler_amd as ea
from euler_amd import models as Z
from euler_amd.dataset import get_dataset
from euler_amd.estimator import NodeEstimator


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
    p = {"model_dir": str(tmp / "ckpt"), "batch_size": 32, "total_step": 30, "optimizer": "adam",
         "learning_rate": 0.02, "log_steps": 10, "train_node_type": tnt, "device": device, "device_graph": True,
         "seed": 11}
    p.update(kw)
    return p


def _model(ds, cls=Z.DeepWalk, **kw):
    torch.manual_seed(0)
    return cls("train", ["train"], ds.max_node_id, 8, walk_len=3, num_negs=3, **kw)


@pytest.mark.parametrize("sharded", [False, True])
def test_model_tables_are_views_of_the_trainer_halves(cora, tmp_path, sharded):
    """the model's two id tables keep their values and become views of the trainer's table
    halves (no second copy of a table while the trainer owns it); per-rank shard files
    round-trip the rows and the optimizer slots"""
    from euler_amd.graph.device_graph import DeviceGraph
    from euler_amd.models.deepwalk_step import DeepWalkEstimatorTrainer

    m = _model(cora, sharded=sharded)
    est = NodeEstimator(m, _params(cora, tmp_path, "cpu"))
    est._prepare(est.get_train_from_input(32, est.params))
    before = {k: v.clone() for k, v in m.state_dict().items()}
    tr = DeepWalkEstimatorTrainer(m, DeviceGraph.from_engine(device="cpu"), 32)
    t = tr.inner.table
    assert len(tr._keys) == 2
    for h, key in enumerate(tr._keys):
        w = m.state_dict()[key]
        assert w.shape[0] == cora.max_node_id + 2  # the pad row max_id + 1 included
        assert torch.equal(w, before[key])
        assert w.data_ptr() == t.weight[h * tr._offw].data_ptr()
    for _ in range(3):
        tr.step()
    trained = {k: v.clone() for k, v in m.state_dict().items()}
    assert any(not torch.equal(trained[k], before[k]) for k in tr._keys)
    slots = {k: getattr(t, k).clone() for k in t.slot_kinds()}
    ck = str(tmp_path / "model.ckpt-3.pt")
    metas = {k: [v] for k, v in tr.checkpoint_shards(ck).items()}
    with torch.no_grad():
        t.weight.zero_()
        for k in t.slot_kinds():
            getattr(t, k).zero_()
    tr.load_shards(str(tmp_path), metas)
    for k in tr._keys:
        assert torch.equal(m.state_dict()[k], trained[k])
    for k, v in slots.items():
        assert torch.equal(getattr(t, k), v)


@pytest.mark.parametrize("cls,kw", [(Z.DeepWalk, {}), (Z.Node2Vec, {"walk_p": 0.5, "walk_q": 2.0})])
def test_deepwalk_device_path_cpu(cora, tmp_path, cls, kw):
    m = _model(cora, cls, **kw)
    before = m.state_dict()["_target_encoder.embedding.weight"].clone()
    res = NodeEstimator(m, _params(cora, tmp_path, "cpu")).train()
    assert res["step"] == 30 and np.isfinite(res["loss"])
    assert not torch.equal(before, m.state_dict()["_target_encoder.embedding.weight"])


def test_deepwalk_device_path_resumes(cora, tmp_path):
    m = _model(cora)
    est = NodeEstimator(m, _params(cora, tmp_path, "cpu", total_step=20))
    est.train()
    ctr = int(est.device_trainer.graph.rng[1])
    m2 = _model(cora)
    est2 = NodeEstimator(m2, _params(cora, tmp_path, "cpu", total_step=30))
    assert est2.train()["step"] == 30
    assert int(est2.device_trainer.graph.rng[1]) == ctr + 10


@pytest.mark.gpu
def test_deepwalk_device_path_gpu_captured(cora, tmp_path, cuda):
    m = _model(cora)
    est = NodeEstimator(m, _params(cora, tmp_path, "cuda", total_step=120, log_steps=40, steps_per_graph=8))
    res = est.train()
    tr = est.device_trainer
    assert res["step"] == 120 and np.isfinite(res["loss"]) and tr.captures >= 1


def _line(ds, order=2):
    torch.manual_seed(0)
    return Z.Line("train", ["train"], ds.max_node_id, 8, num_negs=3, order=order)


def test_line_device_path_cpu(cora, tmp_path):
    """second-order LINE (examples/line/line.py:27-71) on the device path: one (root,
    weighted neighbour) pair per root, negatives from the node sampler"""
    m = _line(cora)
    before = m.state_dict()["_context_encoder.embedding.weight"].clone()
    est = NodeEstimator(m, _params(cora, tmp_path, "cpu"))
    res = est.train()
    assert res["step"] == 30 and np.isfinite(res["loss"])
    assert not torch.equal(before, m.state_dict()["_context_encoder.embedding.weight"])
    inner = est.device_trainer.inner
    assert inner.pairs_per_walk == 1 and inner.walk_len == 1
    src, pos, negs = inner.sample()
    g = est.device_trainer.graph
    assert src.numel() == 32 and negs.shape == (32, 3)
    # every positive is an out-neighbour of its root (or the pad row of a sink)
    indptr, nbr, T = g.indptr.cpu(), g.nbr.cpu(), g.num_types
    for s, p in zip(src.tolist(), pos.tolist()):
        assert p == inner.pad or p in nbr[indptr[s * T]: indptr[(s + 1) * T]].tolist()


def test_line_first_order_device_path_cpu(cora, tmp_path):
    """first-order LINE (one table in both roles) on the autograd device trainer; the
    row-sparse SGNS trainer refuses a shared table"""
    from euler_amd.graph.device_graph import DeviceGraph
    from euler_amd.models.deepwalk_step import DeepWalkEstimatorTrainer

    m = _line(cora, order=1)
    before = m.state_dict()["_target_encoder.embedding.weight"].clone()
    est = NodeEstimator(m, _params(cora, tmp_path, "cpu"))
    res = est.train()
    assert res["step"] == 30 and np.isfinite(res["loss"]) and 0.0 < res["mrr"] <= 1.0
    assert type(est.device_trainer).__name__ == "IdPairTrainer"
    assert not torch.equal(before, m.state_dict()["_target_encoder.embedding.weight"])
    with pytest.raises(ValueError, match="separate target and context"):
        DeepWalkEstimatorTrainer(m, DeviceGraph.from_engine(device="cpu"), 8)


@pytest.mark.gpu
def test_line_device_path_gpu_captured(cora, tmp_path, cuda):
    m = _line(cora)
    est = NodeEstimator(m, _params(cora, tmp_path, "cuda", total_step=120, log_steps=40, steps_per_graph=8))
    res = est.train()
    assert res["step"] == 120 and np.isfinite(res["loss"]) and est.device_trainer.captures >= 1


@pytest.mark.gpu
def test_line_first_order_device_path_gpu_captured(cora, tmp_path, cuda):
    m = _line(cora, order=1)
    est = NodeEstimator(m, _params(cora, tmp_path, "cuda", total_step=120, log_steps=40, steps_per_graph=8))
    res = est.train()
    assert res["step"] == 120 and np.isfinite(res["loss"]) and est.device_trainer.captures >= 1


def test_line_first_order_row_sparse_first_step_equals_dense(cora, tmp_path):
    """RowSparseIdPairTrainer (the shared id table row-sparse: touched rows gathered,
    merged gradients, sparse Adam) against IdPairTrainer (the table in the dense flat
    buffer): Adam's first update of an untouched row is zero, so one step leaves both
    tables equal; then the estimator trains it and checkpoints the table under the
    model's own name"""
    from euler_amd.graph.device_graph import DeviceGraph
    from euler_amd.models.line_trainer import IdPairTrainer, RowSparseIdPairTrainer

    out = {}
    for cls in (IdPairTrainer, RowSparseIdPairTrainer):
        torch.manual_seed(0)
        m = _line(cora, order=1)
        g = DeviceGraph.from_engine(node_type=0, seed=4, device="cpu")
        tr = cls(m, g, 32, learning_rate=0.02)
        tr.step()
        out[cls.__name__] = (float(tr.loss), tr.logical_params())
    (l0, p0), (l1, p1) = out["IdPairTrainer"], out["RowSparseIdPairTrainer"]
    assert abs(l0 - l1) <= 1e-6 * abs(l0) and set(p0) == set(p1)
    for k in p0:
        assert torch.allclose(p0[k].cpu(), p1[k].cpu(), atol=1e-6), k
    m = _line(cora, order=1)
    before = m.state_dict()["_target_encoder.embedding.weight"].clone()
    est = NodeEstimator(m, _params(cora, tmp_path, "cpu", row_sparse_tables=True))
    res = est.train()
    assert type(est.device_trainer).__name__ == "RowSparseIdPairTrainer"
    assert res["step"] == 30 and np.isfinite(res["loss"]) and 0.0 < res["mrr"] <= 1.0
    after = m.state_dict()["_target_encoder.embedding.weight"]
    assert not torch.equal(before, after)
    from euler_amd.estimator.base import latest_checkpoint

    ck = torch.load(latest_checkpoint(str(tmp_path / "ckpt")), map_location="cpu", weights_only=True)
    # the table lives in this rank's shard files, listed under both role names
    assert "_target_encoder.embedding.weight" not in ck["model"]
    assert set(ck["shards"]) >= {"_target_encoder.embedding.weight", "_context_encoder.embedding.weight"}
    m2 = _line(cora, order=1)
    est2 = NodeEstimator(m2, _params(cora, tmp_path, "cpu", device_graph=False))
    est2._prepare(est2.get_train_from_input(32, est2.params))
    assert est2.restore()
    assert torch.equal(m2.state_dict()["_target_encoder.embedding.weight"], after)
