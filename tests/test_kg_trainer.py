"""Device-path training of the TransX family under EdgeEstimator(device_graph=True)
(models/kg_trainer.py; reference euler_estimator/python/edge_estimator.py:27-72,
examples/TransX/transX.py:63-145).  CPU: the torch twin of the samplers and the same
estimator loop; GPU: alias-sample kernels, fused kg_score, captured multi-step graphs."""
import numpy as np
import pytest
import torch

import euler_amd as ea
from euler_amd import models as Z
from euler_amd.dataset import get_dataset
from euler_amd.estimator import EdgeEstimator


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


def _params(tmp, device, **kw):
    p = {"model_dir": str(tmp / "ckpt"), "batch_size": 64, "total_step": 40, "optimizer": "adam",
         "learning_rate": 0.02, "log_steps": 20, "train_edge_type": "train", "device": device,
         "device_graph": True, "seed": 7}
    p.update(kw)
    return p


def _model(fb, kind="transe"):
    torch.manual_seed(0)
    args = ("train", "train", fb.max_node_id, fb.max_edge_id, 16, 16)
    return {"transe": lambda: Z.TransE(*args, num_negs=4), "transh": lambda: Z.TransH(*args, num_negs=4),
            "distmult": lambda: Z.DistMult(*args, num_negs=4)}[kind]()


def test_triple_table_matches_engine(fb):
    """the exported table is the engine's edge set with the relation feature"""
    from euler_amd.models.kg_trainer import TripleTable

    t = TripleTable.from_engine("train", node_type="train", seed=1, device="cpu")
    assert t.src.numel() > 0 and t.src.shape == t.dst.shape == t.rel.shape
    edges = torch.stack([t.src[:50], t.dst[:50], torch.zeros(50, dtype=torch.long)], 1)
    et = int(np.asarray(ea.get_edge_type_id("train")).reshape(-1)[0])
    edges[:, 2] = et
    rel = ea.get_edge_dense_feature(edges.numpy(), ["id"], [1])[0].reshape(-1)
    assert torch.equal(torch.as_tensor(np.asarray(rel)).long(), t.rel[:50])
    s, r, d = t.sample_triples(200)
    assert s.shape == (200,) and bool((r >= 0).all())
    n = t.sample_corruptions(300)
    assert set(n.tolist()) <= set(t.cand.tolist())


@pytest.mark.parametrize("kind", ["transe", "transh", "distmult"])
def test_edge_estimator_device_path_cpu(fb, tmp_path, kind):
    model = _model(fb, kind)
    res = EdgeEstimator(model, _params(tmp_path, "cpu")).train()
    assert res["step"] == 40 and np.isfinite(res["loss"]) and 0.0 < res["mrr"] <= 1.0


def test_edge_estimator_device_path_resumes(fb, tmp_path):
    """the checkpoint carries the tables, the optimizer slots and the sampler's counter"""
    model = _model(fb)
    est = EdgeEstimator(model, _params(tmp_path, "cpu", total_step=60, log_steps=10))
    assert est.train()["step"] == 60
    ctr = int(est.device_trainer.table.rng[1])
    model2 = _model(fb)
    est2 = EdgeEstimator(model2, _params(tmp_path, "cpu", total_step=70, log_steps=10))
    assert est2.train()["step"] == 70
    assert int(est2.device_trainer.table.rng[1]) == ctr + 10
    for k, v in model.state_dict().items():
        assert v.shape == model2.state_dict()[k].shape


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["transe", "transh"])
def test_edge_estimator_device_path_gpu(fb, tmp_path, cuda, kind):
    """the whole run replays captured multi-step graphs on the GPU (samplers in HBM)"""
    model = _model(fb, kind)
    est = EdgeEstimator(model, _params(tmp_path, "cuda", total_step=200, log_steps=20, steps_per_graph=8))
    res = est.train()
    tr = est.device_trainer
    assert res["step"] == 200 and np.isfinite(res["loss"])
    assert tr.captures >= 1, "the step should have been captured"
    assert tr.table.rng.is_cuda


@pytest.mark.gpu
def test_kg_trainer_fused_step_matches_fp32_torch(fb, cuda):
    """the device step's loss (fused kg_score kernels) equals the torch fp32 composition of
    the same model on the same batch, on the CPU"""
    import copy

    from euler_amd.models.kg_trainer import KGTrainer

    model = _model(fb)
    ref_model = copy.deepcopy(model)
    tr = KGTrainer.from_model(model, 64, "train", seed=3, device=cuda)
    with torch.no_grad():
        loss = float(tr._forward_loss())
        src, rel, dst, neg = (x.cpu() for x in tr._samples)
        ref, _, _ = ref_model.loss_scores(src, dst, neg, rel)
    assert abs(loss - float(ref)) < 1e-4 * max(1.0, abs(float(ref)))


def test_row_sparse_kg_first_step_equals_dense_and_trains(fb, tmp_path):
    """RowSparseKGTrainer (row-sparse entity table, sparse Adam on the touched rows only)
    against KGTrainer (the table in the dense flat buffer): Adam's first update of an
    untouched row is 0 / (0 + eps) = 0, so after one step both hold the same tables; then
    the sparse trainer keeps training (loss falls) and its state round-trips through the
    model's own parameter names"""
    from euler_amd.models.kg_trainer import KGTrainer, RowSparseKGTrainer, TripleTable

    out = {}
    for cls in (KGTrainer, RowSparseKGTrainer):
        m = _model(fb)
        t = TripleTable.from_engine("train", node_type="train", seed=3, device="cpu")
        tr = cls(m, t, 64, optimizer="adam", learning_rate=0.02)
        tr.step()
        out[cls.__name__] = (float(tr.loss), tr.logical_params(), tr)
    (l0, p0, _), (l1, p1, sp) = out["KGTrainer"], out["RowSparseKGTrainer"]
    assert abs(l0 - l1) <= 1e-6 * abs(l0)
    assert set(p0) == set(p1)
    for k in p0:
        assert torch.allclose(p0[k], p1[k], atol=1e-6), k
    first = float(sp.loss)
    for _ in range(60):
        sp.step()
    assert float(sp.loss) < first
    # the flat buffer holds no entity rows: per-step work independent of |V|
    assert sp.flat.numel == sp.model.relation_encoder.weight.numel()
    sd = sp.state_dict()
    m2 = _model(fb)
    t2 = TripleTable.from_engine("train", node_type="train", seed=3, device="cpu")
    sp2 = RowSparseKGTrainer(m2, t2, 64)
    sp2.load_logical(sd)
    for k, v in sp2.logical_params().items():
        assert torch.equal(v.cpu(), sd[k]), k
    sp.finish()
    assert torch.equal(sp.model.entity_encoder.weight.detach(), sd["entity_encoder.weight"])


def test_edge_estimator_row_sparse_tables_cpu(fb, tmp_path):
    m = _model(fb)
    est = EdgeEstimator(m, _params(tmp_path, "cpu", row_sparse_tables=True))
    res = est.train()
    assert type(est.device_trainer).__name__ == "RowSparseKGTrainer"
    assert res["step"] == 40 and np.isfinite(res["loss"])
    # the model's own module is back, trained
    from euler_amd.utils.layers import Embedding

    assert isinstance(m.entity_encoder, Embedding) and m.entity_encoder.weight.requires_grad
    # the checkpoint keeps the table in this rank's shard files (rows + Adam slots), not in
    # the .pt; an engine-path restore reads it back
    ck = torch.load(ea_latest(tmp_path), map_location="cpu", weights_only=True)
    assert "entity_encoder.weight" not in ck["model"] and set(ck["shards"]["entity_encoder.weight"]["files"]) == \
        {"weight", "m", "v"}
    m2 = _model(fb)
    est2 = EdgeEstimator(m2, _params(tmp_path, "cpu", device_graph=False))
    assert est2.restore()
    assert torch.equal(m2.entity_encoder.weight.detach(), m.entity_encoder.weight.detach())
    assert torch.equal(m2.relation_encoder.weight.detach(), m.relation_encoder.weight.detach())


def test_row_sparse_kg_resume_equals_continuous_run(fb, tmp_path):
    """20 steps + resume to 40 (per-rank shard files: rows AND sparse Adam slots, the flat
    buffer's slots, the sampler counter) ends on exactly the tables of one 40-step run"""
    runs = {}
    for name, legs in (("cont", (40,)), ("resumed", (20, 40))):
        for total in legs:
            m = _model(fb)
            est = EdgeEstimator(m, _params(tmp_path / name, "cpu", row_sparse_tables=True, total_step=total))
            est.train()
        runs[name] = {k: v.detach().clone() for k, v in m.state_dict().items()}
    for k, v in runs["cont"].items():
        assert torch.equal(v, runs["resumed"][k]), k


def test_row_sparse_kg_refuses_distmult_l2(fb, tmp_path):
    """DistMult's L2 term spans every entity row each step: a row-sparse table cannot
    compute it (explicit request or sharded table: refused; auto: the dense trainer)"""
    from euler_amd.models.kg_trainer import RowSparseKGTrainer, TripleTable

    args = ("train", "train", fb.max_node_id, fb.max_edge_id, 16, 16)
    t = TripleTable.from_engine("train", node_type="train", seed=3, device="cpu")
    with pytest.raises(ValueError, match="l2_regular"):
        RowSparseKGTrainer(Z.DistMult(*args, num_negs=4, l2_regular=True), t, 64)
    with pytest.raises(ValueError, match="l2_regular"):
        EdgeEstimator(Z.DistMult(*args, num_negs=4, l2_regular=True),
                      _params(tmp_path, "cpu", row_sparse_tables=True)).train()
    import euler_amd.estimator.device_trainers as dt

    old = dt.ROW_SPARSE_AUTO_ROWS
    dt.ROW_SPARSE_AUTO_ROWS = 1  # every table counts as large: auto would pick row-sparse
    try:
        est = EdgeEstimator(Z.DistMult(*args, num_negs=4, l2_regular=True), _params(tmp_path / "auto", "cpu",
                                                                                  total_step=4))
        assert np.isfinite(est.train()["loss"])
        assert type(est.device_trainer).__name__ == "KGTrainer"
    finally:
        dt.ROW_SPARSE_AUTO_ROWS = old


def ea_latest(tmp_path):
    from euler_amd.estimator.base import latest_checkpoint

    return latest_checkpoint(str(tmp_path / "ckpt"))
