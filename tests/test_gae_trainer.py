"""GaeEstimator(device_graph=True) for the graph auto-encoder (models/gae_trainer.py;
reference euler_estimator/python/gae_estimator.py:26-51, mp_utils/base_gae.py:23-70) and the
fixed-shape device SageDataFlow it builds the encoder's blocks with."""
import numpy as np
import pytest
import torch

import euler_amd as ea
from euler_amd import models as Z
from euler_amd.dataset import get_dataset
from euler_amd.estimator import GaeEstimator


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


F = 1433


def _params(ds, tmp, device, **kw):
    tnt = ds.train_node_type[0] if isinstance(ds.train_node_type, list) else ds.train_node_type
    p = {"model_dir": str(tmp / "ckpt"), "batch_size": 16, "total_step": 24, "optimizer": "adam",
         "learning_rate": 0.01, "log_steps": 8, "train_node_type": tnt, "device": device, "device_graph": True,
         "seed": 5, "device_feature_dtype": "fp32"}
    p.update(kw)
    return p


def _model(enc, ds):
    torch.manual_seed(0)
    return Z.GraphAutoEncoder(enc, [16, 8], [3], [["train"]], "feature", F, "train", ["train"], ds.max_node_id,
                              num_negs=3)


def test_device_sage_flow_blocks_are_consistent(cora):
    """each hop: the previous set sits at res_n_id inside the new set, every edge joins a
    valid target to a valid source, F draws + one self loop per target"""
    from euler_amd.dataflow.device_flow import DeviceSageFlow
    from euler_amd.graph.device_graph import DeviceGraph

    g = DeviceGraph.from_engine(device="cpu", seed=2)
    flow = DeviceSageFlow(g, [None, None], [4, 3], 32, add_self_loops=True)
    roots = g.sample_node(32).long()
    df = flow.produce(roots)
    prev = roots
    for blk, (e_cap, n_cap) in zip(df.blocks, flow.caps):
        n_id, res = blk.n_id, blk.res_n_id
        assert n_id.numel() == n_cap and blk.edge_index.shape[1] == e_cap
        ok = prev >= 0
        assert torch.equal(n_id[res[ok]], prev[ok])
        t, s = blk.edge_index
        live = t >= 0
        assert bool((s[live] >= 0).all()) and bool((n_id[s[live]] >= 0).all())
        assert int(t[live].max()) < prev.numel()
        # every target keeps its self loop (the last prev.numel() edges)
        assert torch.equal(n_id[s[-prev.numel():][ok]], prev[ok])
        prev = n_id


@pytest.mark.parametrize("enc", ["sage", "gcn"])
def test_gae_device_path_cpu(cora, tmp_path, enc):
    m = _model(enc, cora)
    est = GaeEstimator(m, _params(cora, tmp_path, "cpu"))
    res = est.train()
    assert res["step"] == 24 and np.isfinite(res["loss"]) and 0.0 < res["acc"] <= 1.0
    # resume continues the sampler's counter
    ctr = int(est.device_trainer.graph.rng[1])
    est2 = GaeEstimator(_model(enc, cora), _params(cora, tmp_path, "cpu", total_step=32))
    assert est2.train()["step"] == 32
    assert int(est2.device_trainer.graph.rng[1]) == ctr + 8


@pytest.mark.gpu
@pytest.mark.parametrize("enc", ["sage", "gcn"])
def test_gae_device_path_gpu_captured(cora, tmp_path, cuda, enc):
    m = _model(enc, cora)
    est = GaeEstimator(m, _params(cora, tmp_path, "cuda", total_step=64, log_steps=32, steps_per_graph=8))
    res = est.train()
    tr = est.device_trainer
    assert res["step"] == 64 and np.isfinite(res["loss"]) and tr.captures >= 1


@pytest.mark.gpu
@pytest.mark.parametrize("self_loops", [True, False])
def test_device_sage_flow_fused_block_matches_torch(cora, cuda, monkeypatch, self_loops):
    """flow.hip sage_block / sage_place = the torch block assembly on the same draws, and
    its destination CSR = the stable sort of the edge targets"""
    import euler_amd.dataflow.device_flow as dfm
    from euler_amd.graph.device_graph import DeviceGraph
    from euler_amd.ops.mp_ops import SegmentIndex

    g = DeviceGraph.from_engine(device=cuda, seed=2)
    flow = dfm.DeviceSageFlow(g, [None, None], [4, 3], 32, add_self_loops=self_loops)
    roots = g.sample_node(32).long()
    state = g.rng.clone()
    fused = flow.produce(roots)
    g.rng.copy_(state)
    monkeypatch.setattr(dfm, "_FUSED_BLOCK", False)
    plain = flow.produce(roots)
    for a, b in zip(fused.blocks, plain.blocks):
        assert torch.equal(a.n_id, b.n_id) and torch.equal(a.res_n_id, b.res_n_id)
        assert torch.equal(a.edge_index, b.edge_index)
        seg = a.edge_index._euler_cache["_euler_seg0_%d" % a.size[0]]
        ref = SegmentIndex(b.edge_index[0], a.size[0])
        assert torch.equal(seg.indptr, ref.indptr) and torch.equal(seg.counts, ref.counts)
        n = int(ref.indptr[-1])
        assert torch.equal(seg.perm[:n], ref.perm[:n])


def _vgae(enc, ds, radius=0.5):
    torch.manual_seed(0)
    return Z.VariationalGraphAutoEncoder(radius, enc, [16, 8], [3], [["train"]], "feature", F, "train", ["train"],
                                         ds.max_node_id, num_negs=3)


@pytest.mark.parametrize("enc", ["sage", "gcn"])
def test_vgae_device_path_cpu(cora, tmp_path, enc):
    m = _vgae(enc, cora)
    before = m.state_dict()["log_var_encoder.embedding.weight"].clone()
    est = GaeEstimator(m, _params(cora, tmp_path, "cpu"))
    res = est.train()
    assert res["step"] == 24 and np.isfinite(res["loss"]) and 0.0 < res["acc"] <= 1.0
    assert not torch.equal(before, m.state_dict()["log_var_encoder.embedding.weight"])


def test_vgae_loss_is_gae_loss_plus_kl_cpu(cora, tmp_path):
    """radius 0: the VGAE step's loss = the GAE decoder loss on the same draws + the mean KL
    of (mu, log_var) over every root / positive / negative (gae.py:94-153)"""
    from euler_amd.graph.device_graph import DeviceGraph
    from euler_amd.models.gae_trainer import GaeTrainer, VgaeTrainer

    m = _vgae("sage", cora, radius=0.0)
    est = GaeEstimator(m, _params(cora, tmp_path, "cpu"))
    est._prepare(est.get_train_from_input(8, est.params))  # materialise the lazy layers
    mk = lambda: DeviceGraph.from_engine(features=m.gnn.feature_idx, feature_dims=m.gnn.feature_dim,  # noqa
                                         feature_dtype=torch.float32, seed=9, device="cpu")
    vt, gt = VgaeTrainer(m, mk(), 8), GaeTrainer(m, mk(), 8)
    lv_loss, g_loss = vt._forward_loss(), gt._forward_loss()
    src, pos, neg = vt._samples
    assert all(torch.equal(a, b) for a, b in zip(vt._samples, gt._samples))
    rows = torch.cat([src, pos, neg])
    with torch.no_grad():
        mu = vt._embed(rows)
        ids = torch.where(rows >= 0, vt._ids[rows.clamp(min=0)], torch.full_like(rows, vt._pad_id))
        kl = m.kl(mu, m.log_var_encoder(ids).reshape(mu.shape)).mean()
    assert torch.allclose(lv_loss.detach(), g_loss.detach() + kl, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_vgae_device_path_gpu_captured(cora, tmp_path, cuda):
    m = _vgae("sage", cora)
    est = GaeEstimator(m, _params(cora, tmp_path, "cuda", total_step=64, log_steps=32, steps_per_graph=8))
    res = est.train()
    assert res["step"] == 64 and np.isfinite(res["loss"]) and est.device_trainer.captures >= 1
