"""Historical-embedding encoders on the device path (models/scalable_trainer.py,
graph/device_scope.py; reference tf_euler/python/utils/encoders.py:294-408, 629-748).

CPU: the device trainer (the model's own forward with every graph query answered from the
HBM graph) equals the engine path step for step on the same draws — loss, parameters and
the stale-embedding / gradient stores — for ScalableSageEncoder and ScalableGCNEncoder; the
estimator routes such models to it and trains / resumes; two gloo ranks stay in lockstep.
GPU: the ScalableSage step captured in hipGraphs equals its eager steps and trains."""
import copy

import numpy as np
import pytest
import torch

import euler_amd as ea
import euler_amd.ops.graph_api as G
from euler_amd.dataset import get_dataset
from euler_amd.mp_utils.models import SuperviseModel
from euler_amd.utils import encoders as E


@pytest.fixture(scope="module")
def _ppi(tmp_path_factory):
    ds = get_dataset("ppi", data_dir=str(tmp_path_factory.mktemp("ppi")), scale=0.05)
    ds.get_data_dir()
    return ds


@pytest.fixture
def ppi(_ppi):
    _ppi.load_graph()
    ea.set_seed(3)
    return _ppi


class _Model(SuperviseModel):
    def __init__(self, ds, kind):
        super().__init__(ds.label_idx, ds.label_dim)
        if kind == "sage":
            self.enc = E.ScalableSageEncoder(["train"], 4, 2, 16, feature_idx=ds.feature_idx,
                                             feature_dim=ds.feature_dim, max_id=ds.max_node_id)
        else:
            self.enc = E.ScalableGCNEncoder(["train"], 2, 16, feature_idx=ds.feature_idx,
                                            feature_dim=ds.feature_dim, max_id=ds.max_node_id)

    def embed(self, n_id):
        return self.enc(n_id)


def _materialized(ds, kind, B):
    torch.manual_seed(0)
    m = _Model(ds, kind)
    with torch.no_grad():
        m(G.sample_node(B, ds.train_node_type[0] if isinstance(ds.train_node_type, list) else ds.train_node_type))
    m.enc._pending = None
    for i in range(m.enc._num_stores):
        m.enc.gradient_stores(i).zero_()
    return m


def _trainer(ds, m, B, device="cpu"):
    from euler_amd.graph.device_graph import DeviceGraph
    from euler_amd.models.scalable_trainer import ScalableTrainer

    names, dims = [str(n) for n in m.enc._node_encoder.feature_idx], list(m.enc._node_encoder.feature_dim)
    g = DeviceGraph.from_engine(features=names, feature_dims=dims, label=ds.label_idx, label_dim=ds.label_dim,
                                feature_dtype=torch.float32, seed=9, device=device)
    cols, off = {}, 0
    for n, d in zip(names, dims):
        cols[n] = (off, d)
        off += d
    return ScalableTrainer(m, g, B, cols, label=(ds.label_idx, ds.label_dim), learning_rate=0.01)


@pytest.mark.parametrize("kind", ["sage", "gcn"])
def test_device_path_equals_engine_path_on_the_same_draws_cpu(ppi, kind, monkeypatch):
    """3 steps: the device trainer's loss, parameters and both store kinds equal the engine
    path's (the reference protocol: forward + store loss, backward, store writes, Adam)
    when the engine-path encoder receives the device trainer's draws"""
    B = 16
    m_dev = _materialized(ppi, kind, B)
    m_eng = copy.deepcopy(m_dev)
    tr = _trainer(ppi, m_dev, B)
    opt = torch.optim.Adam([p for p in m_eng.parameters() if p.requires_grad], lr=0.01)
    for step in range(3):
        tr.scope.record = []
        tr.step()
        roots = tr._samples[0].cpu()
        rec = tr.scope.record
        with monkeypatch.context() as mp:  # the engine-path encoder takes the device draws
            if kind == "sage":
                nb = rec[0][1].reshape(-1).cpu()
                mp.setattr(G, "sample_fanout", lambda *a, **k: ([roots, nb], [], []))
            else:
                _, nxt, ind, w = rec[0]
                adj = G.SparseTensor(ind.cpu(), w.cpu(), torch.tensor([roots.numel(), nxt.numel()]))
                mp.setattr(G, "get_multi_hop_neighbor", lambda *a, **k: ([roots, nxt.cpu()], [adj]))
            _, loss, _, _ = m_eng(roots)
        obj = loss + m_eng.enc.store_loss
        opt.zero_grad()
        obj.backward()
        m_eng.enc.after_backward()
        opt.step()
        assert abs(float(tr.loss) - float(loss.detach())) <= 1e-5 * max(1.0, abs(float(loss.detach()))), step
        for (n, a), b in zip(m_dev.state_dict().items(), m_eng.state_dict().values()):
            torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6, msg=lambda s, n=n: f"{n} step {step}: {s}")
        for i in range(m_dev.enc._num_stores):
            torch.testing.assert_close(m_dev.enc.stores(i), m_eng.enc.stores(i), rtol=1e-4, atol=1e-6)
            torch.testing.assert_close(m_dev.enc.gradient_stores(i), m_eng.enc.gradient_stores(i), rtol=1e-4,
                                       atol=1e-7)
    # the stores moved: fresh root embeddings written, neighbour gradients accumulated
    assert float(m_dev.enc.gradient_stores(0).abs().sum()) > 0


@pytest.mark.parametrize("kind", ["sage", "gcn"])
def test_estimator_routes_scalable_models_to_the_device_trainer_and_resumes_cpu(ppi, tmp_path, kind):
    from euler_amd.estimator import NodeEstimator

    tnt = ppi.train_node_type[0] if isinstance(ppi.train_node_type, list) else ppi.train_node_type
    p = {"model_dir": str(tmp_path / "ck"), "batch_size": 16, "total_step": 6, "log_steps": 3, "device": "cpu",
         "device_graph": True, "train_node_type": tnt, "seed": 1, "device_feature_dtype": "fp32"}
    torch.manual_seed(0)
    m = _Model(ppi, kind)
    est = NodeEstimator(m, p)
    res = est.train()
    assert est.device_trainer.device_trainer_kind == "scalable"
    assert res["step"] == 6 and np.isfinite(res["loss"])
    s0 = m.enc.stores(0).clone()
    torch.manual_seed(0)
    m2 = _Model(ppi, kind)
    est2 = NodeEstimator(m2, dict(p, total_step=9))
    assert est2.train()["step"] == 9
    # resumed with the stores of the checkpoint (then trained 3 more steps)
    assert not torch.equal(m2.enc.stores(0), s0) and float(m2.enc.stores(0).abs().sum()) > 0


@pytest.mark.gpu
def test_scalable_sage_captured_equals_eager_and_trains_gpu(ppi):
    B = 64
    losses = {}
    for mode in ("eager", "graph"):
        m = _materialized(ppi, "sage", B).cuda()
        tr = _trainer(ppi, m, B, device="cuda")
        if mode == "graph":
            tr.capture(warmup=2, steps=4)
            tr.replay_steps(40)
        else:
            for _ in range(42):
                tr.step()
        torch.cuda.synchronize()
        losses[mode] = (float(tr.loss), {k: v.detach().clone() for k, v in m.state_dict().items()})
    assert abs(losses["eager"][0] - losses["graph"][0]) <= 1e-4 * max(1.0, abs(losses["eager"][0]))
    # per tensor in norm: the stores' gradient accumulation adds with atomics (order varies
    # between runs), and 42 Adam steps magnify that for near-zero gradients element-wise
    for k, v in losses["eager"][1].items():
        g = losses["graph"][1][k].float()
        rel = float((g - v.float()).norm() / v.float().norm().clamp(min=1e-12))
        assert rel < 2e-3, (k, rel)
