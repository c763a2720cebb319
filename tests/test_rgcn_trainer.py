"""NodeEstimator(device_graph=True) for the estimator's UnsupervisedRGCN
(models/rgcn_trainer.py, dataflow/device_flow.py DeviceRelationFlow; reference
examples/rgcn/rgcn.py:30-105, relation_dataflow.py:25-75)."""
import math

import numpy as np
import pytest
import torch


def _setup(tmp_path, device="cpu", batch=8):
    from euler_amd.tools import runner

    a = runner.parse_args(["--scale", "0.05", "--batch_size", str(batch), "--device", device, "--seed", "1",
                           "--data_dir", str(tmp_path / "data"), "--model_dir", str(tmp_path / "ckpt")], model="rgcn")
    torch.manual_seed(0)
    m, est = runner.build(a)
    return a, m, est


def test_relation_flow_edge_attr_is_the_engine_relation_cpu(tmp_path):
    """every block edge carries the relation the engine's RelationDataFlow + to_edge give
    the same (target, neighbour) pair; the device embedding of the roots equals the engine
    path's gnn output"""
    import euler_amd.ops.graph_api as ge
    from euler_amd.graph.device_graph import DeviceGraph
    from euler_amd.models.rgcn_trainer import UnsupRgcnTrainer

    a, m, est = _setup(tmp_path)
    est._prepare(est.get_train_from_input(8, est.params))
    g = DeviceGraph.from_engine(seed=5, device="cpu")
    tr = UnsupRgcnTrainer(m, g, 8)
    roots = torch.randint(0, g.num_rows, (tr.flow.B,), generator=torch.Generator().manual_seed(3))
    df = tr.flow.produce(roots)
    ids = np.asarray(g.ids).astype(np.int64)
    prev = roots
    for b in df.blocks:
        ei, rel = b.edge_index, b.e_id
        ok = ei[0] >= 0
        assert bool((rel[ok] >= 0).all()) and bool((rel[~ok] < 0).all())
        t_ids = ids[prev[ei[0][ok]].numpy()]
        s_ids = ids[b.n_id[ei[1][ok]].numpy()]
        for t, s_, r in list(zip(t_ids, s_ids, rel[ok].tolist()))[:200]:
            types = [int(x) for x in np.asarray(ge.get_edge_type_id(m.gnn.sampler.metapath[0])).reshape(-1)]
            want = {int(np.asarray(ge.get_edge_dense_feature(torch.tensor([[t, s_, ty]]), m.gnn.feature_idx,
                                                                  m.gnn.feature_dim)[0]).reshape(-1)[0])
                    for ty in types}
            assert r in want
        prev = b.n_id
    with torch.no_grad():
        dev = tr._embed(roots)[: roots.numel()]
        eng = m.gnn(torch.as_tensor(ids[roots.numpy()]))
    assert torch.allclose(dev, eng.float(), atol=1e-4, rtol=1e-4)


def test_rgcn_device_path_trains_cpu(tmp_path):
    from euler_amd.tools.runner import main

    res = main(["--scale", "0.05", "--batch_size", "16", "--total_step", "6", "--log_steps", "3", "--device", "cpu",
                "--seed", "1", "--data_dir", str(tmp_path / "data"), "--model_dir", str(tmp_path / "ckpt"),
                "--device_graph"], model="rgcn")
    assert res["step"] == 6 and math.isfinite(res["loss"]) and 0.0 < res["mrr"] <= 1.0


@pytest.mark.gpu
def test_rgcn_device_path_gpu_captured(tmp_path, cuda):
    from euler_amd.tools.runner import main

    res = main(["--scale", "0.05", "--batch_size", "64", "--total_step", "80", "--log_steps", "40", "--device",
                "cuda", "--seed", "1", "--data_dir", str(tmp_path / "data"), "--model_dir", str(tmp_path / "ckpt"),
                "--device_graph", "--learning_rate", "0.01"], model="rgcn")
    assert res["step"] == 80 and math.isfinite(res["loss"])


def test_row_sparse_rgcn_matches_dense_first_step_cpu(tmp_path):
    """RowSparseRgcnTrainer (id table row-sparse: the blocks' node set gathered, sparse Adam
    on those rows) against UnsupRgcnTrainer (the table in the dense flat buffer): the same
    embedding of the same blocks, and after one Adam step the same parameters (an
    untouched row's first update is zero); the estimator trains it on request and its
    checkpoint keeps the table under the model's name"""
    from euler_amd.graph.device_graph import DeviceGraph
    from euler_amd.models.rgcn_trainer import RowSparseRgcnTrainer, UnsupRgcnTrainer

    out = {}
    for cls in (UnsupRgcnTrainer, RowSparseRgcnTrainer):
        a, m, est = _setup(tmp_path / cls.__name__)
        est._prepare(est.get_train_from_input(8, est.params))
        g = DeviceGraph.from_engine(seed=5, device="cpu")
        tr = cls(m, g, 8)
        roots = torch.randint(0, g.num_rows, (tr.flow.B,), generator=torch.Generator().manual_seed(3))
        with torch.no_grad():
            emb = tr._embed(roots)
        tr.step()
        out[cls.__name__] = (emb, float(tr.loss), tr.logical_params())
    (e0, l0, p0), (e1, l1, p1) = out["UnsupRgcnTrainer"], out["RowSparseRgcnTrainer"]
    assert torch.allclose(e0, e1, atol=1e-6)
    assert abs(l0 - l1) <= 1e-5 * abs(l0) and set(p0) == set(p1)
    for k in p0:
        assert torch.allclose(p0[k], p1[k], atol=1e-6), k
    a, m, est = _setup(tmp_path / "est")
    est.params.update(device_graph=True, row_sparse_tables=True, total_step=6, log_steps=3)
    res = est.train()
    assert type(est.device_trainer).__name__ == "RowSparseRgcnTrainer"
    assert res["step"] == 6 and math.isfinite(res["loss"])
    from euler_amd.estimator.base import latest_checkpoint

    ck = torch.load(latest_checkpoint(str(tmp_path / "est" / "ckpt")), map_location="cpu", weights_only=True)
    key = "gnn._encoder.embedding.weight"
    # the table sits in this rank's shard files (rows + Adam slots); the engine-path
    # restore of a fresh model reads it back
    assert key not in ck["model"] and set(ck["shards"][key]["files"]) == {"weight", "m", "v"}
    a2, m2, est2 = _setup(tmp_path / "est")
    est2._prepare(est2.get_train_from_input(8, est2.params))
    assert est2.restore()
    assert torch.equal(m2.state_dict()[key], m.state_dict()[key])
