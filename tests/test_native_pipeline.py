"""Native C++ SAGE batch pipeline (dataflow/native_loader.py, csrc/pipeline/pipeline.cc)
and the graph-captured estimator step over its static inputs (estimator/graph_step.py).

Batches are checked against the engine's own lookups (features, labels) and the
SageDataFlow contract (the neighbour matrix is exactly the block's edge list); the
capacity padding the captured step relies on (-1 in res / nbr past the valid rows) is
checked on the raw slot.  On the GPU the captured step must train the same trajectory
as the eager estimator step over the same batch stream.
"""
import numpy as np
import pytest
import torch

import euler_amd as ea
from euler_amd.dataflow.dataflows import SageDataFlow
from euler_amd.dataflow.native_loader import NativeSageLoader

N, FD, LD = 5000, 50, 16


@pytest.fixture(scope="module")
def graph():
    return ea.synthetic_graph(N, 8.0, 64, 1, 1, FD, LD, seed=3)


def _loader(flow, device="cpu", workers=3, seed=5, batch=64, **kw):
    return NativeSageLoader(flow, ["feature"], [FD], "label", LD, batch, -1, device, workers=workers, seed=seed, **kw)


@pytest.mark.parametrize("loops", [True, False])
def test_batches_match_engine_lookups(graph, loops):
    ea.use_graph(graph)
    flow = SageDataFlow([6, 4], [["0"], ["0"]], add_self_loops=loops, max_id=N - 1)
    ld = _loader(flow)
    try:
        for _ in range(3):
            p = ld.get()
            df = p.fields["embed_in"].fields["flow"]
            roots = p.fields["inputs"]
            assert roots.shape == (64,)
            prev = roots
            for b, f in zip(df.blocks, [6, 4]):
                n = b.size[0]
                assert n == prev.numel() and tuple(b.nbr.shape) == (n, f + (1 if loops else 0))
                assert b.nbr.dtype == torch.int32 and b.edge_index.shape[0] == 2
                dst = torch.arange(n).repeat_interleave(b.nbr.shape[1])
                got = sorted(zip(dst.tolist(), b.nbr.reshape(-1).tolist()))
                want = sorted(zip(b.edge_index[0].tolist(), b.edge_index[1].tolist()))
                assert got == want
                # res maps the previous level into this level's ids
                assert torch.equal(b.n_id[b.res_n_id], prev)
                prev = b.n_id
            x = p.fields["embed_in"].fields["x"]
            want_x = ea.get_dense_feature(df.blocks[-1].n_id, ["feature"], [FD])[0]
            assert torch.allclose(x, torch.as_tensor(want_x).float())
            want_y = ea.get_dense_feature(roots, ["label"], [LD])[0]
            assert torch.allclose(p.fields["label"], torch.as_tensor(want_y).float())
    finally:
        ld.close()


def test_capacity_padding_in_slot(graph):
    ea.use_graph(graph)
    flow = SageDataFlow([6, 4], [["0"], ["0"]], add_self_loops=False, max_id=N - 1)
    ld = _loader(flow)
    try:
        slot = ld.pipe.next()
        L, n, _, _ = ld._extent(slot)
        I, lay = ld.ints[slot], ld.lay
        cap = lay["cap"]
        for h in range(1, L + 1):
            res = I[lay["off_res"][h]:lay["off_res"][h] + cap[h - 1]]
            assert (res[n[h - 1]:] == -1).all() and (res[:n[h - 1]] >= 0).all()
            w = [6, 4][h - 1]
            o = lay["off_nbr"][h]
            nbr = I[o:o + (cap[h - 1] * w + 1) // 2].view(torch.int32)[: cap[h - 1] * w].view(cap[h - 1], w)
            assert (nbr[n[h - 1]:] == -1).all()
        ld.pipe.release(slot)
    finally:
        ld.close()


def test_batch_stream_reproducible_across_worker_counts(graph):
    ea.use_graph(graph)
    flow = SageDataFlow([5, 3], [["0"], ["0"]], max_id=N - 1)
    streams = []
    for workers in (1, 4):
        ld = _loader(flow, workers=workers, seed=11)
        try:
            streams.append([ld.get().fields["inputs"].clone() for _ in range(6)])
        finally:
            ld.close()
    for a, b in zip(*streams):
        assert torch.equal(a, b)


def test_slots_never_all_held_by_inflight_copies(graph):
    """Back-pressure: with copies that never report completion on their own (events that
    only finish on synchronize), get() must still make progress: the loader waits on its
    oldest in-flight copy instead of blocking forever in next()."""
    ea.use_graph(graph)
    flow = SageDataFlow([4, 3], [["0"], ["0"]], max_id=N - 1)
    ld = _loader(flow, workers=2)

    class SlowEvent:
        def query(self):
            return False

        def synchronize(self):
            pass

    try:
        for _ in range(3 * ld.n_slots):
            ld.get()
            # pretend the copy of the batch just handed out is still in flight
            ld._inflight[-1] = (ld._inflight[-1][0], SlowEvent())
            assert len(ld._inflight) <= ld.n_slots - ld.workers
    finally:
        ld.close()


def _model():
    from euler_amd import models as Z

    torch.manual_seed(0)
    return Z.SupervisedGraphSage([32, 32, LD], [6, 4], [["0"], ["0"]], "feature", FD, "label", LD, max_id=N - 1)


def _train(tmp_path, device, steps, **extra):
    from euler_amd.estimator import NodeEstimator

    ea.set_seed(2)
    params = {"model_dir": str(tmp_path), "batch_size": 64, "total_step": steps, "optimizer": "adam",
              "learning_rate": 0.01, "log_steps": 1, "train_node_type": -1, "device": device, "seed": 4,
              "native_pipeline": True, "pipeline_workers": 2}
    params.update(extra)
    m = _model()
    est = NodeEstimator(m, params)
    res = est.train()
    return m, res


def test_estimator_trains_through_native_pipeline_cpu(graph, tmp_path):
    ea.use_graph(graph)
    m, res = _train(tmp_path, "cpu", 12)
    assert res["step"] == 12 and np.isfinite(res["loss"])


@pytest.mark.gpu
def test_static_loader_serves_one_prepared(graph, cuda):
    ea.use_graph(graph)
    flow = SageDataFlow([6, 4], [["0"], ["0"]], add_self_loops=False, max_id=N - 1)
    ld = _loader(flow, device=cuda, static=True)
    eager = _loader(flow, device=cuda, seed=5)
    try:
        for _ in range(3):
            p, q = ld.get(), eager.get()
            assert p is ld.static_prepared
            torch.cuda.synchronize()
            assert torch.equal(p.fields["inputs"], q.fields["inputs"])
            assert torch.equal(p.fields["label"], q.fields["label"])
            for b, c in zip(p.fields["embed_in"].fields["flow"].blocks, q.fields["embed_in"].fields["flow"].blocks):
                t = c.size[0]
                assert torch.equal(b.nbr[:t], c.nbr) and (b.nbr[t:] == -1).all()
                assert torch.equal(b.res_n_id[:t], c.res_n_id)
            nl = q.fields["embed_in"].fields["x"].shape[0]
            assert torch.equal(p.fields["embed_in"].fields["x"][:nl], q.fields["embed_in"].fields["x"])
    finally:
        ld.close()
        eager.close()


@pytest.mark.gpu
def test_graph_captured_step_tracks_eager_step(graph, cuda, tmp_path):
    """Same seeds -> same batch stream; the hipGraph-replayed step (capacity-padded
    inputs) must follow the eager step's trajectory as closely as a second eager run does.
    (Eager runs are not bitwise reproducible themselves: the fused layer's input-gradient
    scatter accumulates with fp32 atomics, and Adam's per-coordinate normalisation turns
    that rounding into sign noise on near-zero gradients.)"""
    from euler_amd.convolution.convs import SAGEConv

    ea.use_graph(graph)
    steps = 12
    m_e, r_e = _train(tmp_path / "eager", cuda, steps, cuda_graph=False)
    m_e2, r_e2 = _train(tmp_path / "eager2", cuda, steps, cuda_graph=False)
    before = SAGEConv.fused_calls
    m_g, r_g = _train(tmp_path / "graph", cuda, steps, cuda_graph=True)
    # 1 first (raw-input) step + 3 warm eager steps + 1 capture: 5 Python dispatches per conv
    assert SAGEConv.fused_calls - before == 2 * 5
    assert r_g["step"] == steps
    tol = max(0.01 * r_e["loss"], 3 * abs(r_e2["loss"] - r_e["loss"]))
    assert abs(r_g["loss"] - r_e["loss"]) < tol, (r_g["loss"], r_e["loss"], r_e2["loss"])
    cos = torch.nn.functional.cosine_similarity
    sd_e, sd_e2 = m_e.state_dict(), m_e2.state_dict()
    for k, b in m_g.state_dict().items():
        a = sd_e[k]
        if a.is_floating_point() and a.numel() > 1:
            c = float(cos(a.float().reshape(-1), b.float().reshape(-1), dim=0))
            c_ee = float(cos(a.float().reshape(-1), sd_e2[k].float().reshape(-1), dim=0))
            assert c > min(0.999, c_ee - 0.005), (k, c, c_ee)
