"""Device-path training of the full-neighbourhood zoo (dataflow/device_flow.py,
models/full_trainer.py).

CPU: the padded device dataflow equals the engine's GCNDataFlow block by block (same
node sets in the same order, same res_n_id, same edges in the same order once the -1
padding is dropped); NodeEstimator(device_graph=True) trains a GCN through it and resumes.
GPU: the HIP expansion equals the CPU twin; the device step's loss and gradients equal the
engine path's fp32 autograd on the same roots (the numerics oracle); hipGraph replay
equals eager; the GCN-family models train on the device path."""
import math

import numpy as np
import pytest
import torch


def _setup(device, model="gcn", batch=32, extra=()):
    from euler_amd.tools import runner

    a = runner.parse_args(["--dataset", "ppi", "--scale", "0.05", "--batch_size", str(batch), "--device", device,
                           "--seed", "1"] + list(extra), model=model)
    torch.manual_seed(0)
    m, est = runner.build(a)
    return a, m, est


def _device_graph(m, device, fdt=torch.float32):
    from euler_amd.graph.device_graph import DeviceGraph

    return DeviceGraph.from_engine(features=m.gnn.feature_idx, feature_dims=m.gnn.feature_dim, label=m.label_idx,
                                   label_dim=m.label_dim, feature_dtype=fdt, seed=5, device=device)


def _masks(g, flow):
    import euler_amd.ops.graph_api as ge

    out = []
    for mp in flow.metapath:
        ids = None if mp is None else [int(t) for t in np.asarray(ge.get_edge_type_id(mp)).reshape(-1)]
        out.append(g._mask(None if ids is None or any(t < 0 for t in ids) else ids))
    return out


def _compare_flows(dev_df, eng_df, ids):
    """padded device blocks vs engine blocks (raw ids)"""
    ids = torch.as_tensor(np.asarray(ids).astype(np.int64))
    assert len(dev_df.blocks) == len(eng_df.blocks)
    for bd, be in zip(dev_df.blocks, eng_df.blocks):
        nd = bd.n_id.cpu()
        n_real = int((nd >= 0).sum())
        assert bool((nd[:n_real] >= 0).all()) and bool((nd[n_real:] < 0).all()), "padding not at the end"
        assert torch.equal(ids[nd[:n_real]], be.n_id.cpu().long()), "node set / order differs"
        rd = bd.res_n_id.cpu()
        assert torch.equal(rd[rd >= 0], be.res_n_id.cpu().long())
        ei = bd.edge_index.cpu()
        keep = (ei[0] >= 0) & (ei[1] >= 0)
        assert bool(((ei[0] >= 0) == (ei[1] >= 0)).all()), "half-padded edge"
        assert torch.equal(ei[:, keep], be.edge_index.cpu().long()), "edges differ"


def test_device_flow_matches_engine_gcn_flow_cpu():
    from euler_amd.dataflow.device_flow import DeviceFullFlow

    _, m, _ = _setup("cpu")
    g = _device_graph(m, "cpu")
    flow = m.gnn.sampler
    masks = _masks(g, flow)
    dflow = DeviceFullFlow(g, masks, 16, add_self_loops=flow.add_self_loops)
    gen = torch.Generator().manual_seed(3)
    roots = torch.randint(0, g.num_rows, (16,), generator=gen)
    roots[3] = roots[7]  # repeated roots stay repeated (set 0 is not deduped)
    dev_df = dflow.produce(roots)
    eng_df = flow(torch.as_tensor(np.asarray(g.ids)[roots.numpy()].astype(np.int64)))
    _compare_flows(dev_df, eng_df, g.ids)
    assert int(dflow.overflow.item()) == 0


def test_estimator_device_graph_gcn_trains_and_resumes_cpu(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    from euler_amd.tools.runner import main

    base = ["--dataset", "ppi", "--scale", "0.05", "--batch_size", "32", "--log_steps", "5", "--device", "cpu",
            "--seed", "1", "--model_dir", str(tmp_path / "ckpt"), "--device_graph", "--learning_rate", "0.01"]
    r1 = main(base + ["--total_step", "10"], model="gcn")
    assert r1["step"] == 10 and math.isfinite(r1["loss"])
    r2 = main(base + ["--total_step", "15"], model="gcn")
    assert r2["step"] == 15
    st = torch.load(str(tmp_path / "ckpt" / "model.ckpt-15.pt"), weights_only=True)
    assert st["device_trainer"]["step"] == 15


def test_estimator_device_graph_sampled_flow_other_conv_cpu(tmp_path):
    """a non-SAGE convolution on the sampled SageDataFlow trains on the device path through
    the fixed-shape DeviceSageFlow (the fused GraphSAGE kernels take SAGEConv only)"""
    from euler_amd import models as Z
    from euler_amd.dataflow.device_flow import DeviceSageFlow
    from euler_amd.dataset import get_dataset
    from euler_amd.estimator import NodeEstimator
    from euler_amd.models.full_trainer import FullFlowTrainer

    ds = get_dataset("ppi", data_dir=str(tmp_path / "ppi"), scale=0.05)
    ds.load_graph()
    tnt = ds.train_node_type[0] if isinstance(ds.train_node_type, list) else ds.train_node_type
    torch.manual_seed(0)
    m = Z.SupervisedGNN("gcn", "sage", [16, 16, ds.label_dim], [5, 3], [["train"], ["train"]], "feature",
                        ds.feature_dim, "label", ds.label_dim, max_id=ds.max_node_id)
    p = {"model_dir": str(tmp_path / "ckpt"), "batch_size": 32, "total_step": 12, "optimizer": "adam",
         "learning_rate": 0.01, "log_steps": 6, "train_node_type": tnt, "device": "cpu", "device_graph": True,
         "seed": 2, "device_feature_dtype": "fp32"}
    est = NodeEstimator(m, p)
    res = est.train()
    assert res["step"] == 12 and math.isfinite(res["loss"])
    assert isinstance(est.device_trainer, FullFlowTrainer) and isinstance(est.device_trainer.flow, DeviceSageFlow)


# ----------------------------------------------------------------------------------------- GPU

@pytest.mark.gpu
@pytest.mark.parametrize("self_loops", [True, False])
def test_hip_full_neighbors_matches_cpu_twin(self_loops):
    """the HIP expansion + dedup + fused block assembly (flow.hip flow_block) = the CPU
    torch composition: node sets, positions, edges and the cached destination CSR"""
    from euler_amd.dataflow.device_flow import DeviceFullFlow

    _, m, _ = _setup("cuda")
    g = _device_graph(m, "cuda")
    gc = _device_graph(m, "cpu")
    flow = m.gnn.sampler
    masks = _masks(g, flow)
    roots = torch.randint(0, g.num_rows, (64,), generator=torch.Generator().manual_seed(4))
    roots[5] = roots[9]
    fg = DeviceFullFlow(g, masks, 64, add_self_loops=self_loops)
    d_gpu = fg.produce(roots.cuda())
    d_cpu = DeviceFullFlow(gc, masks, 64, add_self_loops=self_loops).produce(roots)
    for a, b in zip(d_gpu.blocks, d_cpu.blocks):
        assert torch.equal(a.n_id.cpu(), b.n_id) and torch.equal(a.res_n_id.cpu(), b.res_n_id)
        assert torch.equal(a.edge_index.cpu(), b.edge_index)
        key = "_euler_seg0_%d" % a.size[0]
        sa, sb = a.edge_index._euler_cache[key], b.edge_index._euler_cache[key]
        assert torch.equal(sa.indptr.cpu(), sb.indptr) and torch.equal(sa.counts.cpu(), sb.counts)
        assert torch.equal(sa.perm.cpu(), sb.perm)
    assert int(fg.overflow.item()) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["gcn", "appnp", "sgcn", "tagcn"])
def test_device_step_matches_engine_oracle(model):
    """one device step's loss and gradients = fp32 autograd of the same model on the
    engine path's GCNDataFlow for the same roots"""
    from euler_amd.models.full_trainer import FullFlowTrainer

    a, m, est = _setup("cuda", model=model, batch=64)
    m.to("cuda")
    g = _device_graph(m, "cuda")
    tr = FullFlowTrainer.from_model(m, g, 64, learning_rate=0.01)
    loss = tr._forward_loss()
    tr.opt.zero_grad()
    loss.backward()
    grads = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
    ref_loss, ref = tr.reference_loss_and_grads(tr._samples)
    assert abs(float(loss) - ref_loss) <= 1e-4 * max(1.0, abs(ref_loss)), (float(loss), ref_loss)
    for n, gr in grads.items():
        r = ref[n]
        err = float((gr - r).norm() / max(float(r.norm()), 1e-12))
        assert err < 1e-3, (n, err)


@pytest.mark.gpu
def test_device_graph_replay_matches_eager():
    from euler_amd.models.full_trainer import FullFlowTrainer

    losses = []
    for captured in (False, True):
        a, m, est = _setup("cuda", batch=64)
        m.to("cuda")
        g = _device_graph(m, "cuda")
        tr = FullFlowTrainer.from_model(m, g, 64, learning_rate=0.01)
        out = []
        if captured:
            tr.capture(warmup=2, steps=4)
            out += [None, None]
            for _ in range(6):
                tr.replay(1)
                out.append(float(tr.loss.item()))
        else:
            for _ in range(8):
                tr.step()
                out.append(float(tr.loss.item()))
        losses.append(out)
    eager, graph = losses
    np.testing.assert_allclose(graph[2:], eager[2:], rtol=1e-4, atol=1e-5)


# held-out F1 floors on the planted-community graph after 200 device-path steps (measured
# on MI355X, profiles/r5_zoo/: gcn 0.896, sgcn 0.894, tagcn 0.889, arma 0.889, solution
# 0.842, gat 0.830, appnp 0.764, adaptivegcn 0.528; the engine path's GCN 0.894).  AGNN,
# DNA, FastGCN, GeniePath and LGCN learn this task slowly on either path (AGNN / DNA /
# FastGCN reach F1 0.0 on the engine path too in 200 steps): for them the held-out loss
# must beat the best constant prediction (0.2338 for 16 one-hot labels).
_ZOO_F1 = {"gcn": 0.8, "sgcn": 0.8, "tagcn": 0.8, "arma": 0.8, "solution": 0.7, "gat": 0.7, "appnp": 0.6}
_CONST_LOSS = 0.2338
# FastGCN / AdaptiveGCN evaluate with their own layer sampling on the engine path (reference
# fast_dataflow / layerwise_dataflow; an exact full-neighbourhood block would report other
# metrics than the model defines): after 200 steps that is near the constant prediction
# (measured: fastgcn 0.2338, adaptivegcn 0.2200), so only divergence is checked
_LAYER_SAMPLED = {"fastgcn", "adaptivegcn"}


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["gcn", "appnp", "sgcn", "tagcn", "agnn", "gat", "arma", "dna", "fastgcn",
                                   "adaptivegcn", "geniepath", "lgcn", "solution"])
def test_estimator_device_graph_gcn_family_gpu(tmp_path, monkeypatch, model):
    monkeypatch.chdir(tmp_path)
    from euler_amd.tools.runner import main

    r, ev = main(["--dataset", "community", "--scale", "0.5", "--batch_size", "64", "--log_steps", "100",
                  "--device", "cuda", "--seed", "1", "--model_dir", str(tmp_path / "ckpt"), "--device_graph",
                  "--total_step", "200", "--learning_rate", "0.01", "--run_mode", "train_and_evaluate",
                  "--data_dir", str(tmp_path / "data")], model=model)
    assert r["step"] == 200 and math.isfinite(r["loss"]) and math.isfinite(ev["loss"])
    if model in _ZOO_F1:
        assert ev["f1"] >= _ZOO_F1[model], ev
    elif model in _LAYER_SAMPLED:
        assert ev["loss"] < _CONST_LOSS + 0.01, ev
    else:
        assert ev["loss"] < _CONST_LOSS - 0.002, ev


def test_device_flow_dst_csr_equals_sorted_csr_cpu():
    """the destination CSR handed to the convolutions equals the stable sort the engine
    path would compute (SegmentIndex on the same edge list)"""
    from euler_amd.dataflow.device_flow import DeviceFullFlow
    from euler_amd.ops.mp_ops import SegmentIndex

    _, m, _ = _setup("cpu")
    g = _device_graph(m, "cpu")
    flow = m.gnn.sampler
    for loops in (True, False):
        dflow = DeviceFullFlow(g, _masks(g, flow), 16, add_self_loops=loops)
        roots = torch.randint(0, g.num_rows, (16,), generator=torch.Generator().manual_seed(9))
        for b in dflow.produce(roots).blocks:
            pre = b.edge_index._euler_cache["_euler_seg0_%d" % b.size[0]]
            ref = SegmentIndex(b.edge_index[0], b.size[0])
            n_real = int(ref.indptr[-1])
            assert torch.equal(pre.indptr, ref.indptr)
            assert torch.equal(pre.perm[:n_real], ref.perm[:n_real])


@pytest.mark.parametrize("model", ["agnn", "gat", "dna"])
def test_attention_convs_on_padded_blocks_stay_finite_cpu(tmp_path, model):
    """attention convolutions on capacity-padded device blocks: the padding edges (index -1)
    get softmax weight 0 on the CPU path too (an out-of-range read divided by an empty
    segment's 0 and turned AGNN's gradients into NaN)"""
    from euler_amd.tools.runner import main

    res = main(["--dataset", "ppi", "--scale", "0.05", "--batch_size", "16", "--log_steps", "3", "--device", "cpu",
                "--seed", "1", "--model_dir", str(tmp_path / model), "--device_graph", "--learning_rate", "0.01",
                "--total_step", "6"], model=model)
    assert res["step"] == 6 and math.isfinite(res["loss"])


@pytest.mark.parametrize("kind", ["fast", "layer"])
def test_device_layer_flow_keeps_exactly_the_edges_into_the_layer_cpu(kind):
    """FastGCN / AdaptiveGCN hops on the device (DeviceLayerFlow): the first hop keeps every
    out-edge of the roots that lands in the sampled layer and nothing else (the engine's
    sparse_get_adj(set, layer)); the last hop is the full neighbourhood"""
    from euler_amd.dataflow.device_flow import DeviceFullFlow, DeviceLayerFlow

    _, m, _ = _setup("cpu")
    g = _device_graph(m, "cpu")
    masks = _masks(g, m.gnn.sampler)
    dflow = DeviceLayerFlow(g, masks, [kind, "full"], [6, 6], 16, True, samplers=[g, None])
    layers = []
    orig = dflow._layer
    dflow._layer = lambda h, n_id: layers.append(orig(h, n_id)) or layers[-1]
    roots = torch.randint(0, g.num_rows, (16,), generator=torch.Generator().manual_seed(4))
    g.reseed_cpu()
    df = dflow.produce(roots)
    assert len(layers) == 1 and layers[0].numel() == 6
    lay = set(int(v) for v in layers[0].tolist() if v >= 0)
    T = g.num_types
    want = set()
    for u in roots.tolist():
        for t in range(T):
            if (masks[0] >> t) & 1:
                for v in g.nbr[g.indptr[u * T + t]: g.indptr[u * T + t + 1]].tolist():
                    if v in lay:
                        want.add((u, v))
    b = df.blocks[0]
    ei, nid = b.edge_index, b.n_id
    n_e = ei.shape[1] - 16  # the last 16 edges are the self loops
    got = set((int(roots[t]), int(nid[s])) for t, s in zip(ei[0, :n_e].tolist(), ei[1, :n_e].tolist()) if t >= 0)
    assert got == want
    assert torch.equal(nid[b.res_n_id[:16]], roots)
    # the last hop: the full flow's expansion of the same set
    full = DeviceFullFlow(g, masks[1:], int(nid.numel()), True)
    ref = full.produce(nid).blocks[0]
    e1 = df.blocks[1].edge_index
    assert int((e1[0] >= 0).sum()) == int((ref.edge_index[0] >= 0).sum())


@pytest.mark.parametrize("model", ["fastgcn", "adaptivegcn"])
def test_layer_sampled_gcn_device_path_cpu(tmp_path, model):
    from euler_amd.tools.runner import main

    res = main(["--dataset", "ppi", "--scale", "0.05", "--batch_size", "16", "--log_steps", "3", "--device", "cpu",
                "--seed", "1", "--model_dir", str(tmp_path / model), "--device_graph", "--learning_rate", "0.01",
                "--total_step", "6"], model=model)
    assert res["step"] == 6 and math.isfinite(res["loss"])


@pytest.mark.parametrize("agg", ["attention", "gcn", "mean"])
def test_encoder_device_path_matches_engine_encoder_cpu(agg, monkeypatch):
    """GeniePath on the device path (models/encoder_trainer.py): the padded device hop sets
    and adjacencies give the roots the same logits as the engine's get_multi_hop_neighbor
    path of the same model"""
    from euler_amd.models.encoder_trainer import EncoderFlowTrainer
    from euler_amd.utils import encoders

    orig = encoders.GenieEncoder.__init__
    monkeypatch.setattr(encoders.GenieEncoder, "__init__",
                        lambda self, mp, dim, aggregator="attention", *a, **k: orig(self, mp, dim, agg, *a, **k))
    _, m, est = _setup("cpu", model="geniepath", batch=8)
    est._prepare(est.get_train_from_input(8, est.params))
    m.eval()
    g = _device_graph(_Feat(m), "cpu")
    tr = EncoderFlowTrainer.from_model(m, g, 8)
    roots = torch.randint(0, g.num_rows, (8,), generator=torch.Generator().manual_seed(2))
    with torch.no_grad():
        dev, _ = tr._forward(roots)
        raw = torch.as_tensor(np.asarray(g.ids)[roots.numpy()].astype(np.int64))
        eng = m.out_fc(m.embed(raw)).float()
    assert torch.allclose(dev, eng, atol=1e-4, rtol=1e-4)


class _Feat:
    """feature / label columns of an encoder model in the shape _device_graph reads"""

    def __init__(self, m):
        ne = m._encoder._node_encoder
        self.gnn = type("G", (), {"feature_idx": ne.feature_idx, "feature_dim": ne.feature_dim})
        self.label_idx, self.label_dim = m.label_idx, m.label_dim


def test_lgcn_device_path_matches_engine_features_cpu(tmp_path):
    """LGCN on the device path: for the neighbours it drew, the logits equal the model's
    engine-side encoder over features read from the engine (default node: zeros); the
    estimator trains it"""
    import euler_amd.ops.graph_api as ge
    from euler_amd.models.encoder_trainer import LgcnTrainer

    a, m, est = _setup("cpu", model="lgcn", batch=8)
    est._prepare(est.get_train_from_input(8, est.params))
    enc = m._encoder
    from euler_amd.graph.device_graph import DeviceGraph

    g = DeviceGraph.from_engine(features=[enc.feature_idx], feature_dims=[enc.feature_dim], label=m.label_idx,
                                label_dim=m.label_dim, feature_dtype=torch.float32, seed=5, device="cpu")
    tr = LgcnTrainer.from_model(m, g, 8)
    roots = torch.randint(0, g.num_rows, (8,), generator=torch.Generator().manual_seed(2))
    state = g.rng.clone()
    g.reseed_cpu()
    with torch.no_grad():
        dev, _ = tr._forward(roots)
    g.rng.copy_(state)
    g.reseed_cpu()
    nbrs = g.sample_neighbor(roots, enc.nb_num, edge_types=tr.types, default=-1, stream_id=6).long().reshape(-1)
    ids = np.asarray(g.ids).astype(np.int64)

    def eng(rows):
        raw = np.where(rows.numpy() >= 0, ids[rows.clamp(min=0).numpy()], -1)
        x = torch.as_tensor(np.asarray(ge.get_dense_feature(raw, [enc.feature_idx], [enc.feature_dim])[0]))
        return x.float().reshape(rows.numel(), -1) * (rows >= 0).unsqueeze(1)

    with torch.no_grad():
        want = m.out_fc(enc.encode(eng(roots), eng(nbrs).view(8, enc.nb_num, -1))).float()
    assert torch.allclose(dev, want, atol=1e-5)
    from euler_amd.tools.runner import main

    res = main(["--dataset", "ppi", "--scale", "0.05", "--batch_size", "16", "--log_steps", "3", "--device", "cpu",
                "--seed", "1", "--model_dir", str(tmp_path / "lgcn"), "--device_graph", "--total_step", "6"],
               model="lgcn")
    assert res["step"] == 6 and math.isfinite(res["loss"])


def test_solution_device_path_matches_engine_features_cpu(tmp_path):
    """SuperviseSolution over a SageEncoder on the device path: for the tree it drew, the
    logits equal the encoder's aggregation over features read from the engine"""
    import euler_amd.ops.graph_api as ge
    from euler_amd.graph.device_graph import DeviceGraph
    from euler_amd.models.encoder_trainer import SolutionTrainer

    a, m, est = _setup("cpu", model="solution", batch=8)
    est._prepare(est.get_train_from_input(8, est.params))
    enc, lab = m.encoder, m.get_label_fn
    ne = enc._node_encoder
    g = DeviceGraph.from_engine(features=ne.feature_idx, feature_dims=ne.feature_dim, label=lab.label_idx,
                                label_dim=lab.label_dim, feature_dtype=torch.float32, seed=5, device="cpu")
    tr = SolutionTrainer.from_model(m, g, 8)
    roots = torch.randint(0, g.num_rows, (8,), generator=torch.Generator().manual_seed(2))
    state = g.rng.clone()
    g.reseed_cpu()
    with torch.no_grad():
        dev, _ = tr._forward(roots)
    g.rng.copy_(state)
    g.reseed_cpu()
    hops = [roots.long()]
    for i, (f, et) in enumerate(zip(enc.fanouts, tr.types)):
        hops.append(g.sample_neighbor(hops[-1], int(f), edge_types=et, default=-1, stream_id=4 + i).long().reshape(-1))
    ids = np.asarray(g.ids).astype(np.int64)

    def eng(rows):
        raw = ids[rows.clamp(min=0).numpy()]
        x = torch.cat([torch.as_tensor(np.asarray(t)).float().reshape(rows.numel(), -1)
                       for t in ge.get_dense_feature(raw, ne.feature_idx, ne.feature_dim)], 1)
        return x * (rows >= 0).unsqueeze(1)

    with torch.no_grad():
        want = m.logit_fn(enc._aggregate([eng(h) for h in hops])).float()
    assert torch.allclose(dev, want, atol=1e-5)


def test_hop0_cap_holds_a_hub_repeated_among_the_roots_cpu():
    """hop 0 expands the roots as drawn (repeats kept): a hub drawn B times needs B times
    its degree, which can exceed the graph's masked edge count; the exact caps cover it"""
    from euler_amd.dataflow.device_flow import DeviceFullFlow, masked_edges

    _, m, _ = _setup("cpu")
    g = _device_graph(m, "cpu")
    masks = _masks(g, m.gnn.sampler)
    sel = torch.tensor([(masks[0] >> t) & 1 for t in range(g.num_types)])
    deg = ((g.indptr[1:] - g.indptr[:-1]).view(g.num_rows, g.num_types) * sel).sum(1)
    hub = int(deg.argmax())
    B = 64
    flow = DeviceFullFlow(g, masks, B, add_self_loops=True)
    assert flow.caps[0][0] >= B * int(deg[hub])
    flow.produce(torch.full((B,), hub, dtype=torch.long))
    assert not flow.overflowed()


def test_bounded_caps_are_smaller_and_overflow_regrows_cpu(tmp_path):
    """caps="bounded" sizes hops from the degree distribution; a chunk whose batch exceeds a
    cap is rolled back and re-run with grown caps: the job finishes with the parameters of
    a job that never overflowed (same draws, complete blocks)"""
    from euler_amd.dataflow.device_flow import bounded_caps, exact_caps
    from euler_amd.tools.runner import main

    _, m, _ = _setup("cpu")
    g = _device_graph(m, "cpu")
    masks = _masks(g, m.gnn.sampler)
    ex, bd = exact_caps(g, masks, 32), bounded_caps(g, masks, 32)
    assert all(b[0] <= e[0] and b[1] <= e[1] for b, e in zip(bd, ex))
    assert sum(b[0] for b in bd) < sum(e[0] for e in ex)

    def run(caps, d):
        import euler_amd.estimator.base as eb

        est_box = {}
        orig = eb.BaseEstimator._train_device_graph

        def spy(self):
            est_box["est"] = self
            if caps is not None:
                self.params["device_flow_caps"] = caps
            return orig(self)

        eb.BaseEstimator._train_device_graph = spy
        torch.manual_seed(0)  # the same initial weights in both jobs
        try:
            r = main(["--dataset", "ppi", "--scale", "0.05", "--batch_size", "32", "--log_steps", "4",
                      "--device", "cpu", "--seed", "1", "--model_dir", str(tmp_path / d), "--device_graph",
                      "--total_step", "12", "--learning_rate", "0.01"], model="gcn")
        finally:
            eb.BaseEstimator._train_device_graph = orig
        est = est_box["est"]
        p = est.device_trainer.logical_params()
        return r, est, torch.cat([p[k].reshape(-1).float() for k in sorted(p)])

    r0, e0, p0 = run("exact", "a")
    tiny = [(256, 256)] * len(masks)  # every batch of this graph overflows these
    r1, e1, p1 = run(tiny, "b")
    assert r1["step"] == 12 and e1.flow_regrows >= 1 and e0.flow_regrows == 0
    assert all(c[0] > 256 for c in e1.device_trainer.flow.caps)
    torch.testing.assert_close(p1, p0, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("model", ["fastgcn", "adaptivegcn"])
def test_layer_sampled_gcn_evaluate_matches_engine_path_cpu(tmp_path, model):
    """FastGCN / AdaptiveGCN sample their layers (reference fast_dataflow / LayerwiseDataFlow):
    after device-path training, evaluate with device_graph=True must take the engine path's
    sampled blocks, not an exact full-neighbourhood block, so both report the same metrics"""
    import euler_amd as ea
    from euler_amd.tools.runner import main

    base = ["--dataset", "ppi", "--scale", "0.05", "--batch_size", "16", "--log_steps", "3", "--device", "cpu",
            "--seed", "1", "--model_dir", str(tmp_path / model), "--learning_rate", "0.01", "--total_step", "6"]
    main(base + ["--device_graph"], model=model)
    res = {}
    for dg in (True, False):
        ea.set_seed(7)
        torch.manual_seed(7)
        res[dg] = main(base + ["--run_mode", "evaluate"] + (["--device_graph"] if dg else []), model=model)
    assert res[True] and res[True] == res[False]


def test_scalable_encoder_is_not_trained_as_plain_gcn_cpu(tmp_path, caplog):
    """a ScalableGCNEncoder model is a GCNEncoder subclass: no device trainer without the
    stores' protocol may take it (it would silently train a full multi-hop GCN without
    stores); without a store-aware trainer the estimator logs and trains on the engine path"""
    import logging

    import euler_amd as ea
    from euler_amd.dataset import get_dataset
    from euler_amd.estimator import NodeEstimator
    from euler_amd.estimator.device_trainers import NoDeviceTrainer, REGISTRY, STORE_AWARE
    from euler_amd.mp_utils.models import SuperviseModel
    from euler_amd.utils import encoders as E

    ds = get_dataset("ppi", data_dir=str(tmp_path / "ppi"), scale=0.05)
    ds.load_graph()
    ea.set_seed(3)

    class M(SuperviseModel):
        def __init__(self):
            super().__init__(ds.label_idx, ds.label_dim)
            self._encoder = E.ScalableGCNEncoder(["train"], 2, 16, feature_idx=ds.feature_idx,
                                                 feature_dim=ds.feature_dim, max_id=ds.max_node_id)

        def embed(self, n_id):
            return self._encoder(n_id)

    m = M()
    tnt = ds.train_node_type[0] if isinstance(ds.train_node_type, list) else ds.train_node_type
    p = {"model_dir": str(tmp_path / "ck"), "batch_size": 16, "total_step": 3, "log_steps": 1, "device": "cpu",
         "device_graph": True, "train_node_type": tnt, "seed": 1}
    est = NodeEstimator(m, p)
    with caplog.at_level(logging.WARNING, logger="euler_amd.estimator"):
        res = est.train()
    assert np.isfinite(res["loss"]) and getattr(est, "device_trainer", None) is None or \
        getattr(est.device_trainer, "device_trainer_kind", None) in STORE_AWARE
    if not any(n in STORE_AWARE for n, _, _ in REGISTRY):
        assert "engine path" in caplog.text
    assert float(m._encoder.stores(0).abs().sum()) > 0
    from euler_amd.estimator.device_trainers import build_device_trainer
    if not any(n in STORE_AWARE for n, _, _ in REGISTRY):
        with pytest.raises(NoDeviceTrainer):
            build_device_trainer(est, m, None)
