"""SageTrainer (the device-path GraphSAGE trainer, csrc/hip/sage_tree.hip).

GPU: every kernel path (1/2/3 hops, class-id / dense labels, bf16 / fp32 features, self
loops, multi-type metapaths, odd widths that need padding) against the fp32 torch
oracle of the same model on the same sampled tree; hipGraph replay against eager;
checkpoint / resume continuing the sample + loss trajectory; a 200-step bf16-vs-fp32
loss trajectory.  CPU: the torch implementation (layout, padding, optimizers, state).
"""
import math

import numpy as np
import pytest
import torch


def _graph(device, n=6000, types=1, seed=3):
    from euler_amd.graph.device_graph import DeviceGraph

    rng = np.random.default_rng(seed)
    deg = rng.integers(0, 12, n * types)
    indptr = np.zeros(n * types + 1, np.int64)
    indptr[1:] = np.cumsum(deg)
    nbr = rng.integers(0, n, int(indptr[-1])).astype(np.int32)
    for s in range(n * types):  # sorted segments like the engine
        a, b = indptr[s], indptr[s + 1]
        nbr[a:b].sort()
    w = rng.uniform(0.5, 1.5, int(indptr[-1]))
    nw = rng.uniform(0.1, 1.0, n)
    g = DeviceGraph.from_csr(indptr, nbr, w, num_types=types, node_weights=nw, seed=seed, device=device)
    return g


def _tables(device, n, D, C, mode, fdt=torch.bfloat16, seed=5):
    gen = torch.Generator().manual_seed(seed)
    x = torch.randn(n, D, generator=gen)
    if mode == "class":
        lab = x[:, :C].argmax(1).to(torch.int16)
    elif mode == "class32":
        lab = x[:, :C].argmax(1).to(torch.int32)
    else:
        lab = (x[:, :C] > 0.3).float()
    return x.to(device=device, dtype=fdt), lab.to(device)


def _cmp(a, b):
    a, b = a.float().reshape(-1).cpu(), b.float().reshape(-1).cpu()
    if b.norm() < 1e-9:
        return 1.0, float(a.norm())
    cos = torch.nn.functional.cosine_similarity(a, b, dim=0).item()
    rel = ((a - b).norm() / b.norm()).item()
    return cos, rel


def _trainer(device, fanouts, dims, C, mode="class", fdt=torch.bfloat16, D=20, types=1, metapath=None, B=64,
             self_loops=False, opt="adam", seed=3, lr=0.01):
    from euler_amd.models.sage_trainer import SageTrainer

    g = _graph(device, types=types, seed=seed)
    g.manual_seed(seed + 17)
    x, lab = _tables(device, g.num_rows, D, C, mode, fdt)
    return SageTrainer(g, B, fanouts, dims, C, features=x, labels=lab, metapath=metapath,
                       add_self_loops=self_loops, optimizer=opt, learning_rate=lr, init_seed=seed)


# ----------------------------------------------------------------------------------------- CPU


def test_slot_layout_and_padding_cpu():
    tr = _trainer("cpu", [25, 10], [40, 40, 24], 10)
    assert tr.logP == [0, 5] and tr.M == [64, 64 * 32]
    assert tr.Dp == 32 and tr.Hp == [64, 64] and tr.Ep == 32 and tr.Cp == 32
    # pack / unpack round trip through the padded flat layout; padding stays zero
    logical = tr.logical_params()
    flat = torch.zeros(tr.offsets[-1])
    tr._pack(logical, flat)
    back = tr._unpack(flat)
    for k in logical:
        assert torch.equal(back[k], logical[k]), k
    nz = sum(int((v != 0).sum()) for v in logical.values())
    assert int((flat != 0).sum()) == nz


@pytest.mark.parametrize("L,fan", [(1, [6]), (2, [5, 3]), (3, [4, 3, 2])])
def test_cpu_training_learns(L, fan):
    dims = [32] * L + [16]
    tr = _trainer("cpu", fan, dims, 5)
    losses = [float(tr.step()) for _ in range(80)]
    assert losses[-1] < 0.6 * losses[0], (losses[0], losses[-1])
    assert 0.0 <= tr.metric() <= 1.0
    r, nodes, leaf = tr.samples()
    assert nodes.numel() == tr.M[L - 1] and leaf.shape == (tr.M[L - 1], fan[-1])


@pytest.mark.parametrize("opt", ["adam", "adagrad", "sgd", "momentum"])
def test_cpu_optimizers_reduce_loss(opt):
    tr = _trainer("cpu", [5, 3], [32, 32, 16], 5, opt=opt, lr=0.05 if opt in ("sgd", "momentum") else 0.01)
    first = np.mean([float(tr.step()) for _ in range(5)])
    for _ in range(60):
        tr.step()
    last = np.mean([float(tr.step()) for _ in range(5)])
    assert last < first, (opt, first, last)


def test_cpu_resume_continues_trajectory():
    a = _trainer("cpu", [5, 3], [32, 32, 16], 5, mode="dense")
    for _ in range(5):
        a.step()
    sd, st = a.state_dict(), a.trainer_state()
    gen_state = a.graph._cpu_gen.get_state()
    cont = [float(a.step()) for _ in range(5)]
    b = _trainer("cpu", [5, 3], [32, 32, 16], 5, mode="dense")
    b.load_logical(sd)
    b.load_trainer_state(st)
    b.graph._cpu_gen.set_state(gen_state)  # CPU sampling uses torch's generator
    again = [float(b.step()) for _ in range(5)]
    np.testing.assert_allclose(again, cont, rtol=1e-5)


def test_from_model_matches_supervised_graphsage_names():
    from euler_amd.models.sage_trainer import sage_param_names

    tr = _trainer("cpu", [5, 3], [32, 32, 16], 5)
    assert list(tr.state_dict()) == sage_param_names(2)


@pytest.mark.parametrize("cfg", [dict(fanouts=[6], dims=[40, 24], C=10),
                                 dict(fanouts=[5, 3], dims=[64, 64, 32], C=10, self_loops=True, mode="dense"),
                                 dict(fanouts=[3, 20, 2], dims=[64, 128, 64, 32], C=16, D=64, mode="dense",
                                      self_loops=True)])
def test_bf16_oracle_is_the_model_without_rounding_cpu(cfg, monkeypatch):
    """the bf16-aware oracle's hand-written forward / backward (head, tree routing, the
    combined Wout Wfc) IS the model's autograd once the bf16 rounding is switched off"""
    tr = _trainer("cpu", fdt=torch.float32, **cfg)
    tr.step()
    orig = torch.Tensor.to

    def no_bf16(self, *a, **k):
        return self if a and a[0] is torch.bfloat16 else orig(self, *a, **k)

    monkeypatch.setattr(torch.Tensor, "to", no_bf16)
    loss_o, grads_o = tr.reference_loss_and_grads_bf16()
    monkeypatch.setattr(torch.Tensor, "to", orig)
    loss_r, grads_r = tr.reference_loss_and_grads()
    assert abs(loss_o - loss_r) <= 1e-6 * abs(loss_r) and set(grads_o) == set(grads_r)
    for k in grads_r:
        assert ((grads_o[k] - grads_r[k]).norm() / grads_r[k].norm()).item() < 1e-5, k


# ----------------------------------------------------------------------------------------- GPU

CASES = [
    dict(fanouts=[6], dims=[40, 24], C=10),                                   # 1 hop (mode-1 gather, no dA)
    dict(fanouts=[5, 3], dims=[64, 64, 32], C=32),
    dict(fanouts=[25, 10], dims=[256, 256, 256], C=64, D=128, B=128),         # bench shapes
    dict(fanouts=[5, 3], dims=[40, 72, 24], C=10, mode="dense"),              # padding everywhere, multi-label
    dict(fanouts=[5, 3], dims=[64, 64, 32], C=32, fdt=torch.float32),         # fp32 feature table
    dict(fanouts=[5, 3], dims=[64, 64, 32], C=32, self_loops=True, mode="class32"),
    dict(fanouts=[17, 3], dims=[64, 64, 32], C=32),                           # 64-row sibling groups
    dict(fanouts=[5, 3], dims=[64, 64, 32], C=32, types=2, metapath=[[0], [0, 1]]),
    dict(fanouts=[4, 3, 2], dims=[64, 64, 64, 32], C=32),                     # 3 hops (inner layer + bwd)
    dict(fanouts=[3, 20, 2], dims=[64, 128, 64, 32], C=16, mode="dense", self_loops=True),
    dict(fanouts=[5, 3], dims=[64, 64, 32], C=32, B=1024),                    # 64 fc-bias slabs: grouped reduce
    # every sibling-group size of the layer-0 kernel at D % 64 == 0
    dict(fanouts=[3, 3], dims=[64, 64, 32], C=32, D=64, B=256),                # 4-row groups
    dict(fanouts=[5, 4], dims=[128, 64, 32], C=32, D=64, B=256, self_loops=True),  # 8-row groups
    dict(fanouts=[10, 3], dims=[64, 64, 32], C=32, D=128, B=512),              # 16-row groups
    dict(fanouts=[40, 2], dims=[64, 64, 32], C=32, D=64, B=64, mode="dense"),  # 64-row groups
]


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", CASES, ids=[f"case{i}" for i in range(len(CASES))])
def test_tree_step_matches_fp32_oracle(cuda, cfg):
    tr = _trainer(cuda, **cfg)
    tr.forward_backward()
    torch.cuda.synchronize()
    loss_k = float(tr.loss_acc.item())
    grads_k = tr.gradients()
    # tight: the bf16-aware fp32 oracle rounds operands exactly where the kernels do, so
    # only fp32 accumulation order separates them
    loss_b, grads_b = tr.reference_loss_and_grads_bf16()
    assert abs(loss_k - loss_b) <= 1e-4 * abs(loss_b), (loss_k, loss_b)
    for name in grads_b:
        cos, rel = _cmp(grads_k[name], grads_b[name])
        assert rel < 1e-3, (name, cos, rel)
    # loose, second check: the plain fp32 model (bf16 operand noise: sums over thousands
    # of routed rows with mixed signs reach ~8 % in the relative norm)
    loss_r, grads_r = tr.reference_loss_and_grads()
    assert abs(loss_k - loss_r) <= 2e-2 * abs(loss_r) + 1e-4, (loss_k, loss_r)
    for name in grads_r:
        cos, rel = _cmp(grads_k[name], grads_r[name])
        assert cos > 0.995 and rel < 0.1, (name, cos, rel)
    # samples are valid rows and roots of the right node population
    roots, nodes, leaf = tr.samples()
    n = tr.graph.num_rows
    assert int(roots.min()) >= 0 and int(roots.max()) < n
    assert int(nodes.max()) < n and int(leaf.max()) < n
    # the update is Adam in fp32 on the reduced gradient
    p0, m0, v0, g = tr.flat.clone(), tr.m.clone(), tr.v.clone(), tr.grad.clone()
    t = float(tr._step.item())
    tr.optimizer_step()
    torch.cuda.synchronize()
    assert math.isfinite(float(tr.loss.item()))
    if tr.opt_name == "adam":
        b1, b2 = tr.betas
        m = b1 * m0 + (1 - b1) * g
        v = b2 * v0 + (1 - b2) * g * g
        p = p0 - tr.lr * (m / (1 - b1 ** t)) / (torch.sqrt(v / (1 - b2 ** t)) + tr.eps)
        assert torch.allclose(tr.flat, p, rtol=1e-5, atol=1e-6)
        assert torch.allclose(tr.m, m, rtol=1e-5, atol=1e-7)


@pytest.mark.gpu
def test_padding_stays_zero_and_step_counter(cuda):
    tr = _trainer(cuda, [5, 3], [40, 72, 24], 10, mode="dense")
    for _ in range(5):
        tr.step()
    torch.cuda.synchronize()
    flat = tr.flat.clone()
    logical = tr.logical_params()
    ref = torch.zeros_like(flat)
    tr._pack(logical, ref)
    assert torch.equal(flat, ref), "padded parameter entries moved"
    assert int(tr._step.item()) == 5 and int(tr.graph.rng[1].item()) == 5


@pytest.mark.gpu
def test_graph_replay_matches_eager(cuda):
    a = _trainer(cuda, [5, 3], [64, 64, 32], 32)
    b = _trainer(cuda, [5, 3], [64, 64, 32], 32)
    la = []
    for _ in range(12):
        a.step()
        la.append(float(a.loss.item()))
    b.capture(warmup=2)
    lb = []
    for _ in range(2):  # the warmup steps ran eagerly inside capture()
        pass
    for _ in range(10):
        b.replay()
        lb.append(float(b.loss.item()))
    np.testing.assert_allclose(lb, la[2:], rtol=2e-3, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("fdt", [torch.bfloat16, torch.float32])
def test_pipelined_step_matches_unpipelined(cuda, fdt, monkeypatch):
    """The pipelined step (the optimizer launch gathers the next batch's layer-0 inputs,
    the forward is GEMM-only) computes exactly what the fused gather+GEMM forward does:
    bit-identical losses and parameters, eager and graph-replayed.  The pipelined step is
    opt-in (EULER_AMD_PIPELINE=1: measured slower on the headline, README), so the test
    turns it on for the trainers it builds."""
    from euler_amd.models import sage_trainer

    monkeypatch.setattr(sage_trainer, "_PIPELINE", True)
    a = _trainer(cuda, [25, 10], [64, 64, 32], 32, fdt=fdt, D=64)
    b = _trainer(cuda, [25, 10], [64, 64, 32], 32, fdt=fdt, D=64)
    assert a.pipelined
    b.pipelined = False
    la, lb = [], []
    for _ in range(5):
        a.step()
        b.step()
        la.append(float(a.loss.item()))
        lb.append(float(b.loss.item()))
    a.capture(warmup=1, steps=2)
    b.capture(warmup=1, steps=2)
    a.replay_steps(5)
    b.replay_steps(5)
    la.append(float(a.loss.item()))
    lb.append(float(b.loss.item()))
    assert la == lb, (la, lb)
    pa, pb = a.logical_params(), b.logical_params()
    assert all(torch.equal(pa[k], pb[k]) for k in pa)
    assert la[-1] < la[0]


@pytest.mark.gpu
def test_sharded_feature_cache_matches_whole_table(cuda):
    """The forward reading a feature cache through cache positions (the sharded-feature
    exchange, here one rank without collectives: unique + gather into the cache) trains
    exactly like the forward reading the whole table, eager and graph-replayed."""
    from euler_amd.graph.sharded_features import ShardedFeatures
    from euler_amd.models.sage_trainer import SageTrainer

    def make(shard):
        g = _graph(cuda, seed=3)
        g.manual_seed(20)
        x, lab = _tables(cuda, g.num_rows, 32, 32, "class", torch.bfloat16)
        fs = ShardedFeatures.from_full(x) if shard else None
        return SageTrainer(g, 64, [5, 3], [64, 64, 32], 32, features=None if shard else x, labels=lab,
                           feature_shard=fs, init_seed=3)

    a, b = make(False), make(True)
    la, lb = [], []
    for _ in range(4):
        a.step()
        b.step()
        la.append(float(a.loss.item()))
        lb.append(float(b.loss.item()))
    a.capture(warmup=1)
    b.capture(warmup=1)
    for _ in range(6):
        a.replay()
        b.replay()
        la.append(float(a.loss.item()))
        lb.append(float(b.loss.item()))
    assert la == lb, (la, lb)
    pa, pb = a.logical_params(), b.logical_params()
    assert all(torch.equal(pa[k], pb[k]) for k in pa)


@pytest.mark.gpu
def test_grad_sync_handoff_fp32_and_bf16(cuda):
    """Data-parallel path: per bucket reduce -> grad_sync(bucket) (two buckets, the head
    bucket first, overlapped with the routed dW) -> optimizer.  With an identity sync the
    fp32 hand-off reproduces the fused single-process step exactly; the bf16 hand-off (half
    the all-reduce bytes) tracks it within bf16 rounding."""
    ref = _trainer(cuda, [5, 3], [64, 64, 32], 32)
    f32 = _trainer(cuda, [5, 3], [64, 64, 32], 32)
    b16 = _trainer(cuda, [5, 3], [64, 64, 32], 32)
    f32.n_buckets = b16.n_buckets = 2  # the overlapped two-bucket path (one bucket: test_bench)
    b16.set_grad_sync_dtype(torch.bfloat16)
    seen = []

    def sync(g):
        seen.append((g.dtype, g.numel()))
        return 1.0

    lr, lf, lb = [], [], []
    for _ in range(30):
        ref.step()
        f32.step(sync)
        b16.step(sync)
        lr.append(float(ref.loss.item()))
        lf.append(float(f32.loss.item()))
        lb.append(float(b16.loss.item()))
    (_, a0, a1), (_, b0, b1) = f32.grad_buckets()
    assert seen[:4] == [(torch.float32, a1 - a0), (torch.float32, b1 - b0), (torch.bfloat16, a1 - a0),
                        (torch.bfloat16, b1 - b0)]
    assert a1 - a0 + b1 - b0 == f32.grad.numel()
    np.testing.assert_allclose(lf, lr, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(lb, lr, rtol=0.03, atol=1e-3)


@pytest.mark.gpu
def test_gpu_resume_continues_trajectory(cuda):
    a = _trainer(cuda, [5, 3], [64, 64, 32], 10, mode="dense")
    for _ in range(6):
        a.step()
    sd, st = a.state_dict(), a.trainer_state()
    cont = []
    for _ in range(6):
        a.step()
        cont.append(float(a.loss.item()))
    b = _trainer(cuda, [5, 3], [64, 64, 32], 10, mode="dense")
    b.load_logical(sd)
    b.load_trainer_state(st)
    again = []
    for _ in range(6):
        b.step()
        again.append(float(b.loss.item()))
    # same Philox stream and state: same samples; only float-atomic order may differ
    np.testing.assert_allclose(again, cont, rtol=2e-3, atol=1e-5)


@pytest.mark.gpu
def test_bf16_trajectory_tracks_fp32_for_200_steps(cuda):
    """200 Adam steps of the bf16 kernels vs an fp32 torch model updated with fp32
    gradients on the SAME sampled trees: the loss curves stay together."""
    from euler_amd.models.sage_trainer import SageTrainer  # noqa: F401

    tr = _trainer(cuda, [10, 5], [64, 64, 32], 16, D=32, B=128, lr=0.01)
    ref = {k: v.clone() for k, v in tr.logical_params().items()}
    m = {k: torch.zeros_like(v) for k, v in ref.items()}
    v2 = {k: torch.zeros_like(v) for k, v in ref.items()}
    b1, b2, eps, lr = 0.9, 0.999, 1e-8, 0.01
    lk, lr_ = [], []
    for t in range(1, 201):
        tr.forward_backward()
        loss_ref, g = tr.reference_loss_and_grads(params=ref)
        tr.optimizer_step()
        lk.append(float(tr.loss.item()))
        lr_.append(loss_ref)
        with torch.no_grad():
            for k in ref:
                m[k].mul_(b1).add_(g[k], alpha=1 - b1)
                v2[k].mul_(b2).addcmul_(g[k], g[k], value=1 - b2)
                ref[k] -= lr * (m[k] / (1 - b1 ** t)) / (torch.sqrt(v2[k] / (1 - b2 ** t)) + eps)
    lk, lr_ = np.asarray(lk), np.asarray(lr_)
    w = 20
    sk = np.convolve(lk, np.ones(w) / w, "valid")
    sr = np.convolve(lr_, np.ones(w) / w, "valid")
    assert np.max(np.abs(sk - sr) / sr) < 0.05, np.max(np.abs(sk - sr) / sr)
    assert sk[-1] < 0.8 * sk[0]
    # Adam turns near-zero gradient entries into full-size steps whose sign follows the
    # bf16 rounding noise, so individual weights drift apart; the models must still agree
    for k in ref:
        cos, _ = _cmp(tr.logical_params()[k], ref[k])
        assert cos > 0.9, (k, cos)


# ----------------------------------------------------------------------------------------- estimator


def _run_graphsage(tmp_path, device, steps, extra=()):
    from euler_amd.tools.runner import main

    args = ["--dataset", "ppi", "--scale", "0.05", "--batch_size", "64", "--total_step", str(steps), "--log_steps",
            "10", "--model_dir", str(tmp_path / "ckpt"), "--device_graph", "--device", device, "--seed", "1",
            "--fanouts", "5", "3"] + list(extra)
    return main(args, model="graphsage")


def test_estimator_device_graph_train_resume_evaluate_cpu(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    r1 = _run_graphsage(tmp_path, "cpu", 20)
    assert r1["step"] == 20 and math.isfinite(r1["loss"])
    r2 = _run_graphsage(tmp_path, "cpu", 30)  # resumes from model.ckpt-20
    assert r2["step"] == 30
    st = torch.load(str(tmp_path / "ckpt" / "model.ckpt-30.pt"), weights_only=True)
    assert st["device_trainer"]["step"] == 30 and "gnn.convs.0.self_fc.weight" in st["model"]
    from euler_amd.tools.runner import main

    ev = main(["--dataset", "ppi", "--scale", "0.05", "--batch_size", "64", "--model_dir", str(tmp_path / "ckpt"),
               "--run_mode", "evaluate", "--device", "cpu", "--fanouts", "5", "3"], model="graphsage")
    assert math.isfinite(ev["loss"])


@pytest.mark.gpu
def test_estimator_device_graph_gpu(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    r1 = _run_graphsage(tmp_path, "cuda", 40)
    assert r1["step"] == 40 and math.isfinite(r1["loss"])
    r2 = _run_graphsage(tmp_path, "cuda", 60)
    assert r2["step"] == 60 and r2["loss"] < 0.7


@pytest.mark.gpu
def test_device_path_tracks_engine_path(tmp_path, monkeypatch):
    """The same SupervisedGraphSage / PPI-schema run through the estimator on the engine
    path (CPU sampling + autograd on the GPU) and on the device path (fused kernels on an
    HBM copy of the graph): after 150 steps both reach the same loss level."""
    monkeypatch.chdir(tmp_path)
    from euler_amd.tools.runner import main

    base = ["--dataset", "ppi", "--scale", "0.05", "--batch_size", "256", "--total_step", "150", "--log_steps",
            "150", "--device", "cuda", "--seed", "3", "--fanouts", "5", "3", "--learning_rate", "0.01"]
    eng = main(base + ["--model_dir", str(tmp_path / "eng")], model="graphsage")
    dev = main(base + ["--model_dir", str(tmp_path / "dev"), "--device_graph"], model="graphsage")
    assert math.isfinite(eng["loss"]) and math.isfinite(dev["loss"])
    assert abs(dev["loss"] - eng["loss"]) < 0.12 * eng["loss"], (eng["loss"], dev["loss"])
