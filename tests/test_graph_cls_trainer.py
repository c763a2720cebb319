"""Fused graph-classification step (models/graph_cls_trainer.py, csrc/hip/graph_cls.hip):
GIN and GraphGCN under GraphEstimator(device_graph=True).

* the fused step's loss and every parameter gradient against the generic GraphTrainer's
  autograd step on the CPU (fp32 torch) for the same drawn graphs and weights;
* a captured, replayed training run through the estimator, trajectory against the generic
  GPU step from the same initialisation;
* the routing: GIN / GraphGCN take the fused trainer on the GPU, other models and the CPU
  the generic one.
Reference semantics: tf_euler/python/convolution/gin_conv.py:26-57, graph_conv.py:26-46,
mp_utils/base_graph.py:24-47, euler_estimator/python/graph_estimator.py:27-85.
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F


def _est(tmp_path, model, device, batch=16, steps=12, extra=()):
    from euler_amd.tools import runner

    a = runner.parse_args(["--model_dir", str(tmp_path / (model + device)), "--batch_size", str(batch),
                           "--total_step", str(steps), "--log_steps", "6", "--device", device, "--seed", "1",
                           "--device_graph", "--learning_rate", "0.01"] + list(extra), model=model)
    torch.manual_seed(0)
    return runner.build(a)


def _trainer(est):
    first = est.get_train_from_input(est.train_input_fn(), est.params)
    return est._device_graph_trainer(first)


@pytest.mark.parametrize("model,kind", [("gin", 0), ("graphgcn", 1), ("set2set", None), ("gated_graph", None)])
def test_fused_support_matrix(model, kind, tmp_path):
    from euler_amd.models.graph_cls_trainer import _conv_kind

    m, _ = _est(tmp_path, model, "cpu")
    assert _conv_kind(m) == kind


def test_graphgcn_flow_adds_self_loops(tmp_path):
    """reference examples/graphgcn/graphgcn.py:32: the GraphGCN flow has self loops, GIN's not"""
    m, _ = _est(tmp_path, "graphgcn", "cpu")
    assert m.gnn.sampler.add_self_loops
    m, _ = _est(tmp_path, "gin", "cpu")
    assert not m.gnn.sampler.add_self_loops


def test_cpu_routes_to_generic_trainer(tmp_path):
    from euler_amd.models.graph_cls_trainer import GraphClsTrainer
    from euler_amd.models.graph_trainer import GraphTrainer

    _, est = _est(tmp_path, "gin", "cpu")
    tr = _trainer(est)
    assert type(tr) is GraphTrainer and not isinstance(tr, GraphClsTrainer)


def _train_eps(est):
    """GIN with a trainable eps per conv (reference gin_conv.py train_eps=True)"""
    for conv in est.model.gnn.convs:
        del conv._buffers["eps"]
        conv.eps = torch.nn.Parameter(torch.tensor([0.25]))


@pytest.mark.gpu
@pytest.mark.parametrize("model,zst", [("gin", True), ("graphgcn", True), ("gin", False), ("graphgcn", False),
                                       ("gin_eps", True)])
def test_fused_step_matches_cpu_autograd(tmp_path, cuda, model, zst, monkeypatch):
    """both kernel variants: every conv's aggregate kept in LDS for the backward (default)
    and recomputed there (the fallback when they do not fit, forced by a small LDS budget);
    GIN with trainable eps (d eps = sum dZ . x)"""
    from euler_amd.models.graph_cls_trainer import GraphClsTrainer

    if not zst:
        monkeypatch.setenv("EULER_AMD_GRAPH_MAX_LDS", "1")
    eps = model == "gin_eps"
    model = "gin" if eps else model
    _, est = _est(tmp_path, model, "cuda")
    if eps:
        _train_eps(est)
    tr = _trainer(est)
    assert isinstance(tr, GraphClsTrainer) and tr.launches_per_step == 2
    assert tr.plan.z_kept == zst
    _, est_c = _est(tmp_path, model, "cpu")
    if eps:
        _train_eps(est_c)
    trc = _trainer(est_c)
    assert len(trc.flat.params) == len(tr.flat.params)
    with torch.no_grad():  # the same weights (random, not the init: every path non-trivial)
        gen = torch.Generator().manual_seed(5)
        for pc, pg in zip(trc.flat.params, tr.flat.params):
            assert pc.shape == pg.shape
            v = torch.randn(pc.shape, generator=gen) * 0.3
            pc.copy_(v)
            pg.copy_(v.to(pg.device))
    tr.flat.zero_grad()
    tr.forward_backward_only()
    torch.cuda.synchronize()
    gidx = tr.plan.gidx().long().cpu()
    assert 0 <= int(gidx.min()) and int(gidx.max()) < tr.onehot.shape[0]
    # the fused draw is the generic trainer's (alias table, Philox stream 3, advanced counter)
    st = tr.graph.rng.clone()
    tr.graph.rng[1] -= 1
    tr._draw()
    ref_g = tr.sample_graphs().long().cpu()
    tr.graph.rng.copy_(st)
    assert torch.equal(ref_g, gidx)
    loss_f = float(tr.loss_out)
    gf = tr.flat.grad[: tr.flat.numel].double().cpu()

    trc.flat.zero_grad()
    logits = trc._forward(gidx)
    loss = F.binary_cross_entropy_with_logits(logits, trc.onehot[gidx])
    loss.backward()
    gc = trc.flat.grad[: trc.flat.numel].double()
    assert math.isclose(loss_f, loss.item(), rel_tol=1e-5, abs_tol=1e-6), (loss_f, loss.item())
    for p, (o, n) in zip(trc.flat.params, trc.flat.offsets):
        a, b = gf[o:o + n], gc[o:o + n]
        err = float((a - b).norm() / b.norm().clamp(min=1e-12))
        assert err < 1e-4, (tuple(p.shape), err)
    # the accuracy counters: one step of B graphs
    assert float(tr.right[1]) == tr.B and 0 <= float(tr.right[0]) <= tr.B


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["gin", "graphgcn"])
def test_fused_training_matches_generic_gpu_step(tmp_path, cuda, model, monkeypatch):
    """20 captured steps from the same initialisation and RNG state: the fused trainer's
    losses follow the generic GPU trainer's (batch 16: fp32 linears on both sides)"""
    from euler_amd.models.graph_cls_trainer import GraphClsTrainer

    def run(fused):
        monkeypatch.setenv("EULER_AMD_GRAPH_FUSED", "1" if fused else "0")
        _, est = _est(tmp_path, model, "cuda")
        tr = _trainer(est)
        assert isinstance(tr, GraphClsTrainer) == fused
        with torch.no_grad():
            gen = torch.Generator().manual_seed(7)
            for p in tr.flat.params:
                p.copy_((torch.randn(p.shape, generator=gen) * 0.2).to(p.device))
        tr.graph.manual_seed(11)
        tr.capture(steps=1)
        out = []
        for _ in range(20):
            tr.replay_steps(1)
            out.append(float(tr.loss_out))
        return np.array(out), tr.metric()

    fused, acc_f = run(True)
    gen, acc_g = run(False)
    assert np.all(np.isfinite(fused))
    np.testing.assert_allclose(fused, gen, rtol=2e-3, atol=1e-5)
    assert abs(acc_f - acc_g) < 1e-9


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["gin", "graphgcn"])
def test_fused_estimator_learns(tmp_path, cuda, model):
    from euler_amd.tools import runner

    res = runner.main(["--model_dir", str(tmp_path / model), "--batch_size", "32", "--total_step", "400",
                       "--log_steps", "200", "--device", "cuda", "--seed", "1", "--device_graph",
                       "--learning_rate", "0.01"], model=model)
    assert res["step"] == 400 and math.isfinite(res["loss"])
    assert res["accuracy"] > 0.7, res


def _worker_graph_dp(rank, world, port, q, tmp, model):
    """one rank of a 2-process fused graph-classification job sharing the GPU (gloo process
    group; the gradient all-reduce between the slab reduce and the flat optimizer)"""
    import os

    try:
        os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                           "WORLD_SIZE": str(world), "LOCAL_RANK": "0"})
        import torch.distributed as dist

        from euler_amd.parallel import dp

        dp.init_distributed(backend="gloo", device=torch.device("cuda", 0))
        from euler_amd.tools import runner

        a = runner.parse_args(["--batch_size", "16", "--total_step", "6", "--log_steps", "3", "--model_dir",
                               os.path.join(tmp, f"ck{rank}"), "--device_graph", "--device", "cuda", "--seed", "1",
                               "--data_dir", os.path.join(tmp, "data")], model=model)
        _, est = runner.build(a)
        est.train()
        tr = est.device_trainer
        flat = tr.flat.flat.detach().cpu().clone()
        allp = [torch.zeros_like(flat) for _ in range(world)]
        dist.all_gather(allp, flat)
        gidx = tr.plan.gidx().cpu().clone()
        allg = [torch.zeros_like(gidx) for _ in range(world)]
        dist.all_gather(allg, gidx)
        ok = (type(tr).__name__ == "GraphClsTrainer" and all(torch.equal(x, allp[0]) for x in allp)
              and not torch.equal(allg[0], allg[1]) and bool(torch.isfinite(flat).all()) and est.global_step == 6)
        q.put((rank, "graph_dp", bool(ok), getattr(est, "grad_sync_name", None)))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["gin", "graphgcn"])
def test_fused_graph_two_ranks_share_the_gpu_in_lockstep(tmp_path, model):
    """the data-parallel form of the fused step (slab reduce into the flat gradient, the
    all-reduce, then the flat optimizer): 2 ranks on one GPU end bit-identical, having
    drawn different graphs"""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker_graph_dp, args=(r, 2, port, q, str(tmp_path), model)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    res = []
    while not q.empty():
        res.append(q.get())
    for p in procs:
        if p.is_alive():
            p.kill()
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 2 and all(r[2] for r in res), res
