"""Unsupervised GraphSAGE device path (models/sage_tower.py, csrc TowerPlan).

CPU: the torch twin learns the planted-community structure (held-out link AUC).
GPU: the fused tower kernels against the fp32 torch oracle on the same sampled trees
(loss and every parameter gradient), hipGraph-captured training, valid samples.
"""
import math
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "benchmarks"))


def _setup(device, n=6000, comm=30, dim=32, dims=(64, 64, 32), B=64, fan=(10, 5), lr=0.01, seed=7, fused=True,
           K=5):
    from bench_unsup_sage import build
    from euler_amd.models.sage_tower import UnsupSageTrainer

    graph, x, test = build(n, comm, 10, dim, 0.5, seed, torch.device(device))
    tr = UnsupSageTrainer(graph, B, list(fan), list(dims), features=x, num_negs=K, learning_rate=lr, init_seed=seed,
                          fused=fused)
    return tr, test


def _cmp(a, b):
    a, b = a.float().reshape(-1).cpu(), b.float().reshape(-1).cpu()
    if b.norm() < 1e-9:
        return 1.0, float(a.norm())
    return (torch.nn.functional.cosine_similarity(a, b, dim=0).item(), ((a - b).norm() / b.norm()).item())


def test_unsup_cpu_learns_communities():
    from bench_unsup_sage import link_auc

    tr, test = _setup("cpu", n=8000, comm=40, B=128)
    auc0 = link_auc(tr, test, 8000, 2000, 7)
    losses = [float(tr.step()) for _ in range(250)]
    auc1 = link_auc(tr, test, 8000, 2000, 7)
    assert sum(losses[-10:]) < 0.6 * sum(losses[:10]), (losses[:3], losses[-3:])
    assert auc1 > 0.85 and auc1 > auc0 + 0.25, (auc0, auc1)
    assert tr.metric() > 0.6


def test_unsup_param_layout_roundtrip_cpu():
    from euler_amd.models.sage_tower import unsup_param_names

    tr, _ = _setup("cpu", n=2000, dims=(40, 72, 24))
    lp = tr.logical_params()
    assert sorted(lp) == sorted(unsup_param_names())
    tr2, _ = _setup("cpu", n=2000, dims=(40, 72, 24), seed=8)
    tr2.load_logical(lp)
    for k, v in tr2.logical_params().items():
        assert torch.equal(v, lp[k]), k
    # padding stays zero after training steps
    for _ in range(5):
        tr.step()
    W1 = tr.params["gnn.W1"].detach()
    assert float(W1[72:].abs().sum()) == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [True, False], ids=["pair_plan", "per_op"])
@pytest.mark.parametrize("dims,fan,K", [((64, 64, 32), (10, 5), 5), ((128, 128, 128), (25, 10), 5),
                                        ((40, 72, 24), (5, 3), 3), ((128, 256, 128), (10, 5), 1)])
def test_unsup_kernels_match_fp32_oracle(cuda, dims, fan, K, fused):
    """the fused 7-launch step (PairPlan: roots drawn in the samplers, pair head kernel, one
    dW and one optimizer launch) and the per-op step against the fp32 torch oracle on the
    same sampled trees: loss and every parameter gradient"""
    tr, _ = _setup(cuda, dims=dims, fan=fan, B=64, fused=fused, K=K)
    assert (tr.pair is not None) == fused, getattr(tr, "fused_error", None)
    loss_k = tr.forward_backward()
    torch.cuda.synchronize()
    gk = tr.gradients()
    loss_r, gr = tr.reference_loss_and_grads()
    assert abs(loss_k - loss_r) <= 2e-2 * abs(loss_r) + 1e-4, (loss_k, loss_r)
    for k in gr:
        cos, rel = _cmp(gk[k], gr[k])
        assert cos > 0.995 and rel < 0.1, (k, cos, rel)
    roots, nodes, leaf = tr.tower_samples("context_gnn")
    n = tr.graph.num_rows
    assert int(nodes.max()) < n and int(leaf.max()) < n and int(roots.max()) < n


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [True, False], ids=["pair_plan", "per_op"])
def test_unsup_graph_replay_trains(cuda, fused):
    from bench_unsup_sage import link_auc

    tr, test = _setup(cuda, n=8000, comm=40, B=128, fused=fused)
    auc0 = link_auc(tr, test, 8000, 2000, 7)
    tr.capture(steps=4)
    first = float(tr.loss)
    tr.replay_steps(300)
    torch.cuda.synchronize()
    last = float(tr.loss)
    assert math.isfinite(last) and last < 0.6 * first, (first, last)
    auc1 = link_auc(tr, test, 8000, 2000, 7)
    assert auc1 > 0.85 and auc1 > auc0 + 0.25, (auc0, auc1)


def test_estimator_unsup_device_graph_train_resume_cpu(tmp_path, monkeypatch):
    """examples/run_graphsage_unsup.py --device_graph: NodeEstimator drives the device
    trainer, checkpoints the reference names + optimizer state + Philox counter, resumes."""
    monkeypatch.chdir(tmp_path)
    from euler_amd.tools.runner import main

    base = ["--dataset", "ppi", "--scale", "0.05", "--batch_size", "64", "--log_steps", "10", "--model_dir",
            str(tmp_path / "ckpt"), "--device_graph", "--device", "cpu", "--seed", "1", "--fanouts", "5", "3",
            "--dim", "32"]
    r1 = main(base + ["--total_step", "20"], model="graphsage_unsup")
    assert r1["step"] == 20 and math.isfinite(r1["loss"]) and "mrr" in r1
    r2 = main(base + ["--total_step", "30"], model="graphsage_unsup")
    assert r2["step"] == 30
    st = torch.load(str(tmp_path / "ckpt" / "model.ckpt-30.pt"), weights_only=True)
    assert "context_gnn.convs.1.neigh_fc.weight" in st["model"] and st["device_trainer"]["step"] >= 20


@pytest.mark.gpu
@pytest.mark.parametrize("E,K", [(128, 5), (64, 1), (40, 15)])
def test_fused_pair_loss_matches_torch(cuda, E, K):
    """pair.hip (loss, logits, reciprocal ranks, gradients) against the torch composition"""
    from euler_amd.models import _tower_ops as T

    torch.manual_seed(3)
    B = 300
    es = (torch.randn(B, E, device=cuda) * 0.3).requires_grad_(True)
    ec = (torch.randn(B * (1 + K), E, device=cuda) * 0.3).requires_grad_(True)
    mrr = torch.zeros(1, device=cuda)
    loss, logits, counted = T.pair_loss(es, ec, B, K, mrr)
    assert counted
    (loss * 1.7).backward()
    es2, ec2 = es.detach().clone().requires_grad_(True), ec.detach().clone().requires_grad_(True)
    loss2, logits2 = T._PairLoss.apply(es2, ec2, B, K)
    (loss2 * 1.7).backward()
    torch.testing.assert_close(loss, loss2, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(logits, logits2, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(es.grad, es2.grad, atol=1e-7, rtol=1e-4)
    torch.testing.assert_close(ec.grad, ec2.grad, atol=1e-7, rtol=1e-4)
    rank = 1 + (logits2[:, 1:] >= logits2[:, :1]).sum(1).float()
    torch.testing.assert_close(mrr[0], (1.0 / rank).sum(), atol=1e-3, rtol=1e-5)
