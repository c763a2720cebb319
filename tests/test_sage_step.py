"""Fused GraphSAGE training step (csrc/hip/sage_train.hip) vs an fp32 torch-autograd
oracle of the same model on the same sampled indices and parameters."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(cuda, B, fanouts, D, H, C, include_self=False, n=20000, seed=3):
    from euler_amd.graph.device_graph import DeviceGraph
    from euler_amd.models.fused_sage import synthetic_features, synthetic_labels
    from euler_amd.models.sage_step import FusedSageTrainer

    torch.manual_seed(seed)
    g = DeviceGraph.synthetic(n, 6.0, 64, seed=seed, device=cuda)
    g.manual_seed(seed + 11)
    feats = synthetic_features(n, D, seed + 1, cuda)
    labels = synthetic_labels(feats, C)
    tr = FusedSageTrainer(g, feats, labels, B, fanouts, H, C, lr=0.01, add_self_loops=include_self)
    return tr


def _cmp(a, b):
    a, b = a.float().reshape(-1), b.float().reshape(-1)
    cos = torch.nn.functional.cosine_similarity(a, b, dim=0).item()
    rel = ((a - b).norm() / b.norm().clamp_min(1e-12)).item()
    return cos, rel


@pytest.mark.parametrize("cfg", [
    dict(B=64, fanouts=(5, 3), D=64, H=64, C=32),
    dict(B=64, fanouts=(4, 3), D=32, H=128, C=64, include_self=True),
    dict(B=256, fanouts=(25, 10), D=128, H=256, C=64),  # the bench shapes, smaller batch
])
def test_fused_step_grads_match_autograd(cuda, cfg):
    tr = _setup(cuda, **cfg)
    tr.forward_backward()
    torch.cuda.synchronize()
    loss_k = float(tr.loss_acc.item())
    grads_k = [tr.gW0, tr.gW1, tr.gWfc, tr.gbfc, tr.gWout]
    grads_k = [g.clone() for g in grads_k]
    loss_r, grads_r = tr.reference_forward_backward()
    assert abs(loss_k - loss_r) <= 2e-2 * abs(loss_r) + 1e-4, (loss_k, loss_r)
    for name, gk, gr in zip(["W0", "W1", "Wfc", "bfc", "Wout"], grads_k, grads_r):
        cos, rel = _cmp(gk, gr)
        assert cos > 0.995 and rel < 0.06, (name, cos, rel)


@pytest.mark.parametrize("fuse,fanouts", [("1", (5, 3)), ("0", (1, 3))])
def test_route_variants_match_autograd(cuda, monkeypatch, fuse, fanouts):
    """g0 rebuilt inside the dW kernel (EULER_AMD_FUSE_ROUTE=1), and the route kernel's
    F1 == 1 identity-division case"""
    monkeypatch.setenv("EULER_AMD_FUSE_ROUTE", fuse)
    tr = _setup(cuda, B=64, fanouts=fanouts, D=64, H=64, C=32)
    assert tr.fuse_route == (fuse == "1")
    tr.forward_backward()
    torch.cuda.synchronize()
    g0 = tr.gW0.clone()
    _, grads_r = tr.reference_forward_backward()
    cos, rel = _cmp(g0, grads_r[0])
    assert cos > 0.995 and rel < 0.06, (cos, rel)


def test_fused_adam_and_shadows(cuda):
    tr = _setup(cuda, B=64, fanouts=(5, 3), D=64, H=64, C=32)
    tr.forward_backward()
    torch.cuda.synchronize()
    p0 = tr.flat.clone()
    g = tr.grad.clone()
    ref = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([ref], lr=0.01, eps=1e-8)
    ref.grad = g.clone()
    opt.step()
    tr.optimizer_step()
    torch.cuda.synchronize()
    assert torch.allclose(tr.flat, ref.detach(), atol=1e-5, rtol=1e-4)
    # bias grad (atomically accumulated) is re-zeroed; loss handed off; shadows refreshed
    assert float(tr.gbfc.abs().sum()) == 0.0
    assert float(tr.loss_acc.item()) == 0.0 and float(tr.loss_out.item()) > 0
    from euler_amd.models.sage_step import fm_to_dense

    assert torch.equal(fm_to_dense(tr.W1b), tr.W1.to(torch.bfloat16))
    assert torch.equal(fm_to_dense(tr.W0b), tr.W0.to(torch.bfloat16))
    assert torch.equal(fm_to_dense(tr.Woutb), tr.Wout.to(torch.bfloat16))
    assert torch.equal(fm_to_dense(tr.W1T), tr.W1.to(torch.bfloat16).t())
    assert torch.equal(fm_to_dense(tr.WoutT), tr.Wout.to(torch.bfloat16).t())
    assert torch.equal(fm_to_dense(tr.WfcT), tr.Wfc.to(torch.bfloat16).t())


def test_fused_step_hipgraph_trains(cuda):
    tr = _setup(cuda, B=128, fanouts=(5, 3), D=64, H=64, C=32)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            tr.step()
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        tr.step()
    losses = []
    roots_seen = set()
    for i in range(60):
        graph.replay()
        if i % 10 == 0:
            torch.cuda.synchronize()
            losses.append(float(tr.loss.item()))
            roots_seen.add(tuple(tr.roots[:8].tolist()))
    torch.cuda.synchronize()
    losses.append(float(tr.loss.item()))
    assert all(l == l for l in losses)  # finite
    assert losses[-1] < losses[0]
    assert len(roots_seen) > 1  # replays draw fresh samples
    assert int(tr.step_count.item()) == 62  # 2 eager + 60 replays (capture does not execute)



def test_fused_step_pipelined_sampling_hipgraph(cuda, monkeypatch):
    """EULER_AMD_PIPELINE_SAMPLING=1: next step's samples drawn on a side stream; one
    captured graph per sample-set parity, replayed alternately, keeps training on fresh
    samples and counts Adam steps like the serial order."""
    monkeypatch.setenv("EULER_AMD_PIPELINE_SAMPLING", "1")
    tr = _setup(cuda, B=128, fanouts=(5, 3), D=64, H=64, C=32)
    assert tr.pipelined
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            tr.step()
    torch.cuda.current_stream().wait_stream(s)
    graphs = {}
    for _ in range(2):
        p = tr.parity
        graphs[p] = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graphs[p]):
            tr.step()
    losses, roots_seen = [], set()
    for i in range(60):
        graphs[tr.parity].replay()
        tr.advance_parity()
        if i % 10 == 0:
            torch.cuda.synchronize()
            losses.append(float(tr.loss.item()))
            roots_seen.add(tuple(tr.roots[:8].tolist()))
    torch.cuda.synchronize()
    losses.append(float(tr.loss.item()))
    assert all(l == l for l in losses)
    assert losses[-1] < losses[0]
    assert len(roots_seen) > 1
    assert int(tr.step_count.item()) == 63  # 3 eager + 60 replays
