"""Numerics of every gfx950 kernel against a plain PyTorch fp32 reference of the same op."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _hip():
    from euler_amd.ops._native import hip

    return hip()


def test_extension_is_native(cuda):
    import euler_amd._hip_ops as h

    assert h.arch == "gfx950"
    assert h.__file__.endswith(".so")


@pytest.mark.parametrize("D,H,F,include_self", [(128, 256, 25, False), (64, 128, 10, True), (32, 47, 3, False),
                                                (256, 64, 7, False), (128, 512, 10, False)])
def test_sage_fwd_matches_reference(cuda, D, H, F, include_self):
    from euler_amd.ops.sage_ops import sage_layer_reference

    torch.manual_seed(0)
    N, M = 5000, 777
    x = torch.randn(N, D, device=cuda).to(torch.bfloat16)
    # asymmetric weights (catches transposed C writes)
    W = (torch.randn(H, 2 * D, device=cuda) * 0.1 + torch.arange(H, device=cuda).view(-1, 1) * 1e-3).to(torch.bfloat16)
    b = torch.randn(H, device=cuda)
    nbr = torch.randint(-1, N, (M, F), device=cuda, dtype=torch.int32)
    si = torch.randint(0, N, (M,), device=cuda, dtype=torch.int32)
    out, a = _hip().sage_fwd(x, si, nbr, W, b, include_self, True, True)
    ref = sage_layer_reference(x, si, nbr, W, b, include_self, True)
    torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=3e-2)
    # saved A tile = [x_self | mean]
    xs = x.float()[si.long()]
    torch.testing.assert_close(a[:, :D].float(), xs)


def test_sage_layer_grads(cuda):
    from euler_amd.ops.sage_ops import sage_layer, sage_layer_reference

    torch.manual_seed(1)
    N, M, D, H, F = 2000, 300, 64, 128, 5
    x = torch.randn(N, D, device=cuda).to(torch.bfloat16).requires_grad_(True)
    W = (torch.randn(H, 2 * D, device=cuda) * 0.1).requires_grad_(True)
    nbr = torch.randint(0, N, (M, F), device=cuda, dtype=torch.int32)
    si = torch.randint(0, N, (M,), device=cuda, dtype=torch.int32)
    out = sage_layer(x, si, nbr, W, None, include_self=False, relu=True)
    g = torch.randn_like(out.float())
    (out.float() * g).sum().backward()
    x2 = x.detach().float().requires_grad_(True)
    W2 = W.detach().to(torch.bfloat16).float().requires_grad_(True)
    ref = sage_layer_reference(x2, si, nbr, W2, None, False, False)
    # apply the ReLU mask of the kernel's own (bf16-rounded) output so the check does
    # not depend on sign flips of near-zero pre-activations
    ((ref * (out.detach().float() > 0)) * g).sum().backward()
    torch.testing.assert_close(W.grad, W2.grad, atol=0.15, rtol=5e-2)
    torch.testing.assert_close(x.grad.float(), x2.grad, atol=5e-2, rtol=5e-2)


def test_sage_bwd_disjoint_equals_atomic(cuda):
    torch.manual_seed(2)
    M, F, D = 256, 4, 32
    dA = torch.randn(M, 2 * D, device=cuda).to(torch.bfloat16)
    nbr = torch.arange(M * F, device=cuda, dtype=torch.int32).view(M, F)
    si = torch.arange(M * F, M * F + M, device=cuda, dtype=torch.int32)
    d1 = torch.zeros(M * F + M, D, device=cuda)
    d2 = torch.zeros_like(d1)
    _hip().sage_bwd_scatter(dA, si, nbr, False, True, d1)
    _hip().sage_bwd_scatter(dA, si, nbr, False, False, d2)
    torch.testing.assert_close(d1, d2)


def test_linear_fwd(cuda):
    torch.manual_seed(3)
    A = torch.randn(1000, 256, device=cuda).to(torch.bfloat16)
    W = torch.randn(192, 256, device=cuda).to(torch.bfloat16)
    b = torch.randn(192, device=cuda)
    out = _hip().linear_fwd(A, W, b, False)
    ref = A.float() @ W.float().t() + b
    torch.testing.assert_close(out.float(), ref, atol=0.25, rtol=2e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("idx_dtype", [torch.int32, torch.int64])
def test_gather_rows(cuda, dtype, idx_dtype):
    x = torch.randn(1000, 40, device=cuda).to(dtype)
    idx = torch.randint(-1, 1000, (5000,), device=cuda, dtype=idx_dtype)
    out = _hip().gather_rows(x, idx)
    ref = torch.where((idx >= 0).view(-1, 1), x[idx.clamp(min=0).long()], torch.zeros((), dtype=dtype, device=cuda))
    torch.testing.assert_close(out, ref)


@pytest.mark.parametrize("reduce", ["add", "mean", "max"])
@pytest.mark.parametrize("D,dtype", [(19, torch.float32), (64, torch.float32), (64, torch.bfloat16)])
def test_scatter_ops_match_cpu(cuda, reduce, D, dtype):
    """scalar path (D = 19) and the 16-byte-vector path (D % 4 fp32, D % 8 bf16)"""
    from euler_amd.ops import mp_ops

    torch.manual_seed(4)
    E, S = 3000, 230   # some segments stay empty
    src = torch.randn(E, D).to(dtype)
    idx = torch.randint(0, S - 20, (E,))
    ref = mp_ops._cpu_scatter(src.float(), idx, S, reduce)
    out = mp_ops.scatter_(reduce, src.to(cuda), idx.to(cuda), S)
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    torch.testing.assert_close(out.float().cpu(), ref, atol=tol, rtol=tol)


@pytest.mark.parametrize("reduce", ["add", "mean", "max"])
def test_scatter_grads(cuda, reduce):
    from euler_amd.ops import mp_ops

    torch.manual_seed(5)
    E, S, D = 500, 40, 8
    src = torch.randn(E, D, dtype=torch.float64)
    idx = torch.randint(0, S, (E,))
    g = torch.randn(S, D, dtype=torch.float64)
    s1 = src.clone().float().to(cuda).requires_grad_(True)
    (mp_ops.scatter_(reduce, s1, idx.to(cuda), S) * g.float().to(cuda)).sum().backward()
    s2 = src.clone().float().requires_grad_(True)
    (mp_ops._cpu_scatter(s2, idx, S, reduce) * g.float()).sum().backward()
    torch.testing.assert_close(s1.grad.cpu(), s2.grad, atol=1e-5, rtol=1e-5)


def test_gather_grad(cuda):
    from euler_amd.ops import mp_ops

    x = torch.randn(100, 16, device=cuda, requires_grad=True)
    idx = torch.randint(0, 100, (1000,), device=cuda)
    out = mp_ops.gather(x, idx)
    g = torch.randn_like(out)
    (out * g).sum().backward()
    ref = torch.zeros(100, 16, device=cuda).index_add_(0, idx, g)
    torch.testing.assert_close(x.grad, ref, atol=1e-4, rtol=1e-4)


def test_scatter_softmax(cuda):
    from euler_amd.ops import mp_ops

    torch.manual_seed(6)
    E, S, H = 2000, 100, 8
    lg = torch.randn(E, H) * 3
    idx = torch.randint(0, S, (E,))
    ref = mp_ops.scatter_softmax(lg, idx, S)
    lgc = lg.to(cuda).requires_grad_(True)
    out = mp_ops.scatter_softmax(lgc, idx.to(cuda), S)
    torch.testing.assert_close(out.cpu(), ref, atol=1e-5, rtol=1e-4)
    g = torch.randn(E, H)
    (out * g.to(cuda)).sum().backward()
    lg2 = lg.clone().requires_grad_(True)
    (mp_ops.scatter_softmax(lg2, idx, S) * g).sum().backward()
    torch.testing.assert_close(lgc.grad.cpu(), lg2.grad, atol=1e-5, rtol=1e-4)


def test_spmm_csr(cuda):
    torch.manual_seed(7)
    S, N, D, nnz = 300, 400, 33, 3000
    rows = torch.randint(0, S, (nnz,))
    cols = torch.randint(0, N, (nnz,))
    w = torch.rand(nnz)
    order = torch.argsort(rows, stable=True)
    rows, cols, w = rows[order], cols[order], w[order]
    indptr = torch.zeros(S + 1, dtype=torch.long)
    indptr[1:] = torch.cumsum(torch.bincount(rows, minlength=S), 0)
    x = torch.randn(N, D)
    ref = torch.zeros(S, D).index_add_(0, rows, x[cols] * w.view(-1, 1))
    out = _hip().spmm_csr(indptr.to(cuda), cols.to(cuda), w.to(cuda), x.to(cuda))
    torch.testing.assert_close(out.cpu(), ref, atol=1e-4, rtol=1e-4)


def test_device_graph_sampling_distribution(cuda):
    """Weighted with-replacement sampling ratios (reference end2end_local_test.cc:66-72 style)."""
    from euler_amd.graph.device_graph import DeviceGraph

    # node 0 -> {1 (w=1), 2 (w=2), 3 (w=3)}; node 1 -> {}; nodes 2,3 -> {0}
    indptr = [0, 3, 3, 4, 5]
    nbr = [1, 2, 3, 0, 0]
    w = [1.0, 2.0, 3.0, 1.0, 1.0]
    g = DeviceGraph.from_csr(indptr, nbr, w, device=cuda, seed=3)
    rows = torch.zeros(20000, dtype=torch.int32, device=cuda)
    out = g.sample_neighbor(rows, 10, default=-1).cpu()
    c = torch.bincount(out.reshape(-1).long(), minlength=4).float()
    assert 1.9 < c[2] / c[1] < 2.1
    assert 2.9 < c[3] / c[1] < 3.1
    empty = g.sample_neighbor(torch.tensor([1], dtype=torch.int32, device=cuda), 4, default=-7).cpu()
    assert (empty == -7).all()
    # counter advance changes the draws
    a = g.sample_neighbor(rows[:100], 4).cpu()
    g.advance()
    b = g.sample_neighbor(rows[:100], 4).cpu()
    assert not torch.equal(a, b)


def test_synthetic_graph_and_alias(cuda):
    from euler_amd.graph.device_graph import DeviceGraph

    g = DeviceGraph.synthetic(100_000, 10.0, 512, seed=5, device=cuda)
    deg = torch.diff(g.indptr).float()
    assert 6.0 < deg.mean().item() < 12.0
    assert deg.min().item() >= 1
    nb = g.nbr.long()
    assert nb.min().item() >= 0 and nb.max().item() < 100_000
    # rows sorted
    ip = g.indptr.cpu()
    s, e = int(ip[10]), int(ip[11])
    seg = g.nbr[s:e].cpu()
    assert torch.equal(seg, torch.sort(seg).values)
    roots = g.sample_node(50_000)
    assert roots.min().item() >= 0 and roots.max().item() < 100_000
    walks = g.random_walk(roots[:100], 3)
    assert walks.shape == (100, 4)


def test_flat_adam_matches_cpu(cuda):
    import torch.nn as nn

    from euler_amd.parallel.flat import FlatOptimizer, FlatParams

    torch.manual_seed(8)
    m1 = nn.Linear(16, 8)
    m2 = nn.Linear(16, 8)
    m2.load_state_dict(m1.state_dict())
    m1 = m1.to(cuda)
    f1, f2 = FlatParams(m1.parameters(), cuda), FlatParams(m2.parameters())
    o1, o2 = FlatOptimizer(f1, "adam", 1e-2), FlatOptimizer(f2, "adam", 1e-2)
    x = torch.randn(32, 16)
    for _ in range(3):
        for m, f, o, xx in ((m1, f1, o1, x.to(cuda)), (m2, f2, o2, x)):
            f.zero_grad()
            m(xx).pow(2).sum().backward()
            o.step()
    torch.testing.assert_close(f1.flat.cpu(), f2.flat, atol=1e-5, rtol=1e-5)
