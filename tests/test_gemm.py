"""Tiled MFMA GEMM (csrc/hip/gemm.hip) against fp32 torch: every layout, dtype, epilogue
and split-K, odd shapes included."""
import pytest
import torch


def _ref(a, b, ta, tb, bias, relu, rmask, alpha):
    A = a.float().t() if ta else a.float()
    B = b.float().t() if tb else b.float()
    y = A @ B * alpha
    if bias is not None:
        y = y + bias
    if relu:
        y = torch.relu(y)
    if rmask is not None:
        y = y * (rmask.float() > 0)
    return y


def test_gemm_cpu_composition():
    from euler_amd.ops.gnn_ops import gemm

    a, b = torch.randn(30, 20), torch.randn(12, 20)
    bias = torch.randn(12)
    y = gemm(a, b, trans_b=True, bias=bias, relu=True)
    torch.testing.assert_close(y, _ref(a, b, False, True, bias, True, None, 1.0))


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(6144, 128, 256), (1024, 128, 128), (100, 70, 50), (257, 64, 33), (64, 256, 6144)])
@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False), (True, True)])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_gemm_matches_fp32(cuda, M, N, K, ta, tb, dt):
    from euler_amd.ops.gnn_ops import gemm

    g = torch.Generator(device=cuda).manual_seed(M + N + K)
    a = torch.randn((K, M) if ta else (M, K), device=cuda, generator=g).to(dt)
    b = torch.randn((N, K) if tb else (K, N), device=cuda, generator=g).to(dt)
    ref = _ref(a, b, ta, tb, None, False, None, 1.0)
    for splits in (1, 4):
        y = gemm(a, b, trans_a=ta, trans_b=tb, splits=splits)
        # bf16 operands: relative error ~ sqrt(K) * 2^-8 of the row norm products
        tol = 0.02 * float(ref.abs().max()) + 1e-3
        assert float((y - ref).abs().max()) <= tol, (splits, float((y - ref).abs().max()), tol)


@pytest.mark.gpu
def test_gemm_epilogues(cuda):
    from euler_amd.ops.gnn_ops import gemm

    M, N, K = 300, 96, 128
    a = torch.randn(M, K, device=cuda)
    w = torch.randn(N, K, device=cuda)
    bias = torch.randn(N, device=cuda)
    rm = torch.randn(M, N, device=cuda).to(torch.bfloat16)
    ref = _ref(a, w, False, True, bias, True, rm, 0.5)
    y = gemm(a, w, trans_b=True, bias=bias, relu=True, rmask=rm, alpha=0.5)
    assert float((y - ref).abs().max()) <= 0.02 * float(ref.abs().max()) + 1e-3
    yb = gemm(a, w, trans_b=True, bias=bias, out_dtype=torch.bfloat16)
    assert yb.dtype == torch.bfloat16
    ref2 = _ref(a, w, False, True, bias, False, None, 1.0)
    assert float((yb.float() - ref2).abs().max()) <= 0.03 * float(ref2.abs().max()) + 1e-2
    # in place into a strided view (a slice of a wider matrix)
    big = torch.zeros(M, N + 32, device=cuda)
    gemm(a, w, out=big[:, :N], trans_b=True)
    assert float((big[:, :N] - _ref(a, w, False, True, None, False, None, 1.0)).abs().max()) <= \
        0.02 * float(ref2.abs().max()) + 1e-3
    assert float(big[:, N:].abs().max()) == 0.0


@pytest.mark.gpu
def test_linear_autograd_matches_torch(cuda):
    from euler_amd.ops.gnn_ops import linear

    x = torch.randn(5000, 128, device=cuda, requires_grad=True)
    w = torch.randn(96, 128, device=cuda, requires_grad=True)
    y = linear(x, w)
    gy = torch.randn_like(y)
    (y * gy).sum().backward()
    x2, w2 = x.detach().clone().requires_grad_(True), w.detach().clone().requires_grad_(True)
    ((x2 @ w2.t()) * gy).sum().backward()
    for p, q in ((y, x2 @ w2.t()), (x.grad, x2.grad), (w.grad, w2.grad)):
        assert float((p - q).abs().max()) <= 0.02 * float(q.abs().max()) + 1e-3
