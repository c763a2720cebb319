"""Numerics of the fused GAT / R-GCN / skip-gram / KG-score / unique kernels against plain
PyTorch fp32 references of the same ops (euler_amd/ops/gnn_ops.py)."""
import pytest
import torch

from euler_amd.ops import gnn_ops as G


def _graph(n_dst, n_src, E, device, seed=0, pad=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    dst = torch.randint(0, n_dst, (E,), generator=g)
    src = torch.randint(0, n_src, (E,), generator=g)
    if pad:
        dst[:pad] = -1
        src[pad:2 * pad] = -1
    return torch.stack([dst, src]).to(device)


# ----------------------------------------------------------------------------- CPU (reference semantics)
def test_unique_first_cpu_order():
    x = torch.tensor([5, 3, 5, 9, 3, 1, 9, 7])
    u, inv = G.unique_first(x)
    assert u.tolist() == [5, 3, 9, 1, 7]
    assert torch.equal(u[inv], x)


def test_gat_reference_matches_composed_convs():
    from euler_amd.ops import mp_ops

    torch.manual_seed(0)
    ei = _graph(30, 50, 400, "cpu")
    H, C = 4, 8
    h = torch.randn(50, H, C)
    al, ar = torch.randn(50, H), torch.randn(30, H)
    out = G.gat_aggregate(h, al, ar, ei, (30, 50), 0.2)
    logit = torch.nn.functional.leaky_relu(al[ei[1]] + ar[ei[0]], 0.2)
    alpha = mp_ops.scatter_softmax(logit, ei[0], 30)
    ref = mp_ops.scatter_add((h[ei[1]] * alpha.unsqueeze(-1)).reshape(-1, H * C), ei[0], 30).view(30, H, C)
    torch.testing.assert_close(out, ref, atol=1e-5, rtol=1e-5)


def test_relation_reference_matches_loop():
    torch.manual_seed(1)
    ei = _graph(20, 40, 300, "cpu")
    rel = torch.randint(0, 5, (300,))
    x, W = torch.randn(40, 12), torch.randn(5, 6, 12)
    out = G.relation_transform(x, rel, W, ei, (20, 40), "mean")
    ref = torch.zeros(20, 6)
    cnt = torch.zeros(20)
    for e in range(300):
        ref[ei[0, e]] += W[rel[e]] @ x[ei[1, e]]
        cnt[ei[0, e]] += 1
    torch.testing.assert_close(out, ref / cnt.clamp(min=1).unsqueeze(1), atol=1e-4, rtol=1e-4)


def test_xent_matches_cross_entropy():
    torch.manual_seed(3)
    logits = torch.randn(500, 47, requires_grad=True)
    y = torch.randint(0, 47, (500,))
    l1 = G.xent(logits, y)
    l1.backward()
    g1 = logits.grad.clone()
    logits.grad = None
    l2 = torch.nn.functional.cross_entropy(logits, y)
    l2.backward()
    torch.testing.assert_close(l1, l2)
    torch.testing.assert_close(g1, logits.grad)


def test_kg_reference_shapes():
    ent, rel = torch.randn(50, 16), torch.randn(7, 16)
    src, dst, r = torch.randint(0, 50, (8,)), torch.randint(0, 50, (8,)), torch.randint(0, 7, (8,))
    neg = torch.randint(0, 50, (8, 3))
    p, n = G.kg_score(ent, rel, src, dst, r, neg, "l1", "both")
    assert p.shape == (8,) and n.shape == (8, 6)
    p, n = G.kg_score(ent, rel, src, dst, r, neg, "distmult", "tail")
    assert n.shape == (8, 3)


# ----------------------------------------------------------------------------- GPU kernels
@pytest.mark.gpu
@pytest.mark.parametrize("H,C,dtype", [(8, 16, torch.bfloat16), (1, 32, torch.float32), (4, 64, torch.bfloat16),
                                       (8, 8, torch.float32), (2, 256, torch.bfloat16)])
def test_gat_fused_matches_reference(cuda, H, C, dtype):
    torch.manual_seed(2)
    n_dst, n_src, E = 700, 1500, 9000
    ei = _graph(n_dst, n_src, E, cuda, seed=3, pad=20)
    h = torch.randn(n_src, H, C, device=cuda).to(dtype).requires_grad_(True)
    al = torch.randn(n_src, H, device=cuda).requires_grad_(True)
    ar = torch.randn(n_dst, H, device=cuda).requires_grad_(True)
    out = G.gat_aggregate(h, al, ar, ei, (n_dst, n_src), 0.2)
    g = torch.randn(out.shape, device=cuda)
    (out.float() * g).sum().backward()
    h2 = h.detach().float().requires_grad_(True)
    al2, ar2 = al.detach().clone().requires_grad_(True), ar.detach().clone().requires_grad_(True)
    ref = G.gat_aggregate_reference(h2, al2, ar2, ei, (n_dst, n_src), 0.2)
    (ref * g).sum().backward()
    tol = dict(atol=3e-2, rtol=3e-2) if dtype == torch.bfloat16 else dict(atol=2e-4, rtol=2e-4)
    torch.testing.assert_close(out.float(), ref, **tol)
    torch.testing.assert_close(h.grad.float(), h2.grad, **tol)
    if dtype == torch.bfloat16:
        # the upstream gradient is rounded to bf16 before the <dout, h_j> dot products:
        # its error grows like sqrt(C)
        tol = dict(atol=3e-2 * max(1.0, (C / 64) ** 0.5), rtol=3e-2)
    torch.testing.assert_close(al.grad, al2.grad, **tol)
    torch.testing.assert_close(ar.grad, ar2.grad, **tol)


@pytest.mark.gpu
def test_gat_composed_mp_ops_grads_match_torch(cuda):
    """The composed GAT of benchmarks/bench_gat.py (--impl composed: mp_ops gather,
    scatter_softmax and scatter_add kernels under autograd) against index ops + a
    per-destination softmax in plain fp32 torch: forward and every input gradient."""
    from euler_amd.ops import mp_ops

    torch.manual_seed(14)
    N, E, H, C = 900, 12000, 4, 8
    ei = _graph(N, N, E, cuda, seed=15)
    ei = ei[:, torch.argsort(ei[0])]  # destination-sorted like EdgeCSR.edge_index
    z = torch.randn(N, H, C, device=cuda, requires_grad=True)
    a_s = (torch.randn(H, C, device=cuda) * 0.3).requires_grad_(True)
    a_d = (torch.randn(H, C, device=cuda) * 0.3).requires_grad_(True)
    seg = mp_ops.SegmentIndex(ei[0].long(), N)

    def composed(z, a_s, a_d):
        al, ar = (z * a_s).sum(-1), (z * a_d).sum(-1)
        logit = torch.nn.functional.leaky_relu(mp_ops.gather(ar, ei[0]) + mp_ops.gather(al, ei[1]), 0.2)
        alpha = mp_ops.scatter_softmax(logit, seg, N)
        msg = mp_ops.gather(z.reshape(-1, H * C), ei[1]).view(-1, H, C) * alpha.unsqueeze(-1)
        return mp_ops.scatter_add(msg.reshape(-1, H * C), seg, N).view(-1, H, C)

    def plain(z, a_s, a_d):
        al, ar = (z * a_s).sum(-1), (z * a_d).sum(-1)
        d, s = ei[0].long(), ei[1].long()
        logit = torch.nn.functional.leaky_relu(ar[d] + al[s], 0.2)
        mx = torch.full((N, H), -1e30, device=cuda).scatter_reduce(0, d.unsqueeze(1).expand(-1, H), logit, "amax")
        ex = torch.exp(logit - mx[d])
        den = torch.zeros(N, H, device=cuda).index_add(0, d, ex)
        alpha = ex / den[d]
        return torch.zeros(N, H, C, device=cuda).index_add(0, d, z[s] * alpha.unsqueeze(-1))

    g = torch.randn(N, H, C, device=cuda)
    out = composed(z, a_s, a_d)
    (out * g).sum().backward()
    grads = [t.grad.clone() for t in (z, a_s, a_d)]
    z2, s2, d2 = (t.detach().clone().requires_grad_(True) for t in (z, a_s, a_d))
    ref = plain(z2, s2, d2)
    (ref * g).sum().backward()
    torch.testing.assert_close(out, ref, atol=1e-4, rtol=1e-4)
    for a, b in zip(grads, (z2.grad, s2.grad, d2.grad)):
        torch.testing.assert_close(a, b, atol=1e-3, rtol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("H,C,dtype", [(8, 16, torch.bfloat16), (4, 8, torch.float32)])
def test_gat_conv_full_graph(cuda, H, C, dtype):
    torch.manual_seed(12)
    N, E = 2000, 30000
    ei = _graph(N, N, E, cuda, seed=13)
    csr = G.EdgeCSR(ei, (N, N))
    z = torch.randn(N, H, C, device=cuda).to(dtype).requires_grad_(True)
    a_s = (torch.randn(H, C, device=cuda) * 0.3).requires_grad_(True)
    a_d = (torch.randn(H, C, device=cuda) * 0.3).requires_grad_(True)
    out = G.gat_conv(z, a_s, a_d, csr, 0.2)
    g = torch.randn(out.shape, device=cuda)
    (out.float() * g).sum().backward()
    z2 = z.detach().float().requires_grad_(True)
    as2, ad2 = a_s.detach().clone().requires_grad_(True), a_d.detach().clone().requires_grad_(True)
    ref = G.gat_conv_reference(z2, as2, ad2, ei, (N, N), 0.2)
    (ref * g).sum().backward()
    tol = dict(atol=4e-2, rtol=4e-2) if dtype == torch.bfloat16 else dict(atol=3e-4, rtol=3e-4)
    torch.testing.assert_close(out.float(), ref, **tol)
    torch.testing.assert_close(z.grad.float(), z2.grad, **tol)
    scale = float(as2.grad.abs().max())
    torch.testing.assert_close(a_s.grad, as2.grad, atol=2e-2 * scale, rtol=3e-2)
    torch.testing.assert_close(a_d.grad, ad2.grad, atol=2e-2 * float(ad2.grad.abs().max()), rtol=3e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("H,C,dtype", [(8, 16, torch.bfloat16), (4, 8, torch.float32), (2, 64, torch.bfloat16)])
def test_gat_recomputed_al_matches_gathered(cuda, H, C, dtype):
    """The edge kernels given a_src recompute al = <z_j, a_src> from the gathered row; the
    result must match the path that gathers the precomputed al (same partial order)."""
    from euler_amd.ops._native import hip

    torch.manual_seed(15)
    N, E = 3000, 40000
    ei = _graph(N, N, E, cuda, seed=16)
    csr = G.EdgeCSR(ei, (N, N))
    z = torch.randn(N, H * C, device=cuda).to(dtype)
    a_s = torch.randn(H, C, device=cuda) * 0.3
    a_d = torch.randn(H, C, device=cuda) * 0.3
    al, ar = hip().gat_att_fwd(z, a_s, a_d, H, C)
    indptr, col = csr.csr()
    cindptr, crow = csr.csc()
    o1, l1 = hip().gat_fwd(indptr, col, csr.csr_order(), z, al, ar, H, C, 0.2)
    o2, l2 = hip().gat_fwd(indptr, col, csr.csr_order(), z, al, ar, H, C, 0.2, a_s)
    torch.testing.assert_close(o2.float(), o1.float(), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(l2, l1, atol=1e-5, rtol=1e-5)
    dout = torch.randn_like(o1)
    r1 = hip().gat_bwd(indptr, col, csr.csr_order(), cindptr, crow, csr.csc_order(), z, al, ar, H, C, 0.2, o1,
                       dout, l1)
    r2 = hip().gat_bwd(indptr, col, csr.csr_order(), cindptr, crow, csr.csc_order(), z, al, ar, H, C, 0.2, o1,
                       dout, l1, a_s)
    for a, b in zip(r2, r1):
        torch.testing.assert_close(a.float(), b.float(), atol=1e-4, rtol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("bias", [False, True])
def test_tall_linear_grads(cuda, bias):
    torch.manual_seed(14)
    x = torch.randn(70001, 96, device=cuda).requires_grad_(True)   # 70001: a remainder chunk
    w = torch.randn(47, 96, device=cuda).requires_grad_(True)
    b = torch.randn(47, device=cuda).requires_grad_(True) if bias else None
    y = G.tall_linear(x, w, b, chunk=4096)
    g = torch.randn_like(y)
    (y * g).sum().backward()
    x2, w2 = x.detach().clone().requires_grad_(True), w.detach().clone().requires_grad_(True)
    b2 = b.detach().clone().requires_grad_(True) if bias else None
    y2 = x2 @ w2.t() + (b2 if bias else 0)
    (y2 * g).sum().backward()
    torch.testing.assert_close(y, y2, atol=1e-3, rtol=1e-3)
    torch.testing.assert_close(w.grad, w2.grad, atol=5e-2, rtol=1e-3)
    torch.testing.assert_close(x.grad, x2.grad, atol=1e-3, rtol=1e-3)
    if bias:
        torch.testing.assert_close(b.grad, b2.grad, atol=5e-2, rtol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("K,N,aggr,R", [(100, 100, "mean", 13), (128, 64, "add", 13), (32, 200, "mean", 13),
                                         (128, 128, "mean", 3), (128, 96, "mean", 13), (320, 320, "mean", 13)])  # R = 3: multi-chunk relations (atomic dW)
def test_relation_transform_matches_reference(cuda, K, N, aggr, R):
    torch.manual_seed(4)
    n_dst, n_src, E = 400, 900, 7000
    ei = _graph(n_dst, n_src, E, cuda, seed=5, pad=10)
    rel = torch.randint(0, R, (E,), device=cuda)
    x = (torch.randn(n_src, K, device=cuda) * 0.5).requires_grad_(True)
    W = (torch.randn(R, N, K, device=cuda) * 0.1).requires_grad_(True)
    out = G.relation_transform(x, rel, W, ei, (n_dst, n_src), aggr)
    g = torch.randn(out.shape, device=cuda)
    (out * g).sum().backward()
    x2 = x.detach().to(torch.bfloat16).float().requires_grad_(True)
    W2 = W.detach().to(torch.bfloat16).float().requires_grad_(True)
    ref = G.relation_transform_reference(x2, rel, W2, ei, (n_dst, n_src), aggr)
    (ref * g).sum().backward()
    torch.testing.assert_close(out, ref, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(x.grad, x2.grad, atol=3e-2, rtol=3e-2)
    # dW sums ~E/R bf16-rounded products: bound the error relative to its magnitude
    torch.testing.assert_close(W.grad, W2.grad, atol=1e-2 * float(W2.grad.abs().max()), rtol=3e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("R", [13, 3])  # 3: multi-chunk relations (atomic partials)
def test_relation_dw_grad_sink_accumulates(cuda, R):
    """enable_grad_sink: dW accumulates into the weight's existing .grad (solo chunks add
    to their slab, shared ones use atomics) and equals grad + the autograd dW."""
    torch.manual_seed(5)
    n_dst, n_src, E, K, N = 300, 700, 6000, 128, 128
    ei = _graph(n_dst, n_src, E, cuda, seed=6, pad=10)
    rel = torch.randint(0, R, (E,), device=cuda)
    x = torch.randn(n_src, K, device=cuda) * 0.5
    W = torch.nn.Parameter(torch.randn(R, N, K, device=cuda) * 0.1)
    g = torch.randn(n_dst, N, device=cuda)
    (G.relation_transform(x, rel, W, ei, (n_dst, n_src), "mean") * g).sum().backward()
    plain = W.grad.clone()
    base = torch.randn_like(W) * 0.01
    W.grad = base.clone()
    G.enable_grad_sink(W)
    (G.relation_transform(x, rel, W, ei, (n_dst, n_src), "mean") * g).sum().backward()
    torch.testing.assert_close(W.grad, base + plain, atol=1e-4 * float(plain.abs().max()), rtol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("D,dtype", [(128, torch.bfloat16), (32, torch.float32), (100, torch.float32)])
def test_sgns_matches_reference(cuda, D, dtype):
    torch.manual_seed(6)
    B, P, K = 333, 2, 5
    emb = (torch.randn(B, D, device=cuda) * 0.3).to(dtype).requires_grad_(True)
    pos = (torch.randn(B, P, D, device=cuda) * 0.3).to(dtype).requires_grad_(True)
    neg = (torch.randn(B, K, D, device=cuda) * 0.3).to(dtype).requires_grad_(True)
    loss, lp, ln = G.sgns_loss(emb, pos, neg)
    (loss * 3.0).backward()
    e2, p2, n2 = (t.detach().float().requires_grad_(True) for t in (emb, pos, neg))
    ref, rlp, rln = G.sgns_loss_reference(e2, p2, n2)
    (ref * 3.0).backward()
    tol = dict(atol=2e-2, rtol=2e-2) if dtype == torch.bfloat16 else dict(atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(loss, ref, **tol)
    torch.testing.assert_close(lp, rlp.detach(), **tol)
    torch.testing.assert_close(ln, rln.detach(), **tol)
    for a, b in ((emb, e2), (pos, p2), (neg, n2)):
        torch.testing.assert_close(a.grad.float(), b.grad, **tol)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,corrupt,normalize,D,Ne", [("l1", "both", True, 100, 500), ("l2", "front", True, 100, 500),
                                                          ("distmult", "tail", True, 100, 500),
                                                          ("l2", "both", False, 100, 500),
                                                          # D / 4 a power of two: occurrence rows + segment sums
                                                          # (Ne = 40: hot rows shared by many triples)
                                                          ("l1", "both", True, 128, 40), ("l2", "tail", True, 64, 500)])
@pytest.mark.parametrize("occ", [False, True])
def test_kg_score_matches_reference(cuda, kind, corrupt, normalize, D, Ne, occ, monkeypatch):
    # occ: per-occurrence gradient rows + segment sums instead of atomics (EULER_AMD_KG_OCC)
    monkeypatch.setattr(G, "_KG_OCC", occ)
    torch.manual_seed(7)
    Nr, B, K = 20, 128, 4
    ent = torch.randn(Ne, D, device=cuda).requires_grad_(True)
    rel = torch.randn(Nr, D, device=cuda).requires_grad_(True)
    src, dst = torch.randint(0, Ne, (B,), device=cuda), torch.randint(0, Ne, (B,), device=cuda)
    r = torch.randint(0, Nr, (B,), device=cuda)
    neg = torch.randint(0, Ne, (B, K), device=cuda)
    ps, ns = G.kg_score(ent, rel, src, dst, r, neg, kind, corrupt, normalize)
    gp, gn = torch.randn_like(ps), torch.randn_like(ns)
    ((ps * gp).sum() + (ns * gn).sum()).backward()
    ent2, rel2 = ent.detach().clone().requires_grad_(True), rel.detach().clone().requires_grad_(True)
    rp, rn = G.kg_score_reference(ent2, rel2, src, dst, r, neg, kind, corrupt, normalize)
    ((rp * gp).sum() + (rn * gn).sum()).backward()
    torch.testing.assert_close(ps, rp, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(ns, rn, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(ent.grad, ent2.grad, atol=1e-4, rtol=1e-3)
    torch.testing.assert_close(rel.grad, rel2.grad, atol=1e-4, rtol=1e-3)


def test_unique_first_padded_skips_padding_cpu():
    x = torch.tensor([5, -1, 3, 5, -1, -1, 9, 3])
    u, inv, cnt = G.unique_first_padded(x)
    assert u.tolist() == [5, 3, 9, -1, -1, -1, -1, -1] and int(cnt) == 3
    assert inv.tolist() == [0, -1, 1, 0, -1, -1, 2, 1]
    u, inv2, _ = G.unique_first_padded(x, offset=100)  # distinct values shifted, fill kept
    assert u.tolist() == [105, 103, 109, -1, -1, -1, -1, -1] and torch.equal(inv2, inv)


@pytest.mark.gpu
def test_unique_first_padded_gpu_matches_cpu(cuda):
    """padding ids (< 0, many copies) are not keys on the GPU either: same uniq / inverse /
    count as the CPU composition"""
    torch.manual_seed(9)
    x = torch.randint(0, 3000, (50000,))
    x[torch.rand(50000) < 0.3] = -1
    u_c, i_c, n_c = G.unique_first_padded(x)
    u_g, i_g, n_g = G.unique_first_padded(x.to(cuda))
    assert torch.equal(u_g.cpu(), u_c) and torch.equal(i_g.cpu(), i_c) and int(n_g) == int(n_c)
    u_o, i_o, _ = G.unique_first_padded(x.to(cuda), offset=7001)
    assert torch.equal(u_o.cpu(), torch.where(u_c >= 0, u_c + 7001, u_c)) and torch.equal(i_o.cpu(), i_c)


@pytest.mark.gpu
def test_unique_first_gpu_matches_cpu(cuda):
    torch.manual_seed(8)
    x = torch.randint(0, 5000, (20000,))
    u_c, inv_c = G.unique_first(x)
    u_g, inv_g = G.unique_first(x.to(cuda))
    assert torch.equal(u_g.cpu(), u_c)
    assert torch.equal(inv_g.cpu(), inv_c)
    e_u, _ = G.unique_first(torch.empty(0, dtype=torch.long, device=cuda))
    assert e_u.numel() == 0


@pytest.mark.gpu
def test_gat_conv_uses_fused_kernel(cuda):
    from euler_amd.convolution import MultiHeadGATConv

    torch.manual_seed(9)
    conv = MultiHeadGATConv(64, heads=8).to(cuda)
    x = torch.randn(300, 32, device=cuda)
    ei = _graph(100, 300, 2000, cuda, seed=10)
    out = conv([x[:100], x], ei, (100, 300))
    out.sum().backward()
    assert out.shape == (100, 64)
    cache = ei._euler_cache
    assert any(k.startswith("_euler_csr") for k in cache), "fused GAT path not taken"


@pytest.mark.gpu
@pytest.mark.parametrize("combiner", ["sum", "mean"])
def test_embedding_bag_matches_reference(cuda, combiner):
    from euler_amd.ops import mp_ops

    torch.manual_seed(15)
    table = torch.randn(1000, 64, device=cuda).requires_grad_(True)
    bag_of = torch.sort(torch.randint(0, 300, (5000,), device=cuda))[0]
    ids = torch.randint(0, 1000, (5000,), device=cuda)
    w = torch.rand(5000, device=cuda)
    out = mp_ops.embedding_bag(table, ids, bag_of, 310, combiner, w)
    g = torch.randn_like(out)
    (out * g).sum().backward()
    t2 = table.detach().clone().requires_grad_(True)
    ww = w / torch.bincount(bag_of, minlength=310).clamp(min=1)[bag_of] if combiner == "mean" else w
    ref = torch.zeros(310, 64, device=cuda).index_add(0, bag_of, t2[ids] * ww.unsqueeze(1))
    (ref * g).sum().backward()
    torch.testing.assert_close(out, ref, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(table.grad, t2.grad, atol=1e-4, rtol=1e-4)


@pytest.mark.gpu
def test_deepwalk_step_gpu(cuda):
    from euler_amd.graph.device_graph import DeviceGraph
    from euler_amd.models.deepwalk_step import DeepWalkTrainer

    g = DeviceGraph.synthetic(20000, 8.0, 64, seed=2, device=cuda)
    tr = DeepWalkTrainer(g, 20000, dim=64, batch_size=512, lr=0.05, optimizer="adam", seed=1)
    losses = [float(tr.step()) for _ in range(40)]
    assert all(l == l for l in losses)
    assert sum(losses[-5:]) < sum(losses[:5])
    assert int(tr.table.step.item()) == 40  # one optimizer step per training step (Adam bias correction)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,D", [(torch.float32, 48), (torch.bfloat16, 64), (torch.float32, 7)])
def test_weighted_aggregate_spmm(cuda, dtype, D):
    from euler_amd.ops import mp_ops

    torch.manual_seed(16)
    n_dst, n_src, E = 300, 800, 6000
    ei = _graph(n_dst, n_src, E, cuda, seed=17, pad=15)
    x = torch.randn(n_src, D, device=cuda).to(dtype).requires_grad_(True)
    w = torch.rand(E, device=cuda)
    out = mp_ops.weighted_aggregate(x, ei, (n_dst, n_src), w)
    g = torch.randn(out.shape, device=cuda)
    (out.float() * g).sum().backward()
    x2 = x.detach().float().requires_grad_(True)
    keep = (ei[0] >= 0) & (ei[1] >= 0)
    ref = torch.zeros(n_dst, D, device=cuda).index_add(0, ei[0][keep], x2[ei[1][keep]] * w[keep].unsqueeze(1))
    (ref * g).sum().backward()
    tol = dict(atol=3e-2, rtol=3e-2) if dtype == torch.bfloat16 else dict(atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(out.float(), ref, **tol)
    torch.testing.assert_close(x.grad.float(), x2.grad, **tol)


# ----------------------------------------------------------------------------- index-driven SGNS
def _sgns_case(device, P=300, K=5, D=32, n_t=40, n_c=120, seed=21):
    g = torch.Generator().manual_seed(seed)
    T = torch.randn(n_t + 7, D, generator=g).to(device)
    C = torch.randn(n_c + 9, D, generator=g).to(device)
    src = torch.randint(0, n_t, (P,), generator=g).to(device)
    ctx = torch.randint(0, n_c, (P * (1 + K),), generator=g).to(device)
    return T, C, src, ctx


def _sgns_autograd(T, C, src, ctx, K):
    P = src.numel()
    Tg = T.detach().clone().requires_grad_(True)
    Cg = C.detach().clone().requires_grad_(True)
    c = Cg[ctx]
    loss, _, _ = G.sgns_loss_reference(Tg[src], c[:P].view(P, 1, -1), c[P:].view(P, K, -1))
    loss.backward()
    return loss.detach(), Tg.grad, Cg.grad


def test_sgns_idx_reference_matches_autograd():
    K = 5
    T, C, src, ctx = _sgns_case("cpu", K=K)
    P = src.numel()
    u_t, inv_t = G.unique_first(src)
    u_c, inv_c = G.unique_first(ctx)
    gscale = 1.0 / (P * (1 + K))
    coef, loss_rows = G.sgns_fwd_idx(T, u_t, inv_t, C, u_c, inv_c, K, gscale)
    ptr_t, lst_t = G.occ_csr(inv_t, u_t.numel())
    ptr_c, lst_c = G.occ_csr(inv_c, u_c.numel())
    g_t = G.sgns_grad(0, ptr_t, lst_t, coef, K, C, u_c, inv_c, inv_self=inv_t)
    g_c = G.sgns_grad(1, ptr_c, lst_c, coef, K, T, u_t, inv_t, inv_self=inv_c)
    loss, dT, dC = _sgns_autograd(T, C, src, ctx, K)
    torch.testing.assert_close(loss_rows.sum() * gscale, loss, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(g_t, dT[u_t], atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(g_c, dC[u_c], atol=1e-6, rtol=1e-5)
    # occurrence lists: every occurrence once, grouped by its unique id
    assert torch.equal(torch.sort(lst_c.long())[0], torch.arange(ctx.numel()))
    assert torch.equal(inv_c[lst_c.long()], torch.repeat_interleave(torch.arange(u_c.numel()), ptr_c.diff()))


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["adam", "adagrad", "sgd"])
def test_sgns_idx_kernels_match_cpu(cuda, kind):
    from euler_amd.parallel.sparse_table import ShardedTable

    K, D = 5, 64
    T, C, src, ctx = _sgns_case("cpu", P=2000, K=K, D=D, n_t=300, n_c=900, seed=22)
    P = src.numel()
    gscale = 1.0 / (P * (1 + K))
    u_t, inv_t = G.unique_first(src)
    u_c, inv_c = G.unique_first(ctx)
    coef, loss_rows = G.sgns_fwd_idx(T, u_t, inv_t, C, u_c, inv_c, K, gscale)
    _, dT, dC = _sgns_autograd(T, C, src, ctx, K)
    dv = [t.to(cuda) for t in (T, C, src, ctx)]
    Tg, Cg, srcg, ctxg = dv
    ug_t, ig_t = G.unique_first(srcg)
    ug_c, ig_c = G.unique_first(ctxg)
    assert torch.equal(ug_t.cpu(), u_t) and torch.equal(ig_c.cpu(), inv_c)
    coef_g, loss_g = G.sgns_fwd_idx(Tg, ug_t, ig_t, Cg, ug_c, ig_c, K, gscale)
    torch.testing.assert_close(coef_g.cpu(), coef, atol=1e-7, rtol=1e-4)
    torch.testing.assert_close(loss_g.cpu(), loss_rows, atol=1e-4, rtol=1e-5)
    ptr_t, lst_t = G.occ_csr(ig_t, ug_t.numel())
    ptr_c, lst_c = G.occ_csr(ig_c, ug_c.numel())
    assert torch.equal(torch.sort(lst_c.long())[0].cpu(), torch.arange(ctx.numel()))
    g_t = G.sgns_grad(0, ptr_t, lst_t, coef_g, K, Cg, ug_c, ig_c)
    g_c = G.sgns_grad(1, ptr_c, lst_c, coef_g, K, Tg, ug_t, ig_t)
    torch.testing.assert_close(g_t.cpu(), dT[u_t], atol=1e-7, rtol=1e-4)
    torch.testing.assert_close(g_c.cpu(), dC[u_c], atol=1e-7, rtol=1e-4)
    # fused in-place optimizer == plain optimizer on the reference gradients
    n_rows = C.shape[0]
    fused = ShardedTable(n_rows, D, cuda, optimizer=kind, lr=0.05, seed=3)
    plain = ShardedTable(n_rows, D, "cpu", optimizer=kind, lr=0.05, seed=3)
    plain.weight.copy_(fused.weight.cpu())
    for _ in range(2):
        fused.apply_sgns(1, ptr_c, lst_c, coef_g, K, Tg, ug_t, ig_t, ug_c)
        plain._update(u_c, dC[u_c])
    # Adam / Adagrad normalise each gradient element (g / (|g| + eps) on the first step), so
    # elements whose gradient cancels to ~eps amplify the 1e-4 relative gradient differences
    torch.testing.assert_close(fused.weight.cpu(), plain.weight, atol=1e-3 if kind != "sgd" else 1e-5, rtol=1e-4)
    if kind != "sgd":
        torch.testing.assert_close(fused.v.cpu(), plain.v, atol=1e-9, rtol=1e-3)
    assert int(fused.step.item()) == 2


@pytest.mark.gpu
@pytest.mark.parametrize("D,n_t,n_c,P", [
    (128, 40000, 60000, 20000),  # ids fill the chip: one lp-lane group per row (split 1)
    (128, 5000, 5000, 8000),     # split 2 inside a wave
    (32, 3000, 3000, 6000),      # 128-lane groups across two waves
    (16, 100, 300, 6000),        # block-wide groups, long occurrence lists
])
def test_sgns_grad_split_regimes_match_cpu(cuda, D, n_t, n_c, P):
    """sgns_update_kernel widens each row's lane group while the unique ids underfill the chip
    (embed.hip eh_sgns_update); every regime reduces to the CPU reference gradients."""
    K = 5
    T, C, src, ctx = _sgns_case("cpu", P=P, K=K, D=D, n_t=n_t, n_c=n_c, seed=23)
    gscale = 1.0 / (P * (1 + K))
    u_t, inv_t = G.unique_first(src)
    u_c, inv_c = G.unique_first(ctx)
    coef, _ = G.sgns_fwd_idx(T, u_t, inv_t, C, u_c, inv_c, K, gscale)
    ref_t = G.sgns_grad(0, *G.occ_csr(inv_t, u_t.numel()), coef, K, C, u_c, inv_c, inv_self=inv_t)
    ref_c = G.sgns_grad(1, *G.occ_csr(inv_c, u_c.numel()), coef, K, T, u_t, inv_t, inv_self=inv_c)
    Tg, Cg, coef_g = T.to(cuda), C.to(cuda), coef.to(cuda)
    ug_t, ig_t, ug_c, ig_c = (x.to(cuda) for x in (u_t, inv_t, u_c, inv_c))
    g_t = G.sgns_grad(0, *G.occ_csr(ig_t, ug_t.numel()), coef_g, K, Cg, ug_c, ig_c)
    g_c = G.sgns_grad(1, *G.occ_csr(ig_c, ug_c.numel()), coef_g, K, Tg, ug_t, ig_t)
    torch.testing.assert_close(g_t.cpu(), ref_t, atol=1e-7, rtol=1e-4)
    torch.testing.assert_close(g_c.cpu(), ref_c, atol=1e-7, rtol=1e-4)


@pytest.mark.gpu
def test_sgns_idx_bf16_rows_match_fp32(cuda):
    """bf16 exchanged rows (sharded-table keep_wire path): the index-driven SGNS kernels
    read bf16 rows and write bf16 gradients, the converting gather packs fp32 rows as bf16
    and the row-sparse optimizer reads bf16 gradients — each against the fp32 composition
    of the same (bf16-rounded) inputs."""
    from euler_amd.ops._native import hip

    K, D = 5, 64
    T, C, src, ctx = _sgns_case("cpu", P=2000, K=K, D=D, n_t=300, n_c=900, seed=23)
    Tb, Cb = T.bfloat16(), C.bfloat16()
    P = src.numel()
    gscale = 1.0 / (P * (1 + K))
    u_t, inv_t = G.unique_first(src)
    u_c, inv_c = G.unique_first(ctx)
    coef, loss_rows = G.sgns_fwd_idx(Tb.float(), u_t, inv_t, Cb.float(), u_c, inv_c, K, gscale)
    ptr_t, lst_t = G.occ_csr(inv_t, u_t.numel())
    g_t = G.sgns_grad(0, ptr_t, lst_t, coef, K, Cb.float(), u_c, inv_c, inv_self=inv_t)
    d = lambda *ts: [t.to(cuda) for t in ts]  # noqa: E731
    Tg, Cg, ug_t, ig_t, ug_c, ig_c = d(Tb, Cb, u_t, inv_t, u_c, inv_c)
    coef_g, loss_g = G.sgns_fwd_idx(Tg, ug_t, ig_t, Cg, ug_c, ig_c, K, gscale)
    torch.testing.assert_close(coef_g.cpu(), coef, atol=1e-7, rtol=1e-4)
    torch.testing.assert_close(loss_g.cpu(), loss_rows, atol=1e-4, rtol=1e-5)
    pg, lg = G.occ_csr(ig_t, ug_t.numel())
    out = torch.zeros(ug_t.numel(), D, dtype=torch.bfloat16, device=cuda)
    G.sgns_grad(0, pg, lg, coef_g, K, Cg, ug_c, ig_c, out=out)
    torch.testing.assert_close(out.float().cpu(), g_t, atol=1e-6, rtol=1e-2)
    # converting gather: rows (and -1 -> zeros) of an fp32 table as bf16
    x = torch.randn(500, D, device=cuda)
    idx = torch.randint(-1, 500, (777,), device=cuda)
    got = hip().gather_f32_bf16(x, idx)
    want = torch.where((idx >= 0).unsqueeze(1), x[idx.clamp(min=0)], torch.zeros_like(x[:1])).bfloat16()
    assert torch.equal(got, want)
    # row-sparse Adam from bf16 gradients == from their fp32 widening
    rows = torch.randperm(500, device=cuda)[:300]
    rows[::7] = -1  # empty exchange slots are skipped
    gb = torch.randn(300, D, device=cuda).bfloat16()
    w0 = torch.randn(500, D, device=cuda)
    res = []
    for g in (gb, gb.float()):
        w, m, v, st = w0.clone(), torch.zeros_like(w0), torch.zeros_like(w0), torch.zeros(1, dtype=torch.long,
                                                                                             device=cuda)
        hip().sparse_optim_(w, m, v, rows, g.contiguous(), st, 0.01, 0.9, 0.999, 1e-8, 0)
        res.append((w, m, v))
    for a, b in zip(*res):
        assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_splitk_linear_grads_match(cuda, dtype):
    """Dense / fused-SAGE weight gradients as split-K batched GEMMs (gnn_ops.splitk_*)
    equal the plain linear backward (fp32 reference)."""
    from euler_amd.ops.gnn_ops import splitk_linear, splitk_mm_t

    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(5632 + 37, 256, generator=g).to(cuda, dtype).requires_grad_(True)
    w = torch.randn(121, 256, generator=g).to(cuda, dtype).requires_grad_(True)
    b = torch.randn(121, generator=g).to(cuda, dtype).requires_grad_(True)
    y = splitk_linear(x, w, b)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    torch.nn.functional.linear(xr, wr, br).backward(dy.float())
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    for got, ref in ((x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        rel = (got.float() - ref).norm() / ref.norm()
        assert rel < tol, rel
    m = splitk_mm_t(dy, x.detach())
    assert m.dtype == torch.float32 and m.shape == (121, 256)
    assert ((m - dy.float().t() @ x.detach().float()).norm() / m.norm()) < tol


@pytest.mark.gpu
def test_rel_weight_bf16_shadows(cuda):
    from euler_amd.ops._native import hip
    W = torch.randn(5, 128, 192, device=cuda)
    wb, wt = hip().rel_weight_bf16(W)
    ref = W.to(torch.bfloat16)
    assert torch.equal(wb, ref)
    assert torch.equal(wt, ref.transpose(1, 2).contiguous())


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,D,op,use_perm", [(torch.bfloat16, 128, 1, False), (torch.float32, 128, 0, True),
                                                 (torch.bfloat16, 64, 0, True), (torch.float32, 16, 1, False)])
def test_segment_reduce_wave_matches_reference(cuda, dtype, D, op, use_perm):
    from euler_amd.ops._native import hip
    torch.manual_seed(7)
    S = 300
    lens = (torch.rand(S) ** 6 * 900).long()  # skewed: a few long segments, many short / empty
    lens[::37] = 0
    indptr = torch.zeros(S + 1, dtype=torch.long)
    indptr[1:] = torch.cumsum(lens, 0)
    n = int(indptr[-1])
    x = torch.randn(n, D, device=cuda).to(dtype)
    perm = torch.randperm(n, device=cuda) if use_perm else None
    out = hip().segment_reduce_wave(x, indptr.to(cuda), perm, op)
    xs = (x[perm] if use_perm else x).float().cpu()
    ref = torch.zeros(S, D)
    for s in range(S):
        a, b = int(indptr[s]), int(indptr[s + 1])
        if b > a:
            ref[s] = xs[a:b].sum(0) / (b - a if op == 1 else 1)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    torch.testing.assert_close(out.float().cpu(), ref, atol=tol * 10, rtol=tol)


@pytest.mark.gpu
def test_per_item_kernels_cover_more_than_2pow32_items(cuda):
    """A dispatch counts work-items in 32 bits: one-thread-per-item kernels over > 2^32
    items (an [E, 128] message tensor of a 50M-edge graph) run on a capped grid with a
    grid-stride loop (common.h grid_for / grid_stride) instead of silently wrapping — the
    bug behind the composed GAT's wrong gradients at 1M nodes (profiles/r3_learning/gat_ab/)."""
    from euler_amd.ops._native import hip

    E, D = (1 << 25) + (1 << 20), 128          # 4.43e9 elements (8.9 GB of bf16 ones)
    src = torch.ones(E, D, dtype=torch.bfloat16, device=cuda)
    idx = torch.div(torch.arange(E, device=cuda), 64, rounding_mode="floor")
    out = torch.zeros(E // 64, D, device=cuda)
    hip().index_add_rows_(out, idx, src)
    del src
    assert float(out.min()) == 64.0 and float(out.max()) == 64.0


@pytest.mark.gpu
def test_seg_count_skips_padding(cuda):
    """SegmentIndex.counts without the sort (csrc/hip/flow.hip seg_count) vs bincount"""
    from euler_amd.ops.mp_ops import SegmentIndex

    torch.manual_seed(0)
    idx = torch.randint(-1, 500, (200_000,), device=cuda)
    idx[:100_000] = -1  # a capacity-padded tail of padding entries
    cnt = SegmentIndex(idx, 500).counts
    ref = torch.bincount(idx[idx >= 0].cpu(), minlength=500)
    assert cnt.dtype == torch.long and torch.equal(cnt.cpu(), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("pad", [0, 300])
def test_gcn_conv_gpu_matches_cpu(cuda, pad):
    """GCNConv (degree norm from the segment counts, SpMM forward, lazy CSC backward) on the
    GPU against the CPU torch composition, with and without padding edges"""
    import copy

    from euler_amd.convolution.convs import GCNConv

    torch.manual_seed(1)
    n_dst, n_src = 200, 500
    ei = _graph(n_dst, n_src, 3000, "cpu", seed=3, pad=pad)
    conv = GCNConv(32)
    x = torch.randn(n_src, 48)
    conv((x, None), ei, (n_dst, n_src))  # materialise
    gconv = copy.deepcopy(conv).to(cuda)
    xc = x.clone().requires_grad_(True)
    xg = x.to(cuda).requires_grad_(True)
    yc = conv((xc, None), ei, (n_dst, n_src))
    yg = gconv((xg, None), ei.to(cuda), (n_dst, n_src))
    assert torch.allclose(yg.cpu(), yc, atol=2e-3, rtol=2e-3)
    w = torch.randn_like(yc)
    (yc * w).sum().backward()
    (yg * w.to(cuda)).sum().backward()
    assert torch.allclose(xg.grad.cpu(), xc.grad, atol=2e-3, rtol=2e-3)
    assert torch.allclose(gconv.fc.weight.grad.cpu(), conv.fc.weight.grad, atol=2e-2, rtol=2e-3)


@pytest.mark.gpu
def test_zero_kernel_sizes(cuda):
    """hip().zero_ (vector-store kernel; memset fallback for unaligned views) on odd sizes"""
    from euler_amd.ops._native import hip

    for n in (1, 3, 4, 5, 17, 1000, 100_003):
        t = torch.full((n + 1,), 7.0, device=cuda)
        hip().zero_(t[:n])
        assert bool((t[:n] == 0).all()) and float(t[n]) == 7.0
        u = torch.full((n + 2,), 7.0, device=cuda)
        hip().zero_(u[1:n + 1])  # 4-byte-aligned view (byte kernel)
        assert float(u[0]) == 7.0 and bool((u[1:n + 1] == 0).all()) and float(u[n + 1]) == 7.0


@pytest.mark.gpu
def test_bce_f1_loss_matches_torch(cuda):
    """fused multi-label sigmoid CE + F1 counts (embed.hip bce_f1_*) vs the torch composition"""
    import torch.nn.functional as F

    torch.manual_seed(0)
    labels = (torch.rand(700, 121, device=cuda) < 0.3).float()
    rows = torch.randint(0, 700, (512,), device=cuda)
    x = (torch.randn(512, 121, device=cuda) * 3).requires_grad_(True)
    counts = torch.zeros(3, dtype=torch.long, device=cuda)
    loss = G.bce_f1_loss(x, labels, rows, counts)
    loss.backward()
    xr = x.detach().clone().requires_grad_(True)
    y = labels[rows]
    ref = F.binary_cross_entropy_with_logits(xr, y)
    ref.backward()
    assert abs(float(loss) - float(ref)) < 1e-5 * max(1.0, abs(float(ref)))
    assert torch.allclose(x.grad, xr.grad, atol=1e-7, rtol=1e-4)
    pred, pos = xr.detach() >= 0, y > 0.5
    want = [int((pred & pos).sum()), int((pred & ~pos).sum()), int((~pred & pos).sum())]
    assert counts.tolist() == want


@pytest.mark.gpu
def test_gather_rows_odd_bf16_width(cuda):
    """gather of bf16 rows with an odd width (Cora's 1433 features: 2866-byte rows)"""
    from euler_amd.ops import mp_ops

    x = torch.randn(50, 1433, device=cuda).to(torch.bfloat16)
    idx = torch.tensor([3, -1, 49, 0, 3], device=cuda)
    out = mp_ops.gather(x, idx)
    ref = x[idx.clamp(min=0)]
    ref[1] = 0
    assert torch.equal(out, ref)
