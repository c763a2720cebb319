"""Fused R-GCN + TransE step (models/rgcn_kg_step.py; BASELINE config 5, reference
examples/rgcn/rgcn.py:30-105 + examples/TransX/transX.py:63-145) against the plain fp32
torch composition of the same model on the same drawn batch, and the gemm addend epilogue
it relies on."""
import copy

import pytest
import torch

from euler_amd.dataset.synthetic import lattice_kg
from euler_amd.models.rgcn_kg_step import RgcnTransE, RgcnTransEStep
from euler_amd.ops import gnn_ops
from euler_amd.parallel.flat import FlatOptimizer, FlatParams


def test_autograd_model_cpu_trains():
    (src, rel, dst), _ = lattice_kg(300, 12, 3000, 10, seed=1)
    torch.manual_seed(0)
    m = RgcnTransE(300, 12, 16, layers=1, margin=1.0)
    opt = torch.optim.Adam(m.parameters(), lr=0.01)
    ei = torch.stack([dst, src])
    losses = []
    for _ in range(20):
        idx = torch.randint(0, src.numel(), (128,))
        negs = torch.randint(0, 300, (128, 4))
        loss = m(ei, rel, src[idx], rel[idx], dst[idx], negs)
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(float(loss))
    assert losses[-1] < losses[0]


def _setup(dev, layers, D=64, num_ent=640, num_rel=24, B=256, K=4, seed=2, bases=0, drop=0.0, det=None):
    (src, rel, dst), _ = lattice_kg(num_ent, num_rel, 8000, 10, seed=seed)
    src, rel, dst = src.to(dev), rel.to(dev), dst.to(dev)
    torch.manual_seed(seed)
    m = RgcnTransE(num_ent, num_rel, D, layers=layers, margin=1.0, num_bases=bases).to(dev)
    ei = torch.stack([dst, src])
    m(ei, rel, src[:8], rel[:8], dst[:8], torch.zeros(8, K, dtype=torch.long, device=dev)).backward()
    m.self_drop = drop
    flat = FlatParams(m.parameters(), dev)
    opt = FlatOptimizer(flat, "adam", 1e-3)
    pool = torch.arange(src.numel(), device=dev)
    step = RgcnTransEStep(m, flat, opt, ei, rel, (src, rel, dst), pool, B, K, seed=11, deterministic=det)
    return m, flat, opt, step, ei, rel


def _oracle_loss(ref, ei, erel, batch, keeps):
    """RgcnTransE.forward with the fused step's keep masks in place of torch.rand"""
    import torch.nn.functional as F

    s, r, d, negs = batch
    n = ref.ent.shape[0]
    h = ref.ent
    for i, conv in enumerate(ref.convs):
        x0 = h if keeps is None else h * keeps[i].view(n, 1)
        h = conv([x0, h], ei, (n, n), edge_attr=erel)
        if i + 1 < len(ref.convs):
            h = F.relu(h)
    pos, neg = gnn_ops.kg_score(h.float(), ref.rel, s, d, r, negs, "l2", "both", ref.norm)
    return F.relu(ref.margin + neg.mean(-1) - pos).mean()


@pytest.mark.gpu
@pytest.mark.parametrize("layers,bases,drop", [(0, 0, 0.0), (1, 0, 0.0), (2, 0, 0.0), (1, 4, 0.0), (1, 0, 0.5),
                                               (2, 4, 0.5)])
def test_fused_step_matches_fp32_torch(cuda, layers, bases, drop):
    m, flat, opt, step, ei, erel = _setup(cuda, layers, bases=bases, drop=drop)
    loss = float(step.forward_backward()[0])
    g_fused = [p.grad.detach().float().cpu().clone() for p in flat.params]
    s, r, d, n = (t.cpu() for t in step.batch())
    assert int(s.min()) >= 0 and int(n.max()) < m.ent.shape[0] and int(r.max()) < m.rel.shape[0]
    keeps = None
    if drop > 0:
        keeps = [k.cpu().clone() for k in step.keep_masks()]
        frac = float(torch.cat(keeps).mean())
        assert 0.4 < frac < 0.6 and set(torch.cat(keeps).unique().tolist()) <= {0.0, 1.0}
    ref = copy.deepcopy(m).cpu()
    for p in ref.parameters():
        p.grad = None
    ref_loss = _oracle_loss(ref, ei.cpu(), erel.cpu(), (s, r, d, n), keeps)
    ref_loss.backward()
    errs = {}
    for (name, p), gf in zip(ref.named_parameters(), g_fused):
        gr = p.grad.float()
        errs[name] = float((gf - gr).norm() / gr.norm().clamp(min=1e-12))
    print("loss", loss, float(ref_loss), "relative gradient errors", errs)
    # bf16 operands (messages, relation-transformed rows, MFMA inputs) against fp32 torch;
    # bounds per parameter from MI355X runs (profiles/r5_zoo/kg_step_fp32_oracle.log):
    # <= 1 layer every gradient 0.3-0.5 % (bound 1 %); with 2 layers the first layer's
    # and the entity table's gradients pass through two bf16 message hops, 2.8-3.6 %
    # (bound 5 %), the rest 0.3-0.5 % (bound 1 %); the loss agrees to 3e-5 (bound 1e-4)
    assert abs(loss - float(ref_loss)) <= 1e-4 * abs(float(ref_loss)) + 1e-5
    deep = layers >= 2
    for name, err in errs.items():
        bound = 5e-2 if deep and (name == "ent" or name.startswith("convs.0.")) else 1e-2
        if layers == 0:
            bound = 1e-5  # no message passing: the scores are the only bf16-free path
        assert err < bound, (name, err, bound)
    # same optimizer step count -> same draws; after the update -> new draws
    before = [t.clone() for t in step.batch()]
    step.forward_backward()
    assert all(torch.equal(a, b) for a, b in zip(before, step.batch()))
    step.optimizer_step()
    step.forward_backward()
    assert not torch.equal(before[3], step.batch()[3])


def test_deterministic_dw_slots_cpu():
    """rel_gemm_dw slot layout: solo chunks -1, each multi-chunk relation's chunks take
    consecutive slots (chunk order), the CSR over the multi-chunk relations covers them"""
    g = torch.Generator().manual_seed(0)
    E = 5000
    rel = torch.cat([torch.zeros(3000, dtype=torch.long), torch.randint(1, 6, (E - 3000,), generator=g)])
    ei = torch.randint(0, 300, (2, E), generator=g)
    t = gnn_ops.RelationTiles(ei, rel, (300, 300), 6, tile=64)
    slot, mrel, mrp, n = t.det_slots()
    cr, solo = t.chunk_rel.long(), t.chunk_solo.bool()
    assert n == int((~solo).sum()) and n >= 3  # relation 0: 3000 edges -> 3 chunks of 1024
    assert (slot[solo] == -1).all() and torch.equal(slot[~solo].long(), torch.arange(n))
    assert mrel.tolist() == sorted(set(cr[~solo].tolist())) and mrel[0] == 0
    for i, r in enumerate(mrel.tolist()):
        assert torch.equal(slot[cr == r].long(), torch.arange(int(mrp[i]), int(mrp[i + 1])))


@pytest.mark.gpu
@pytest.mark.parametrize("layers,bases,num_rel", [(0, 0, 24), (1, 0, 24), (1, 0, 4), (2, 4, 4), (1, 4, 3)])
def test_deterministic_step_matches_atomic_step(cuda, layers, bases, num_rel):
    """the atomic-free step (occurrence rows + fixed-order sums, per-chunk dW slabs) computes
    the same loss and gradients as the atomic step on the same draws, to fp32 summation order;
    with 3-4 relations over 8000 edges every relation spans several dW chunks (slot mode)"""
    grads, losses = {}, {}
    for det in (False, True):
        m, flat, opt, step, ei, erel = _setup(cuda, layers, num_rel=num_rel, bases=bases, det=det)
        losses[det] = float(step.forward_backward()[0])
        grads[det] = flat.grad.detach().clone()
        if det and layers:
            assert step.layers[0][2].det_slots()[3] > (0 if num_rel <= 4 else -1)
    assert losses[True] == losses[False]  # the forward and its loss reduction are order-fixed
    err = float((grads[True] - grads[False]).norm() / grads[False].norm())
    print("deterministic vs atomic relative gradient difference", err)
    assert err <= 1e-5


@pytest.mark.gpu
def test_deterministic_step_2000_replays_bit_identical(cuda):
    """two runs of 2 eager steps + 2,000 captured replays of the deterministic step (2
    layers, basis relations, multi-chunk relations) end with bit-identical parameters,
    optimizer state and loss"""
    out = []
    for _ in range(2):
        m, flat, opt, step, ei, erel = _setup(cuda, 2, num_rel=4, bases=2, det=True)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                step.step()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            step.step()
        for _ in range(2000):
            g.replay()
        torch.cuda.synchronize()
        assert int(opt.step_count.item()) == 2002 and bool(torch.isfinite(flat.flat).all())
        out.append((flat.flat.detach().clone(), [opt.m.clone(), opt.v.clone()],
                    step.loss.detach().clone()))
        del g
    (a, sa, la), (b, sb, lb) = out
    assert torch.equal(a, b) and torch.equal(la, lb)
    assert all(torch.equal(x, y) for x, y in zip(sa, sb))


@pytest.mark.gpu
def test_fused_step_captures_and_trains(cuda):
    m, flat, opt, step, ei, erel = _setup(cuda, 1)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            step.step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    first = float(step.loss[0])
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        step.step()
    for _ in range(60):
        g.replay()
    torch.cuda.synchronize()
    assert int(opt.step_count.item()) == 62  # 2 eager steps + 60 replays (capture runs nothing)
    last = float(step.loss[0])
    assert last == last and last < first


@pytest.mark.gpu
def test_gemm_addend_epilogue(cuda):
    torch.manual_seed(0)
    a = torch.randn(300, 96, device=cuda)
    b = torch.randn(80, 96, device=cuda)
    add = torch.randn(300, 80, device=cuda).to(torch.bfloat16)
    rm = torch.randn(300, 80, device=cuda)
    out = gnn_ops.gemm(a, b, trans_b=True, addend=add, rmask=rm)
    ref = (a.bfloat16().float() @ b.bfloat16().float().t() + add.float()) * (rm > 0).float()
    assert torch.allclose(out, ref, atol=2e-2, rtol=1e-2)
    # split-K transposed product with an fp32 addend aliasing the output
    g = torch.randn(4096, 64, device=cuda)
    x = torch.randn(4096, 64, device=cuda)
    c = torch.randn(64, 64, device=cuda)
    c0 = c.clone()
    gnn_ops.gemm(g, x, out=c, trans_a=True, splits=8, addend=c)
    ref = g.bfloat16().float().t() @ x.bfloat16().float() + c0
    assert torch.allclose(c, ref, atol=0.5, rtol=2e-2)
