"""Full-graph GAT (BASELINE config 3) in the product (models/gat_full.py; reference
examples/gat/gat.py:27-86).

CPU: the trainer's flat-Adam step equals torch autograd + torch.optim.Adam on the same
model; fused and composed convolutions agree.  GPU: the captured epoch equals the eager
epochs and learns a planted neighbourhood task."""
import copy

import pytest
import torch

from euler_amd.models.gat_full import FullGraphGAT, FullGraphGatTrainer, add_self_loops
from euler_amd.ops import gnn_ops


def _graph(n=300, deg=6, seed=0, device="cpu"):
    g = torch.Generator().manual_seed(seed)
    d = torch.randint(1, deg * 2, (n,), generator=g)
    indptr = torch.zeros(n + 1, dtype=torch.int64)
    indptr[1:] = torch.cumsum(d, 0)
    col = torch.randint(0, n, (int(indptr[-1]),), generator=g).to(torch.int32)
    indptr, col = add_self_loops(indptr.to(device), col.to(device))
    csr = gnn_ops.EdgeCSR.from_csr(indptr, col, n)
    x = torch.randn(n, 20, generator=g).to(device)
    # planted: class of the neighbourhood-mean projection
    w = torch.repeat_interleave(1.0 / torch.diff(indptr).float(), torch.diff(indptr))
    dst = torch.repeat_interleave(torch.arange(n, device=device), torch.diff(indptr))
    agg = torch.zeros(n, 20, device=device).index_add_(0, dst, x[col.long()] * w.unsqueeze(1))
    y = (agg @ torch.randn(20, 5, generator=g).to(device)).argmax(1)
    return x, csr, y


def test_add_self_loops_cpu():
    indptr = torch.tensor([0, 2, 2, 3])
    col = torch.tensor([1, 2, 0], dtype=torch.int32)
    ip, c = add_self_loops(indptr, col)
    assert ip.tolist() == [0, 3, 4, 6] and c.tolist() == [0, 1, 2, 1, 2, 0]


def test_trainer_step_equals_autograd_adam_cpu():
    x, csr, y = _graph()
    torch.manual_seed(0)
    m = FullGraphGAT(20, 4, 8, 5, 2)
    ref = copy.deepcopy(m)
    idx = torch.arange(0, 300, 3)
    tr = FullGraphGatTrainer(m, x, csr, y, idx, "adam", 0.01)
    opt = torch.optim.Adam(ref.parameters(), lr=0.01)
    for _ in range(4):
        loss = float(tr.step())
        lr_ = gnn_ops.xent(ref(x, csr, idx), y[idx])
        opt.zero_grad()
        lr_.backward()
        opt.step()
        assert abs(loss - float(lr_)) <= 1e-5 * max(1.0, abs(loss))
    for (k, a), b in zip(m.state_dict().items(), ref.state_dict().values()):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6, msg=k)


def test_fused_and_composed_agree_cpu():
    x, csr, y = _graph()
    torch.manual_seed(1)
    a = FullGraphGAT(20, 4, 8, 5, 2, impl="fused")
    b = copy.deepcopy(a)
    b.impl = "composed"
    torch.testing.assert_close(a(x, csr), b(x, csr), rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
def test_captured_epochs_equal_eager_and_learn_gpu():
    x, csr, y = _graph(n=4000, device="cuda")
    idx = torch.arange(0, 4000, 2, device="cuda")
    test = torch.arange(1, 4000, 2, device="cuda")
    out = {}
    for mode in ("eager", "graph"):
        torch.manual_seed(0)
        m = FullGraphGAT(20, 8, 16, 5, 2).cuda()
        tr = FullGraphGatTrainer(m, x, csr, y, idx, "adam", 5e-3)
        acc0 = tr.accuracy(test)
        if mode == "graph":
            tr.capture(warmup=2, steps=1)
            tr.replay_steps(118)
        else:
            for _ in range(120):
                tr.step()
        torch.cuda.synchronize()
        out[mode] = (float(tr.loss.item()), tr.flat.flat.clone(), acc0, tr.accuracy(test))
    (le, pe, a0, ae), (lg, pg, _, ag) = out["eager"], out["graph"]
    assert abs(le - lg) <= 1e-3 * max(1.0, abs(le)), (le, lg)
    assert float((pe - pg).norm() / pe.norm()) < 1e-3
    assert ae > a0 + 0.2 and ag > a0 + 0.2, (a0, ae, ag)
