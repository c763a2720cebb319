"""Owner routing of the fixed-capacity all-to-all exchanges (csrc/hip/route.hip vs the
torch composition and a brute-force definition)."""
import pytest
import torch


def _brute(ids, W, C):
    n = ids.numel()
    pos = torch.full((n,), W * C, dtype=torch.long)
    send = torch.full((W * C + 1,), -1, dtype=torch.long)
    seen = [0] * W
    over = 0
    for k in range(n):
        v = int(ids[k])
        if v < 0:
            continue
        o = v % W
        if seen[o] < C:
            pos[k] = o * C + seen[o]
            send[o * C + seen[o]] = v
        else:
            over = 1
        seen[o] += 1
    return pos, send, over


@pytest.mark.parametrize("W,C,n", [(1, 300, 300), (2, 90, 160), (8, 64, 700), (8, 20, 700), (63, 4, 500)])
def test_route_by_owner_cpu(W, C, n):
    from euler_amd.ops.gnn_ops import route_by_owner

    g = torch.Generator().manual_seed(W * 7 + n)
    ids = torch.randint(-3, 10_000, (n,), generator=g)
    ov = torch.zeros(1, dtype=torch.int32)
    pos, send = route_by_owner(ids, W, C, ov)
    bp, bs, bo = _brute(ids, W, C)
    assert torch.equal(pos, bp) and torch.equal(send, bs) and int(ov) == bo


@pytest.mark.gpu
@pytest.mark.parametrize("W,C,n", [(1, 700_001, 700_001), (2, 400_000, 700_001), (8, 90_000, 700_001),
                                   (8, 80_000, 700_001), (63, 50, 3000), (8, 64, 100)])
def test_route_by_owner_kernel_matches_torch(cuda, W, C, n):
    from euler_amd.ops import gnn_ops

    g = torch.Generator().manual_seed(n + W)
    ids = torch.randint(-5, 1 << 40, (n,), generator=g)
    ov_k = torch.zeros(1, dtype=torch.int32, device=cuda)
    pk, sk = gnn_ops.route_by_owner(ids.to(cuda), W, C, ov_k)
    ov_r = torch.zeros(1, dtype=torch.int32)
    pr, sr = _torch_route(ids, W, C, ov_r)
    assert torch.equal(pk.cpu(), pr) and torch.equal(sk.cpu(), sr) and int(ov_k.cpu()) == int(ov_r)


def _torch_route(ids, W, C, ov):
    from euler_amd.ops.gnn_ops import route_by_owner

    return route_by_owner(ids, W, C, ov)  # CPU tensors: the torch composition
