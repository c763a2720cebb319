"""Owner routing of the fixed-capacity all-to-all exchanges (csrc/hip/route.hip vs the
torch composition and a brute-force definition)."""
import pytest
import torch


def _brute(ids, W, C, self_rank=-1):
    n = ids.numel()

    def blk(o):  # self_rank >= 0: own block last, peers in rank order
        if self_rank < 0:
            return o
        return o if o < self_rank else (o - 1 if o > self_rank else W - 1)

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
            pos[k] = blk(o) * C + seen[o]
            send[blk(o) * C + seen[o]] = v
        else:
            over = 1
        seen[o] += 1
    return pos, send, over


@pytest.mark.parametrize("self_rank", [-1, 0, 1, 5])
@pytest.mark.parametrize("W,C,n", [(1, 300, 300), (2, 90, 160), (8, 64, 700), (8, 20, 700), (63, 4, 500)])
def test_route_by_owner_cpu(W, C, n, self_rank):
    from euler_amd.ops.gnn_ops import route_by_owner

    if self_rank >= W:
        pytest.skip("self_rank outside the world")
    g = torch.Generator().manual_seed(W * 7 + n)
    ids = torch.randint(-3, 10_000, (n,), generator=g)
    ov = torch.zeros(1, dtype=torch.int32)
    pos, send = route_by_owner(ids, W, C, ov, self_rank)
    bp, bs, bo = _brute(ids, W, C, self_rank)
    assert torch.equal(pos, bp) and torch.equal(send, bs) and int(ov) == bo


@pytest.mark.gpu
@pytest.mark.parametrize("W,C,n,self_rank", [(1, 700_001, 700_001, -1), (2, 400_000, 700_001, -1),
                                             (8, 90_000, 700_001, -1), (8, 80_000, 700_001, -1), (63, 50, 3000, -1),
                                             (8, 64, 100, -1), (1, 700_001, 700_001, 0), (2, 400_000, 700_001, 1),
                                             (8, 90_000, 700_001, 3), (8, 80_000, 700_001, 7), (63, 50, 3000, 20)])
def test_route_by_owner_kernel_matches_torch(cuda, W, C, n, self_rank):
    from euler_amd.ops import gnn_ops

    g = torch.Generator().manual_seed(n + W)
    ids = torch.randint(-5, 1 << 40, (n,), generator=g)
    ov_k = torch.zeros(1, dtype=torch.int32, device=cuda)
    pk, sk = gnn_ops.route_by_owner(ids.to(cuda), W, C, ov_k, self_rank)
    ov_r = torch.zeros(1, dtype=torch.int32)
    pr, sr = _torch_route(ids, W, C, ov_r, self_rank)
    assert torch.equal(pk.cpu(), pr) and torch.equal(sk.cpu(), sr) and int(ov_k.cpu()) == int(ov_r)


def _torch_route(ids, W, C, ov, self_rank=-1):
    from euler_amd.ops.gnn_ops import route_by_owner

    return route_by_owner(ids, W, C, ov, self_rank)  # CPU tensors: the torch composition
