"""CPU checks of the fused kernels' memory layouts."""
import torch


def test_fm_layout_roundtrip_cpu():
    """fm_to_dense inverts the kernels' fm_off index map (sage_train.hip)"""
    from euler_amd.models.sage_step import fm_to_dense

    N, K = 32, 64
    buf = torch.empty(N * K, dtype=torch.float32)
    for n in range(N):
        for k in range(K):
            off = (((n >> 4) * (K >> 5) + (k >> 5)) * 64 + ((k & 31) >> 3) * 16 + (n & 15)) * 8 + (k & 7)
            buf[off] = n * K + k
    assert torch.equal(fm_to_dense(buf.view(N, K)), torch.arange(N * K, dtype=torch.float32).view(N, K))
