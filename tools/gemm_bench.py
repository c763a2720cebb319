#!/usr/bin/env python3
"""Times the tiled MFMA GEMM (gnn_ops.gemm) against torch (hipBLASLt) on the shapes the
model code uses: unsupervised tower heads (R = 1024 / 6144 rows) and the R-GCN self-loop
(14951 rows).  Prints one JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps=50):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) * 1000.0 / reps, 2)


def main():
    from euler_amd.ops.gnn_ops import _gemm_splits, gemm

    dev = torch.device("cuda", 0)
    cases = [  # (name, M, N, K, trans_a, trans_b, a dtype)
        ("tower h1 = A1 W1^T", 6144, 128, 256, False, True, torch.bfloat16),
        ("tower e = h1 Wfc^T", 6144, 128, 128, False, True, torch.float32),
        ("tower dh1 = de Wfc", 6144, 128, 128, False, False, torch.float32),
        ("tower dA1 = dh1 W1", 6144, 256, 128, False, False, torch.float32),
        ("tower dW1 = dh1^T A1", 128, 256, 6144, True, False, torch.float32),
        ("tower dWfc = de^T h1", 128, 128, 6144, True, False, torch.float32),
        ("rgcn self-loop x W^T", 14951, 128, 128, False, True, torch.float32),
        ("rgcn dW = g^T x", 128, 128, 14951, True, False, torch.float32),
    ]
    for name, M, N, K, ta, tb, dt in cases:
        a = torch.randn((K, M) if ta else (M, K), device=dev).to(dt)
        b = torch.randn((N, K) if tb else (K, N), device=dev)
        out = torch.empty(M, N, device=dev)
        splits = _gemm_splits(K, -(-M // 64) * -(-N // 64)) if ta else 1
        ours = timeit(lambda: gemm(a, b, out=out, trans_a=ta, trans_b=tb, splits=splits))
        A = a.float().t() if ta else a.float()
        B = b.t() if tb else b
        ref = timeit(lambda: torch.mm(A, B))
        print(json.dumps({"case": name, "M": M, "N": N, "K": K, "splits": splits, "gemm_us": ours,
                          "torch_us": ref}), flush=True)


if __name__ == "__main__":
    main()
