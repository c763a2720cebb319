#!/usr/bin/env python3
"""Kernels with known HBM traffic, to calibrate what rocprofv3's memory counters report on
this box (e.g. whether TCC-derived FETCH_SIZE / WRITE_SIZE cover all 8 XCDs):

  copy     : y.copy_(x) of a 512 MiB fp32 buffer            -> 512 MiB read, 512 MiB written
  gather   : gather_rows of 262,144 random rows x 256 B out of a 4 GiB bf16 table
                                                            -> 64 MiB read (+1 MiB ids), 64 MiB written
  fill     : x.zero_() of 512 MiB                           -> 0 read, 512 MiB written
Each op runs 3 times after a warm-up.  Pair with tools/pmc_passes.sh.
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from euler_amd.ops._native import hip

    dev = torch.device("cuda", 0)
    x = torch.randn(128 << 20, device=dev)   # 512 MiB
    y = torch.empty_like(x)
    table = torch.empty(8 << 20, 256, dtype=torch.bfloat16, device=dev)  # 4 GiB
    table.view(torch.int16).random_(-1000, 1000)
    ids = torch.randint(0, table.shape[0], (262144,), device=dev)
    for _ in range(4):
        y.copy_(x)
        hip().gather_rows(table, ids)
        y.zero_()
    torch.cuda.synchronize()
    print("calibration done", flush=True)


if __name__ == "__main__":
    main()
