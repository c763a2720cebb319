#!/usr/bin/env python3
"""Do independent branches of a captured hipGraph run concurrently on this ROCm?  Two
torch.cuda._sleep kernels captured on two forked streams vs on one stream."""
import time

import torch


def timed(g, n=50):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e6


def main():
    cyc = 200_000  # ~ 80-100 us per sleep kernel at ~2.4 GHz
    s0 = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    # warm
    torch.cuda._sleep(cyc)
    torch.cuda.synchronize()
    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1):
        torch.cuda._sleep(cyc)
        torch.cuda._sleep(cyc)
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2):
        cap = torch.cuda.current_stream()
        side.wait_stream(cap)
        torch.cuda._sleep(cyc)
        with torch.cuda.stream(side):
            torch.cuda._sleep(cyc)
        cap.wait_stream(side)
    g0 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g0):
        torch.cuda._sleep(cyc)
    print(f"one sleep {timed(g0):.1f} us; two serial {timed(g1):.1f} us; two forked branches {timed(g2):.1f} us",
          flush=True)


if __name__ == "__main__":
    main()
