#!/usr/bin/env python3
"""cProfile of the engine-path GraphSAGE estimator loop (benchmarks/bench_engine_sage.py,
serial input pipeline) — where the host time of a reference-architecture step goes."""
import argparse
import cProfile
import os
import pstats
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))

import torch  # noqa: E402

import bench_engine_sage as b  # noqa: E402
from euler_amd.dataset import get_dataset  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=40)
    p.add_argument("--out", default=None)
    a = p.parse_args()
    ds = get_dataset("ppi", data_dir=tempfile.mkdtemp(prefix="euler_amd_ppi_"), scale=1.0)
    ds.load_graph()
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    args = argparse.Namespace(steps=a.steps, warmup=3, batch=512, scale=1.0)
    b.run(ds, args, 0, dev, 1)
    prof = cProfile.Profile()
    prof.enable()
    el, _ = b.run(ds, args, 0, dev, 1)
    prof.disable()
    print(f"{a.steps} steps in {el:.3f}s = {el * 1e3 / a.steps:.2f} ms/step", flush=True)
    st = pstats.Stats(prof)
    st.sort_stats("tottime").print_stats(30)
    st.sort_stats("cumtime").print_stats(40)


if __name__ == "__main__":
    main()
