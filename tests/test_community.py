"""The planted-community dataset is learnable through aggregation, and the device
(fused-trainer) path of NodeEstimator reaches the engine path's held-out F1
(benchmarks/bench_community_f1.py runs the same comparison at full size on the GPU)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "benchmarks"))


def test_community_heldout_f1_engine_and_device_paths_cpu(tmp_path, monkeypatch):
    monkeypatch.setenv("EULER_AMD_DATA", str(tmp_path / "data"))
    monkeypatch.chdir(tmp_path)
    from bench_community_f1 import main

    out = main(["--steps", "150", "--device", "cpu"])
    eng, dev = out["engine"]["heldout"]["f1"], out["device"]["heldout"]["f1"]
    assert eng > 0.75 and dev > 0.75, (eng, dev)
    assert abs(eng - dev) < 0.05, (eng, dev)
