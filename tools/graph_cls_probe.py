"""Phase stamps of the fused graph-classification step (csrc/hip/graph_cls.hip): one eager
step with per-block wall-clock stamps (100 MHz), mean phase durations over blocks.

    python tools/graph_cls_probe.py [--model gin|graphgcn] [--batch 64]
"""
import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gin")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--hidden", type=int, default=32)
    a = ap.parse_args()
    import torch
    from euler_amd.tools import runner

    work = tempfile.mkdtemp()
    args = runner.parse_args(["--model_dir", os.path.join(work, "m"), "--batch_size", str(a.batch), "--total_step", "10",
                              "--device", "cuda", "--device_graph", "--hidden_dim", str(a.hidden),
                              "--data_dir", os.path.join(work, "data")], model=a.model)
    _, est = runner.build(args)
    first = est.get_train_from_input(est.train_input_fn(), est.params)
    tr = est._device_graph_trainer(first)
    for _ in range(5):
        tr.step()
    torch.cuda.synchronize()
    prof = tr.plan.profile().cpu().double()
    torch.cuda.synchronize()
    n = int((prof[0] > 0).sum())
    d = (prof[:, 1:n] - prof[:, : n - 1]) * 0.01  # us
    out = {"model": a.model, "batch": a.batch, "lds_bytes": tr.plan.lds_bytes, "z_kept": tr.plan.z_kept,
           "phase_us_mean": [round(float(x), 2) for x in d.mean(0)],
           "block_us_mean": round(float(((prof[:, n - 1] - prof[:, 0]) * 0.01).mean()), 2),
           "start_skew_us": round(float((prof[:, 0].max() - prof[:, 0].min()) * 0.01), 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
