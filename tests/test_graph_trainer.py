"""GraphEstimator(device_graph=True) for graph classification (models/graph_trainer.py;
reference euler_estimator/python/graph_estimator.py:27-85, mp_utils/base_graph.py:24-47):
the device step against the engine path on the same graphs, training, resume, capture."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F


def _est(tmp_path, model, device, steps=12, extra=()):
    from euler_amd.tools import runner

    a = runner.parse_args(["--model_dir", str(tmp_path / model), "--batch_size", "16", "--total_step", str(steps),
                           "--log_steps", "6", "--device", device, "--seed", "1", "--device_graph",
                           "--learning_rate", "0.01"] + list(extra), model=model)
    torch.manual_seed(0)
    return runner.build(a)


@pytest.mark.parametrize("model", ["gin", "set2set"])
def test_device_step_matches_engine_path_cpu(tmp_path, model):
    """same graphs, same weights: the device blocks + padded pooling give the engine path's
    loss (fp32, CPU twin of every kernel)"""
    m, est = _est(tmp_path, model, "cpu")
    first = est.get_train_from_input(est.train_input_fn(), est.params)
    tr = est._device_graph_trainer(first)
    gidx = torch.tensor([0, 3, 3, 7, 11, 2, 5, 1, 9, 4, 6, 8, 10, 12, 13, 14])
    with torch.no_grad():
        logits = tr._forward(gidx)
        loss = F.binary_cross_entropy_with_logits(logits, tr.onehot[gidx])
        inputs = est._graph_inputs(tr.graph_labels_of(gidx))
        _, ref_loss, _, _ = m(inputs)
    assert math.isclose(float(loss), float(ref_loss), rel_tol=1e-4, abs_tol=1e-6)


def test_graph_estimator_device_path_trains_and_resumes_cpu(tmp_path):
    from euler_amd.models.graph_trainer import GraphTrainer
    from euler_amd.tools import runner

    base = ["--model_dir", str(tmp_path / "ckpt"), "--batch_size", "16", "--log_steps", "6", "--device", "cpu",
            "--seed", "1", "--device_graph", "--learning_rate", "0.01"]
    r1 = runner.main(base + ["--total_step", "12"], model="gin")
    assert r1["step"] == 12 and math.isfinite(r1["loss"]) and 0.0 <= r1["accuracy"] <= 1.0
    r2 = runner.main(base + ["--total_step", "18"], model="gin")
    assert r2["step"] == 18
    st = torch.load(str(tmp_path / "ckpt" / "model.ckpt-18.pt"), weights_only=True)
    assert st["device_trainer"]["step"] == 18
    _, est = _est(tmp_path, "gin", "cpu")
    first = est.get_train_from_input(est.train_input_fn(), est.params)
    assert isinstance(est._device_graph_trainer(first), GraphTrainer)


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["gin", "gated_graph"])
def test_graph_estimator_device_path_gpu_captured(tmp_path, cuda, model):
    from euler_amd.tools import runner

    res = runner.main(["--model_dir", str(tmp_path / model), "--batch_size", "32", "--total_step", "64",
                       "--log_steps", "32", "--device", "cuda", "--seed", "1", "--device_graph",
                       "--learning_rate", "0.01"], model=model)
    assert res["step"] == 64 and math.isfinite(res["loss"])
