"""Device-path evaluate / infer (estimator/base.py ``_device_inference_trainer``; VERDICT
r4 item 7, reference euler_estimator/python/base_estimator.py:145-179).

After a device-path train, ``infer()`` runs the device trainer's own flow and model on the
id file and writes the same ``embedding_<rank>.npy`` / ``ids_<rank>.npy`` as the engine
path; ``evaluate()`` reports the model's metric from device logits.  The full-neighbourhood
models are deterministic per batch, so the device and engine outputs on the same checkpoint
agree to fp32 rounding; the sampled GraphSAGE tree is a fresh draw on either path, so
there the test checks shapes, finiteness and the metric's range."""
import math
import os

import numpy as np
import pytest
import torch


def _est(tmp, model, extra, device, device_graph=True):
    from euler_amd.tools import runner

    a = runner.parse_args(["--dataset", "ppi", "--scale", "0.05", "--batch_size", "64", "--total_step", "6",
                           "--log_steps", "3", "--model_dir", os.path.join(tmp, "ckpt"), "--infer_dir",
                           os.path.join(tmp, "infer_dev" if device_graph else "infer_eng"), "--device", device,
                           "--seed", "1"] + extra + (["--device_graph"] if device_graph else []), model=model)
    torch.manual_seed(0)
    return runner.build(a)[1]


def _gcn_parity(tmp, device, rtol):
    est = _est(tmp, "gcn", [], device)
    est.train()
    ids_d, emb_d = est.infer()
    assert getattr(est, "infer_rate", 0) > 0  # the device path wrote them
    ev_d = est.evaluate()
    eng = _est(tmp, "gcn", [], device, device_graph=False)
    ids_e, emb_e = eng.infer()
    ev_e = eng.evaluate()
    assert ids_d.shape == ids_e.shape and (ids_d == ids_e).all()
    assert emb_d.shape == emb_e.shape and emb_d.shape[0] > 64  # several batches, the last one short
    np.testing.assert_allclose(emb_d, emb_e, rtol=rtol, atol=rtol)
    for f in ("embedding_0.npy", "ids_0.npy"):
        assert os.path.exists(os.path.join(tmp, "infer_dev", f))
    assert math.isclose(ev_d["loss"], ev_e["loss"], rel_tol=rtol)
    assert abs(ev_d["f1"] - ev_e["f1"]) <= 0.01
    return est


def test_gcn_device_infer_matches_engine_cpu(tmp_path):
    est = _gcn_parity(str(tmp_path), "cpu", 1e-4)
    assert type(est.device_trainer).__name__ == "FullFlowTrainer"


def test_device_infer_restores_checkpoint_in_a_fresh_estimator(tmp_path):
    tmp = str(tmp_path)
    est = _est(tmp, "gcn", [], "cpu")
    est.train()
    ids_a, emb_a = est.infer()
    fresh = _est(tmp, "gcn", [], "cpu")  # run_mode infer: builds the device trainer from model_dir
    ids_b, emb_b = fresh.infer()
    assert fresh.global_step == 6 and (ids_a == ids_b).all()
    np.testing.assert_allclose(emb_a, emb_b, rtol=1e-6, atol=1e-6)


def test_sage_device_infer_and_evaluate_cpu(tmp_path):
    tmp = str(tmp_path)
    est = _est(tmp, "graphsage", ["--fanouts", "5", "3"], "cpu")
    est.train()
    ids, emb = est.infer()
    assert getattr(est, "infer_rate", 0) > 0
    assert emb.shape == (ids.shape[0], 32) and np.isfinite(emb).all()
    ev = est.evaluate()
    assert math.isfinite(ev["loss"]) and 0.0 <= ev["f1"] <= 1.0


@pytest.mark.gpu
def test_gcn_fused_device_infer_matches_engine_gpu(tmp_path):
    est = _gcn_parity(str(tmp_path), "cuda", 2e-3)
    assert type(est.device_trainer).__name__ == "GcnTrainer"
    assert getattr(est, "infer_rate", 0) > 0


@pytest.mark.gpu
def test_sage_device_infer_gpu(tmp_path):
    tmp = str(tmp_path)
    est = _est(tmp, "graphsage", ["--fanouts", "5", "3"], "cuda")
    est.train()
    ids, emb = est.infer()
    assert getattr(est, "infer_rate", 0) > 0
    assert emb.shape == (ids.shape[0], 32) and np.isfinite(emb).all()
    ev = est.evaluate()
    assert math.isfinite(ev["loss"]) and 0.0 <= ev["f1"] <= 1.0
