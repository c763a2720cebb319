"""contrib back ends (reference tf_euler/python/contrib) against plain fp32 PyTorch, and
the sample-solution example end to end."""
import os
import sys

import pytest
import torch

from euler_amd.contrib import py_scatter, spmm


def _ref_adj(edge_index, size):
    a = torch.zeros(size)
    a.index_put_((edge_index[0], edge_index[1]), torch.ones(edge_index.shape[1]), accumulate=True)
    return a


def _case(device="cpu"):
    g = torch.Generator().manual_seed(0)
    ei = torch.stack([torch.randint(0, 7, (40,), generator=g), torch.randint(0, 11, (40,), generator=g)])
    x = torch.randn(11, 5, generator=g)
    return ei.to(device), x.to(device)


def _check_spmm(device):
    ei, x = _case(device)
    a = _ref_adj(ei.cpu(), (9, 11))
    torch.testing.assert_close(spmm.spmm_add(x, ei, (9, 11)).cpu(), a @ x.cpu(), atol=1e-5, rtol=1e-5)
    mean = (a @ x.cpu()) / a.sum(1, keepdim=True).clamp(min=1)
    torch.testing.assert_close(spmm.spmm_("mean", x, ei, (9, 11)).cpu(), mean, atol=1e-5, rtol=1e-5)


def _check_scatter(device):
    ei, x = _case(device)
    idx, src = ei[0][:11], x
    size = 9
    ref = torch.full((size, 5), 2.0).index_add(0, idx.cpu(), src.cpu())
    torch.testing.assert_close(py_scatter.scatter_add(src, idx, size, fill_value=2.0).cpu(), ref)
    mx = py_scatter.scatter_("max", src, idx, size, fill_value=-3.0).cpu()
    for r in range(size):
        rows = src.cpu()[idx.cpu() == r]
        want = rows.max(0).values if len(rows) else torch.full((5,), -3.0)
        torch.testing.assert_close(mx[r], want)


def test_contrib_cpu():
    _check_spmm("cpu")
    _check_scatter("cpu")
    with pytest.raises(ValueError):
        spmm.spmm_("min", *_case()[::-1], (9, 11))


@pytest.mark.gpu
def test_contrib_gpu():
    _check_spmm("cuda")
    _check_scatter("cuda")


def test_run_sample_solution(tmp_path):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples"))
    import run_sample_solution

    res = run_sample_solution.main(["--scale", "0.05", "--data_dir", str(tmp_path / "cora"), "--num_samples", "64",
                                    "--batch_size", "16", "--epoch", "1", "--model_dir", str(tmp_path / "ckpt")])
    assert res["loss"] == res["loss"]
