"""Every model-zoo runner (examples/run_*.py) trains two steps on a tiny same-schema
synthetic dataset (reference: each examples/*/run_*.py)."""
import numpy as np
import pytest

from euler_amd.tools import runner

MODELS = ["graphsage", "graphsage_unsup", "gcn", "gat", "fastgcn", "adaptivegcn", "agnn", "appnp", "arma", "dna",
          "sgcn", "tagcn", "geniepath", "lgcn", "deepwalk", "node2vec", "line", "dgi", "gae", "vgae", "rgcn",
          "transe", "transh", "transr", "transd", "distmult", "gin", "gated_graph", "graphgcn", "set2set",
          "solution", "scalable_sage", "scalable_gcn"]
SCALE = {"cora": 0.04, "fb15k": 0.004, "wn18": 0.003, "mutag": 0.1, "ppi": 0.02}


@pytest.fixture(scope="module")
def data_root(tmp_path_factory):
    return tmp_path_factory.mktemp("runner_data")


@pytest.mark.parametrize("model", MODELS)
def test_runner_trains(model, data_root, tmp_path):
    ds = runner._models()[model][0]
    args = ["--model", model, "--data_dir", str(data_root / ds), "--scale", str(SCALE[ds]), "--total_step", "2",
            "--log_steps", "1", "--batch_size", "8", "--fanouts", "3", "3", "--hidden_dim", "8", "--dim", "8",
            "--model_dir", str(tmp_path / "ckpt"), "--device", "cpu", "--num_negs", "2"]
    res = runner.main(args)
    assert np.isfinite(res["loss"])


def test_runner_covers_all_examples():
    import os

    here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples")
    scripts = sorted(f[4:-3] for f in os.listdir(here) if f.startswith("run_") and f.endswith(".py"))
    # standalone scripts with their own main (covered by their own tests, e.g. test_contrib.py)
    standalone = {"sample_solution"}
    assert [s for s in scripts if s not in standalone] == sorted(MODELS)
    assert set(MODELS) == set(runner._models())
