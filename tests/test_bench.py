"""bench.py contract: one JSON line with the driver's fields, on the single-GPU path and on
the multi-GPU path (RCCL process group + all-reduce captured in the hipGraph) run with one
rank under torch.distributed.run."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(cmd):
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    assert KEYS <= set(out), set(KEYS) - set(out)
    return out


SMALL = ["--num-nodes", "200000", "--steps", "20", "--warmup", "5"]


@pytest.mark.gpu
def test_bench_single_gpu_json():
    out = _run([sys.executable, "bench.py"] + SMALL)
    assert out["n_gpus"] == 1 and out["value"] > 0 and out["config"]["parallelism"] == "dp1"


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [[], ["--no-graph"], ["--grad-reduce-dtype", "bf16"], ["--grad-buckets", "2"]],
                         ids=["captured", "eager", "bf16_allreduce", "two_buckets"])
def test_bench_distributed_path_one_rank(extra):
    out = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--force-dist"]
               + extra + SMALL)
    assert "all-reduce" in out["config"]["grad_sync"] and out["value"] > 0
    first, last = out["config"]["loss_first_last"]
    assert last == last and first == first


@pytest.mark.gpu
def test_bench_gpus_flag_launches_ranks():
    # plain `python bench.py --gpus 2` (the driver's BENCH invocation) starts 2 ranks itself;
    # --shared-gpu puts both on the one GPU of the box (gloo group, xGMI all-reduce kernel)
    out = _run([sys.executable, "bench.py", "--gpus", "2", "--shared-gpu"] + SMALL)
    # a rehearsal is one physical GPU: n_gpus counts devices, "ranks" processes, no vs_baseline
    assert out["n_gpus"] == 1 and out["ranks"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["vs_baseline"] is None
    assert out["config"]["global_batch"] == 2 * 1024
    assert "xgmi" in out["config"]["grad_sync"] and out["value"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("ranks", [4, 8])
def test_bench_shared_gpu_rehearsal_many_ranks(ranks):
    # the whole-node path at the driver's rank counts, every rank on the one GPU of the box:
    # W-rank xGMI reduce-scatter shard math, per-block flags and epochs inside the captured
    # step; the loss must fall and stay finite on every rank's replicas
    out = _run([sys.executable, "bench.py", "--gpus", str(ranks), "--shared-gpu", "--num-nodes", "200000",
                "--steps", "40", "--warmup", "5"])
    assert out["ranks"] == ranks and out["config"]["parallelism"] == "dp%d" % ranks
    assert out["n_gpus"] == 1 and out["vs_baseline"] is None
    first, last = out["config"]["loss_first_last"]
    assert last == last and last < first
