"""Single-node launcher (euler_amd/parallel/launch.py) and bench.py's --gpus handling on the
CPU: rank env, stdout forwarding, failure propagation, the WORLD_SIZE consistency check."""
import json
import os
import subprocess
import sys
import textwrap
import time

import pytest

from euler_amd.parallel.launch import rank_env, spawn_local

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _script(tmp_path, body):
    p = tmp_path / "child.py"
    p.write_text(textwrap.dedent(body))
    return str(p)


class _Sink:
    def __init__(self):
        self.parts = []

    def write(self, s):
        self.parts.append(s)

    def flush(self):
        pass

    @property
    def text(self):
        return "".join(self.parts)


def test_rank_env_fields():
    e = rank_env({"FOO": "1"}, 2, 4, 12345)
    assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"], e["MASTER_ADDR"], e["MASTER_PORT"]) == \
        ("2", "2", "4", "127.0.0.1", "12345")
    assert e["FOO"] == "1" and e["EULER_AMD_LAUNCHED"] == "1" and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_spawn_forwards_rank0_stdout_and_env(tmp_path):
    script = _script(tmp_path, """
        import json, os, sys
        keys = ["RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"]
        print(json.dumps({k: os.environ[k] for k in keys} | {"argv": sys.argv[1:]}))
        print("hello from", os.environ["RANK"], file=sys.stderr)
    """)
    out, err = _Sink(), _Sink()
    rc = spawn_local(3, ["--x", "1"], script=script, stdout=out, stderr=err)
    assert rc == 0
    lines = [json.loads(l) for l in out.text.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.text  # only rank 0's stdout is the job's stdout
    assert lines[0]["RANK"] == "0" and lines[0]["WORLD_SIZE"] == "3" and lines[0]["argv"] == ["--x", "1"]
    ranks_seen = sorted(int(l.split()[1][:-1]) for l in err.text.splitlines() if l.startswith("[rank ") and
                        "stdout]" not in l)
    assert ranks_seen == [0, 1, 2]
    # ranks 1, 2 stdout arrive on stderr, prefixed, all with the same rendezvous port
    others = [json.loads(l.split("] ", 1)[1]) for l in err.text.splitlines() if "stdout]" in l]
    assert sorted(o["RANK"] for o in others) == ["1", "2"]
    assert {o["MASTER_PORT"] for o in others} == {lines[0]["MASTER_PORT"]}


def test_spawn_failure_stops_other_ranks(tmp_path):
    script = _script(tmp_path, """
        import os, sys, time
        if os.environ["RANK"] == "1":
            print("boom: rank one failed", file=sys.stderr)
            sys.exit(3)
        time.sleep(60)
    """)
    out, err = _Sink(), _Sink()
    t0 = time.time()
    rc = spawn_local(2, [], script=script, stdout=out, stderr=err, grace_s=2.0)
    assert rc == 3
    assert time.time() - t0 < 30, "the surviving rank was not stopped"
    assert "rank 1 of 2 exited with code 3" in err.text and "boom: rank one failed" in err.text


def _bench(args, env_extra=None, timeout=120):
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, "bench.py"] + args, cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=timeout)


def test_bench_gpus_must_match_world_size():
    r = _bench(["--gpus", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "disagrees with WORLD_SIZE=2" in r.stderr


@pytest.mark.skipif(__import__("torch").cuda.is_available(), reason="CPU-only check of the failure path")
def test_bench_gpus_launches_ranks_and_propagates_failure():
    # on a CPU box every rank fails at device set-up: the launcher must start --gpus ranks
    # and exit non-zero with a failing rank's stderr tail
    r = _bench(["--gpus", "2", "--num-nodes", "1000", "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0
    assert "[launch] rank" in r.stderr and "of 2 exited with code" in r.stderr, r.stderr[-2000:]


# ------------------------------------------------------------------ every multi-GPU entry point
_ENTRY_POINTS = ["bench.py", "benchmarks/bench_deepwalk.py", "benchmarks/bench_kg.py",
                 "benchmarks/bench_deepwalk_estimator.py", "euler_amd/tools/runner.py", "euler_amd/__init__.py"]


@pytest.mark.parametrize("path", _ENTRY_POINTS)
def test_entry_points_set_dmabuf_ipc_before_torch(path):
    """RCCL needs HSA_ENABLE_IPC_MODE_LEGACY=0 before HIP loads: every multi-GPU entry point
    sets it above its first torch import (the package init covers the examples)"""
    lines = open(os.path.join(ROOT, path)).read().splitlines()
    env = next(i for i, l in enumerate(lines) if 'HSA_ENABLE_IPC_MODE_LEGACY", "0"' in l and "setdefault" in l)
    torch_imp = [i for i, l in enumerate(lines) if l.startswith("import torch") or l.startswith("from torch")]
    assert not torch_imp or env < torch_imp[0], (path, env, torch_imp[:1])


def _run_script(args, timeout=600, env_extra=None):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "EULER_AMD_LAUNCHED", "HSA_ENABLE_IPC_MODE_LEGACY"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable] + args, cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=timeout)


@pytest.mark.skipif(__import__("torch").cuda.is_available(), reason="CPU-only check of the failure path")
def test_bench_deepwalk_gpus_spawns_ranks_that_fail_cleanly_without_gpus():
    r = _run_script(["benchmarks/bench_deepwalk.py", "--gpus", "2", "--num-nodes", "1000", "--steps", "1",
                     "--eval-nodes", "0"])
    assert r.returncode != 0
    assert "of 2 exited with code" in r.stderr and "needs a GPU" in r.stderr, r.stderr[-2000:]


def test_bench_kg_gpus_two_ranks_run_on_cpu():
    """bench_kg.py --gpus 2 --device cpu: two self-spawned gloo ranks train data parallel;
    rank 0's JSON line is the job's stdout and names the parallelism"""
    r = _run_script(["benchmarks/bench_kg.py", "--gpus", "2", "--device", "cpu", "--steps", "2", "--warmup", "1",
                     "--num-ent", "2000", "--num-rel", "20", "--num-triples", "20000", "--eval-after", "0"])
    assert r.returncode == 0, r.stderr[-3000:]
    out = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(out) == 1 and out[0]["n_gpus"] == 2 and out[0]["ranks"] == 2 and out[0]["parallelism"] == "dp2"


def test_runner_gpus_two_ranks_train_on_cpu(tmp_path):
    """the model-zoo runner (and through it every examples/run_*.py): --gpus 2 starts two
    ranks whose estimators all-reduce over gloo on the CPU"""
    r = _run_script(["-m", "euler_amd.tools.runner", "--model", "graphsage", "--dataset", "cora", "--scale", "0.05",
                     "--data_dir", str(tmp_path / "cora"), "--gpus", "2", "--device", "cpu", "--total_step", "2",
                     "--log_steps", "1", "--batch_size", "8", "--model_dir", str(tmp_path / "ck")])
    assert r.returncode == 0, r.stderr[-3000:]
    assert "[rank 1]" in r.stderr
    assert os.path.exists(tmp_path / "ck" / "checkpoint")


def test_maybe_spawn_contract(monkeypatch):
    from euler_amd.parallel.launch import maybe_spawn

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert maybe_spawn(None, [], "x.py") is None and maybe_spawn(1, [], "x.py") is None
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert maybe_spawn(4, [], "x.py") is None and maybe_spawn(None, [], "x.py") is None
    with pytest.raises(SystemExit, match="disagrees"):
        maybe_spawn(2, [], "x.py")
