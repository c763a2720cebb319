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
