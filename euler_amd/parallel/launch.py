"""Single-node multi-process launcher: one rank per GPU, started from a plain
``python script.py --gpus N`` (reference ``tf_euler/scripts/dist_tf_euler.sh:1-49``, which
starts the ps / worker processes of one between-graph job by hand).

The parent never touches the GPU: it picks a free rendezvous port on 127.0.0.1, starts N
child processes of the same script with ``RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
MASTER_PORT`` set (what ``torch.distributed.run`` would export), forwards rank 0's stdout
verbatim (the script's result line) and every rank's stderr with a ``[rank r]`` prefix, and
waits.  A child that exits non-zero makes the parent stop the others (SIGTERM, then SIGKILL
after a grace period; only the PIDs it started) and return that exit code with the child's
stderr tail.  No ``exec``: each child is a fresh ``subprocess`` of a parent that never
initialised HIP, so every rank does its own device set-up.
"""
from __future__ import annotations

import collections
import os
import socket
import subprocess
import sys
import threading
import time

__all__ = ["free_port", "rank_env", "spawn_local", "maybe_spawn", "require_gpu", "LAUNCHED_ENV"]

# set in every child: a script seeing it never launches again
LAUNCHED_ENV = "EULER_AMD_LAUNCHED"


def free_port(host: str = "127.0.0.1") -> int:
    s = socket.socket()
    try:
        s.bind((host, 0))
        return int(s.getsockname()[1])
    finally:
        s.close()


def rank_env(base: dict, rank: int, world: int, port: int, addr: str = "127.0.0.1") -> dict:
    """The environment of rank ``rank`` of a ``world``-rank single-node job."""
    env = dict(base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0", "MASTER_ADDR": addr,
                "MASTER_PORT": str(port), LAUNCHED_ENV: "1"})
    # dmabuf IPC (the only mode the host driver supports): RCCL and the xGMI all-reduce's
    # peer mappings fail without it
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def _pump(stream, sink, prefix: str, tail: collections.deque | None):
    for line in iter(stream.readline, ""):
        if tail is not None:
            tail.append(line)
        sink.write(prefix + line)
        sink.flush()
    stream.close()


def spawn_local(nprocs: int, argv: list, script: str | None = None, env: dict | None = None,
                grace_s: float = 10.0, poll_s: float = 0.05, stdout=None, stderr=None) -> int:
    """Run ``python script *argv`` as ``nprocs`` ranks on this node; return the job's exit
    code (0 when every rank exited 0, else the first failing rank's code, or 1 for a
    signal).  ``script`` defaults to the running program (``sys.argv[0]``)."""
    nprocs = int(nprocs)
    if nprocs < 1:
        raise ValueError("nprocs must be >= 1")
    script = os.path.abspath(script or sys.argv[0])
    stdout = stdout or sys.stdout
    stderr = stderr or sys.stderr
    port = free_port()
    base = dict(os.environ if env is None else env)
    procs, pumps, tails = [], [], []
    try:
        for r in range(nprocs):
            p = subprocess.Popen([sys.executable, "-u", script] + list(argv), env=rank_env(base, r, nprocs, port),
                                 stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, bufsize=1)
            procs.append(p)
            tail = collections.deque(maxlen=40)
            tails.append(tail)
            # rank 0's stdout is the job's stdout (the one result line); the others' go to stderr
            out_sink, out_pre = (stdout, "") if r == 0 else (stderr, f"[rank {r} stdout] ")
            for stream, sink, pre, tl in ((p.stdout, out_sink, out_pre, None), (p.stderr, stderr, f"[rank {r}] ", tail)):
                t = threading.Thread(target=_pump, args=(stream, sink, pre, tl), daemon=True)
                t.start()
                pumps.append(t)
        failed = None
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                failed = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(poll_s)
    finally:
        _stop(procs, grace_s)
        for t in pumps:
            t.join(timeout=5.0)
    if failed is None:
        return 0
    r, code = failed
    stderr.write(f"[launch] rank {r} of {nprocs} exited with code {code}; stopped the other ranks. "
                 f"stderr tail of rank {r}:\n" + "".join(tails[r]))
    stderr.flush()
    return code if code > 0 else 1


def _stop(procs, grace_s):
    live = [p for p in procs if p.poll() is None]
    for p in live:
        p.terminate()
    deadline = time.time() + grace_s
    for p in live:
        try:
            p.wait(timeout=max(0.0, deadline - time.time()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()


_REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def maybe_spawn(gpus, argv, script):
    """The ``--gpus N`` contract of every multi-GPU entry point (bench.py,
    benchmarks/bench_deepwalk.py, benchmarks/bench_kg.py, tools/runner.py and the
    examples): a plain ``python script --gpus N`` (no WORLD_SIZE) starts N ranks here and
    returns the job's exit code; a rank (torchrun's or ours) gets None and runs.  ``gpus``
    None: whatever WORLD_SIZE says.  A WORLD_SIZE that disagrees with an explicit --gpus
    is an error.  Call before anything touches the GPU."""
    env_world = os.environ.get("WORLD_SIZE")
    if gpus is None:
        return None
    gpus = int(gpus)
    if gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if env_world is None:
        if gpus > 1 and LAUNCHED_ENV not in os.environ:
            env = dict(os.environ)
            env["PYTHONPATH"] = _REPO + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
            return spawn_local(gpus, list(argv), script=os.path.abspath(script), env=env)
        return None
    if int(env_world) != gpus:
        raise SystemExit(f"--gpus {gpus} disagrees with WORLD_SIZE={env_world} (torchrun --nproc-per-node)")
    return None


def require_gpu(local_rank: int, world: int, what: str = "this script"):
    """Fail cleanly (SystemExit naming the shortfall) when rank ``local_rank`` has no GPU of
    its own: one rank per GPU, no device sharing under RCCL."""
    import torch

    n = torch.cuda.device_count()
    if n == 0:
        raise SystemExit(f"{what} needs a GPU (run through gpurun on an MI355X)")
    if local_rank >= n:
        raise SystemExit(f"{what}: rank with LOCAL_RANK={local_rank} of {world} needs its own GPU, but only {n} "
                         f"visible (one rank per GPU)")
