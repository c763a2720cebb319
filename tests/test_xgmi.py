"""xGMI two-shot all-reduce (csrc/hip/xgmi_ar.hip, parallel/xgmi.py).

W = 2, 4 and 8 processes share the box's one GPU: each maps the others' IPC buffers exactly
as ranks on different GPUs of a node do, so the protocol (staging, per-block flags, epochs
across calls and hipGraph replays, shard arithmetic for the driver's rank counts) runs for
real; only the xGMI transport is replaced by local HBM.  Results are compared with an fp32 sum of every rank's input
gathered over gloo.
"""
import os
import socket
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    try:
        dist.init_process_group("gloo", rank=rank, world_size=world, init_method=f"tcp://127.0.0.1:{port}")
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        from euler_amd.parallel.xgmi import XgmiAllReduce

        res = {}
        ar = XgmiAllReduce(2 << 20, timeout_s=10.0)
        res["self_test_fp32"] = ar.self_test(dtype=torch.float32)
        res["self_test_bf16"] = ar.self_test(numel=4096, dtype=torch.bfloat16)
        res["self_test_fp32_in_place"] = ar.self_test(numel=278784, dtype=torch.float32, in_place=True)
        res["self_test_bf16_in_place"] = ar.self_test(numel=278784, dtype=torch.bfloat16, in_place=True)
        # random data, sizes that do not divide evenly into shards / blocks
        for n in (278784, 8, 4104, 131080):
            for dtype in (torch.float32, torch.bfloat16):
                if dtype == torch.float32 and n % 4 or dtype == torch.bfloat16 and n % 8:
                    continue
                g = torch.Generator().manual_seed(100 * rank + n)
                x = torch.randn(n, generator=g).to(dtype)
                parts = [torch.empty_like(x.float()) for _ in range(world)]
                dist.all_gather(parts, x.float())
                want = torch.stack(parts).sum(0)
                xd = x.to(dev)
                ar(xd)
                torch.cuda.synchronize()
                tol = 1e-6 if dtype == torch.float32 else 1e-2
                err = float(((xd.float().cpu() - want).abs() / (want.abs() + 1.0)).max())
                res[f"eager_{n}_{str(dtype)[6:]}"] = err <= tol
        # captured: replays with new inputs each time (epochs advance inside the graph)
        n = 278784
        xd = torch.zeros(n, device=dev)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            ar(xd)  # warm-up call outside the capture
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            ar(xd)
        ok = True
        for k in range(5):
            val = torch.full((n,), float(rank + 1 + 10 * k))
            xd.copy_(val.to(dev))
            graph.replay()
            torch.cuda.synchronize()
            want = sum(float(r + 1 + 10 * k) for r in range(world))
            ok = ok and bool(torch.all(xd == want).item())
        res["graph_replays"] = ok
        # in place inside a captured graph: a producer kernel (copy_) writes the IPC input
        # view, the all-reduce reduces it there; and slices of the view (2-bucket trainer)
        xv = ar.input_view(n, torch.float32)
        src = torch.zeros(n, device=dev)
        graph2 = torch.cuda.CUDAGraph()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            xv.copy_(src)
            ar(xv[: n // 2])
            ar(xv[n // 2:])
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        with torch.cuda.graph(graph2, capture_error_mode="thread_local"):
            xv.copy_(src)
            ar(xv[: n // 2])
            ar(xv[n // 2:])
        ok = True
        for k in range(4):
            src.copy_(torch.arange(n, dtype=torch.float32).to(dev) * (rank + 1) + k)
            graph2.replay()
            torch.cuda.synchronize()
            want = torch.arange(n, dtype=torch.float32) * (world * (world + 1) // 2) + k * world
            ok = ok and bool(torch.equal(xv.cpu(), want))
        res["graph_in_place_slices"] = ok
        res["error"] = ar.error()
        dist.barrier()
        del graph, graph2
        q.put((rank, res))
    except Exception as e:  # reported to the parent, which fails the test
        q.put((rank, {"exception": repr(e)}))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4, 8])
def test_xgmi_allreduce_ranks_one_gpu(world):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            r, res = q.get(timeout=60 + 20 * world)
            out[r] = res
    finally:
        for p in procs:
            p.join(timeout=20)
            if p.is_alive():
                p.kill()
    for r in range(world):
        res = out[r]
        assert "exception" not in res, res
        assert res.pop("error") == 0, res
        bad = [k for k, v in res.items() if not v]
        assert not bad, (r, bad, res)


def test_xgmi_block_count():
    pytest.importorskip("euler_amd._hip_ops")
    from euler_amd.parallel import xgmi

    # 4 16-byte vectors per thread and shard sweep, 256 threads per block, at least 16
    # blocks when the tensor has that many 256-vector chunks, at most 64
    assert xgmi._blocks_for(278784, 8, 4) == 16
    assert xgmi._blocks_for(278784, 8, 2) == 16
    assert xgmi._blocks_for(278784, 1, 4) == 64
    assert xgmi._blocks_for(4096, 2, 4) == 4
    assert xgmi._blocks_for(8, 2, 2) == 1
    assert xgmi._blocks_for(1 << 30, 2, 4) == 64


def _worker_estimator_timeout(rank, world, port, q, tmp):
    """NodeEstimator(device_graph=True) on 2 ranks sharing the GPU with the xGMI all-reduce
    forced and a 0.5 s wait bound; rank 1 arrives 3 s late at its first chunk, so rank 0's
    waits time out.  The estimator must notice at the next boundary on BOTH ranks, drop the
    graphs, re-synchronise rank 0's parameters and finish over the fallback all-reduce with
    the ranks in lockstep."""
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    try:
        os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                           "WORLD_SIZE": str(world), "LOCAL_RANK": "0"})
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from euler_amd.tools import runner

        torch.manual_seed(0)
        a = runner.parse_args(["--dataset", "ppi", "--scale", "0.05", "--batch_size", "64", "--total_step", "24",
                               "--log_steps", "8", "--model_dir", os.path.join(tmp, f"ckpt{rank}"),
                               "--device_graph", "--device", "cuda:0", "--seed", "1", "--fanouts", "5", "3"],
                              model="graphsage")
        _, est = runner.build(a)
        est.params.update(grad_sync="xgmi", xgmi_timeout_s=0.5, debug_delay_rank=1, debug_delay_s=3.0)
        est.train()
        p = est.device_trainer.logical_params()
        flat = torch.cat([p[k].reshape(-1).float().cpu() for k in sorted(p)])
        allp = [torch.zeros_like(flat) for _ in range(world)]
        dist.all_gather(allp, flat)
        same = all(torch.equal(x, allp[0]) for x in allp)
        q.put((rank, {"fallback": bool(getattr(est, "grad_sync_fallback", False)), "lockstep": same,
                      "steps": est.global_step == 24, "finite": bool(torch.isfinite(flat).all())}))
    except Exception:  # reported to the parent, which fails the test
        import traceback

        q.put((rank, {"exception": traceback.format_exc()}))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.gpu
def test_estimator_falls_back_when_xgmi_wait_times_out(tmp_path):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    procs = [ctx.Process(target=_worker_estimator_timeout, args=(r, world, port, q, str(tmp_path)))
             for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            r, res = q.get(timeout=110)
            out[r] = res
    finally:
        for p in procs:
            p.join(timeout=20)
            if p.is_alive():
                p.kill()
    for r in range(world):
        res = out[r]
        assert "exception" not in res, res
        bad = [k for k, v in res.items() if not v]
        assert not bad, (r, bad, res)
