"""Per-call time of the xGMI two-shot all-reduce (parallel/xgmi.py) next to RCCL's
all_reduce on the headline gradient sizes, both replayed from a hipGraph of 100 calls.

One rank:   python tools/xgmi_bench.py
N ranks:    torchrun --nproc-per-node N --master-addr 127.0.0.1 tools/xgmi_bench.py
            (--shared-gpu: every rank on cuda:0, gloo group, xGMI path only)
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, calls, reps):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        for _ in range(calls):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        if dist.is_initialized():
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / calls * 1e6)
    del g
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shared-gpu", action="store_true")
    ap.add_argument("--calls", type=int, default=100)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--numel", type=int, nargs="+", default=[278784])
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.shared_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29581")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    if args.shared_gpu:
        dist.init_process_group("gloo")
    else:
        dist.init_process_group("nccl", device_id=dev)
    from euler_amd.parallel.xgmi import XgmiAllReduce, _blocks_for

    cap = max(args.numel) * 4
    ar = XgmiAllReduce(cap, timeout_s=5.0)
    assert ar.self_test(numel=max(args.numel), dtype=torch.float32)
    out = {"world": world, "shared_gpu": args.shared_gpu, "blocks_env": os.environ.get("EULER_AMD_XAR_BLOCKS"),
           "uncached_data": os.environ.get("EULER_AMD_HIP_FLAGS", "")}
    for n in args.numel:
        for dt in (torch.float32, torch.bfloat16):
            x = torch.randn(n, device=dev).to(dt)
            key = f"{n}_{str(dt)[6:]}"
            out[f"xgmi_us_{key}"] = round(timed(lambda: ar(x), args.calls, args.reps), 2)
            xi = ar.input_view(n, dt).copy_(x)  # in place: the producer wrote the IPC region
            out[f"xgmi_inplace_us_{key}"] = round(timed(lambda: ar(xi), args.calls, args.reps), 2)
            out[f"xgmi_blocks_{key}"] = _blocks_for(n, world, x.element_size())
            if not args.shared_gpu:
                out[f"rccl_us_{key}"] = round(timed(lambda: dist.all_reduce(x), args.calls, args.reps), 2)
    out["error"] = ar.error()
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
