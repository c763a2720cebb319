#!/usr/bin/env python3
"""One-rank probe of DeepWalkTrainer(micro_batches=2) through the all-to-all path: eager
steps, then capture + replay, on a small graph; prints each phase so a crash names it.
Run: RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 python -X faulthandler tools/dw_overlap_probe.py"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    from euler_amd.graph.device_graph import DeviceGraph
    from euler_amd.models.deepwalk_step import DeepWalkTrainer

    g = DeviceGraph.synthetic(20000, 6.0, 64, seed=3, device=dev)
    mode = sys.argv[1] if len(sys.argv) > 1 else "both"
    tr = DeepWalkTrainer(g, 20000, dim=32, batch_size=256, lr=0.05, optimizer="adagrad", seed=5, static=True,
                         force_comm=True, micro_batches=2)
    print("eager step 1", flush=True)
    l = tr.step()
    torch.cuda.synchronize()
    print("eager loss", float(l), flush=True)
    for _ in range(3):
        tr.step()
    torch.cuda.synchronize()
    print("eager ok", flush=True)
    if mode in ("both", "graph"):
        tr.capture(warm=1)
        print("captured", flush=True)
        for _ in range(5):
            tr.step()
        torch.cuda.synchronize()
        print("replay loss", float(tr.loss), flush=True)
        tr.release()
    tr.table.check_overflow()
    dist.barrier()
    dist.destroy_process_group()
    print("probe ok", flush=True)


if __name__ == "__main__":
    main()
