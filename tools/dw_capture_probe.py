#!/usr/bin/env python3
"""Stage-by-stage probe of the DeepWalk fixed-capacity step with a one-rank RCCL group:
init, eager static steps, capture, replays.  Prints after every stage (hang triage)."""
import os
import socket
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def say(*a):
    print(f"[{time.strftime('%X')}]", *a, flush=True)


def main():
    from euler_amd.graph.device_graph import DeviceGraph
    from euler_amd.models.deepwalk_step import DeepWalkTrainer

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    mode = sys.argv[1] if len(sys.argv) > 1 else "explicit"
    say("init", mode)
    if mode == "explicit":
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    else:
        os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
        dist.init_process_group("nccl", device_id=dev)
    say("init done")
    g = DeviceGraph.synthetic(20000, 8.0, 64, seed=3, device=dev)
    g.manual_seed(7)
    tr = DeepWalkTrainer(g, 20000, dim=64, batch_size=2048, lr=0.05, optimizer="adam", seed=5, force_comm=True,
                         static=True)
    for i in range(2):
        tr.step()
        torch.cuda.synchronize()
        say("eager step", i, float(tr.loss))
    tr.capture(warm=1)
    say("captured")
    for i in range(3):
        tr.step()
        torch.cuda.synchronize()
        say("replay", i, float(tr.loss))
    tr.table.check_overflow()
    tr.release()
    say("released")
    dist.destroy_process_group()
    say("done")


if __name__ == "__main__":
    main()
