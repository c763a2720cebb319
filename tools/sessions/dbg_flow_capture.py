"""where the sampled sharded flow's capture stops (faulthandler dumps every 40 s)"""
import faulthandler
import os
import sys

_ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path[:0] = [_ROOT, os.path.join(_ROOT, "tests")]
faulthandler.dump_traceback_later(40, repeat=True)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from test_parallel import _free_port  # noqa: E402
from test_sharded_graph import _graph  # noqa: E402

from euler_amd import models as Z  # noqa: E402
from euler_amd.dataflow.device_flow import DeviceSageFlow  # noqa: E402
from euler_amd.graph.sharded_graph import ShardedDeviceGraph  # noqa: E402
from euler_amd.models.full_trainer import ShardedFlowTrainer  # noqa: E402

dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
g, indptr, nbr, w, nw = _graph(device="cuda")
sg = ShardedDeviceGraph.from_full(g, force_comm=True, node_weights=nw)
torch.manual_seed(0)
m = Z.SupervisedGNN("gcn", "sage", [16, 16, 3], [4, 3], [[0], [0]], "f", 12, "l", 3, max_id=300).cuda()
tr = ShardedFlowTrainer(m, sg, 32, DeviceSageFlow(sg, [None, None], [4, 3], 32, True))
print("built", flush=True)
tr.step()
torch.cuda.synchronize()
print("eager ok", float(tr.loss.item()), flush=True)
mode = sys.argv[1] if len(sys.argv) > 1 else "warm"
tr.capture(None, warmup=0 if mode == "cold" else 2, steps=1)
print("captured", flush=True)
tr.replay(3)
torch.cuda.synchronize()
print("replayed", float(tr.loss.item()), flush=True)
tr.release_graphs()
dist.destroy_process_group()
print("done", flush=True)
