"""Graph shard server launcher (reference ``euler/python/start_service.py``).

    python -m euler_amd.tools.service --data_path DIR --shard_idx 0 --shard_num 2 \
        --registry /shared/registry_dir [--port 0] [--threads 32]

Loads shard ``shard_idx`` of a reference-format graph directory (files whose
partition p satisfies p % shard_num == shard_idx), starts the RPC server, writes
"<shard>#<host>:<port>" + shard meta into the registry and serves until SIGTERM /
SIGINT (the entry is removed on exit so clients stop routing to it; the server refreshes
it every --heartbeat_ms so that after a SIGKILL clients drop it once it is older than
their registry_ttl).  --module / --load_data_type / --global_sampler_type choose the
loaded tables and global samplers (reference start_service.py Module flags).
"""
from __future__ import annotations

import argparse
import signal
import sys
import threading


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--data_path", required=True)
    p.add_argument("--shard_idx", type=int, default=0)
    p.add_argument("--shard_num", type=int, default=1)
    p.add_argument("--registry", default="", help="registry directory (or memory:<name>)")
    p.add_argument("--zk_path", default="", help="alias of --registry (reference flag name)")
    p.add_argument("--port", type=int, default=0)
    p.add_argument("--threads", type=int, default=32)
    p.add_argument("--host", default="127.0.0.1")
    p.add_argument("--module", type=int, default=None,
                   help="reference Module flags: NODE=1 EDGE=2 NODE_SAMPLER=4 EDGE_SAMPLER=8 (OR-ed)")
    p.add_argument("--load_data_type", default=None, choices=["none", "node", "edge", "all"])
    p.add_argument("--global_sampler_type", default=None, choices=["none", "node", "edge", "all"])
    p.add_argument("--heartbeat_ms", type=int, default=1000, help="registry entry refresh period")
    a = p.parse_args(argv)
    from euler_amd.ops.base import start_service

    srv = start_service(a.data_path, a.shard_idx, a.shard_num, a.registry or a.zk_path, a.port, a.threads, a.host,
                        module=a.module, load_data_type=a.load_data_type, global_sampler_type=a.global_sampler_type,
                        heartbeat_ms=a.heartbeat_ms)
    print("euler_amd graph server shard %d/%d on port %d" % (a.shard_idx, a.shard_num, srv.port), flush=True)
    done = threading.Event()

    def stop(*_):
        done.set()

    signal.signal(signal.SIGTERM, stop)
    signal.signal(signal.SIGINT, stop)
    while not done.wait(0.5):
        pass
    srv.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
