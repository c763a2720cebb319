"""Graph shard server launcher (reference ``euler/python/start_service.py``).

    python -m euler_amd.tools.service --data_path DIR --shard_idx 0 --shard_num 2 \
        --registry /shared/registry_dir [--port 0] [--threads 32]

Loads shard ``shard_idx`` of a reference-format graph directory (files whose
partition p satisfies p % shard_num == shard_idx), starts the RPC server, writes
"<shard>#<host>:<port>" + shard meta into the registry and serves until SIGTERM /
SIGINT (the entry is removed on exit so clients stop routing to it).
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
    a = p.parse_args(argv)
    from euler_amd.ops.base import start_service

    srv = start_service(a.data_path, a.shard_idx, a.shard_num, a.registry or a.zk_path, a.port, a.threads, a.host)
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
