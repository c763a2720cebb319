"""Network registry service: ``python -m euler_amd.tools.registry --port 2379``.

Holds the shard -> replica table for deployments without a shared filesystem (the role of
the reference's ZooKeeper ensemble, euler/common/zk_server_register.cc and
zk_server_monitor.cc).  Shard servers take ``--registry tcp://<host>:<port>`` and refresh
their entry every heartbeat; clients use the same spec in ``initialize_shared_graph`` and
see only entries refreshed within the TTL (csrc/rpc/rpc.cc RegistryServer / TcpRegistry).
"""
from __future__ import annotations

import argparse
import signal
import threading


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--port", type=int, default=0, help="0: ephemeral (printed)")
    args = p.parse_args(argv)
    from euler_amd import _engine

    srv = _engine.RegistryServer(args.port)
    print(f"registry listening on {srv.port}", flush=True)
    done = threading.Event()
    for sig in (signal.SIGINT, signal.SIGTERM):
        signal.signal(sig, lambda *_: done.set())
    done.wait()
    srv.stop()


if __name__ == "__main__":
    main()
