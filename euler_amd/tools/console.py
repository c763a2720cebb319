"""Interactive console against a live (remote / sharded / local) graph
(reference ``euler/tools/remote_console/remote_console.cc:27-157``).

Commands (one per line; ``help`` lists them)::

    query_nb <node_id> <edge_type>            full out-neighbours (ids, weights, types)
    query_sp_fea <node_id> <feature_name>     sparse feature values
    query_dense_fea <node_id> <feature_name>  dense feature values
    query_bin_fea <node_id> <feature_name>    binary feature bytes
    sample_nb <node_id> <edge_type> <count>   weighted neighbour sampling
    gql <query> [-- key=v1,v2 ...]            run a GQL query (uint64 inputs), print every output
    explain <query>                           the compiled (physical) DAG
    meta | stats | quit

Usage::

    python -m euler_amd.tools.console --registry /shared/reg --shard_num 2   # remote shards
    python -m euler_amd.tools.console --data_path /data/euler                # embedded graph

The reference prompted for ``zk_addr``/``zk_path``/``shard_num`` on stdin; here they are
flags (the registry directory replaces ZooKeeper).
"""
from __future__ import annotations

import argparse
import re
import shlex
import sys

import numpy as np

import euler_amd as ea
from euler_amd.utils import trace

HELP = __doc__.split("Commands (one per line; ``help`` lists them)::")[1].split("Usage::")[0]


def _print(label, arr):
    a = np.asarray(arr)
    print("%s: %s" % (label, " ".join(str(x) for x in a.reshape(-1).tolist())))


def handle(line: str, out=print) -> bool:
    """Execute one console command; returns False on quit."""
    parts = shlex.split(line)
    if not parts:
        return True
    cmd, args = parts[0], parts[1:]
    if cmd in ("quit", "exit"):
        return False
    if cmd == "help":
        out(HELP)
    elif cmd == "query_nb":
        ids, w, t = ea.get_full_neighbor([int(args[0])], [args[1]])
        _print("nb", ids.values)
        _print("weights", w.values)
        _print("types", t.values)
    elif cmd == "query_sp_fea":
        sp = ea.get_sparse_feature([int(args[0])], [args[1]])[0]
        _print("feature", sp.values)
    elif cmd == "query_dense_fea":
        feats = ea.get_engine().meta().get("node_features", {})  # name -> (type, index, dim)
        dim = int(args[2]) if len(args) > 2 else int(feats.get("dense_" + args[1], (0, 0, 1))[2])
        _print("feature", ea.get_dense_feature([int(args[0])], [args[1]], [dim])[0])
    elif cmd == "query_bin_fea":
        out("feature: %r" % (ea.get_binary_feature([int(args[0])], [args[1]])[0][0],))
    elif cmd == "sample_nb":
        ids, w, t = ea.sample_neighbor([int(args[0])], [args[1]], int(args[2]))
        _print("nb", ids)
        _print("weights", w)
    elif cmd == "gql":
        # gql v(nodes).outV(et).as(nb) -- nodes=1,2 et=0 [out=nb:1,nb:2]
        q, _, rest = " ".join(args).partition("--")
        inputs, outs = {}, None
        for kv in rest.split():
            k, v = kv.split("=", 1)
            if k == "out":
                outs = v.split(",")
            elif k in ("et", "edge_types", "e_types"):
                inputs[k] = np.asarray([int(x) for x in v.split(",")], dtype=np.int32)
            else:
                inputs[k] = np.asarray([int(x) for x in v.split(",")], dtype=np.uint64)
        if outs is None:
            aliases = re.findall(r"\.as\((\w+)\)", q)
            outs = ["%s:%d" % (aliases[-1], i) for i in range(2)] if aliases else []
        res = ea.run_gql(q.strip(), inputs, outs) if outs else []
        for name, val in zip(outs, res):
            _print(name, val)
    elif cmd == "explain":
        out(ea.explain_gql(" ".join(args)))
    elif cmd == "meta":
        out(str(ea.get_engine().meta()))
    elif cmd == "stats":
        out(str(trace.engine_stats()))
    else:
        out("unknown command %r (try help)" % cmd)
    return True


def main(argv=None):
    p = argparse.ArgumentParser(description="euler_amd graph console")
    p.add_argument("--registry", default=None, help="shared registry directory of the shard servers")
    p.add_argument("--shard_num", type=int, default=0)
    p.add_argument("--data_path", default=None, help="embedded graph directory (local mode)")
    a = p.parse_args(argv)
    if a.data_path:
        ea.initialize_embedded_graph(a.data_path)
    elif a.registry:
        ea.initialize_shared_graph(a.registry, shard_num=a.shard_num)
    else:
        p.error("give --registry (remote shards) or --data_path (embedded graph)")
    print("connected; type help for commands")
    for line in sys.stdin:
        try:
            if not handle(line.strip()):
                break
        except Exception as e:  # keep the console alive on bad input
            print("error: %s" % e)


if __name__ == "__main__":
    main()
