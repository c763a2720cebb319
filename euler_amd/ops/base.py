"""Graph-engine session for the Python API (reference ``tf_euler/python/euler_ops/base.py``).

``initialize_graph(config)`` takes a dict or a ``"k=v;k=v"`` string, exactly like the
reference (``base.py:37-60``); keys: ``mode`` (local | remote | local_sharded),
``data_path``, ``shard_num``, ``registry`` (shared directory or ``memory:<name>``; the
reference's ``zk_server``/``zk_path`` are accepted and mapped to it), ``num_retries``,
``bad_host_timeout``, ``num_channels_per_host``, ``seed``.

Besides reference-format directories an engine can also adopt an in-process graph
(``use_graph``): a ``GraphBuilder`` result or the native synthetic generator.
"""
from __future__ import annotations

import threading

from euler_amd.ops._native import engine as _engine_mod

__all__ = ["initialize_graph", "initialize_embedded_graph", "initialize_shared_graph", "get_engine",
           "use_graph", "set_seed", "synthetic_graph", "GraphBuilder", "start_service"]

_ENGINE = None
_LOCK = threading.Lock()


def _parse(config):
    if isinstance(config, dict):
        return {str(k): str(v) for k, v in config.items()}
    if isinstance(config, bytes):
        config = config.decode()
    if not isinstance(config, str):
        raise TypeError("Expect str or dict for graph config, got {}.".format(type(config).__name__))
    out = {}
    for kv in config.split(";"):
        if "=" in kv:
            k, v = kv.split("=", 1)
            out[k.strip()] = v.strip()
    return out


def initialize_graph(config) -> bool:
    global _ENGINE
    cfg = _parse(config)
    if "registry" not in cfg and "zk_path" in cfg:
        cfg["registry"] = cfg["zk_path"]
    eng = _engine_mod().Engine.from_config(cfg)
    with _LOCK:
        _ENGINE = eng
    return True


def initialize_embedded_graph(data_dir, sampler_type="all", data_type="all") -> bool:
    return initialize_graph({"mode": "local", "data_path": data_dir, "data_type": data_type,
                             "sampler_type": sampler_type})


def initialize_shared_graph(data_dir_or_registry, zk_addr=None, zk_path=None, shard_num=0, **kw) -> bool:
    """Remote mode.  ``zk_path`` / the first argument name the shared registry directory."""
    reg = zk_path or data_dir_or_registry
    cfg = {"mode": "remote", "registry": reg, "shard_num": shard_num, "num_retries": kw.get("num_retries", 1)}
    cfg.update({k: v for k, v in kw.items() if k != "num_retries"})
    return initialize_graph(cfg)


def use_graph(engine_obj):
    """Make an already-built engine (builder / synthetic) the current graph."""
    global _ENGINE
    with _LOCK:
        _ENGINE = engine_obj
    return engine_obj


def get_engine():
    if _ENGINE is None:
        raise RuntimeError("graph not initialized: call euler_amd.initialize_graph(...) first")
    return _ENGINE


_WALK_SEED = [0x9E3779B97F4A7C15, 0]  # (global seed, calls): per-call walk seeds


def set_seed(seed: int):
    """Seed the engine's samplers and the per-call seeds of the walk ops."""
    _engine_mod().set_seed(int(seed))
    _WALK_SEED[0], _WALK_SEED[1] = int(seed), 0


def next_walk_seed() -> int:
    """A fresh, reproducible seed for one walk call (a function of the global seed and the
    number of calls since it was set)."""
    _WALK_SEED[1] += 1
    x = (_WALK_SEED[0] * 0x9E3779B97F4A7C15 + _WALK_SEED[1] * 0xBF58476D1CE4E5B9) & (2 ** 64 - 1)
    x ^= x >> 31
    return x & (2 ** 63 - 1)


def synthetic_graph(num_nodes, avg_degree=10.0, max_degree=1024, node_types=1, edge_types=1, feature_dim=0,
                    label_dim=0, seed=0, make_current=True, out_only=False):
    """Power-law synthetic graph inside the C++ engine.  ``out_only`` keeps only the out
    CSR (no in-adjacency / edge table): enough for neighbour sampling at 100M-node scale."""
    e = _engine_mod().synthetic(int(num_nodes), float(avg_degree), int(max_degree), int(node_types),
                                int(edge_types), int(feature_dim), int(label_dim), int(seed), bool(out_only))
    if make_current:
        use_graph(e)
    return e


def GraphBuilder():
    return _engine_mod().GraphBuilder()


class Module:
    """What a shard server loads and which global samplers it builds (reference
    ``euler/python/start_service.py:33-67``): data tables NODE / EDGE, samplers
    NODE_SAMPLER / EDGE_SAMPLER, OR-ed together."""
    NODE = 1
    EDGE = 2
    NODE_SAMPLER = 4
    EDGE_SAMPLER = 8
    DEFAULT_MODULE = NODE | NODE_SAMPLER

    @staticmethod
    def _two(module, a, b):
        m = module & (a | b)
        return {0: "none", a: "node", b: "edge", a | b: "all"}[m]

    @classmethod
    def to_load_data_type_string(cls, module):
        return cls._two(int(module), cls.NODE, cls.EDGE)

    @classmethod
    def to_global_sampler_type_string(cls, module):
        return cls._two(int(module), cls.NODE_SAMPLER, cls.EDGE_SAMPLER)


def start_service(data_path, shard_idx, shard_num, registry="", port=0, threads=32, host="127.0.0.1",
                  module=None, load_data_type=None, global_sampler_type=None, heartbeat_ms=1000):
    """Start a graph shard server in this process.  ``module`` (Module flags) or the
    explicit ``load_data_type`` / ``global_sampler_type`` strings ("none" / "node" /
    "edge" / "all") select the loaded tables and global samplers (default: everything);
    the registry entry is refreshed every ``heartbeat_ms`` (clients drop entries older
    than their ``registry_ttl``)."""
    if module is not None:
        load_data_type = load_data_type or Module.to_load_data_type_string(module)
        global_sampler_type = global_sampler_type or Module.to_global_sampler_type_string(module)
    return _engine_mod().GraphServer(data_path, int(shard_idx), int(shard_num), registry, int(port), int(threads),
                                     host, load_data_type or "all", global_sampler_type or "all", int(heartbeat_ms))


def start(directory="", shard_idx=0, shard_num=1, zk_addr="", zk_path="", module=Module.DEFAULT_MODULE,
          server_thread_num=None):
    """Reference ``euler.start`` signature (``euler/python/start_service.py:70-80``): the
    ZooKeeper path names the shared registry directory here."""
    import multiprocessing

    reg = zk_path or zk_addr
    return start_service(directory, shard_idx, shard_num, reg, 0, int(server_thread_num or multiprocessing.cpu_count()),
                         module=module)
