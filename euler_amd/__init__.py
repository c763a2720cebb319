"""euler_amd — an MI355X-native large-scale graph-learning framework with the
capabilities of Euler-2.0 (renyi533/euler).

Layers:
  * C++ engine (``euler_amd._engine``): sharded columnar graph store, attribute
    indexes, GQL compiler + dataflow executor, RPC graph servers;
  * graph-query API with the reference's ``tf_euler`` names (this module's top level);
  * message passing on hand-written gfx950 HIP kernels (``euler_amd.ops``), the
    convolution / dataflow / encoder / solution libraries, estimators and the
    model zoo, data parallelism and sharded embeddings over RCCL (``euler_amd.parallel``).
"""
__version__ = "0.1.0"

import os as _os

# dmabuf IPC, the only mode the host driver supports: RCCL and the xGMI all-reduce's peer
# mappings fail without it ("hipIpcGetMemHandle: invalid argument").  Set before the
# package (or a script importing it first) loads torch / HIP, so every entry point —
# tools/runner.py, the examples, the benchmarks under torchrun — gets it.
_os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

from euler_amd.ops.base import (  # noqa: F401
    GraphBuilder, Module, get_engine, initialize_embedded_graph, initialize_graph, initialize_shared_graph, set_seed,
    start, start_service, synthetic_graph, use_graph)
from euler_amd.ops.graph_api import *  # noqa: F401,F403
from euler_amd.ops.graph_api import __all__ as _graph_all
# message-passing ops (reference tf_euler euler_ops/mp_ops.py re-exported at top level)
from euler_amd.ops.mp_ops import gather, scatter_, scatter_add, scatter_max, scatter_mean, scatter_softmax  # noqa: F401


__all__ = ["initialize_graph", "initialize_embedded_graph", "initialize_shared_graph", "use_graph", "get_engine",
           "set_seed", "synthetic_graph", "GraphBuilder", "Module", "start_service", "start", "gather", "scatter_",
           "scatter_add", "scatter_max", "scatter_mean", "scatter_softmax"] + list(_graph_all)
