"""Graph pooling (reference tf_euler/python/graph_pool)."""
from euler_amd.graph_pool.pools import *  # noqa: F401,F403
from euler_amd.graph_pool.pools import __all__  # noqa: F401
