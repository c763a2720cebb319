"""Message-passing GNN nets (reference tf_euler/python/mp_utils)."""
from euler_amd.mp_utils.models import *  # noqa: F401,F403
from euler_amd.mp_utils.models import __all__  # noqa: F401
