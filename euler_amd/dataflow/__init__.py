"""Sampling dataflows (reference tf_euler/python/dataflow)."""
from euler_amd.dataflow.dataflows import *  # noqa: F401,F403
from euler_amd.dataflow.dataflows import __all__  # noqa: F401
