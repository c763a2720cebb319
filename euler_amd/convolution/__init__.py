"""Graph convolutions (reference tf_euler/python/convolution)."""
from euler_amd.convolution.convs import *  # noqa: F401,F403
from euler_amd.convolution.convs import __all__  # noqa: F401
