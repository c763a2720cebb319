"""Reference module name ``tf_euler/python/utils/optimizers.py``; the implementation lives in
:mod:`euler_amd.utils.misc`."""
from euler_amd.utils.misc import get_optimizer, optimizers  # noqa: F401
