"""Reference module name ``tf_euler/python/utils/flags.py``; the implementation lives in
:mod:`euler_amd.utils.misc`."""
from euler_amd.utils.misc import FLAGS, set_defaults  # noqa: F401
