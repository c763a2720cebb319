"""Reference module name ``tf_euler/python/utils/hooks.py``; the implementation lives in
:mod:`euler_amd.utils.misc`."""
from euler_amd.utils.misc import SyncExitHook  # noqa: F401
