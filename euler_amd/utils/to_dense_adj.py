"""Reference module name ``tf_euler/python/utils/to_dense_adj.py``; the implementation lives in
:mod:`euler_amd.utils.misc`."""
from euler_amd.utils.misc import to_dense_adj  # noqa: F401
