"""Reference module name ``tf_euler/python/utils/to_dense_batch.py``; the implementation lives in
:mod:`euler_amd.utils.misc`."""
from euler_amd.utils.misc import to_dense_batch  # noqa: F401
