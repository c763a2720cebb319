"""Reference module name ``tf_euler/python/utils/embedding.py``; the implementation lives in
:mod:`euler_amd.utils.misc`."""
from euler_amd.utils.misc import embedding_update, embedding_add  # noqa: F401
