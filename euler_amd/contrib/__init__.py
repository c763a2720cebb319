"""Alternate message-passing back ends (reference ``tf_euler/python/contrib``).

The reference kept two fallbacks next to its main MP ops: ``spmm.py`` (aggregation as a
``tf.SparseTensor`` x dense matmul, ``contrib/spmm.py:23-41``) and ``py_scatter.py``
(numpy ``py_func`` scatters with hand-registered gradients, ``contrib/py_scatter.py:25-58``).
Here both names exist for drop-in parity, but neither is a separate slow path: every
function routes to the same gfx950 kernels as :mod:`euler_amd.ops.mp_ops` (CSR SpMM and
segment reduce), so switching back ends changes nothing about speed or numerics.
"""
from euler_amd.contrib import py_scatter, spmm  # noqa: F401
from euler_amd.contrib.spmm import spmm_, spmm_add, spmm_mean  # noqa: F401

__all__ = ["spmm", "py_scatter", "spmm_", "spmm_add", "spmm_mean"]
