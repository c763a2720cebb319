"""Loaders for the two native extensions.

``hip()`` returns the gfx950 kernel module.  On a machine with a GPU the kernels
are the ONLY compute path for the ops that have them: if the extension is
missing we raise instead of silently falling back to eager torch, so a GPU run
can never pass on a fallback (set ``EULER_AMD_ALLOW_FALLBACK=1`` to opt out, e.g.
for debugging).  On CPU-only hosts the pure-torch reference implementations in
the op modules are used (they are also the numerics oracle in tests).
"""
from __future__ import annotations

import importlib
import os

_HIP = None
_ENGINE = None


class NativeExtensionMissing(RuntimeError):
    pass


def _try_build(target: str) -> None:
    if os.environ.get("EULER_AMD_NO_AUTOBUILD") == "1":
        return
    from euler_amd import _build

    if target == "hip":
        _build.build_hip()
    else:
        _build.build_engine()


def hip():
    """Return the ``euler_amd._hip_ops`` module (building it in-tree if needed)."""
    global _HIP
    if _HIP is None:
        import torch  # noqa: F401  (loads torch's HIP runtime first: one runtime per process)

        try:
            _HIP = importlib.import_module("euler_amd._hip_ops")
        except ImportError:
            _try_build("hip")
            try:
                _HIP = importlib.import_module("euler_amd._hip_ops")
            except ImportError as e:  # pragma: no cover - only on broken installs
                raise NativeExtensionMissing(
                    "euler_amd._hip_ops is not built; run `python -m euler_amd._build hip`") from e
    return _HIP


def engine():
    """Return the ``euler_amd._engine`` module (C++ graph engine)."""
    global _ENGINE
    if _ENGINE is None:
        try:
            _ENGINE = importlib.import_module("euler_amd._engine")
        except ImportError:
            _try_build("engine")
            _ENGINE = importlib.import_module("euler_amd._engine")
    return _ENGINE


def use_hip(*tensors) -> bool:
    """True when the HIP kernels must run for these tensors (all on a GPU)."""
    if not tensors:
        return False
    on_gpu = all(getattr(t, "is_cuda", False) for t in tensors if t is not None)
    if not on_gpu:
        return False
    if os.environ.get("EULER_AMD_ALLOW_FALLBACK") == "1":
        try:
            hip()
        except NativeExtensionMissing:
            return False
    return True
