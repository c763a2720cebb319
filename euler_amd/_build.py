"""In-tree native build for euler_amd.

Two shared objects are produced next to the Python sources so that they travel
with a repo snapshot (``gpurun`` copies the tree, not a JIT cache):

* ``euler_amd/_engine*.so``  — the C++17 CPU graph engine (graph store, samplers,
  attribute indexes, GQL compiler + executor, RPC).  Plain pybind11 + numpy,
  no torch / HIP dependency, built with g++.
* ``euler_amd/_hip_ops*.so`` — hand-written CDNA4 (gfx950) HIP kernels plus the
  torch binding.  Every ``.hip`` file is compiled by ``hipcc --offload-arch=gfx950``
  directly (no hipify step, no CUDA sources), the binding links against the
  HIP runtime that ships inside torch (same soname, so one runtime per process).

The reference builds ``libeuler_core.so`` + ``libtf_euler.so`` with CMake
(``/root/reference/cmake/euler_core.cmake:1-144``, ``tf_euler/CMakeLists.txt:24-76``);
this file plays that role with an mtime-cached, parallel compile driver.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(ROOT)
# object files live outside the tree (only the linked .so files travel with a snapshot)
BUILD = os.environ.get("EULER_AMD_BUILD_DIR", os.path.join(os.path.expanduser("~"), ".cache", "euler_amd_build"))
CSRC = os.path.join(ROOT, "csrc")
ARCH = os.environ.get("EULER_AMD_ARCH", "gfx950")

_EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _log(msg: str) -> None:
    if os.environ.get("EULER_AMD_BUILD_QUIET") != "1":
        print(f"[euler_amd build] {msg}", file=sys.stderr, flush=True)


def _newest(paths) -> float:
    m = 0.0
    for p in paths:
        try:
            m = max(m, os.path.getmtime(p))
        except OSError:
            pass
    return m


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("command failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def _compile_all(jobs, max_workers):
    """jobs: list of (cmd, obj, deps_mtime, src)."""
    todo = []
    for cmd, obj, dep_m, src in jobs:
        if os.path.exists(obj) and os.path.getmtime(obj) >= max(dep_m, os.path.getmtime(src)):
            continue
        todo.append((cmd, obj, src))
    if not todo:
        return False
    with cf.ThreadPoolExecutor(max_workers=max_workers) as ex:
        futs = {ex.submit(_run, cmd): src for cmd, obj, src in todo}
        for f in cf.as_completed(futs):
            f.result()
            _log("compiled " + os.path.relpath(futs[f], REPO))
    return True


def _pybind_includes():
    import pybind11

    return [pybind11.get_include(), sysconfig.get_paths()["include"]]


# ----------------------------------------------------------------------------
# C++ engine (CPU)
# ----------------------------------------------------------------------------
ENGINE_DIRS = ["common", "graph", "index", "framework", "gql", "ops", "rpc", "pipeline", "bindings"]


def engine_sources():
    srcs = []
    for d in ENGINE_DIRS:
        srcs += sorted(glob.glob(os.path.join(CSRC, d, "*.cc")))
    return srcs


def engine_headers():
    hs = []
    for d in ENGINE_DIRS:
        hs += glob.glob(os.path.join(CSRC, d, "*.h"))
    return hs


def engine_target():
    return os.path.join(ROOT, "_engine" + _EXT_SUFFIX)


def build_engine(max_workers: int = 8, extra_flags=None) -> str:
    out = engine_target()
    objdir = os.path.join(BUILD, "engine")
    os.makedirs(objdir, exist_ok=True)
    flags = ["-O3", "-g1", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-pthread",
             "-fno-omit-frame-pointer", "-Wall", "-Wno-sign-compare", "-Wno-unused-function"]
    flags += list(extra_flags or [])
    inc = ["-I" + CSRC] + ["-I" + p for p in _pybind_includes()]
    hdr_m = _newest(engine_headers() + [__file__])
    if os.path.exists(out) and os.path.getmtime(out) >= max(hdr_m, _newest(engine_sources())):
        return out  # up to date (object files need not be present, e.g. on a fresh snapshot)
    jobs, objs = [], []
    for s in engine_sources():
        rel = os.path.relpath(s, CSRC).replace(os.sep, "_")
        o = os.path.join(objdir, rel + ".o")
        objs.append(o)
        jobs.append((["g++"] + flags + inc + ["-c", s, "-o", o], o, hdr_m, s))
    changed = _compile_all(jobs, max_workers)
    if changed or not os.path.exists(out) or os.path.getmtime(out) < _newest(objs):
        _run(["g++", "-shared", "-pthread", "-o", out] + objs)
        _log("linked " + os.path.relpath(out, REPO))
    return out


def console_target():
    return os.path.join(ROOT, "bin", "remote_console")


def build_console(max_workers: int = 8) -> str:
    """Native remote console (csrc/tools/remote_console.cc; reference
    euler/tools/remote_console): the engine objects (minus the pybind module) + main()."""
    build_engine(max_workers)
    out = console_target()
    objdir = os.path.join(BUILD, "engine")
    src = os.path.join(CSRC, "tools", "remote_console.cc")
    flags = ["-O2", "-std=c++17", "-pthread", "-Wall", "-Wno-sign-compare", "-I" + CSRC]
    obj = os.path.join(objdir, "tools_remote_console.cc.o")
    hdr_m = _newest(engine_headers() + [__file__])
    _compile_all([(["g++"] + flags + ["-c", src, "-o", obj], obj, hdr_m, src)], 1)
    objs = []
    for s in engine_sources():
        if os.sep + "bindings" + os.sep in s:
            continue
        o = os.path.join(objdir, os.path.relpath(s, CSRC).replace(os.sep, "_") + ".o")
        if not os.path.exists(o):  # engine .so was up to date but objects are gone: rebuild them
            _compile_all([(["g++", "-O3", "-std=c++17", "-fPIC", "-pthread", "-I" + CSRC] +
                           ["-I" + p for p in _pybind_includes()] + ["-c", s, "-o", o], o, hdr_m, s)], 1)
        objs.append(o)
    if not os.path.exists(out) or os.path.getmtime(out) < _newest(objs + [obj]):
        os.makedirs(os.path.dirname(out), exist_ok=True)
        _run(["g++", "-pthread", "-o", out, obj] + objs + ["-ldl"])
        _log("linked " + os.path.relpath(out, REPO))
    return out


_SANITIZERS = {
    "thread": ["-fsanitize=thread"],
    "address": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
    "none": [],
}


def build_selftest(sanitize: str = "thread", max_workers: int = 8) -> str:
    """Engine self-test binary (csrc/tests/engine_selftest.cc) under a sanitizer:
    ``thread`` (TSAN) or ``address`` (ASAN + UBSan).  Host code only; the pybind
    module is not part of it.  Returns the binary path (mtime-cached under build/)."""
    if sanitize not in _SANITIZERS:
        raise ValueError("sanitize must be one of %s" % sorted(_SANITIZERS))
    objdir = os.path.join(BUILD, "selftest_" + sanitize)
    os.makedirs(objdir, exist_ok=True)
    out = os.path.join(objdir, "engine_selftest")
    san = _SANITIZERS[sanitize]
    flags = ["-O1", "-g", "-std=c++17", "-pthread", "-fno-omit-frame-pointer", "-Wno-sign-compare"] + san
    srcs = [s for s in engine_sources() if os.sep + "bindings" + os.sep not in s]
    srcs.append(os.path.join(CSRC, "tests", "engine_selftest.cc"))
    hdr_m = _newest(engine_headers() + [__file__])
    jobs, objs = [], []
    for s in srcs:
        rel = os.path.relpath(s, CSRC).replace(os.sep, "_")
        o = os.path.join(objdir, rel + ".o")
        objs.append(o)
        jobs.append((["g++"] + flags + ["-I" + CSRC, "-c", s, "-o", o], o, hdr_m, s))
    changed = _compile_all(jobs, max_workers)
    if changed or not os.path.exists(out) or os.path.getmtime(out) < _newest(objs):
        _run(["g++"] + san + ["-pthread", "-o", out] + objs + ["-ldl"])
        _log("linked " + os.path.relpath(out, REPO))
    return out


# ----------------------------------------------------------------------------
# HIP kernels (gfx950) + torch binding
# ----------------------------------------------------------------------------
def hip_target():
    return os.path.join(ROOT, "_hip_ops" + _EXT_SUFFIX)


def _torch_paths():
    import torch

    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    return tdir, inc, os.path.join(tdir, "lib"), bool(torch._C._GLIBCXX_USE_CXX11_ABI)


def build_hip(max_workers: int = 8) -> str:
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    out = hip_target()
    objdir = os.path.join(BUILD, "hip")
    os.makedirs(objdir, exist_ok=True)
    tdir, tinc, tlib, abi = _torch_paths()
    hdir = os.path.join(CSRC, "hip")
    kernels = sorted(glob.glob(os.path.join(hdir, "*.hip")))
    bindings = sorted(glob.glob(os.path.join(hdir, "*.cpp")))
    hdrs = glob.glob(os.path.join(hdir, "*.h")) + [__file__]
    hdr_m = _newest(hdrs)
    if os.path.exists(out) and os.path.getmtime(out) >= max(hdr_m, _newest(kernels + bindings)):
        return out
    kflags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
              "-D__HIP_PLATFORM_AMD__=1", "-I" + CSRC, "-Wno-unused-result"]
    kflags += os.environ.get("EULER_AMD_HIP_FLAGS", "").split()  # tuning experiments (-DNAME=value)
    bflags = ["-O2", "-std=c++17", "-fPIC", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
              f"-D_GLIBCXX_USE_CXX11_ABI={int(abi)}", "-DTORCH_API_INCLUDE_EXTENSION_H",
              "-DTORCH_EXTENSION_NAME=_hip_ops", "-I" + CSRC, "-I/opt/rocm/include",
              "-Wno-unused-result", "-Wno-deprecated-declarations"]
    bflags += ["-I" + p for p in tinc + _pybind_includes()]
    jobs, objs = [], []
    for s in kernels:
        o = os.path.join(objdir, os.path.basename(s) + ".o")
        objs.append(o)
        jobs.append(([hipcc] + kflags + ["-c", s, "-o", o], o, hdr_m, s))
    for s in bindings:
        o = os.path.join(objdir, os.path.basename(s) + ".o")
        objs.append(o)
        # host-only translation unit: torch headers + HIP runtime API, no device code
        jobs.append((["g++"] + bflags + ["-c", s, "-o", o], o, hdr_m, s))
    changed = _compile_all(jobs, max_workers)
    if changed or not os.path.exists(out) or os.path.getmtime(out) < _newest(objs):
        link = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out] + objs + [
            "-L" + tlib, "-Wl,-rpath," + tlib, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
            "-ltorch_hip", "-ltorch_python", "-lamdhip64"]
        _run(link)
        _log("linked " + os.path.relpath(out, REPO))
    return out


def build_all(max_workers: int = 8) -> None:
    if engine_sources():
        build_engine(max_workers)
        build_console(max_workers)
    build_hip(max_workers)


if __name__ == "__main__":
    what = sys.argv[1:] or ["all"]
    if "all" in what:
        build_all()
    else:
        if "engine" in what:
            build_engine()
        if "hip" in what:
            build_hip()
        if "console" in what:
            build_console()
