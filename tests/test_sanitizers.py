"""Race detection and memory checking of the C++ engine: the engine's
executor, plan cache, RPC server/client and counters are hammered from many threads
by csrc/tests/engine_selftest.cc, built with ThreadSanitizer and with
AddressSanitizer + UBSan (host code only; GPU sanitizers are not used)."""
import os
import subprocess

import pytest

from euler_amd import _build


@pytest.mark.parametrize("sanitizer", ["thread", "address"])
def test_engine_selftest_under_sanitizer(sanitizer):
    exe = _build.build_selftest(sanitizer)
    env = dict(os.environ)
    env["TSAN_OPTIONS"] = "halt_on_error=1 second_deadlock_stack=1"
    # the environment may preload a library of its own: tolerate it rather than touch it
    env["ASAN_OPTIONS"] = "detect_leaks=1 halt_on_error=1 verify_asan_link_order=0"
    env["UBSAN_OPTIONS"] = "halt_on_error=1 print_stacktrace=1"
    r = subprocess.run([exe, "8", "40"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "engine_selftest OK" in r.stdout
    assert "ThreadSanitizer" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
