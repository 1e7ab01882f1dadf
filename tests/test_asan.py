"""Host-code AddressSanitizer + UBSan run.

hummingbird_amd/build.py build_asan() builds libhbec with the sanitizers on
the host code only (device code is not instrumented; this pool runs no GPU
ASan) plus the C driver tests/native/host_asan.c.  The test runs the
host-only entry points.  (A GPU variant existed until round 5; the sanitizer
build does not travel to the GPU box, so it could only ever skip there.)"""
import os
import subprocess

import pytest

from hummingbird_amd import build as Bd

ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:protect_shadow_gap=0:abort_on_error=0",
           UBSAN_OPTIONS="print_stacktrace=1")


def _exe():
    if not Bd.ASAN_EXE.exists():
        pytest.skip("sanitizer build missing: run __graft_entry__.build()")
    return str(Bd.ASAN_EXE)


def test_host_asan_cpu():
    out = subprocess.run([_exe()], capture_output=True, text=True, env=ENV, timeout=120)
    assert out.returncode == 0, out.stderr[-4000:]
    assert "host_asan cpu ok" in out.stdout

