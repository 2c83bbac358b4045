"""The C-ABI's host-side argument checks under AddressSanitizer (SURVEY.md 5,
sanitizers): build_ext.py --asan compiles libmoe_hip's host code and
tools/capi_asan.cpp with -fsanitize=address; the driver hands every hot-path
entry point an invalid argument and requires a non-zero code plus a
moe_last_error() message, with no ASan report (out-of-bounds, use-after-free,
leaks).  No GPU: every call is rejected before a launch."""
from __future__ import annotations

import os
import subprocess

import pytest


@pytest.mark.timeout(1200)
def test_capi_argument_checks_under_asan():
    import build_ext

    driver = build_ext.build_asan_driver()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=23")
    r = subprocess.run([str(driver)], capture_output=True, text=True, timeout=300, env=env)
    assert "ERROR: AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert "LeakSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert " 0 failed" in r.stdout
