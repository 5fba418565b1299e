"""The oracle under AddressSanitizer + UndefinedBehaviorSanitizer (host only): oracle/asan_check.c
builds tables with the oracle Builder, then parses, opens, decodes and merges them -- valid, and
with random corruption, truncation and undersized outputs -- in a sanitized build.  Every GPU
parity test trusts these readers, so an over-read here would hide everywhere else."""
import os
import subprocess

import pytest

ORACLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")


def test_oracle_under_asan():
    mk = subprocess.run(["make", "-C", ORACLE, "-s", "build/asan_check"], capture_output=True,
                        text=True, timeout=300)
    if mk.returncode != 0 and "asan" in (mk.stderr + mk.stdout).lower():
        pytest.skip("no sanitizer runtime for the host compiler: " + mk.stderr[-300:])
    assert mk.returncode == 0, mk.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    run = subprocess.run([os.path.join(ORACLE, "build", "asan_check"), "120"], capture_output=True,
                         text=True, timeout=300, env=env)
    assert run.returncode == 0, (run.stdout[-1000:], run.stderr[-4000:])
    assert "0 failures" in run.stdout
