"""The CPU oracle under AddressSanitizer and UndefinedBehaviorSanitizer (host
code only): oracle/asan_driver.c links oracle/sst_oracle.c built with
-fsanitize=address,undefined and calls every entry point the tests use
(is_valid, explain with and without the memo, the recursion, both length
bounds) on a canonical + modification alphabet.  A sanitizer report or a
leak fails the run.  TEST INFRASTRUCTURE: checks the checker."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no host C compiler")
def test_oracle_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "asan_driver")
    cmd = ["gcc", "-O1", "-g", "-fno-omit-frame-pointer", "-std=c11", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", "-Wno-unknown-pragmas", "-o", exe,
           os.path.join(REPO, "oracle", "asan_driver.c"), os.path.join(REPO, "oracle", "sst_oracle.c"), "-lm"]
    b = subprocess.run(cmd, capture_output=True, text=True)
    if b.returncode != 0 and "sanitize" in b.stderr:
        pytest.skip("gcc without the sanitizer runtimes: " + b.stderr[-300:])
    assert b.returncode == 0, b.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    assert r.stdout.startswith("checksum "), r.stdout
