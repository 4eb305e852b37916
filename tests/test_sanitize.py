"""Host sanitizers (ASan + UBSan), CPU only (GPU sanitizers are not available
on the pool):
* the CPU oracle: oracle/sanitize_main.cpp drives every oracle entry point the
  parity tests use, multi-threaded sweep included;
* the product library's host code (fantoch_amd/csrc/bote_host.cpp: colex
  ranks, the group walk and its chunk/shard cuts, quad layouts, result
  unpacking): tests/native/host_check.cpp checks each against a direct
  restatement."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_oracle_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", ORACLE, "build/oracle_sanitize"], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([os.path.join(ORACLE, "build", "oracle_sanitize")], capture_output=True, text=True,
                       env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "calls ok" in r.stdout and "error path ok" in r.stdout, r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_library_host_code_under_asan_ubsan():
    native = os.path.join(ROOT, "tests", "native")
    subprocess.run(["make", "-s", "-C", native, "build/host_check"], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([os.path.join(native, "build", "host_check")], capture_output=True, text=True, env=env,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host ok" in r.stdout, r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr
