"""Host-side sanitizer runs: the ASan + UBSan
builds of libtcbee_host (it parses untrusted pcap / .tcp input) and of the C
oracle, driven over valid, truncated and malformed files and random records by
tests/sanitize_driver.py in a child process with the sanitizer runtimes
preloaded (Python itself is not instrumented). UB aborts (-fno-sanitize-recover);
leak checking is off (the interpreter's own allocations). CPU only."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _runtime(name):
    try:
        p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True,
                           timeout=30).stdout.strip()
    except (OSError, subprocess.SubprocessError):
        return None
    return p if os.path.isabs(p) and os.path.exists(p) else None


def test_host_and_oracle_under_asan_ubsan():
    asan, ubsan = _runtime("libasan.so"), _runtime("libubsan.so")
    if not asan or not ubsan:
        pytest.skip("gcc sanitizer runtimes not installed")
    for d in (os.path.join(ROOT, "tcbee_amd", "host"), os.path.join(ROOT, "oracle")):
        subprocess.run(["make", "-C", d, "asan"], check=True, capture_output=True, timeout=600)
    host_lib = os.path.join(ROOT, "tcbee_amd", "lib", "libtcbee_host_asan.so")
    orc_lib = os.path.join(ROOT, "oracle", "liboracle_asan.so")
    env = dict(os.environ, LD_PRELOAD=f"{asan} {ubsan}",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               TCBEE_HOST_LIB=host_lib, TCBEE_ORACLE_LIB=orc_lib, TCBEE_NO_TORCH="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "sanitize_driver.py")],
                       env=env, capture_output=True, text=True, timeout=900)
    tail = (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0, tail
    assert "SANITIZE_OK" in r.stdout, tail
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, tail
    loaded = [ln for ln in r.stdout.splitlines() if ln.startswith("LOADED")][0]
    assert "libtcbee_host_asan.so" in loaded and "liboracle_asan.so" in loaded, loaded
