import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")
    _ensure_built()


def _stale(targets, src_dirs, exts=(".hip", ".h", ".c", ".cpp", "Makefile")) -> bool:
    """A target missing, or older than any source it is built from (make's own rule for
    these link targets; object files are not consulted: tcbee_amd/csrc/build does not
    travel to the GPU box, whose snapshot keeps the built libraries and every mtime)."""
    if not all(os.path.exists(t) for t in targets):
        return True
    oldest = min(os.path.getmtime(t) for t in targets)
    for d in src_dirs:
        for n in os.listdir(d):
            if n.endswith(exts) and os.path.getmtime(os.path.join(d, n)) > oldest + 1.0:
                return True
    return False


def _ensure_built():
    """Build the oracle and the HIP / host libraries in-tree when a fresh checkout lacks
    them or a source is newer than the library (a stale library used to
    be tested as if it were the tree's)."""
    inc = os.path.join(ROOT, "include")
    oracle_dir = os.path.join(ROOT, "oracle")
    if _stale([os.path.join(oracle_dir, "liboracle.so")], [oracle_dir]):
        subprocess.run(["make", "-C", oracle_dir], check=True, stdout=subprocess.DEVNULL)
    csrc = os.path.join(ROOT, "tcbee_amd", "csrc")
    libs = [os.path.join(ROOT, "tcbee_amd", "lib", n)
            for n in ("libtcbee_amd.so", "libtcbee_amd_variants.so")]
    if _stale(libs, [csrc, inc]):
        subprocess.run(["make", "-C", csrc, "-j8"], check=True, stdout=subprocess.DEVNULL)
    hdir = os.path.join(ROOT, "tcbee_amd", "host")
    host = [os.path.join(ROOT, "tcbee_amd", "lib", "libtcbee_host.so"),
            os.path.join(ROOT, "tcbee_amd", "bin", "tcbee-record-gpu")]
    if _stale(host, [hdir, inc]):  # (the C host program links both)
        subprocess.run(["make", "-C", hdir], check=True, stdout=subprocess.DEVNULL)


def _have_gpu() -> bool:
    try:
        import tcbee_amd
        return tcbee_amd.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def oracle():
    from oracle_py import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def gpu():
    if not _have_gpu():
        pytest.fail("GPU test selected but no HIP device is visible")
    return 0


@pytest.fixture(scope="session")
def parser(gpu):
    import tcbee_amd
    p = tcbee_amd.PacketParser(device=0, max_frames=1 << 21, max_arena=1 << 28,
                               max_flows=1 << 18)
    yield p
    p.close()
