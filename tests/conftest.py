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


def _ensure_built():
    """Build the oracle and the HIP library in-tree if a fresh checkout lacks them."""
    oracle_so = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(oracle_so):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True,
                       stdout=subprocess.DEVNULL)
    libs = [os.path.join(ROOT, "tcbee_amd", "lib", n)
            for n in ("libtcbee_amd.so", "libtcbee_amd_variants.so")]
    if not all(os.path.exists(x) for x in libs):
        subprocess.run(["make", "-C", os.path.join(ROOT, "tcbee_amd", "csrc")], check=True,
                       stdout=subprocess.DEVNULL)
    host = [os.path.join(ROOT, "tcbee_amd", "lib", "libtcbee_host.so"),
            os.path.join(ROOT, "tcbee_amd", "bin", "tcbee-record-gpu")]
    if not all(os.path.exists(x) for x in host):  # (the C host program links both)
        subprocess.run(["make", "-C", os.path.join(ROOT, "tcbee_amd", "host")], check=True,
                       stdout=subprocess.DEVNULL)


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
