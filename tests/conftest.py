import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "raytracing-potato_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

REFERENCE = "/root/reference"
HAVE_REFERENCE = os.path.isdir(os.path.join(REFERENCE, "src"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through librp.so on the device)")
    config.addinivalue_line("markers", "slow: long-running")


def _ensure_built():
    libs = [os.path.join(PKG, "lib", "librp.so"), os.path.join(PKG, "lib", "librp_host.so"),
            os.path.join(REPO, "oracle", "liboracle.so")]
    if not all(os.path.exists(p) for p in libs):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
        subprocess.run(["make", "-s", "-j8", "-C", PKG], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle_py
    return oracle_py


@pytest.fixture(scope="session")
def gpu():
    """Fails loudly (no skip, no fallback) when the HIP library or the device is missing."""
    from rtpotato import render
    n = render.device_count()
    assert n > 0, "no HIP device visible: -m gpu tests need an MI355X"
    return render
