import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def built():
    """Make sure the in-tree libraries exist (build() compiles them)."""
    need = [os.path.join(ROOT, "bling_amd", "_lib", "libbling_host.so"),
            os.path.join(ROOT, "oracle", "_build", "liboracle.so")]
    if not all(os.path.exists(p) for p in need):
        import subprocess
        subprocess.check_call(["make", "-j8", "host", "oracle"], cwd=ROOT)
    return True
