import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# Every device context of the session fills each buffer it allocates with 0xFF bytes
# (LUMO_OPT_POISON, read at lumo_create): a kernel that reads a buffer before the render has
# written it then sees NaN / -1 instead of zeros an earlier test left, so a missing
# initialisation or cross-stream wait fails deterministically, not depending on test order.
os.environ.setdefault("LUMO_POISON", "1")
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session", autouse=True)
def _built():
    lib = os.path.join(ROOT, "lumo_amd", "liblumo_amd.so")
    orc = os.path.join(ROOT, "oracle", "_build", "liblumo_oracle.so")
    if not (os.path.exists(lib) and os.path.exists(orc)):
        import subprocess
        subprocess.run(["make", "-C", ROOT, "-j8"], check=True)
