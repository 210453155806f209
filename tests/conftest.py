import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


# Eager zero-copy is opt-in (NCCL_AMD_EAGER_REGISTER); a caller's environment that turns it on must
# not change what the staged-kernel tests test. The eager tests set it explicitly.
os.environ.setdefault("NCCL_AMD_EAGER_REGISTER", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")


@pytest.fixture(scope="session")
def built():
    """Make sure libnccl.so and the oracle are built (CPU-side cross compile)."""
    import subprocess
    lib = os.path.join(ROOT, "nccl_amd", "lib", "libnccl.so")
    orc = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
    if not (os.path.exists(lib) and os.path.exists(orc)):
        subprocess.check_call(["make", "-j8"], cwd=ROOT)
    return True
