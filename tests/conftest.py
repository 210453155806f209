import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


# The GPU tests of the staged kernels spawn multi-process communicators, where eager zero-copy is the default since
# round 6: they keep testing what they name. The eager tests set it on explicitly, and the default
# itself is tested with the variable removed (tests/test_gpu_eager.py, tests/test_gpu_bench.py).
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
