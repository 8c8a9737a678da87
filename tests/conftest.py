import os
import sys

import pytest
# torch first: libmastic_hip.so then binds the HIP runtime torch already loaded
# (same soname), as in bench.py.  A test module that creates a Mastic ctx
# before anything imports torch would otherwise load /opt/rocm's runtime
# first, and torch's own copy, loaded second, then sees no GPU
# (torch.cuda.is_available() False: gpurun_out r06_v6, tests/test_gpu_comm.py
# after tests/test_gpu_serial_sponges.py).
import torch  # noqa: F401,E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(ROOT, "draft-mouris-cfrg-mastic_amd")
for p in (ROOT, PKG_ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C-ABI)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def golden_files():
    return sorted(os.path.join(GOLDEN, f) for f in os.listdir(GOLDEN)
                  if f.startswith("Mastic") and f.endswith(".json"))


@pytest.fixture(scope="session")
def gpu_available():
    import torch  # noqa: F401  (device presence only; the product does not use torch)
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return True
