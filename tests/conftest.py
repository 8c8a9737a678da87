import os
import sys

import pytest

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
