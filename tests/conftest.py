import os
import sys

import pytest

# the library honours its measurement / test switches (PYR_FILTER_CERR, PYR_STREAM_*, ...) only with this set
# before it is loaded (kernels.h knob())
os.environ.setdefault("PYR_DEV_KNOBS", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device; calls the HIP path through the C ABI")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def hiplib():
    """The product library; on a GPU box a missing .so or device is a failure, not a skip.

    PyTorch-ROCm bundles its own HIP runtime; when the library's (/opt/rocm) runtime opens the
    device first, torch's later lazy init reports no GPU.  Tests that hand torch tensors to the
    library therefore need torch's runtime up first (bench.py does the same)."""
    import torch
    if torch.cuda.is_available():
        torch.cuda.init()
    from pyrope_amd import _lib
    from pyrope_amd.build import build
    build()
    return _lib.load()
