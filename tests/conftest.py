import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")


@pytest.fixture(scope="session")
def built():
    """Build the product library, the synth helper and the oracle in-tree (idempotent)."""
    import __graft_entry__ as g
    g.build_native()
    return True


@pytest.fixture(scope="session", autouse=True)
def torch_hip_first():
    """torch ships its own HIP/HSA runtime next to the system one libldso_ba.so links; when both
    live in one process, torch's must initialise first or its device enumeration comes back
    empty.  Tests that hand torch buffers to the C ABI rely on this ordering."""
    try:
        import torch

        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:  # CPU container: nothing to order
        pass
    yield
