import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")

# torch ships its own HIP/HSA runtime (torch/lib/libamdhip64.so); libcocoa_hip.so
# links /opt/rocm's.  A process that uses both must bring torch's runtime up
# first: once libcocoa_hip.so has opened the GPU, torch's copy finds no device.
# The multi-rank tests hand device buffers to torch, so torch is loaded here.
try:
    import torch  # noqa: F401
except ImportError:  # pragma: no cover
    torch = None


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built libcocoa_hip.so")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
