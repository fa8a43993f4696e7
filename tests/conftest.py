"""pytest configuration: the `gpu` marker and import paths.

`-m "not gpu"` tests run on the CPU-only container (oracle vs golden vectors,
host logic, C-ABI symbols); `-m gpu` tests are the parity tests proper and run
on an MI355X through libcip_hip.so.
"""
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "ska-sdp-continuum-imaging-pipeline_amd", ROOT / "oracle"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and libcip_hip.so")


@pytest.fixture(scope="session")
def has_gpu():
    import torch

    return torch.cuda.is_available()


@pytest.fixture(scope="session")
def gpu_device():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)
