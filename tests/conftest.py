import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "cmu-11785-idl-1.58bit-asr_amd"
for p in (str(ROOT), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and libonebit_hip.so")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU visible")
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
