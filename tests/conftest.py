"""Shared pytest configuration: the `gpu` marker and repo-root imports.

`-m "not gpu"` runs here (no GPU): oracle vs reference fixtures, host logic, the native
library's exports and host-side RNG. `-m gpu` runs on an MI355X and checks the HIP path
against the oracle."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP (MI355X) device")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def dev():
    import torch

    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch.device("cuda", 0)
