import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REFERENCE = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP ops")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from replisense_rfq_amd.ops import _native

    _native.require()
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def reference_root():
    if not os.path.isdir(REFERENCE):
        pytest.skip("reference snapshot not mounted")
    return REFERENCE
