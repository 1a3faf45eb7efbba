import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "3d_gaussian_magic_change-segment_3dgs_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libgsr.so on cuda:0)")
    config.addinivalue_line("markers", "slow: full-size (BASELINE config) parity checks")


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def gpu_available():
    # gpu-marked tests never skip: on the MI355X box a missing GPU is a failure.
    import torch
    assert torch.cuda.is_available(), "gpu test selected but torch.cuda.is_available() is False"
    return True
