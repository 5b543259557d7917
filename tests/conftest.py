import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "vq-vae-transformer-arc-welding_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")


def golden(name):
    import numpy as np
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture
def gold():
    return golden
