import os
import sys

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
PKG = os.path.join(ROOT, "face-detection-recognization-pca_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def local_golden(name):
    """Real-face fixtures live only in the git-ignored tests/golden/local/ (privacy:
    they hold photographs of real people); regenerate them with
    tests/golden/make_goldens.py where /root/reference is mounted."""
    path = os.path.join(GOLDEN, "local", name)
    if not os.path.exists(path):
        pytest.skip(f"local real-face fixture {name} absent (not committed; see make_goldens.py)")
    return np.load(path, allow_pickle=False)


@pytest.fixture(scope="session")
def eng():
    # torch's HIP runtime must initialise before libeigenface creates its context in this
    # process (device tensors are used by some tests); otherwise torch reports no GPU.
    import torch
    if torch.cuda.is_available():
        torch.cuda.init()
    from eigenface import Engine
    e = Engine(0)
    yield e
    e.close()
