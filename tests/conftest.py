import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs under gpurun)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))
    return load


def pytest_sessionstart(session):
    """Measurement knobs passed through the environment (HH_PCA_P,
    HH_PCA_METHOD) apply to GPU test runs too."""
    for key in ("pca_p", "pca_method"):
        v = os.environ.get("HH_" + key.upper())
        if v:
            from hichap_master_amd._lib import call
            call("hh_tune", key.encode(), int(v))
