import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import agilerl_amd  # noqa: E402,F401  (before any device call: its hardware-queue setting, agilerl_amd/__init__.py)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


@pytest.fixture
def golden():
    import numpy as np

    def load(name):
        return dict(np.load(os.path.join(GOLDEN, f"{name}.npz")))

    return load
