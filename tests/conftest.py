import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
# before any test touches the HIP runtime: the package turns hipGraph packet capture off for the process
# (ouzelum_amd/__init__.py), which only takes effect if the runtime has not started yet
import ouzelum_amd  # noqa: E402,F401


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    d = os.path.join(ROOT, "tests", "golden")

    def load(name):
        return np.load(os.path.join(d, name))
    return load
