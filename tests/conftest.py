import os
import sys

import pytest

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
for p in (os.path.join(REPO, "2dsfs-scan_amd"), REPO, os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests through the C-ABI")
    config.addinivalue_line("markers", "slow: larger CPU cases")


def pytest_collection_modifyitems(config, items):
    # -m gpu runs on the GPU box; a GPU test must not silently pass without a device
    pass


@pytest.fixture(scope="session")
def golden():
    import golden_util
    return golden_util.Golden()
