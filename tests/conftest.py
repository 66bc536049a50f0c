import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")


def pytest_collection_modifyitems(config, items):
    # A GPU test collected without a GPU present fails loudly rather than
    # skipping, unless the run explicitly deselected GPU tests (-m "not gpu").
    pass


@pytest.fixture(scope="session")
def repo_root():
    return ROOT
