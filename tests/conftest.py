import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as o

    o.lib()
    return o


@pytest.fixture(scope="session")
def pkg():
    """The product package (flink-cooccurrence_amd/) imported as flink_cooccurrence_amd."""
    from __graft_entry__ import load_package

    return load_package()
