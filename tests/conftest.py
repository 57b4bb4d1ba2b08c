"""Test configuration: registers the `gpu` marker and puts the package on sys.path."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "optical-flow-using-dense-inverse-search_amd")
for p in (PKG, ROOT, os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


@pytest.fixture(scope="session")
def oracle():
    import oracle_binding
    return oracle_binding


@pytest.fixture(scope="session")
def disflow_mod():
    import disflow
    return disflow
