"""Test configuration: `gpu` marks tests that need an MI355X (HIP device)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X / HIP device and libcairo_amd.so")


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle

    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def cairo():
    import cairo_amd

    cairo_amd.lib()
    return cairo_amd
