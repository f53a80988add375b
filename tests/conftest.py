import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "erasure-codes-prototype_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C ABI)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import ref
    ref.build()
    ref.lib()
    return ref


@pytest.fixture(scope="session")
def ecg():
    import ecg as E
    E.lib()
    return E
