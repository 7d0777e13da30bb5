"""Test configuration: `gpu` marker, import paths, and shared fixtures.

`-m "not gpu"` runs everywhere (oracle vs golden vectors, host logic, ABI load/exports);
`-m gpu` needs a visible MI355X and exercises the HIP path through the C-ABI.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "sparse-matrix-linear-equations_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a visible MI355X (HIP device)")


@pytest.fixture(scope="session")
def orc():
    import _oracle
    return _oracle.Oracle()


@pytest.fixture(scope="session")
def mspmv():
    import mspmv as m
    return m


@pytest.fixture(scope="session")
def gpu_available():
    import mspmv as m
    if m.device_count() == 0:
        pytest.skip("no HIP device visible")
    return True


def pytest_collection_modifyitems(config, items):
    """Run test_gpu_fullsize.py (one test per BASELINE config at its full size) first, then the
    rest in file order: a round-end run cut short still has covered every config."""
    first = [it for it in items if it.fspath.basename == "test_gpu_fullsize.py"]
    if first:
        rest = [it for it in items if it.fspath.basename != "test_gpu_fullsize.py"]
        items[:] = first + rest
