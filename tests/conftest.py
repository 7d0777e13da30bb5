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


# Modules that run the library's default plan choice.  The others exercise the tile kernels' own
# features (reductions, node blocks, dictionaries, slabs, plan queries) on stencil-shaped matrices too,
# which by default take the offset-window plan (csrc/mspmv_dia.hip): they pin MSPMV_DIA=0.
DEFAULT_PLAN_MODULES = {"test_gpu_dia.py", "test_gpu_fullsize.py", "test_gpu_cg.py"}


@pytest.fixture(autouse=True)
def _tile_plans_for_tile_tests(request, monkeypatch):
    if request.node.fspath.basename not in DEFAULT_PLAN_MODULES:
        monkeypatch.setenv("MSPMV_DIA", "0")


def pytest_collection_modifyitems(config, items):
    """Run test_gpu_fullsize.py (one test per BASELINE config at its full size) first, then the
    rest in file order: a round-end run cut short still has covered every config."""
    first = [it for it in items if it.fspath.basename == "test_gpu_fullsize.py"]
    if first:
        rest = [it for it in items if it.fspath.basename != "test_gpu_fullsize.py"]
        items[:] = first + rest
