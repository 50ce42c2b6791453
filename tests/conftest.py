import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and libmmba.so")


@pytest.fixture(scope="session")
def oracle():
    from oracle import refcpu
    refcpu.lib()
    return refcpu


@pytest.fixture
def paths():
    """Pin plan-builder choices for one test (mmba_debug_set_path);
    everything is restored afterwards.  paths(abi.PATH_X, value)."""
    from mayamatchmovesolver_amd import abi
    from mayamatchmovesolver_amd.solver import set_path
    yield set_path
    for k in range(1, abi.PATH_NUM):
        set_path(k, -1)


@pytest.fixture(scope="session")
def gpu_ctx():
    from mayamatchmovesolver_amd import solver
    if solver.device_count() < 1:
        pytest.fail("no gfx950 device visible to libmmba.so")
    ctx = solver.Context(0)
    yield ctx
    ctx.close()
