"""Shared fixtures.  `-m gpu` tests need a gfx950 device and the built
libsurf_hip.so; they never fall back to the CPU.  Everything else runs on CPU."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "surf-path-tracer_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built HIP library")


@pytest.fixture(scope="session")
def oracle_scene():
    import oracle
    s = oracle.OracleScene()
    yield s
    s.close()


@pytest.fixture(scope="session")
def product_scene():
    import surf_amd
    s = surf_amd.Scene.indoor()
    yield s
    s.close()
