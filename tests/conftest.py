import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libfm3d.so on the GPU)")


@pytest.fixture(scope="session")
def fm3d():
    return importlib.import_module("3dfeaturematcher_amd")


@pytest.fixture(scope="session")
def synth():
    return importlib.import_module("3dfeaturematcher_amd.synth")


@pytest.fixture(scope="session")
def orc():
    import oracle
    return oracle


def oracle_threads():
    return int(os.environ.get("FM3D_ORACLE_THREADS", "16"))
