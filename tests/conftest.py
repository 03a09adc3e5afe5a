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


def full_fixture(name):
    """tests/golden/full_<name>.npz (tests/golden/make_full_fixtures.py): the oracle's records of a
    whole BASELINE workload plus the digests of its generated inputs."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_full_fixtures",
                                                  os.path.join(ROOT, "tests", "golden", "make_full_fixtures.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod, mod.load_fixture(name)


def assert_inputs(mod, fx, fp):
    """the frame pair this box generated is the one the fixture was made from (numpy's generators
    and SIMD paths differ across machines only if something is wrong -- fail loudly)"""
    got = mod.input_digests(fp)
    bad = [k for k, v in fx["digests"].items() if got[k] != v]
    assert not bad, f"synthetic inputs differ from the fixture's: {bad}"
