"""Host-side sanitizer builds: the CPU oracle, the settings.yml / PGM parsers and
the host algebra of libfm3d compiled with -fsanitize=address,undefined (tests/native/Makefile)
and run on well-formed and malformed inputs.  Any sanitizer report fails the run.  CPU only:
no GPU code is sanitized (the host half of fm3d_host.cpp is, via hipcc -Xarch_host)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

NATIVE = os.path.join(ROOT, "tests", "native")


@pytest.fixture(scope="module")
def build_dir(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("san"))
    targets = [f"{out}/san_oracle", f"{out}/san_star", f"{out}/san_mser", f"{out}/san_parse"]
    csrc = os.path.join(ROOT, "3dfeaturematcher_amd", "csrc", "_build")
    if all(os.path.exists(os.path.join(csrc, f"{k}.hip.o")) for k in ("fm3d_match", "fm3d_misc", "fm3d_lm2", "fm3d_patch")):
        targets.append(f"{out}/san_host")
    r = subprocess.run(["make", "-C", NATIVE, f"OUT={out}", "-j3"] + targets, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return out


def _run(exe, *args, env=None):
    e = dict(os.environ)
    e.update(env or {})
    e["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    r = subprocess.run([exe, *args], capture_output=True, text=True, timeout=300, env=e)
    assert r.returncode == 0 and "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, \
        r.stdout[-2000:] + r.stderr[-4000:]
    return r.stdout


def test_oracle_under_asan_ubsan(build_dir):
    assert "san_oracle: ok" in _run(f"{build_dir}/san_oracle", env={"OMP_NUM_THREADS": "2"})


def test_star_oracle_under_asan_ubsan(build_dir):
    assert "san_star: ok" in _run(f"{build_dir}/san_star")


def test_mser_oracle_under_asan_ubsan(build_dir):
    assert "san_mser: ok" in _run(f"{build_dir}/san_mser")


def test_settings_and_pgm_parsers_malformed_inputs(build_dir, tmp_path):
    assert "san_parse: ok" in _run(f"{build_dir}/san_parse", str(tmp_path))


def test_host_algebra_under_asan_ubsan(build_dir):
    exe = f"{build_dir}/san_host"
    if not os.path.exists(exe):
        pytest.skip("libfm3d objects not built (run __graft_entry__.build())")
    # the ROCm runtime linked into the binary keeps allocations alive at exit: no leak check
    assert "san_host: ok" in _run(exe, env={"ASAN_OPTIONS": "detect_leaks=0"})


def test_toolchain_present():
    assert shutil.which("gcc") and shutil.which("g++")
