"""OpenCV 2.4's SVD where the hot path calls it: cvTriangulatePoints' per-point
cvSVD (Triangulator/singlecameratriangulator.cpp:186) and cvRodrigues2's orthonormalisation in
decomposeTransformation (tools.cpp:110), both JacobiSVDImpl_<double> (OpenCV 2.4.9 core/src/lapack.cpp).

Two restatements are pinned against each other and against numpy, CPU only:
  * the oracle's (oracle/fm3d_oracle.c orc_cv_jacobi_svd: generic m x n, strided loops, physical row
    swaps in the sort);
  * the product's (include/fm3d_cvsvd.h: fixed sizes, the sort on a permutation), which the
    triangulation kernel, the host's R2 and the patch frames run -- built here for the host with g++
    (tests/native/cvsvd_shim.cpp) under the same no-FMA rule as the kernels.
The GPU side of the same header is pinned bit for bit by tests/test_gpu_parity.py."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT


@pytest.fixture(scope="module")
def shim(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("cvsvd") / "libcvsvd_shim.so")
    r = subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-shared", "-fPIC",
                        "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "native", "cvsvd_shim.cpp"),
                        "-o", out], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return ctypes.CDLL(out)


def _p(a, t=ctypes.c_double):
    return a.ctypes.data_as(ctypes.POINTER(t))


def _systems(n, seed=0):
    """n DLT inputs: the reference pose's g12 and keypoint pairs of points 1.5-2.4 m away, their
    projections perturbed at the float32 keypoint rounding level (and a few far off)"""
    import importlib
    synth = importlib.import_module("3dfeaturematcher_amd.synth")
    g12 = synth.reference_g12()
    rng = np.random.default_rng(seed)
    X = np.stack([rng.uniform(-1, 1, n), rng.uniform(-0.8, 0.8, n), rng.uniform(1.5, 2.4, n)], 1)
    Y = X @ g12[:3, :3].T + g12[:3, 3]
    u = np.concatenate([X[:, :2] / X[:, 2:], Y[:, :2] / Y[:, 2:]], 1)
    u += rng.normal(0, 3e-5, u.shape) * rng.choice([1.0, 1.0, 1.0, 100.0], (n, 1))
    return g12, np.ascontiguousarray(u)


def _numpy_dlt(g12, u, rows=(0, 1, 2, 3, 4, 5)):
    P1, P2 = np.eye(4)[:3], g12[:3]
    out = np.zeros((len(u), 4))
    for i, (a, b, c, d) in enumerate(u):
        A = np.array([a * P1[2] - P1[0], b * P1[2] - P1[1], a * P1[1] - b * P1[0],
                      c * P2[2] - P2[0], d * P2[2] - P2[1], c * P2[1] - d * P2[0]])[list(rows)]
        out[i] = np.linalg.svd(A)[2][-1]
    return out


def test_oracle_svd_vs_numpy(orc):
    rng = np.random.default_rng(1)
    for m, n in ((6, 4), (3, 3), (4, 4), (5, 2), (8, 8)):
        for _ in range(40):
            A = rng.normal(size=(m, n)) * rng.choice([1e-3, 1.0, 1e3])
            w, u, vt = orc.cv_svd(A)
            assert np.all(np.diff(w) <= 0)
            np.testing.assert_allclose(w, np.linalg.svd(A, compute_uv=False), rtol=1e-13, atol=1e-13 * w[0])
            assert np.abs(u @ np.diag(w) @ vt - A).max() <= 1e-13 * max(1.0, np.abs(A).max())
            assert np.abs(vt @ vt.T - np.eye(n)).max() < 1e-14
            assert np.abs(u.T @ u - np.eye(n)).max() < 1e-13


def test_oracle_svd_rank_deficient_left_vectors(orc):
    """a zero singular value: JacobiSVDImpl_'s cv::RNG vector, orthogonalised -- U stays orthonormal"""
    A = np.array([[1.0, 2.0, 3.0], [2.0, 4.0, 6.0], [1.0, 0.0, 1.0]]).T.copy()  # rank 2
    A[:, 2] = 0.0
    w, u, vt = orc.cv_svd(A)
    assert w[2] == 0.0
    assert np.abs(u.T @ u - np.eye(3)).max() < 1e-14
    assert np.abs(u @ np.diag(w) @ vt - A).max() < 1e-14


def test_oracle_dlt_vs_numpy(orc):
    g12, u = _systems(2000)
    X = np.array([orc.triangulate1(g12, r[:2], r[2:]) for r in u])
    ref = _numpy_dlt(g12, u)
    p, q = X[:, :3] / X[:, 3:], ref[:, :3] / ref[:, 3:]
    assert (np.abs(p - q) / np.maximum(1.0, np.abs(q))).max() < 1e-9
    with orc.geometry_mode(orc.GEOM_DLT_LEGACY):
        X4 = np.array([orc.triangulate1(g12, r[:2], r[2:]) for r in u])
    q4 = _numpy_dlt(g12, u, rows=(0, 1, 3, 4))
    assert (np.abs(X4[:, :3] / X4[:, 3:] - q4[:, :3] / q4[:, 3:]) / np.maximum(1.0, np.abs(q))).max() < 1e-9


def test_header_dlt_bitwise_vs_oracle(orc, shim):
    g12, u = _systems(20000, seed=2)
    X = np.zeros((len(u), 4))
    shim.shim_triangulate(_p(np.ascontiguousarray(g12.ravel())), _p(u), ctypes.c_int(len(u)), _p(X))
    ref = np.array([orc.triangulate1(g12, r[:2], r[2:]) for r in u])
    assert np.array_equal(X.view(np.int64), ref.view(np.int64))


def test_header_svd64_bitwise_vs_oracle(orc, shim):
    rng = np.random.default_rng(3)
    for _ in range(500):
        A = np.ascontiguousarray(rng.normal(size=(6, 4)))
        if rng.random() < 0.2:
            A[:, 3] = A[:, 1]  # equal and zero singular values: the sort's ties
        W, Vt, perm = np.zeros(4), np.zeros((4, 4)), np.zeros(4, dtype=np.int32)
        shim.shim_svd64(_p(A), _p(W), _p(Vt), _p(perm, ctypes.c_int))
        w, _, vt = orc.cv_svd(A)
        assert np.array_equal(W, w) and np.array_equal(Vt, vt)


def test_header_polar_bitwise_vs_oracle(orc, shim):
    rng = np.random.default_rng(4)
    Rs = [orc.rodrigues_v2m(r) + rng.normal(0, s, (3, 3)) for r, s in
          zip(rng.normal(0, 1, (300, 3)), rng.choice([0.0, 1e-15, 1e-9, 1e-3], 300))]
    Rs += [np.eye(3), np.diag([1.0, -1.0, -1.0]), np.array([[1.0, 0, 0], [0, 1.0, 0], [0, 0, 0.0]])]
    Rs = np.ascontiguousarray(np.array(Rs))
    out = np.zeros_like(Rs)
    shim.shim_polar3(_p(Rs), ctypes.c_int(len(Rs)), _p(out))
    ref = np.array([orc.cv_polar3(R) for R in Rs])
    assert np.array_equal(out.view(np.int64), ref.view(np.int64))
    U, _, Vt = np.linalg.svd(Rs[:-1])
    assert np.abs(out[:-1] - U @ Vt).max() < 1e-13


def test_camera2_from_g12_host_equals_oracle(orc, fm3d):
    """libfm3d's host R2 (decomposeTransformation's cvRodrigues2 round trip, fm3d_host.cpp) is the
    oracle's, bit for bit, and equals numpy's SVD polar route within rounding"""
    import importlib
    synth = importlib.import_module("3dfeaturematcher_amd.synth")
    rng = np.random.default_rng(5)
    gs = [synth.reference_g12()]
    for r in rng.normal(0, 0.5, (20, 3)):
        g = np.eye(4)
        g[:3, :3] = orc.rodrigues_v2m(r) + rng.normal(0, 1e-12, (3, 3))
        g[:3, 3] = rng.normal(size=3)
        gs.append(g)
    for g in gs:
        R2, t2 = fm3d.camera2_from_g12(g)
        R2o, t2o = orc.camera2_from_g12(g)
        assert np.array_equal(R2, R2o) and np.array_equal(t2, t2o)
        U, _, Vt = np.linalg.svd(g[:3, :3])
        assert np.abs(R2 - U @ Vt).max() < 1e-13


def test_polar_newton_legacy_differs_in_last_bits(orc):
    """the legacy Newton polar factor (GEOM_POLAR_NEWTON, rounds 1-5) is not the SVD's bit for bit: the
    reference pose's R2 moves by a few ulps (1.8e-15; acos near 1 amplifies the trace's rounding)"""
    import importlib
    synth = importlib.import_module("3dfeaturematcher_amd.synth")
    g = synth.reference_g12()
    R2, _ = orc.camera2_from_g12(g)
    with orc.geometry_mode(orc.GEOM_POLAR_NEWTON):
        R2n, _ = orc.camera2_from_g12(g)
    d = np.abs(R2 - R2n).max()
    assert 0 < d < 1e-14
