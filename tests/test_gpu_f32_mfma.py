"""The float-row matcher's bf16 MFMA prefilter (csrc/fm3d_match.hip, knn2_bf16_kernel + recheck):
knnMatch(k = 2) of SURF-type float descriptors (descriptorsmatcher.cpp:89-131) must return exactly
what the full FLANN-order scan returns -- the same two train rows per query, lowest index on equal
distances, bit-identical float distances -- against the oracle and against the VALU scan of the
same library (FM3D_F32_MFMA=0).  The prefilter serves calls with nA * nB >= 2^22 at dim 64 / 128."""
import os

import numpy as np
import pytest

from conftest import oracle_threads

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(fm3d):
    c = fm3d.Context(fm3d.Settings.default())
    yield c
    c.close()


def _knn(dm, A, B, **env):
    for k, v in env.items():
        os.environ[k] = v
    try:
        return dm.knn_match(A, B)
    finally:
        for k in env:
            del os.environ[k]


def _check(fm3d, orc, ctx, A, B, eps=0.7):
    """the fused prefilter (default), the two-pass prefilter (FM3D_F32_FUSED=0) and the VALU scan
    (FM3D_F32_MFMA=0) byte-identical, and equal to the oracle"""
    dm = fm3d.DescriptorsMatcher(ctx)
    got = dm.knn_match(A, B)
    assert got.tobytes() == _knn(dm, A, B, FM3D_F32_FUSED="0").tobytes()
    ref = _knn(dm, A, B, FM3D_F32_MFMA="0")
    assert got.tobytes() == ref.tobytes()
    idx, dist = orc.knn2(A, B, orc.F32, oracle_threads())
    assert np.array_equal(got["trainIdx"], idx)
    ok = idx >= 0
    assert np.array_equal(got["distance"][ok], dist[ok])
    m = dm.compareWithNNDR(eps, A, B)
    q, t, d = orc.nndr(idx, dist, eps)
    assert np.array_equal(m["queryIdx"], q) and np.array_equal(m["trainIdx"], t) and np.array_equal(m["distance"], d)


@pytest.mark.parametrize("dim", [128, 64])
def test_f32_mfma_surf_descriptors(fm3d, orc, synth, ctx, dim):
    """SURF descriptors of the synthetic frames (unit rows), extended and not"""
    fp = synth.make_frame_pair(4000, seed=3)
    s = fm3d.Settings.default()
    s.surfExtended = 1 if dim == 128 else 0
    c = fm3d.Context(s)
    try:
        _, da = fm3d.SURF(c).detect(fp.img1, with_descriptors=True)
        _, db = fm3d.SURF(c).detect(fp.img2, with_descriptors=True)
    finally:
        c.close()
    assert da.shape[1] == dim and len(da) * len(db) >= 1 << 22
    _check(fm3d, orc, ctx, da, db)


@pytest.mark.parametrize("dim,nA,nB", [(128, 3000, 9000), (64, 2500, 12000)])
def test_f32_mfma_random_rows(fm3d, orc, ctx, dim, nA, nB):
    """near neighbours among clutter, un-normalised rows of varied length"""
    rng = np.random.default_rng(dim + nA)
    B = (rng.normal(0, 1, (nB, dim)) * rng.uniform(0.2, 3, (nB, 1))).astype(np.float32)
    A = np.concatenate([B[: nA // 2] + rng.normal(0, 0.05, (nA // 2, dim)),
                        rng.normal(0, 1, (nA - nA // 2, dim))]).astype(np.float32)
    _check(fm3d, orc, ctx, A, B)


def test_f32_mfma_ties_and_duplicates(fm3d, orc, ctx):
    """exact duplicates among the train rows (equal distances: the lowest index first), queries equal
    to train rows (distance 0), many rows inside the prefilter's bound (more than either candidate
    list holds: those queries are rescanned)"""
    rng = np.random.default_rng(7)
    B = rng.normal(0, 0.1, (4096, 128)).astype(np.float32)
    B[2000] = B[17]
    B[3000] = B[17]
    B[100:300] = B[99]  # 201 identical rows: one query's bound holds them all
    A = np.concatenate([B[17:18], B[99:100], B[:1500], rng.normal(0, 0.1, (1000, 128))]).astype(np.float32)
    _check(fm3d, orc, ctx, A, B)
    got = fm3d.DescriptorsMatcher(ctx).knn_match(A, B)
    assert list(got["trainIdx"][0]) == [17, 2000] and list(got["trainIdx"][1]) == [99, 100]


def test_f32_mfma_nonfinite_rows_rescanned(fm3d, orc, ctx):
    """a NaN / inf in the train rows voids the prefilter's bound: every query takes the exact rescan"""
    rng = np.random.default_rng(8)
    B = rng.normal(0, 0.1, (3000, 64)).astype(np.float32)
    A = rng.normal(0, 0.1, (1500, 64)).astype(np.float32)
    B[5, 3] = np.inf
    dm = fm3d.DescriptorsMatcher(ctx)
    got = dm.knn_match(A, B)
    assert got.tobytes() == _knn(dm, A, B, FM3D_F32_FUSED="0").tobytes()
    assert got.tobytes() == _knn(dm, A, B, FM3D_F32_MFMA="0").tobytes()
