"""GPU parity: libfm3d.so (HIP, gfx950) against the CPU oracle on the same inputs.

Bar (north_star): bit-exact match indices and pixel neighbourhoods; normals
within 1e-4.  The LM kernel replays the reference's sequential MINPACK sums, so
it is compared BIT FOR BIT with the oracle run with the same deterministic
transcendentals (oracle.DETMATH), and at 1e-4 with the libm-based oracle
(oracle.STRICT).
"""
import importlib

import os

import numpy as np
import pytest

from conftest import assert_inputs, full_fixture, oracle_threads

pytestmark = pytest.mark.gpu


def _settings(fm3d, cam, **kw):
    s = fm3d.Settings.default()
    s.set_camera(cam)
    for k, v in kw.items():
        setattr(s, k, v)
    return s


@pytest.fixture(scope="module")
def pair(synth):
    return synth.make_frame_pair(3000, seed=11)


@pytest.fixture(scope="module")
def ctx(fm3d, pair):
    c = fm3d.Context(_settings(fm3d, pair.cam, pixelsRay=16))
    yield c
    c.close()


# ---------------------------------------------------------------- matching
@pytest.mark.parametrize("shape", [(3000, 3000), (777, 1500), (1, 5), (130, 1), (0, 10)])
def test_knn2_u8_exact(fm3d, orc, ctx, pair, shape):
    nA, nB = shape
    rng = np.random.default_rng(nA * 7 + nB)
    A = pair.desc1[:nA] if nA <= len(pair.desc1) else None
    B = pair.desc2[:nB]
    if nA <= 1 or nB <= 1:
        A = rng.integers(0, 256, (nA, 128), dtype=np.uint8)
        B = rng.integers(0, 256, (nB, 128), dtype=np.uint8)
    dm = fm3d.DescriptorsMatcher(ctx)
    if nA == 0:
        assert len(dm.compareWithNNDR(0.55, A, B)) == 0
        return
    got = dm.knn_match(A, B)
    idx, dist = orc.knn2(A, B, orc.U8, oracle_threads())
    assert np.array_equal(got["trainIdx"], idx)
    ok = idx >= 0
    assert np.array_equal(got["distance"][ok], dist[ok])
    m = dm.compareWithNNDR(0.55, A, B)
    q, t, d = orc.nndr(idx, dist, 0.55)
    assert np.array_equal(m["queryIdx"], q) and np.array_equal(m["trainIdx"], t) and np.array_equal(m["distance"], d)


def test_knn2_u8_ties_lowest_index(fm3d, orc, ctx):
    # duplicated train rows: equal distances must resolve to the lowest trainIdx
    rng = np.random.default_rng(5)
    B = rng.integers(0, 256, (300, 128), dtype=np.uint8)
    B[200] = B[17]
    B[250] = B[17]
    A = np.concatenate([B[17:18], B[:40]])
    got = fm3d.DescriptorsMatcher(ctx).knn_match(A, B)
    idx, dist = orc.knn2(A, B, orc.U8, 1)
    assert np.array_equal(got["trainIdx"], idx)
    assert got["trainIdx"][0, 0] == 17 and got["trainIdx"][0, 1] == 200


def test_knn2_u8_dims(fm3d, orc, ctx):
    rng = np.random.default_rng(9)
    for dim in (64, 100, 256):
        A = rng.integers(0, 256, (500, dim), dtype=np.uint8)
        B = rng.integers(0, 256, (700, dim), dtype=np.uint8)
        got = fm3d.DescriptorsMatcher(ctx).knn_match(A, B)
        idx, dist = orc.knn2(A, B, orc.U8, oracle_threads())
        assert np.array_equal(got["trainIdx"], idx), dim
        assert np.array_equal(got["distance"], dist), dim


@pytest.mark.parametrize("dim", [128, 64, 36])
def test_knn2_f32_flann_order(fm3d, orc, ctx, dim):
    # SURF-like non-integer floats: FLANN L2 accumulation order, float32
    rng = np.random.default_rng(dim)
    A = rng.normal(0, 0.1, (1200, dim)).astype(np.float32)
    B = np.concatenate([A[:900] + rng.normal(0, 0.01, (900, dim)).astype(np.float32),
                        rng.normal(0, 0.1, (700, dim)).astype(np.float32)])
    dm = fm3d.DescriptorsMatcher(ctx)
    got = dm.knn_match(A, B)
    idx, dist = orc.knn2(A, B, orc.F32, oracle_threads())
    assert np.array_equal(got["trainIdx"], idx)
    assert np.array_equal(got["distance"], dist)
    m = dm.compareWithNNDR(0.6, A, B)
    q, t, d = orc.nndr(idx, dist, 0.6)
    assert np.array_equal(m["queryIdx"], q) and np.array_equal(m["trainIdx"], t)


@pytest.mark.parametrize("dim", [128, 64])
def test_knn2_f32_train_parts_and_ties(fm3d, orc, ctx, dim):
    # a train set large enough to be split into parts (merged afterwards), an odd row count (the
    # last row pair has one row) and exact duplicates across parts (ties: lower train index first)
    rng = np.random.default_rng(100 + dim)
    nB = 20001
    B = rng.normal(0, 0.1, (nB, dim)).astype(np.float32)
    B[15000:15400] = B[100:500]          # duplicates in a later part
    B[nB - 1] = B[7]                     # and in the last, single-row pair
    A = np.concatenate([B[:600] + rng.normal(0, 0.01, (600, dim)).astype(np.float32),
                        B[100:300], B[[7, 7]],  # zero distances, tied twice
                        rng.normal(0, 0.1, (2200, dim)).astype(np.float32)])
    got = fm3d.DescriptorsMatcher(ctx).knn_match(A, B)
    idx, dist = orc.knn2(A, B, orc.F32, oracle_threads())
    assert np.array_equal(got["trainIdx"], idx)
    assert np.array_equal(got["distance"], dist)
    assert (idx[600:800, 0] == np.arange(100, 300)).all() and (idx[600:800, 1] == np.arange(15000, 15200)).all()


@pytest.mark.parametrize("kind", ["f32_128", "f32_64", "bits"])
@pytest.mark.parametrize("shape", [(1, 5), (130, 1), (5, 2), (40, 0), (300, 4099)])
def test_knn2_ragged_f32_and_bits(fm3d, orc, ctx, kind, shape):
    # one query, one or two train rows, no train rows (trainIdx -1), odd sizes past a part
    nA, nB = shape
    rng = np.random.default_rng(nA * 13 + nB)
    if kind == "bits":
        A = rng.integers(0, 256, (nA, 32), dtype=np.uint8)
        B = rng.integers(0, 256, (nB, 32), dtype=np.uint8)
        ty = orc.BITS
    else:
        d = int(kind.split("_")[1])
        A = rng.normal(0, 0.1, (nA, d)).astype(np.float32)
        B = rng.normal(0, 0.1, (nB, d)).astype(np.float32)
        ty = orc.F32
    got = fm3d.DescriptorsMatcher(ctx, binary=kind == "bits").knn_match(A, B)
    idx, dist = orc.knn2(A, B, ty, oracle_threads())
    assert np.array_equal(got["trainIdx"], idx)
    ok = idx >= 0
    assert np.array_equal(got["distance"][ok], dist[ok])
    assert (idx[:, 0] >= 0).all() == (nB >= 1) and (idx[:, 1] >= 0).all() == (nB >= 2)


def test_knn2_f32_integer_valued_sift(fm3d, orc, ctx, pair):
    # OpenCV SIFT floats are integer valued: routed to the int8-MFMA kernel, same results
    A = pair.desc1[:1500].astype(np.float32)
    B = pair.desc2[:2000].astype(np.float32)
    got = fm3d.DescriptorsMatcher(ctx).knn_match(A, B)
    idx, dist = orc.knn2(A, B, orc.F32, oracle_threads())
    assert np.array_equal(got["trainIdx"], idx)
    assert np.array_equal(got["distance"], dist)


def test_knn2_hamming(fm3d, orc, ctx, synth):
    fp = synth.make_frame_pair(1500, seed=3, desc="orb")
    dm = fm3d.DescriptorsMatcher(ctx, binary=True)
    got = dm.knn_match(fp.desc1, fp.desc2)
    idx, dist = orc.knn2(fp.desc1, fp.desc2, orc.BITS, oracle_threads())
    assert np.array_equal(got["trainIdx"], idx)
    assert np.array_equal(got["distance"], dist)
    m = dm.compareWithNNDR(0.8, fp.desc1, fp.desc2)
    q, t, d = orc.nndr(idx, dist, 0.8)
    assert np.array_equal(m["queryIdx"], q) and np.array_equal(m["trainIdx"], t)
    assert np.mean(fp.true_train[m["queryIdx"]] == m["trainIdx"]) > 0.95


def test_nndr_appends(fm3d, ctx, pair):
    dm = fm3d.DescriptorsMatcher(ctx)
    m1 = dm.compareWithNNDR(0.55, pair.desc1[:500], pair.desc2)
    m2 = dm.compareWithNNDR(0.55, pair.desc1[:500], pair.desc2, matches=m1)
    assert len(m2) == 2 * len(m1)


# ---------------------------------------------------------------- geometry
def test_camera2_and_g12(fm3d, orc, ctx, pair):
    sct = fm3d.SingleCameraTriangulator(ctx)
    s = ctx.settings
    g = sct.setg12(s.pos1[:3], s.pos2[:3], s.pos1[3:], s.pos2[3:])
    go = orc.setg12(list(s.rodriguesIC), list(s.translationIC), s.pos1[:3], s.pos2[:3], s.pos1[3:], s.pos2[3:])
    assert np.array_equal(g, go)
    R2, t2 = sct.camera2()
    R2o, t2o = orc.camera2_from_g12(g)
    assert np.array_equal(R2, R2o) and np.array_equal(t2, t2o)


def test_undistort_bitwise(fm3d, orc, ctx):
    rng = np.random.default_rng(1)
    xy = np.stack([rng.uniform(-50, 700, 5000), rng.uniform(-50, 530, 5000)], 1)
    out = np.zeros_like(xy)
    lib = fm3d.lib()
    import ctypes
    ctx.check(lib.fm3d_undistort(ctx.handle, xy.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), len(xy),
                                 out.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
    cam = type("C", (), {})()
    cam.fx, cam.fy, cam.cx, cam.cy, cam.k = ctx.settings.camera()
    assert np.array_equal(out, orc.undistort(cam, xy))


def test_triangulate_bitwise(fm3d, orc, ctx, pair):
    dm = fm3d.DescriptorsMatcher(ctx)
    m = dm.compareWithNNDR(0.55, pair.desc1, pair.desc2)
    sct = fm3d.SingleCameraTriangulator(ctx)
    sct.set_g12(pair.g12)
    sct.setKeypoints(pair.kp1, pair.kp2, m)
    pts, mask = sct.triangulate()
    pto, masko = orc.triangulate(pair.cam, pair.g12, 1.5, 2.4, pair.kp1, pair.kp2, m["queryIdx"], m["trainIdx"])
    assert np.array_equal(mask, masko)
    assert np.array_equal(pts, pto)
    assert 0 < len(pts) <= len(m)


def test_triangulate_legacy_solver_bitwise(fm3d, orc, pair):
    """dltSolver = 1 (opt-in): the 4-row system and round-robin Jacobi of rounds 1-5, bit for bit the
    oracle's GEOM_DLT_LEGACY mode; the default (cvTriangulatePoints' 6 x 4 JacobiSVD) differs from it"""
    c = fm3d.Context(_settings(fm3d, pair.cam, pixelsRay=16, dltSolver=1))
    try:
        dm = fm3d.DescriptorsMatcher(c)
        m = dm.compareWithNNDR(0.55, pair.desc1, pair.desc2)
        sct = fm3d.SingleCameraTriangulator(c)
        sct.set_g12(pair.g12)
        sct.setKeypoints(pair.kp1, pair.kp2, m)
        pts, mask = sct.triangulate()
    finally:
        c.close()
    with orc.geometry_mode(orc.GEOM_DLT_LEGACY):
        pto, masko = orc.triangulate(pair.cam, pair.g12, 1.5, 2.4, pair.kp1, pair.kp2, m["queryIdx"], m["trainIdx"])
    assert np.array_equal(mask, masko) and np.array_equal(pts, pto)
    ptn, maskn = orc.triangulate(pair.cam, pair.g12, 1.5, 2.4, pair.kp1, pair.kp2, m["queryIdx"], m["trainIdx"])
    assert np.array_equal(maskn, mask) and not np.array_equal(ptn, pts)


def test_triangulate_degenerate_systems_bitwise(fm3d, orc, pair):
    """OpenCV's JacobiSVD where its branches matter: DLT systems with zero and repeated singular
    values. Cases: a pure rotation (t = 0, so the 6 x 4 system has a zero column), the same keypoint
    in both views, both keypoints at the principal point, keypoints far outside the frame, and
    repeated matches. With the z filter opened wide, every point and mask bit equals the oracle's
    (NaN included)."""
    rng = np.random.default_rng(41)
    n = 512
    kp1 = np.ascontiguousarray(rng.uniform(0, 640, (n, 2)).astype(np.float32))
    kp2 = np.ascontiguousarray(rng.uniform(0, 480, (n, 2)).astype(np.float32))
    cx, cy = pair.cam.cx, pair.cam.cy
    kp2[:64] = kp1[:64]                                 # the same pixel in both views
    kp1[64:96] = kp2[64:96] = (np.float32(cx), np.float32(cy))  # the principal point
    kp1[96:128] *= np.float32(1e4)                      # far outside the frame
    kp2[128:160] = np.float32(-3e5)
    m = np.zeros(n + 64, dtype=fm3d.DMATCH)
    m["queryIdx"][:n] = np.arange(n)
    m["trainIdx"][:n] = np.arange(n)
    m["queryIdx"][n:] = 7                               # repeated matches
    m["trainIdx"][n:] = 9
    g_rot = np.array(pair.g12, dtype=np.float64).copy()
    g_rot[:3, 3] = 0.0
    c = fm3d.Context(_settings(fm3d, pair.cam, pixelsRay=16, zThresholdMin=-1e300, zThresholdMax=1e300))
    try:
        for g in (np.asarray(pair.g12, dtype=np.float64), g_rot):
            sct = fm3d.SingleCameraTriangulator(c)
            sct.set_g12(g)
            sct.setKeypoints(kp1, kp2, m)
            pts, mask = sct.triangulate()
            pto, masko = orc.triangulate(pair.cam, g, -1e300, 1e300, kp1, kp2, m["queryIdx"], m["trainIdx"])
            assert np.array_equal(mask, masko)
            assert np.array_equal(pts, pto, equal_nan=True)
            assert mask.sum() > n // 2
    finally:
        c.close()


def test_pyramid_bitwise(fm3d, orc, ctx, pair):
    no = fm3d.NormalOptimizer(ctx)
    no.setImages(pair.img1, pair.img2)
    for which, img in ((1, pair.img1), (2, pair.img2)):
        ref = img
        for L in range(ctx.settings.pyramids + 1):
            got = no.pyramid(which, L)
            assert np.array_equal(got, ref), (which, L)
            ref = orc.pyrdown(ref)
    # odd sizes
    rng = np.random.default_rng(2)
    for h, w in ((37, 53), (1, 9), (8, 1), (121, 160)):
        img = rng.integers(0, 256, (h, w), dtype=np.uint8)
        out = np.zeros(((h + 1) // 2, (w + 1) // 2), dtype=np.uint8)
        import ctypes
        ctx.check(fm3d.lib().fm3d_pyrdown(ctx.handle, img.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), w, h,
                                          out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))))
        assert np.array_equal(out, orc.pyrdown(img)), (h, w)


# ---------------------------------------------------------------- normals
def _normals_case(fm3d, orc, pair, points, ray, bound=(1024, 768), levels=3):
    s = _settings(fm3d, pair.cam, pixelsRay=ray, boundWidth=bound[0], boundHeight=bound[1], pyramids=levels)
    ctx = fm3d.Context(s)
    try:
        sct = fm3d.SingleCameraTriangulator(ctx)
        sct.set_g12(pair.g12)
        R2, t2 = sct.camera2()
        no = fm3d.NormalOptimizer(ctx, sct)
        no.setImages(pair.img1, pair.img2)
        kept, normals = no.computeOptimizedNormals(points)
        st, info, nfev = no.last_status, no.last_info, no.last_nfev
    finally:
        ctx.close()
    ref = orc.optimize_normals(pair.cam, R2, t2, pair.img1, pair.img2, levels, points, ray, bound[0], bound[1],
                               mode=orc.DETMATH, nthreads=oracle_threads())
    return kept, normals, st, info, nfev, ref, (R2, t2)


@pytest.mark.parametrize("ray,safe", [(8, 0), (16, 0), (16, 1)])
def test_normals_bitwise_vs_oracle(fm3d, orc, pair, ray, safe, monkeypatch):
    # safe = 1: every pass takes the guarded form (per-lane division guards, general flags) that
    # the kernel otherwise keeps for out-of-range weights and numerators
    monkeypatch.setenv("FM3D_LM_SAFE", str(safe))
    # triangulated points of the pair (oracle chain), plus border / degenerate cases
    q, t, _ = orc.match_nndr(pair.desc1, pair.desc2, orc.U8, 0.55, oracle_threads())
    pts, _ = orc.triangulate(pair.cam, pair.g12, 1.5, 2.4, pair.kp1, pair.kp2, q, t)
    extra = np.array([[-1.3, -0.95, 2.0],    # projects near the top-left corner: trimmed neighbourhood
                      [5.0, 5.0, 2.0],       # outside every image: no pixels
                      [0.0, 0.0, 2.0]])
    P = np.concatenate([pts[:120], extra])
    kept, normals, st, info, nfev, ref, _ = _normals_case(fm3d, orc, pair, P, ray)
    assert np.array_equal(st, ref["status"])
    assert np.array_equal(info[:, :4], ref["info"][:, :4])
    assert np.array_equal(nfev[:, :4], ref["nfev"][:, :4])
    ok = ref["status"] == 0
    assert np.array_equal(normals, ref["normals"][ok])
    assert np.array_equal(kept, P[ok])
    assert ok.sum() > 10


def test_normals_vs_strict_oracle_1e4(fm3d, orc, pair):
    q, t, _ = orc.match_nndr(pair.desc1, pair.desc2, orc.U8, 0.55, oracle_threads())
    pts, _ = orc.triangulate(pair.cam, pair.g12, 1.5, 2.4, pair.kp1, pair.kp2, q, t)
    P = pts[:80]
    kept, normals, st, info, nfev, _, (R2, t2) = _normals_case(fm3d, orc, pair, P, 16)
    strict = orc.optimize_normals(pair.cam, R2, t2, pair.img1, pair.img2, 3, P, 16, mode=orc.STRICT,
                                  nthreads=oracle_threads())
    assert np.array_equal(st, strict["status"])
    ok = strict["status"] == 0
    assert np.abs(normals - strict["normals"][ok]).max() < 1e-4   # north_star tolerance


def test_normals_reference_config_ray64(fm3d, orc, pair):
    # build/settings.yml: pixelsRay 64, pyramids 3 (12,853-pixel residuals)
    q, t, _ = orc.match_nndr(pair.desc1, pair.desc2, orc.U8, 0.55, oracle_threads())
    pts, _ = orc.triangulate(pair.cam, pair.g12, 1.5, 2.4, pair.kp1, pair.kp2, q, t)
    P = pts[:24]
    kept, normals, st, info, nfev, ref, _ = _normals_case(fm3d, orc, pair, P, 64)
    assert np.array_equal(st, ref["status"])
    assert np.array_equal(nfev[:, :4], ref["nfev"][:, :4])
    ok = ref["status"] == 0
    assert np.array_equal(normals, ref["normals"][ok])


def test_normals_ray128_largest_neighbourhood(fm3d, orc, pair):
    # pixelsRay 128: 51,445-pixel residuals (4x the reference's), the largest slab rows
    q, t, _ = orc.match_nndr(pair.desc1, pair.desc2, orc.U8, 0.55, oracle_threads())
    pts, _ = orc.triangulate(pair.cam, pair.g12, 1.5, 2.4, pair.kp1, pair.kp2, q, t)
    P = pts[:12]
    kept, normals, st, info, nfev, ref, _ = _normals_case(fm3d, orc, pair, P, 128)
    assert np.array_equal(st, ref["status"])
    assert np.array_equal(nfev[:, :4], ref["nfev"][:, :4])
    ok = ref["status"] == 0
    assert np.array_equal(normals, ref["normals"][ok])


@pytest.mark.parametrize("levels", [0, 1])
def test_normals_pyramid_depths(fm3d, orc, pair, levels):
    # no pyramid (level 0 only) and one pyramid level
    q, t, _ = orc.match_nndr(pair.desc1, pair.desc2, orc.U8, 0.55, oracle_threads())
    pts, _ = orc.triangulate(pair.cam, pair.g12, 1.5, 2.4, pair.kp1, pair.kp2, q, t)
    kept, normals, st, info, nfev, ref, _ = _normals_case(fm3d, orc, pair, pts[:40], 16, levels=levels)
    assert np.array_equal(st, ref["status"])
    assert np.array_equal(nfev[:, :levels + 1], ref["nfev"][:, :levels + 1])
    ok = ref["status"] == 0
    assert np.array_equal(normals, ref["normals"][ok])
    assert ok.sum() > 5


@pytest.mark.parametrize("coop", ["0", "1"])
def test_normals_more_points_than_slots(fm3d, orc, pair, coop, monkeypatch):
    # 6,000 points > 3,840 slots: slots pull second points from the queue while idle slots help
    # busy ones (FM3D_LM_COOP=1, the default) or leave (0); both must give the oracle's bits
    monkeypatch.setenv("FM3D_LM_COOP", coop)
    q, t, _ = orc.match_nndr(pair.desc1, pair.desc2, orc.U8, 0.55, oracle_threads())
    pts, _ = orc.triangulate(pair.cam, pair.g12, 1.5, 2.4, pair.kp1, pair.kp2, q, t)
    reps = -(-6000 // len(pts))
    P = np.concatenate([pts * (1.0 + 2e-3 * r) for r in range(reps)])[:6000]
    kept, normals, st, info, nfev, ref, _ = _normals_case(fm3d, orc, pair, P, 6)
    assert np.array_equal(st, ref["status"])
    assert np.array_equal(nfev[:, :4], ref["nfev"][:, :4])
    ok = ref["status"] == 0
    assert np.array_equal(normals, ref["normals"][ok])
    assert np.array_equal(kept, P[ok])
    assert ok.sum() > 1000


def test_normals_vga_bounds(fm3d, orc, pair):
    # image bound = the VGA size instead of the reference's literal 1024x768
    q, t, _ = orc.match_nndr(pair.desc1, pair.desc2, orc.U8, 0.55, oracle_threads())
    pts, _ = orc.triangulate(pair.cam, pair.g12, 1.5, 2.4, pair.kp1, pair.kp2, q, t)
    kept, normals, st, info, nfev, ref, _ = _normals_case(fm3d, orc, pair, pts[:60], 12, bound=(640, 480))
    assert np.array_equal(st, ref["status"])
    ok = ref["status"] == 0
    assert np.array_equal(normals, ref["normals"][ok])


# ---------------------------------------------------------------- whole path
def test_pipeline_end_to_end(fm3d, orc, pair):
    s = _settings(fm3d, pair.cam, pixelsRay=12)
    ctx = fm3d.Context(s)
    try:
        sct = fm3d.SingleCameraTriangulator(ctx)
        sct.set_g12(pair.g12)
        R2, t2 = sct.camera2()
        pipe = fm3d.Pipeline(ctx)
        pipe.upload(pair.desc1, pair.desc2, pair.kp1, pair.kp2, pair.img1, pair.img2)
        n, stats = pipe.run()
        rec = pipe.records(n)
        n2, _ = pipe.run()      # idempotent re-run on resident inputs
        rec2 = pipe.records(n2)
    finally:
        ctx.close()
    assert n == n2 and np.array_equal(rec, rec2)
    q, t, d = orc.match_nndr(pair.desc1, pair.desc2, orc.U8, 0.55, oracle_threads())
    assert stats["matches"] == len(q)
    pts, mask = orc.triangulate(pair.cam, pair.g12, 1.5, 2.4, pair.kp1, pair.kp2, q, t)
    assert stats["inliers"] == len(pts)
    ref = orc.optimize_normals(pair.cam, R2, t2, pair.img1, pair.img2, 3, pts, 12, mode=orc.DETMATH,
                               nthreads=oracle_threads())
    ok = ref["status"] == 0
    assert n == ok.sum()
    assert np.array_equal(rec["queryIdx"], q[mask][ok])
    assert np.array_equal(rec["trainIdx"], t[mask][ok])
    assert np.array_equal(rec["point"], pts[ok])
    assert np.array_equal(rec["normal"], ref["normals"][ok])


def test_sharded_blocks_equal_single_run(fm3d, pair):
    """Both multi-GPU partitions, run here one share after the other on one GPU: contiguous
    query blocks with queryOffset concatenate to the single-run records byte for byte, and
    the block-cyclic shares (gathered queries, local indices mapped back) merge to them."""
    import importlib
    shard = importlib.import_module("3dfeaturematcher_amd.shard")
    s = _settings(fm3d, pair.cam, pixelsRay=10, pyramids=2)
    n = len(pair.desc1)
    full = shard.run_shard(pair, s, 0, n)
    parts = [shard.run_shard(pair, s, *shard.partition(n, 3, r)) for r in range(3)]
    merged = np.concatenate(parts)
    assert len(full) > 100
    assert merged.tobytes() == full.tobytes()
    cyc = np.concatenate([shard.run_shard_queries(pair, s, shard.query_blocks(n, 3, r, 64)) for r in range(3)])
    cyc = cyc[np.argsort(cyc["queryIdx"], kind="stable")]
    assert cyc.tobytes() == full.tobytes()


# ---------------------------------------------------------------- patch export (§8(f))
def test_features_frames_and_patches_bitwise(fm3d, orc, pair):
    """computeFeaturesFrames + getReferenceSquaredNeighborhood + projectReferencePointsToImageWithFrames
    on the GPU: frames bit-exact, 128x128 patches and projected points bit-exact against the oracle's
    deterministic-math mode, and within the truncation flips of the libm oracle."""
    q, t, _ = orc.match_nndr(pair.desc1, pair.desc2, orc.U8, 0.55, oracle_threads())
    pts, _ = orc.triangulate(pair.cam, pair.g12, 1.5, 2.4, pair.kp1, pair.kp2, q, t)
    kept, normals, st, info, nfev, ref, _ = _normals_case(fm3d, orc, pair, pts[:60], 12)
    assert len(kept) > 20
    s = _settings(fm3d, pair.cam)
    ctx = fm3d.Context(s)
    try:
        no = fm3d.NormalOptimizer(ctx)
        no.setImages(pair.img1, pair.img2)
        g = no.getGravity()
        frames = no.computeFeaturesFrames(kept, normals)
        ng = fm3d.NeighborhoodsGenerator(s)
        sct = fm3d.SingleCameraTriangulator(ctx)
        patches, ipts = sct.projectReferencePointsToImageWithFrames(ng.getReferenceSquaredNeighborhood(), frames,
                                                                    image_points=True)
    finally:
        ctx.close()
    assert np.array_equal(g, orc.gravity(list(s.rodriguesIC)))
    assert np.array_equal(frames, orc.features_frames(kept, normals, g))
    assert patches.shape == (len(kept), 128, 128)
    ref_p, ref_pts = orc.export_patches(pair.cam, pair.img1, frames, mode=orc.DETMATH, image_points=True)
    assert np.array_equal(ipts, ref_pts)
    assert np.array_equal(patches, ref_p)
    strict = orc.export_patches(pair.cam, pair.img1, frames, mode=orc.STRICT)
    d = np.abs(patches.astype(int) - strict.astype(int))
    assert d.max() <= 1 and (d == 0).mean() > 0.999
    assert (patches > 0).mean() > 0.5  # the patches see the textured scene


def test_square_neighborhoods_bitwise(fm3d, orc, pair):
    """computeSquareNeighborhoodsByNormals (main.cpp:187) on the GPU: every frame's 128x128 grid
    bit-exact against the oracle, plus a non-rigid frame (the 1/w branch) and a small grid whose
    point count is not a multiple of the block."""
    q, t, _ = orc.match_nndr(pair.desc1, pair.desc2, orc.U8, 0.55, oracle_threads())
    pts, _ = orc.triangulate(pair.cam, pair.g12, 1.5, 2.4, pair.kp1, pair.kp2, q, t)
    normals = pts / np.linalg.norm(pts, axis=1, keepdims=True)
    frames = orc.features_frames(pts[:50], normals[:50], orc.gravity([0.1, -0.2, 0.05])).reshape(-1, 16)
    frames = np.concatenate([frames, [[1, 0.5, 0.25, 0.1, 0, 1, 0, 0.2, 0.3, 0, 1, 2.0, 0.01, -0.02, 0.5, 0.9]]])
    for eps, cmpp in ((0.16, 0.25), (0.0151, 0.25)):
        s = _settings(fm3d, pair.cam, neighEpsilon=eps, cmPerPixel=cmpp)
        ctx = fm3d.Context(s)
        try:
            got = fm3d.NeighborhoodsGenerator(s).computeSquareNeighborhoodsByNormals(ctx, frames)
        finally:
            ctx.close()
        ref = orc.square_neighborhoods(frames, eps, cmpp)
        assert got.shape == ref.shape and got.shape[1] == orc.patch_size(eps, cmpp) ** 2
        assert np.array_equal(got, ref), (eps, cmpp)


# ---------------------------------------------------------------- BASELINE configs as parity cases
@pytest.mark.parametrize("given_normals", [True, False])
def test_circular_neighborhoods_bitwise(fm3d, orc, pair, given_normals):
    """computeCircularNeighborhoodsByNormals (neighborhoodsgenerator.cpp:160-224) on the GPU against the
    oracle, bit for bit: triangulated points of the frame pair with their LM-free initial normals
    perturbed (given) or the empty-normals branch (X/|X|), the reference's 15 x 5 samples."""
    rng = np.random.default_rng(32)
    X = np.stack([rng.uniform(-0.6, 0.6, 700), rng.uniform(-0.4, 0.4, 700), rng.uniform(1.6, 2.3, 700)], 1)
    N = X + rng.normal(0, 0.3, X.shape)
    N /= np.linalg.norm(N, axis=1, keepdims=True)
    s = _settings(fm3d, pair.cam, neighMethod=1, neighThetas=15, neighRays=5)
    ctx = fm3d.Context(s)
    try:
        ng = fm3d.NeighborhoodsGenerator(s)
        got = ng.computeCircularNeighborhoodsByNormals(ctx, X, N if given_normals else None)
        ref = orc.circular_neighborhoods(X, N if given_normals else None, s.neighEpsilon, 15, 5)
        assert got.shape == (700, 75, 3) and np.array_equal(got, ref)
        one = ng.computeCircularNeighborhoodByNormal(ctx, X[3], N[3] if given_normals else (0.0, 0.0, 0.0))
        assert np.array_equal(one, ref[3])
        assert ng.computeCircularNeighborhoodsByNormals(ctx, np.zeros((0, 3))).shape == (0, 75, 3)
    finally:
        ctx.close()


# (3, 4) and (5, 5): the partial instances (H 9..15 four hypotheses per wave, H 17..31 eight)
@pytest.mark.parametrize("ray,hphi,htheta", [(16, 4, 4), (32, 8, 4), (8, 1, 3), (16, 3, 4), (16, 5, 5)])
def test_ncc_hypotheses_bitwise(fm3d, orc, pair, ray, hphi, htheta):
    """NCC scoring of candidate normals (fm3d_ncc_hypotheses) on the GPU against the oracle, bit for
    bit: scores of every hypothesis, the best normal and its index (16 and 32 hypotheses, VGA bounds
    so that border points fail, a degenerate 1 x 3 grid)."""
    s = _settings(fm3d, pair.cam, pixelsRay=ray, boundWidth=640, boundHeight=480)
    ctx = fm3d.Context(s)
    try:
        sct = fm3d.SingleCameraTriangulator(ctx)
        sct.set_g12(pair.g12)
        R2, t2 = sct.camera2()
        no = fm3d.NormalOptimizer(ctx, sct)
        no.setImages(pair.img1, pair.img2)
        X = np.concatenate([pair.points[:300], [[0.0, 0.0, 0.0], [5.0, 5.0, 2.0]]])
        sc, nb, b = no.nccHypotheses(X, hphi, htheta, 0.4)
    finally:
        ctx.close()
    rs, rn, rb = orc.ncc_hypotheses(pair.cam, R2, t2, pair.img1, pair.img2, X, ray, hphi, htheta, 0.4, bound=(640, 480))
    assert np.array_equal(b, rb) and np.array_equal(sc, rs) and np.array_equal(nb, rn, equal_nan=True)
    assert np.isnan(nb[-2]).all() and b[-2] == -1  # X = 0: no pixel, the initial guess 0/0
    assert (b >= 0).mean() > 0.5


@pytest.mark.parametrize("cx,cy", [(0.0, 0.0), (-20.0, 10.0)])
def test_ncc_hypotheses_principal_point(fm3d, orc, pair, cx, cy):
    """NCC scoring with a principal point on / outside the image edge: the kernel's bit-pattern
    isPixelGood and fast divisions give the oracle's scores bit for bit."""
    import dataclasses
    cam = dataclasses.replace(pair.cam, cx=cx, cy=cy)
    s = _settings(fm3d, cam, pixelsRay=12, boundWidth=640, boundHeight=480)
    ctx = fm3d.Context(s)
    try:
        sct = fm3d.SingleCameraTriangulator(ctx)
        sct.set_g12(pair.g12)
        R2, t2 = sct.camera2()
        no = fm3d.NormalOptimizer(ctx, sct)
        no.setImages(pair.img1, pair.img2)
        X = np.concatenate([np.abs(pair.points[:200]), [[0.0, 0.0, 2.0], [0.05, 0.02, 2.0]]])
        sc, nb, b = no.nccHypotheses(X, 4, 4, 0.4)
    finally:
        ctx.close()
    rs, rn, rb = orc.ncc_hypotheses(cam, R2, t2, pair.img1, pair.img2, X, 12, 4, 4, 0.4, bound=(640, 480))
    assert np.array_equal(b, rb) and np.array_equal(sc, rs) and np.array_equal(nb, rn, equal_nan=True)
    assert (b >= 0).sum() > 0


def test_c2_sift10k_match_and_dlt(fm3d, orc, synth):
    """BASELINE configs[1] (C2): 10k SIFT-128 per frame, brute-force L2 match + NNDR + DLT --
    match indices, distances, inlier mask and points bit-exact against the oracle."""
    fp = synth.make_frame_pair(10_000, seed=101)
    ctx = fm3d.Context(_settings(fm3d, fp.cam))
    try:
        m = fm3d.DescriptorsMatcher(ctx).compareWithNNDR(0.55, fp.desc1, fp.desc2)
        sct = fm3d.SingleCameraTriangulator(ctx)
        sct.set_g12(fp.g12)
        sct.setKeypoints(fp.kp1, fp.kp2, m)
        pts, mask = sct.triangulate()
    finally:
        ctx.close()
    q, t, d = orc.match_nndr(fp.desc1, fp.desc2, orc.U8, 0.55, oracle_threads())
    assert np.array_equal(m["queryIdx"], q) and np.array_equal(m["trainIdx"], t) and np.array_equal(m["distance"], d)
    pto, masko = orc.triangulate(fp.cam, fp.g12, 1.5, 2.4, fp.kp1, fp.kp2, q, t)
    assert np.array_equal(mask, masko) and np.array_equal(pts, pto)
    assert len(q) > 8000 and np.mean(fp.true_train[q] == t) > 0.99


@pytest.mark.parametrize("ray,k", [(32, 150), (64, 96)])
def test_c3_orb10k_pipeline(fm3d, orc, synth, ray, k):
    """BASELINE configs[2] (C3): 10k ORB-256 (Hamming) + normals, through the device-resident
    pipeline, in SURVEY.md §8(d)'s two variants: 64x64-pixel neighbourhoods (pixelsRay 32) and
    pixelsRay 64.  Matching and DLT are checked in full; the LM on a seeded random sample of k
    inliers bit-exact against the oracle's DETMATH mode run here (which points survive, and their
    normals), and every survivor record byte for byte against the committed oracle run over ALL
    inliers (tests/golden/full_c3r<ray>.npz; the generated inputs' digests are checked first)."""
    mod, fx = full_fixture(f"c3r{ray}")
    fp = synth.make_frame_pair(10_000, seed=102, desc="orb")
    assert_inputs(mod, fx, fp)
    s = _settings(fm3d, fp.cam, pixelsRay=ray, nndrEpsilon=0.8)
    ctx = fm3d.Context(s)
    try:
        sct = fm3d.SingleCameraTriangulator(ctx)
        sct.set_g12(fp.g12)
        R2, t2 = sct.camera2()
        pipe = fm3d.Pipeline(ctx)
        pipe.upload(fp.desc1, fp.desc2, fp.kp1, fp.kp2, fp.img1, fp.img2, binary=True)
        n, stats = pipe.run()
        rec = pipe.records(n)
    finally:
        ctx.close()
    q, t, d = orc.match_nndr(fp.desc1, fp.desc2, orc.BITS, 0.8, oracle_threads())
    assert stats["matches"] == len(q)
    pts, mask = orc.triangulate(fp.cam, fp.g12, 1.5, 2.4, fp.kp1, fp.kp2, q, t)
    assert stats["inliers"] == len(pts)
    # survivors: in match order, each carrying its match and its triangulated point
    pos = np.searchsorted(q[mask], rec["queryIdx"])
    assert (np.diff(rec["queryIdx"]) > 0).all() and np.array_equal(q[mask][pos], rec["queryIdx"])
    assert np.array_equal(rec["trainIdx"], t[mask][pos]) and np.array_equal(rec["distance"], d[mask][pos])
    assert np.array_equal(rec["point"], pts[pos])
    # every survivor record against the oracle's DETMATH run over all inliers (full_c3r<ray>.npz)
    assert rec.tobytes() == fx["records"].tobytes()
    sel = np.sort(np.random.default_rng(1000 + ray).choice(len(pts), k, replace=False))
    ref = orc.optimize_normals(fp.cam, R2, t2, fp.img1, fp.img2, 3, pts[sel], ray, mode=orc.DETMATH,
                               nthreads=oracle_threads())
    ok = ref["status"] == 0
    assert np.array_equal(np.isin(sel, pos), ok)
    assert np.array_equal(rec[np.isin(pos, sel)]["normal"], ref["normals"][ok])
    assert ok.sum() > k // 4 and n > 0.3 * len(pts)


def test_c3_ncc_leg_16_hypotheses_r32(fm3d, orc, synth):
    """the C3 NCC leg -- 16 normal hypotheses (4 x 4 over a 0.4 rad span) scored by NCC
    over pixelsRay-32 neighbourhoods for EVERY DLT inlier of the 10k-ORB pair (configs[2]); a seeded
    1,000-point sample bit-exact against the oracle (scores, best normal, best index)."""
    fp = synth.make_frame_pair(10_000, seed=102, desc="orb")
    q, t, _ = orc.match_nndr(fp.desc1, fp.desc2, orc.BITS, 0.8, oracle_threads())
    pts, _ = orc.triangulate(fp.cam, fp.g12, 1.5, 2.4, fp.kp1, fp.kp2, q, t)
    s = _settings(fm3d, fp.cam, pixelsRay=32, nndrEpsilon=0.8, boundWidth=640, boundHeight=480)
    ctx = fm3d.Context(s)
    try:
        sct = fm3d.SingleCameraTriangulator(ctx)
        sct.set_g12(fp.g12)
        R2, t2 = sct.camera2()
        no = fm3d.NormalOptimizer(ctx, sct)
        no.setImages(fp.img1, fp.img2)
        sc, nb, b = no.nccHypotheses(pts, 4, 4, 0.4)
    finally:
        ctx.close()
    assert sc.shape == (len(pts), 16) and len(pts) > 5000
    sel = np.sort(np.random.default_rng(33).choice(len(pts), 1000, replace=False))
    rs, rn, rb = orc.ncc_hypotheses(fp.cam, R2, t2, fp.img1, fp.img2, pts[sel], 32, 4, 4, 0.4, bound=(640, 480))
    assert np.array_equal(b[sel], rb) and np.array_equal(sc[sel], rs) and np.array_equal(nb[sel], rn, equal_nan=True)
    assert (b >= 0).mean() > 0.5


# ---------------------------------------------------------------- error paths and part boundaries
def test_knn2_u8_train_parts_ties(fm3d, orc, ctx):
    """A small query set against >= 4096 train rows: the u8 kernel splits the train tiles into
    parts (knn2_u8_parts) merged by knn2_int_merge.  Duplicated train rows in different parts
    must resolve to the lowest trainIdx for both neighbours."""
    rng = np.random.default_rng(21)
    nB = 9001
    B = rng.integers(0, 256, (nB, 128), dtype=np.uint8)
    # 402 queries leave CUs idle, so the train tiles split into parts; row 2304 starts a tile at either
    # tile size (18 x 128 = 9 x 256) and started part 1 with round 4's 128-row tiles
    B[5000:5100] = B[10:110]        # duplicates in a later part
    B[nB - 1] = B[3]                # and in the last, partial tile
    B[2304] = B[3]                  # and on the first row of part 1
    A = np.concatenate([B[10:110], B[[3, 3]], rng.integers(0, 256, (300, 128), dtype=np.uint8)])
    got = fm3d.DescriptorsMatcher(ctx).knn_match(A, B)
    idx, dist = orc.knn2(A, B, orc.U8, oracle_threads())
    assert np.array_equal(got["trainIdx"], idx)
    assert np.array_equal(got["distance"], dist)
    assert (idx[:100, 0] == np.arange(10, 110)).all() and (idx[:100, 1] == np.arange(5000, 5100)).all()
    assert idx[100, 0] == 3 and idx[100, 1] == 2304


@pytest.mark.parametrize("nA", [402, 3000])
def test_knn2_u8_256_row_tiles_ties(fm3d, orc, ctx, nA):
    """Round 5: 128-byte u8 rows run in 256-row train tiles with an 8-bit row index in the packed key
    (knn2_i8_kernel<4, false, 2, 256>, 256 queries per workgroup).  Exact duplicates of one row in the
    tile's upper half (row index > 127: the eighth bit), on the first row of the next tile, on the
    first row of a part (402 queries: 9 parts of 4 tiles, part 1 from row 1024), in the last partial
    tile, and distances at the 24-bit key's extremes (all-0 and all-255 rows) must resolve exactly as
    the scan does: the lowest trainIdx first, for both neighbours."""
    rng = np.random.default_rng(31 + nA)
    nB = 9001
    B = rng.integers(0, 256, (nB, 128), dtype=np.uint8)
    for r in (200, 256, 1024, nB - 1):
        B[r] = B[3]
    B[700] = 0
    B[701] = 255
    A = np.concatenate([B[[3, 3, 200, 700, 701]], np.zeros((1, 128), np.uint8), np.full((1, 128), 255, np.uint8),
                        rng.integers(0, 256, (nA - 7, 128), dtype=np.uint8)])
    got = fm3d.DescriptorsMatcher(ctx).knn_match(A, B)
    idx, dist = orc.knn2(A, B, orc.U8, oracle_threads())
    assert np.array_equal(got["trainIdx"], idx)
    assert np.array_equal(got["distance"], dist)
    assert tuple(idx[0]) == (3, 200) and tuple(idx[2]) == (3, 200)
    assert idx[5, 0] == 700 and idx[6, 0] == 701


@pytest.mark.parametrize("mfma", ["1", "0"])
@pytest.mark.parametrize("nA", [402, 3000])
def test_knn2_bits_parts_and_ties(fm3d, orc, ctx, mfma, nA, monkeypatch):
    """256-bit rows on the int8-MFMA kernel (unpacked bits, packed per-tile keys) and on the
    popcount kernel: duplicated train rows inside one tile (different 32-row blocks), across tiles
    and across parts, plus the many natural Hamming ties of random strings, must all resolve to the
    lowest trainIdx for both neighbours."""
    monkeypatch.setenv("FM3D_BITS_MFMA", mfma)
    rng = np.random.default_rng(23 + nA)
    nB = 9001
    B = rng.integers(0, 256, (nB, 32), dtype=np.uint8)
    B[115] = B[3]; B[125] = B[3]        # same tile, other row blocks (other chain)
    B[5000:5100] = B[10:110]            # later tile / part
    B[nB - 1] = B[3]; B[2304] = B[3]    # last partial tile, first row of a part
    A = np.concatenate([B[10:110], B[[3, 3]], rng.integers(0, 256, (nA - 102, 32), dtype=np.uint8)])
    got = fm3d.DescriptorsMatcher(ctx, binary=True).knn_match(A, B)
    idx, dist = orc.knn2(A, B, orc.BITS, oracle_threads())
    assert np.array_equal(got["trainIdx"], idx)
    assert np.array_equal(got["distance"], dist)
    assert (idx[:100, 0] == np.arange(10, 110)).all() and (idx[:100, 1] == np.arange(5000, 5100)).all()
    assert idx[100, 0] == 3 and idx[100, 1] == 115


def test_knn2_u8_ties_inside_tile_chains(fm3d, orc, ctx):
    """Equal distances at rows of the same 128-row tile held by the two epilogue chains (even and
    odd 32-row blocks) and by the two lane halves: the packed per-tile key orders them by row."""
    rng = np.random.default_rng(24)
    B = rng.integers(0, 256, (700, 128), dtype=np.uint8)
    for r in (36, 68, 100, 133, 165, 4, 5):
        B[r] = B[1]
    A = np.concatenate([B[[1, 36, 133]], rng.integers(0, 256, (200, 128), dtype=np.uint8)])
    got = fm3d.DescriptorsMatcher(ctx).knn_match(A, B)
    idx, dist = orc.knn2(A, B, orc.U8, 1)
    assert np.array_equal(got["trainIdx"], idx)
    assert np.array_equal(got["distance"], dist)
    assert list(got["trainIdx"][0]) == [1, 4]


def test_knn2_integer_valued_f32_wider_than_u8_kernel(fm3d, orc, ctx):
    """Integer-valued f32 rows longer than the u8 kernel's 256 bytes stay on the f32 kernel."""
    rng = np.random.default_rng(22)
    A = rng.integers(0, 256, (300, 300)).astype(np.float32)
    B = rng.integers(0, 256, (500, 300)).astype(np.float32)
    got = fm3d.DescriptorsMatcher(ctx).knn_match(A, B)
    idx, dist = orc.knn2(A, B, orc.F32, oracle_threads())
    assert np.array_equal(got["trainIdx"], idx)
    assert np.array_equal(got["distance"], dist)


def test_optimize_normals_empty_on_fresh_context(fm3d, pair):
    """computeOptimizedNormals on an empty vector returns at once (the reference loop body never
    runs); the LM counters of a fresh context are reset, not read uninitialised."""
    ctx = fm3d.Context(_settings(fm3d, pair.cam, pixelsRay=8))
    try:
        sct = fm3d.SingleCameraTriangulator(ctx)
        sct.set_g12(pair.g12)
        no = fm3d.NormalOptimizer(ctx, sct)
        no.setImages(pair.img1, pair.img2)
        kept, normals = no.computeOptimizedNormals(np.zeros((0, 3)))
        assert kept.shape == (0, 3) and normals.shape == (0, 3)
        assert no.last_stats["evaluations"] == 0
    finally:
        ctx.close()


def test_pipeline_watchdog_raises(fm3d, pair, monkeypatch):
    """A tripped LM watchdog (FM3D_LM_MAX_SECONDS) is an error of fm3d_pipeline_run, not a
    silent drop of the unfinished points; the context stays usable afterwards."""
    s = _settings(fm3d, pair.cam, pixelsRay=24)
    ctx = fm3d.Context(s)
    try:
        sct = fm3d.SingleCameraTriangulator(ctx)
        sct.set_g12(pair.g12)
        pipe = fm3d.Pipeline(ctx)
        pipe.upload(pair.desc1, pair.desc2, pair.kp1, pair.kp2, pair.img1, pair.img2)
        monkeypatch.setenv("FM3D_LM_MAX_SECONDS", "0.0002")
        with pytest.raises(fm3d.Fm3dError, match="guard"):
            pipe.run()
        monkeypatch.setenv("FM3D_LM_MAX_SECONDS", "300")
        n, stats = pipe.run()
        assert n > 0 and stats["kept"] == n
    finally:
        ctx.close()


# ---------------------------------------------------------------- C4 and C5 at full size
@pytest.mark.timeout(600)
def test_c4_sift100k_full_pipeline(fm3d, orc, synth):
    """BASELINE configs[3] (C4) -- the bench workload itself (seed 7): 100k SIFT-128 per 640x480
    frame, pixelsRay 64, pyramids 3, through the device-resident pipeline.
      * knn: a seeded 16k-query sample bit-exact against the oracle (trainIdx, distance);
      * NNDR: every one of the 100k queries (the oracle's NNDR on the GPU's knn lists);
      * DLT: all matches, inlier mask and points bit-exact;
      * records: every survivor's (queryIdx, trainIdx, distance, point) equal to its match / point;
      * the whole result: the generated inputs' digests equal the fixture's, then ALL 36,143
        survivor records byte for byte against the oracle's DETMATH run over all 71,238 inliers
        (tests/golden/full_c4.npz, made by tests/golden/make_full_fixtures.py in the container);
      * LM vs libm (STRICT) on a seeded random 128-point sample: the same statuses, and each kept
        point's |n - n_libm| exactly the one tools/full_parity.py measured for it over the whole
        set (tests/golden/full_parity_c4.npz, DESIGN.md §4: with the correctly rounded
        transcendentals 36,141 of the 36,143 kept normals are within 1e-4 of libm's, the other two
        within 4.4e-3 through glibc's sin; measured over the whole set, not a sampled 99 %)."""
    mod, fx = full_fixture("c4")
    fp = synth.make_frame_pair(100_000, 640, 480, seed=7)
    assert_inputs(mod, fx, fp)
    s = _settings(fm3d, fp.cam, pixelsRay=64, pyramids=3)
    ctx = fm3d.Context(s)
    try:
        sct = fm3d.SingleCameraTriangulator(ctx)
        sct.set_g12(fp.g12)
        R2, t2 = sct.camera2()
        pipe = fm3d.Pipeline(ctx)
        pipe.upload(fp.desc1, fp.desc2, fp.kp1, fp.kp2, fp.img1, fp.img2)
        n, stats = pipe.run()
        rec = pipe.records(n)
        dm = fm3d.DescriptorsMatcher(ctx)
        knn = dm.knn_match(fp.desc1, fp.desc2)
        m = dm.compareWithNNDR(0.55, fp.desc1, fp.desc2)
        sct.setKeypoints(fp.kp1, fp.kp2, m)
        pts, mask = sct.triangulate()
    finally:
        ctx.close()
    rng = np.random.default_rng(44)
    qs = np.sort(rng.choice(len(fp.desc1), 16_384, replace=False))
    idx, dist = orc.knn2(fp.desc1[qs], fp.desc2, orc.U8, oracle_threads())
    assert np.array_equal(knn["trainIdx"][qs], idx) and np.array_equal(knn["distance"][qs], dist)
    q, t, d = orc.nndr(knn["trainIdx"], knn["distance"], 0.55)
    assert np.array_equal(m["queryIdx"], q) and np.array_equal(m["trainIdx"], t) and np.array_equal(m["distance"], d)
    assert stats["matches"] == len(q) > 80_000
    pto, masko = orc.triangulate(fp.cam, fp.g12, 1.5, 2.4, fp.kp1, fp.kp2, q, t)
    assert np.array_equal(mask, masko) and np.array_equal(pts, pto)
    assert stats["inliers"] == len(pts)
    # survivors: in match order, each carrying its match and its triangulated point
    pos = np.searchsorted(q[mask], rec["queryIdx"])
    assert (np.diff(rec["queryIdx"]) > 0).all() and np.array_equal(q[mask][pos], rec["queryIdx"])
    assert np.array_equal(rec["trainIdx"], t[mask][pos]) and np.array_equal(rec["distance"], d[mask][pos])
    assert np.array_equal(rec["point"], pts[pos])
    # EVERY survivor record (all 71,238 inliers through the LM) byte for byte against the oracle's
    # DETMATH run of the whole frame pair (tests/golden/full_c4.npz)
    assert n == len(fx["records"]) and tuple(fx["counts"]) == (100_000, stats["matches"], stats["inliers"], n)
    assert rec.tobytes() == fx["records"].tobytes()
    assert mod.records_digest(rec) == str(fx["records_sha256"])
    # libm (STRICT) on a seeded random sample of the inliers
    sel = np.sort(rng.choice(len(pts), 128, replace=False))
    kept_sel = np.isin(sel, pos)
    ok = kept_sel
    got = rec[np.isin(pos, sel)]
    strict = orc.optimize_normals(fp.cam, R2, t2, fp.img1, fp.img2, 3, pts[sel], 64, mode=orc.STRICT,
                                  nthreads=oracle_threads())
    assert np.array_equal(strict["status"] == 0, kept_sel)
    dev = np.abs(got["normal"] - strict["normals"][ok]).max(axis=1)
    print(f"C4 LM sample: {ok.sum()} of 128 kept; max |n - n_libm| {dev.max():.3g}, "
          f"{int((dev > 1e-4).sum())} beyond 1e-4")
    fpar = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "full_parity_c4.npz"),
                   allow_pickle=False)
    # the full-set measurement belongs to the fixture's contract (tools/full_parity.py records the
    # records digest of the DETMATH run it compared; a fixture of an earlier contract has none)
    same = "records_sha256" in fpar.files and str(fpar["records_sha256"]) == str(fx["records_sha256"])
    if same:
        assert np.array_equal(fpar["status_strict"][sel] == 0, kept_sel)
        assert np.array_equal(dev, fpar["dn_strict"][sel][ok])  # the full-set measurement, point for point
        both = (fpar["status_detmath"] == 0) & (fpar["status_strict"] == 0)
        # the whole set: 36,141 of the 36,143 kept normals within 1e-4 of libm's; the two
        # others (4.4e-3 at most) move with glibc's sin, which is not correctly rounded everywhere
        assert int((fpar["dn_strict"][both] > 1e-4).sum()) <= 2 and fpar["dn_strict"][both].max() < 1e-2
    else:
        print("full_parity_c4.npz is of an earlier contract: the sample alone is checked")
        assert (dev <= 1e-4).all()
    assert ok.sum() > 40


@pytest.mark.timeout(900)
def test_c5_1m_keypoints_query_blocks(fm3d, orc, synth):
    """BASELINE configs[4] (C5) on one GPU: one 1M-keypoint frame pair (640x480, sub-pixel
    keypoints; pixelsRay 64, pyramids 3) run whole and as the 4 block-cyclic
    shares of a 4-GPU run (bench.py --gpus 4): the merged share records are byte-identical to
    the whole run.  Every 10th 4,096-query block (102,400 queries, 36,455 survivors) against the
    committed oracle run over all 1M train rows (tests/golden/full_c5sub.npz),
    record for record; and a seeded 2,000-query sample through the oracle here (match, NNDR, DLT, LM
    in DETMATH mode): the whole run's records of those queries are exactly the oracle's survivors."""
    shard = importlib.import_module("3dfeaturematcher_amd.shard")
    mod, fx = full_fixture("c5sub")
    fp = synth.make_frame_pair(1_000_000, 640, 480, seed=7)
    assert_inputs(mod, fx, fp)
    s = _settings(fm3d, fp.cam, pixelsRay=64, pyramids=3)
    n = len(fp.desc1)
    full = shard.run_shard(fp, s, 0, n)
    qsel = mod.subset_queries(mod.WORKLOADS["c5sub"], n)
    sub10 = full[np.isin(full["queryIdx"], qsel)]
    assert len(sub10) == len(fx["records"]) == 36_455 and sub10.tobytes() == fx["records"].tobytes()
    parts = [shard.run_shard_queries(fp, s, shard.query_blocks(n, 4, r)) for r in range(4)]
    merged = np.concatenate(parts)
    merged = merged[np.argsort(merged["queryIdx"], kind="stable")]
    assert len(full) > 200_000
    assert merged.tobytes() == full.tobytes()
    rng = np.random.default_rng(55)
    qs = np.sort(rng.choice(n, 2000, replace=False))
    q, t, d = orc.match_nndr(fp.desc1[qs], fp.desc2, orc.U8, 0.55, oracle_threads())
    pts, mask = orc.triangulate(fp.cam, fp.g12, 1.5, 2.4, fp.kp1[qs], fp.kp2, q, t)
    R2, t2 = fm3d.camera2_from_g12(fp.g12)
    ref = orc.optimize_normals(fp.cam, R2, t2, fp.img1, fp.img2, 3, pts, 64, mode=orc.DETMATH,
                               nthreads=oracle_threads())
    ok = ref["status"] == 0
    sub = full[np.isin(full["queryIdx"], qs)]
    assert np.array_equal(sub["queryIdx"], qs[q[mask][ok]])
    assert np.array_equal(sub["trainIdx"], t[mask][ok]) and np.array_equal(sub["distance"], d[mask][ok])
    assert np.array_equal(sub["point"], pts[ok])
    assert np.array_equal(sub["normal"], ref["normals"][ok])
    assert ok.sum() > 500


# ---------------------------------------------------------------- multi-GPU behind the C ABI (fm3d_mgpu)
@pytest.mark.parametrize("n,block,shares", [(3000, 256, 4), (20_000, 4096, 4), (5, 4096, 4)])
def test_mgpu_one_device_shares_equal_pipeline_run(fm3d, synth, n, block, shares):
    """fm3d_mgpu with an ndev = 1 RCCL communicator and `shares` logical shares
    (block-cyclic query blocks, run one after the other on the device, records written into the
    all-gather send buffer, ncclAllGather, C++ merge): byte-identical to fm3d_pipeline_run of the
    whole frame pair.  (5 queries: three of the four shares are empty.)"""
    pair = synth.make_frame_pair(n, seed=31)
    s = _settings(fm3d, pair.cam, pixelsRay=12, pyramids=1)
    ctx = fm3d.Context(s)
    try:
        sct = fm3d.SingleCameraTriangulator(ctx)
        sct.set_g12(pair.g12)
        pipe = fm3d.Pipeline(ctx)
        pipe.upload(pair.desc1, pair.desc2, pair.kp1, pair.kp2, pair.img1, pair.img2)
        k, st = pipe.run()
        full = pipe.records(k)
    finally:
        ctx.close()
    mg = fm3d.MultiGPU(s, devices=[0], shares=shares, block=block)
    try:
        mg.set_g12(pair.g12)
        mg.upload(pair.desc1, pair.desc2, pair.kp1, pair.kp2, pair.img1, pair.img2)
        rec, mst = mg.run()
        rec2, _ = mg.run()  # re-run on the staged inputs
    finally:
        mg.close()
    assert rec.tobytes() == full.tobytes() and rec2.tobytes() == full.tobytes()
    assert mst["kept"] == k and mst["matches"] == st["matches"] and mst["inliers"] == st["inliers"]
    if n >= 3000:
        assert k > 50


@pytest.mark.parametrize("cx,cy", [(0.0, 0.0), (-0.0, -0.0), (-20.0, 10.0)])
def test_principal_point_zero_and_negative(fm3d, orc, pair, cx, cy):
    """computeOptimizedNormals with a principal point on or outside the image's
    top/left edge (the reference has no limit there) -- bit-exact against the oracle, which runs the
    reference's comparisons with the same camera.  The kernel's bit-pattern isPixelGood differs
    from `0 <= u` only for u == -0.0, which only cx == -0.0 can produce; the host hands the kernel
    +0.0 there (fm3d_host.cpp lm_camera)."""
    import dataclasses
    cam = dataclasses.replace(pair.cam, cx=cx, cy=cy)
    q, t, _ = orc.match_nndr(pair.desc1, pair.desc2, orc.U8, 0.55, oracle_threads())
    pts, _ = orc.triangulate(pair.cam, pair.g12, 1.5, 2.4, pair.kp1, pair.kp2, q, t)
    # points around the optical axis: with cx = cy = 0 their neighbourhoods straddle u = 0 / v = 0
    extra = np.array([[0.0, 0.0, 2.0], [1e-3, 1e-3, 2.0], [0.05, 0.02, 2.0], [0.2, 0.15, 2.1], [0.4, 0.3, 1.9]])
    P = np.concatenate([np.abs(pts[:40]), extra])
    s = _settings(fm3d, cam, pixelsRay=8, pyramids=1)
    ctx = fm3d.Context(s)
    try:
        sct = fm3d.SingleCameraTriangulator(ctx)
        sct.set_g12(pair.g12)
        R2, t2 = sct.camera2()
        no = fm3d.NormalOptimizer(ctx, sct)
        no.setImages(pair.img1, pair.img2)
        kept, normals = no.computeOptimizedNormals(P)
        st, info, nfev = no.last_status, no.last_info, no.last_nfev
    finally:
        ctx.close()
    ref = orc.optimize_normals(cam, R2, t2, pair.img1, pair.img2, 1, P, 8, mode=orc.DETMATH,
                               nthreads=oracle_threads())
    assert np.array_equal(st, ref["status"])
    assert np.array_equal(info[:, :2], ref["info"][:, :2])
    assert np.array_equal(nfev[:, :2], ref["nfev"][:, :2])
    ok = ref["status"] == 0
    assert np.array_equal(normals, ref["normals"][ok])
    assert np.array_equal(kept, P[ok])
    assert ok.sum() > 0


def _pipe_ctx(fm3d, s, g12):
    ctx = fm3d.Context(s)
    fm3d.SingleCameraTriangulator(ctx).set_g12(g12)
    return ctx, fm3d.Pipeline(ctx)


def test_pipeline_submit_wait_stream_equals_run(fm3d, synth):
    """fm3d_pipeline_submit / fm3d_pipeline_wait (the headline's stream: inputs from host memory,
    device-side counts, two contexts in flight) give the records of fm3d_pipeline_run, byte for byte,
    for two different frame pairs taken in turn; the pending guards fail loudly."""
    pairs = [synth.make_frame_pair(3000, seed=11), synth.make_frame_pair(2500, seed=12)]
    s = _settings(fm3d, pairs[0].cam, pixelsRay=12, pyramids=2)
    ref = []
    ctx, pipe = _pipe_ctx(fm3d, s, pairs[0].g12)
    try:
        for fp in pairs:
            pipe.upload(fp.desc1, fp.desc2, fp.kp1, fp.kp2, fp.img1, fp.img2)
            k, st = pipe.run()
            ref.append((pipe.records(k), st))
    finally:
        ctx.close()
    cs = [_pipe_ctx(fm3d, s, pairs[0].g12) for _ in range(2)]
    try:
        got = []
        order = [0, 1, 0, 1, 1]
        pend = [None, None]
        for i, w in enumerate(order):
            j = i % 2
            if pend[j] is not None:
                got.append((pend[j], cs[j][1].wait()))
            fp = pairs[w]
            cs[j][1].submit(fp.desc1, fp.desc2, fp.kp1, fp.kp2, fp.img1, fp.img2)
            pend[j] = w
        for i in range(len(order), len(order) + 2):
            j = i % 2
            got.append((pend[j], cs[j][1].wait()))
        with pytest.raises(fm3d.Fm3dError):
            cs[0][1].wait()  # nothing pending
        fp = pairs[0]
        cs[0][1].submit(fp.desc1, fp.desc2, fp.kp1, fp.kp2, fp.img1, fp.img2)
        with pytest.raises(fm3d.Fm3dError):
            cs[0][1].run()  # a submit is pending
        got.append((0, cs[0][1].wait()))
    finally:
        for c, _ in cs:
            c.close()
    assert len(got) == len(order) + 1
    for w, (rec, st) in got:
        assert rec.tobytes() == ref[w][0].tobytes()
        for key in ("matches", "inliers", "kept"):
            assert st[key] == ref[w][1][key]
        assert st["lm"]["pixel_evaluations"] == ref[w][1]["lm"]["pixel_evaluations"]
        assert st["pyramid_ms"] > 0 and st["total_ms"] >= st["lm_ms"]
    assert len(ref[0][0]) > 50


def test_pipeline_linked_lm_launch_equals_run(fm3d, synth):
    """fm3d_pipeline_link: two contexts' frame pairs in ONE LM launch (the slots of a workgroup that
    run out of one pair's points take the other's): each pair's records, counts and evaluation
    counts equal its own fm3d_pipeline_run, bit for bit -- in both orders of different pairs, and
    for a member waited for before its leader's submit (its LM alone)."""
    pairs = [synth.make_frame_pair(3000, seed=11), synth.make_frame_pair(2500, seed=12)]
    s = _settings(fm3d, pairs[0].cam, pixelsRay=12, pyramids=2)
    ref = []
    ctx, pipe = _pipe_ctx(fm3d, s, pairs[0].g12)
    try:
        for fp in pairs:
            pipe.upload(fp.desc1, fp.desc2, fp.kp1, fp.kp2, fp.img1, fp.img2)
            k, st = pipe.run()
            ref.append((pipe.records(k), st))
    finally:
        ctx.close()
    cs = [_pipe_ctx(fm3d, s, pairs[0].g12) for _ in range(2)]
    member, leader = cs[0][1], cs[1][1]
    try:
        member.link(leader)
        got = []
        for wm, wl in ((0, 1), (1, 0), (1, 1)):
            a, b = pairs[wm], pairs[wl]
            member.submit(a.desc1, a.desc2, a.kp1, a.kp2, a.img1, a.img2)
            leader.submit(b.desc1, b.desc2, b.kp1, b.kp2, b.img1, b.img2)
            got += [(wm, member.wait()), (wl, leader.wait())]
        a = pairs[0]
        member.submit(a.desc1, a.desc2, a.kp1, a.kp2, a.img1, a.img2)
        got.append((0, member.wait()))  # no leader submit: the member's LM alone
        with pytest.raises(fm3d.Fm3dError):
            leader.link(member)  # linked already
    finally:
        for c, _ in cs:
            c.close()
    for w, (rec, st) in got:
        assert rec.tobytes() == ref[w][0].tobytes()
        for key in ("matches", "inliers", "kept"):
            assert st[key] == ref[w][1][key]
        assert st["lm"]["pixel_evaluations"] == ref[w][1]["lm"]["pixel_evaluations"]
        assert st["lm"]["evaluations"] == ref[w][1]["lm"]["evaluations"]


def test_pipeline_linked_member_waited_after_leader_resubmit(fm3d, synth):
    """submit(member), submit(leader), wait(leader), submit(leader), wait(member).  The
    leader's second launch resets its own LM counters; the member's epilogue reads its own copy of
    the linked launch's counters, so it reports that launch's (equal to what the leader reported for
    it) and its records equal its own fm3d_pipeline_run."""
    pairs = [synth.make_frame_pair(3000, seed=11), synth.make_frame_pair(2500, seed=12)]
    s = _settings(fm3d, pairs[0].cam, pixelsRay=12, pyramids=2)
    ctx, pipe = _pipe_ctx(fm3d, s, pairs[0].g12)
    try:
        ref = []
        for fp in pairs:
            pipe.upload(fp.desc1, fp.desc2, fp.kp1, fp.kp2, fp.img1, fp.img2)
            k, _ = pipe.run()
            ref.append(pipe.records(k))
    finally:
        ctx.close()
    cs = [_pipe_ctx(fm3d, s, pairs[0].g12) for _ in range(2)]
    member, leader = cs[0][1], cs[1][1]
    try:
        member.link(leader)
        a, b = pairs[0], pairs[1]
        member.submit(a.desc1, a.desc2, a.kp1, a.kp2, a.img1, a.img2)
        leader.submit(b.desc1, b.desc2, b.kp1, b.kp2, b.img1, b.img2)
        rec_l1, st_l1 = leader.wait()
        leader.submit(a.desc1, a.desc2, a.kp1, a.kp2, a.img1, a.img2)  # its own launch: counters reset
        rec_m, st_m = member.wait()
        rec_l2, st_l2 = leader.wait()
    finally:
        for c, _ in cs:
            c.close()
    assert rec_m.tobytes() == ref[0].tobytes()
    assert rec_l1.tobytes() == ref[1].tobytes() and rec_l2.tobytes() == ref[0].tobytes()
    for key in ("passes", "cycles_total", "cycles_terms", "wall_ticks_max"):
        assert st_m["lm"][key] == st_l1["lm"][key] > 0, key


def test_pipeline_linked_four_pairs(fm3d, synth):
    """A leader with three members: four frame pairs in one LM launch, each pair's records equal
    its own fm3d_pipeline_run; a member without a queued pair is skipped by its leader."""
    pairs = [synth.make_frame_pair(2000, seed=11), synth.make_frame_pair(1500, seed=12)]
    s = _settings(fm3d, pairs[0].cam, pixelsRay=10, pyramids=1)
    ref = []
    ctx, pipe = _pipe_ctx(fm3d, s, pairs[0].g12)
    try:
        for fp in pairs:
            pipe.upload(fp.desc1, fp.desc2, fp.kp1, fp.kp2, fp.img1, fp.img2)
            k, st = pipe.run()
            ref.append(pipe.records(k))
    finally:
        ctx.close()
    cs = [_pipe_ctx(fm3d, s, pairs[0].g12) for _ in range(4)]
    ps = [p for _, p in cs]
    try:
        for m in ps[:3]:
            m.link(ps[3])
        with pytest.raises(fm3d.Fm3dError):
            cs2 = _pipe_ctx(fm3d, s, pairs[0].g12)
            try:
                cs2[1].link(ps[3])  # a fourth member
            finally:
                cs2[0].close()
        for order, members in (((0, 1, 0, 1), (0, 1, 2)), ((1, 1, 0, 0), (0, 2))):
            for j in members:
                fp = pairs[order[j]]
                ps[j].submit(fp.desc1, fp.desc2, fp.kp1, fp.kp2, fp.img1, fp.img2)
            fp = pairs[order[3]]
            ps[3].submit(fp.desc1, fp.desc2, fp.kp1, fp.kp2, fp.img1, fp.img2)
            for j in list(members) + [3]:
                rec, _ = ps[j].wait()
                assert rec.tobytes() == ref[order[j]].tobytes(), (order, j)
    finally:
        for c, _ in cs:
            c.close()


def test_pipeline_linked_lm_two_poses(fm3d, synth):
    """Linked frame pairs with different camera-2 poses take the LM kernel's per-problem pose
    (lm2_kernel<true>): each pair's records equal its own fm3d_pipeline_run."""
    g12b = synth.reference_g12() @ _small_motion()
    pairs = [synth.make_frame_pair(3000, seed=11), synth.make_frame_pair(3000, seed=14, g12=g12b)]
    s = _settings(fm3d, pairs[0].cam, pixelsRay=12, pyramids=2)
    ref = []
    for fp in pairs:
        ctx, pipe = _pipe_ctx(fm3d, s, fp.g12)
        try:
            pipe.upload(fp.desc1, fp.desc2, fp.kp1, fp.kp2, fp.img1, fp.img2)
            k, st = pipe.run()
            ref.append((pipe.records(k), st))
        finally:
            ctx.close()
    cs = [_pipe_ctx(fm3d, s, fp.g12) for fp in pairs]
    try:
        cs[1][1].link(cs[0][1])  # pair 1's context (pose b) joins pair 0's launches (pose a)
        for _ in range(2):
            b, a = pairs[1], pairs[0]
            cs[1][1].submit(b.desc1, b.desc2, b.kp1, b.kp2, b.img1, b.img2)
            cs[0][1].submit(a.desc1, a.desc2, a.kp1, a.kp2, a.img1, a.img2)
            got = [cs[0][1].wait(), cs[1][1].wait()]
            for w in (0, 1):
                assert got[w][0].tobytes() == ref[w][0].tobytes()
                assert got[w][1]["lm"]["pixel_evaluations"] == ref[w][1]["lm"]["pixel_evaluations"]
    finally:
        for c, _ in cs:
            c.close()
    assert len(ref[0][0]) > 50 and len(ref[1][0]) > 50


def _small_motion():
    c, s_ = np.cos(0.03), np.sin(0.03)
    M = np.eye(4)
    M[:3, :3] = [[c, 0, s_], [0, 1, 0], [-s_, 0, c]]
    M[:3, 3] = [0.02, -0.01, 0.0]
    return M


def test_pipeline_ncc_download_after_other_runs(fm3d, synth):
    """fm3d_pipeline_ncc_download returns the rows of the last successful run_ncc,
    even after a run_dlt / run on a larger pair (which rewrite the inlier count)."""
    small, big = synth.make_frame_pair(1200, seed=41), synth.make_frame_pair(4000, seed=42)
    s = _settings(fm3d, small.cam, pixelsRay=8)
    ctx, pipe = _pipe_ctx(fm3d, s, small.g12)
    try:
        pipe.upload(small.desc1, small.desc2, small.kp1, small.kp2, small.img1, small.img2)
        P1, _ = pipe.run_ncc(4, 4, 0.4)
        sc1, nb1, b1 = pipe.ncc_results(P1, 16)
        pipe.upload(big.desc1, big.desc2, big.kp1, big.kp2, big.img1, big.img2)
        P2, _ = pipe.run_dlt()
        assert P2 > P1 > 0
        sc2, nb2, b2 = pipe.ncc_results(P1, 16)
        pipe.run()
        sc3, _, _ = pipe.ncc_results(P1, 16)
    finally:
        ctx.close()
    assert np.array_equal(sc1, sc2) and np.array_equal(b1, b2) and np.array_equal(nb1, nb2, equal_nan=True)
    assert np.array_equal(sc1, sc3)


def test_mgpu_submit_wait_stream_equals_run(fm3d, synth):
    """fm3d_mgpu_submit / fm3d_mgpu_wait (bench.py --gpus N's path) on one device with three logical
    shares (one replica, linked context sets: two pairs per LM launch, RCCL all-gather, host merge):
    byte-identical to fm3d_pipeline_run of the whole frame pair, pair after pair."""
    fp = synth.make_frame_pair(9000, seed=31)
    s = _settings(fm3d, fp.cam, pixelsRay=12, pyramids=1)
    ctx, pipe = _pipe_ctx(fm3d, s, fp.g12)
    try:
        pipe.upload(fp.desc1, fp.desc2, fp.kp1, fp.kp2, fp.img1, fp.img2)
        k, st = pipe.run()
        full = pipe.records(k)
    finally:
        ctx.close()
    mg = fm3d.MultiGPU(s, devices=[0], shares=3, block=1024)
    try:
        mg.set_g12(fp.g12)
        outs = []
        for i in range(4):
            if i >= 2:
                outs.append(mg.wait())
            mg.submit(fp.desc1, fp.desc2, fp.kp1, fp.kp2, fp.img1, fp.img2)
        outs += [mg.wait(), mg.wait()]
        with pytest.raises(fm3d.Fm3dError):
            mg.wait()
        # a pair on a member set waited for before its leader set takes one: its LM alone
        mg.submit(fp.desc1, fp.desc2, fp.kp1, fp.kp2, fp.img1, fp.img2)
        outs.append(mg.wait())
        # a submit restaged set 0: run without a new upload fails loudly, with one it works
        with pytest.raises(fm3d.Fm3dError):
            mg.run()
        mg.upload(fp.desc1, fp.desc2, fp.kp1, fp.kp2, fp.img1, fp.img2)
        outs.append(mg.run())
    finally:
        mg.close()
    assert k > 50
    for rec, mst in outs:
        assert rec.tobytes() == full.tobytes()
        assert mst["kept"] == k and mst["inliers"] == st["inliers"]


def test_mgpu_eight_aliased_devices_equal_run(fm3d, synth, monkeypatch):
    """The 8-device code of fm3d_mgpu on a one-GPU box. In test mode FM3D_DEBUG_MGPU_ALIAS=1 device 0
    may be listed eight times. Each entry runs as its own device: its own four context sets, its
    host submit thread, its block-cyclic share of the queries (12 shares of 512-query blocks) and its
    memory pre-flight (summed per physical GPU). The all-gather becomes the same copies on the
    streams, since RCCL refuses a device twice. Both fm3d_mgpu_pipeline_run and the submit / wait
    stream merge the eight lists into records byte-identical to one fm3d_pipeline_run of the whole
    pair. Without the variable, a repeated device is refused."""
    fp = synth.make_frame_pair(9000, seed=33)
    s = _settings(fm3d, fp.cam, pixelsRay=12, pyramids=1)
    ctx, pipe = _pipe_ctx(fm3d, s, fp.g12)
    try:
        pipe.upload(fp.desc1, fp.desc2, fp.kp1, fp.kp2, fp.img1, fp.img2)
        k, st = pipe.run()
        full = pipe.records(k)
    finally:
        ctx.close()
    with pytest.raises(fm3d.Fm3dError) as e:
        fm3d.MultiGPU(s, devices=[0, 0])
    assert e.value.code == fm3d.ERR_INVALID
    monkeypatch.setenv("FM3D_DEBUG_MGPU_ALIAS", "1")
    mg = fm3d.MultiGPU(s, devices=[0] * 8, shares=12, block=512)
    try:
        mg.set_g12(fp.g12)
        mg.upload(fp.desc1, fp.desc2, fp.kp1, fp.kp2, fp.img1, fp.img2)
        outs = [mg.run()]
        for i in range(6):
            if i >= 4:
                outs.append(mg.wait())
            mg.submit(fp.desc1, fp.desc2, fp.kp1, fp.kp2, fp.img1, fp.img2)
        outs += [mg.wait() for _ in range(4)]
    finally:
        mg.close()
    assert k > 50 and len(outs) == 7
    for rec, mst in outs:
        assert rec.tobytes() == full.tobytes()
        assert mst["kept"] == k and mst["inliers"] == st["inliers"] and mst["queries"] == 9000


def test_mgpu_more_devices_than_visible_fails(fm3d, pair):
    """fm3d_mgpu_create over more devices than the box has: FM3D_ERR_INVALID, never a silent
    one-GPU run (bench.py --gpus N relies on it)."""
    s = _settings(fm3d, pair.cam)
    import torch
    vis = torch.cuda.device_count()
    with pytest.raises(fm3d.Fm3dError) as e:
        fm3d.MultiGPU(s, devices=list(range(vis + 1)))
    assert e.value.code == fm3d.ERR_INVALID


def test_mgpu_memory_preflight_nomem(fm3d, synth, monkeypatch):
    """fm3d_mgpu pre-flights device memory before anything grows.  With the device
    pretending to have 1 GiB free (FM3D_DEBUG_FREE_MB), creation fails cleanly with FM3D_ERR_NOMEM
    and the shortfall in fm3d_mgpu_last_error(NULL) (four context sets' LM slabs do not fit); a
    created one given 300 MiB refuses a 20k-keypoint pair's buffers at upload, before staging; with
    the real free memory the same object then takes the pair, and its records equal
    fm3d_pipeline_run's."""
    fp = synth.make_frame_pair(20_000, seed=61)
    s = _settings(fm3d, fp.cam, pixelsRay=64, pyramids=3)
    monkeypatch.setenv("FM3D_DEBUG_FREE_MB", "1024")
    with pytest.raises(fm3d.Fm3dError) as e:
        fm3d.MultiGPU(s, devices=[0])
    assert e.value.code == fm3d.ERR_NOMEM
    assert "MiB more needed" in str(e.value), str(e.value)
    monkeypatch.delenv("FM3D_DEBUG_FREE_MB")
    mg = fm3d.MultiGPU(s, devices=[0])
    try:
        mg.set_g12(fp.g12)
        monkeypatch.setenv("FM3D_DEBUG_FREE_MB", "300")
        with pytest.raises(fm3d.Fm3dError) as e:
            mg.upload(fp.desc1, fp.desc2, fp.kp1, fp.kp2, fp.img1, fp.img2)
        assert e.value.code == fm3d.ERR_NOMEM and "MiB more needed" in str(e.value)
        monkeypatch.delenv("FM3D_DEBUG_FREE_MB")
        mg.upload(fp.desc1, fp.desc2, fp.kp1, fp.kp2, fp.img1, fp.img2)
        rec, _ = mg.run()
    finally:
        mg.close()
    ctx = fm3d.Context(s)
    try:
        fm3d.SingleCameraTriangulator(ctx).set_g12(fp.g12)
        pipe = fm3d.Pipeline(ctx)
        pipe.upload(fp.desc1, fp.desc2, fp.kp1, fp.kp2, fp.img1, fp.img2)
        n, _ = pipe.run()
        ref = pipe.records(n)
    finally:
        ctx.close()
    assert rec.tobytes() == ref.tobytes() and len(rec) > 1000


def test_bench_gpus_more_than_visible_exits_nonzero():
    """`bench.py --gpus N` with fewer than N GPUs visible exits non-zero with a clear
    message, never a one-GPU line labelled otherwise."""
    import os
    import subprocess
    import sys
    import torch
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    n = torch.cuda.device_count() + 1
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(n), "--steps", "1", "--warmup",
                        "0", "--no-cpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert f"--gpus {n}" in r.stderr and "visible" in r.stderr
    assert '"metric"' not in r.stdout


@pytest.mark.timeout(400)
def test_bench_mgpu_one_gpu_line_without_torch(tmp_path):
    """`bench.py --gpus 1 --mgpu` (the one-process multi-GPU route on this box's
    one GPU) never imports torch before fm3d_mgpu_create (the visible-device count comes from
    libfm3d's fm3d_device_count), and its line carries the same-workload one-GPU value and the
    efficiency the N-GPU lines report."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / "line.json"
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "1", "--mgpu", "--keypoints",
                        "200000", "--steps", "2", "--warmup", "1", "--no-cpu", "--out", str(out)],
                       capture_output=True, text=True, timeout=380)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(out.read_text())
    assert line["torch_imported_at_mgpu_create"] is False
    assert line["n_gpus"] == 1 and line["efficiency"] == 1.0 and line["value_one_gpu"] == line["value"] > 0
    assert line["records_identical_across_steps"] is True


@pytest.mark.timeout(500)
def test_bench_torchrun_stream_two_ranks_one_gpu(fm3d, synth, tmp_path):
    """bench.py's torchrun route (one process per GPU, frame pairs in flight, all-gather of every
    step's records, rank-0 merge) with two ranks on this one GPU and a gloo all-gather
    (FM3D_BENCH_BACKEND / FM3D_BENCH_SHARE_DEVICE): the merged records of the last step equal one
    fm3d_pipeline_run of the whole frame pair, byte for byte."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dump = tmp_path / "merged.npy"
    env = dict(os.environ, FM3D_BENCH_BACKEND="gloo", FM3D_BENCH_SHARE_DEVICE="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", "29631", os.path.join(root, "bench.py"), "--gpus", "2", "--workload", "c5",
           "--keypoints", "30000", "--steps", "3", "--warmup", "1", "--dump-records", str(dump)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["scaling"] == "strong" and line["value"] > 0
    merged = np.load(dump)
    # the same frame pair whole, one run
    pair = synth.make_frame_pair(30000, 640, 480, seed=7, desc="sift")
    s = fm3d.Settings.default()
    s.set_camera(pair.cam)
    s.nndrEpsilon, s.pixelsRay, s.pyramids = 0.55, 64, 3
    ctx = fm3d.Context(s)
    try:
        fm3d.SingleCameraTriangulator(ctx).set_g12(pair.g12)
        pipe = fm3d.Pipeline(ctx)
        pipe.upload(pair.desc1, pair.desc2, pair.kp1, pair.kp2, pair.img1, pair.img2)
        k, st = pipe.run()
        ref = pipe.records(k)
    finally:
        ctx.close()
    assert len(merged) == k > 1000
    assert merged.tobytes() == ref.tobytes()
