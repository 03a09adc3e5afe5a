"""The SIFT oracle (oracle/orc_sift.c): OpenCV 2.4.9's nonfree SIFT, the detector / extractor of
FeatureOptions DetectorType / ExtractorType SIFT (descriptorsmatcher.cpp:243-257, 302-315).

OpenCV is not in this image, so the restatement is pinned piece by piece:
  * getGaussianKernel, GaussianBlur on float (row taps in order, then the symmetric column sum with
    REFLECT_101 borders, repeated reflections on tiny images), resize INTER_LINEAR (float
    coefficients) and INTER_NEAREST, the pyramid sigmas: independent numpy restatements, bit for bit;
  * cv::exp's two code paths (the SSE2 lane in float, the scalar lane in double) restated in numpy,
    bit for bit, and both within 2 ulp of the true exponential; the element's position in the array
    picks the path;
  * the deterministic cosf / sinf / powf(2, y) of include/fm3d_cvmath.h are the correctly rounded
    floats on the inputs the detector produces (this image's glibc is not: the reference's libm
    stays unpinned);
  * Matx33f::solve (Cramer's rule) against numpy.linalg.solve, and its zero-determinant rule;
  * removeDuplicated against a numpy restatement;
  * properties of the whole detector: a Gaussian blob is found at its centre + 0.25 px (the
    INTER_LINEAR doubling's half-pixel shift every OpenCV 2.4 SIFT has), content translated by 32 px
    moves keypoints by 32 px with identical descriptors, compute() on detect()'s keypoints, the
    descriptor's norm and clamp.
Parity with OpenCV's own build stays unpinned where no fixture exists."""
import math

import numpy as np
import pytest

f32 = np.float32


def _reflect101(p, n):
    if n == 1:
        return 0
    while p < 0 or p >= n:
        p = -p if p < 0 else 2 * n - 2 - p
    return p


def _np_kernel(sigma):
    n = int(np.rint(sigma * 8 + 1)) | 1
    x = np.arange(n) - (n - 1) * 0.5
    cf = np.exp((-0.5 / (sigma * sigma)) * x * x).astype(f32)
    s = 0.0
    for v in cf:
        s += float(v)
    return (cf.astype(np.float64) * (1.0 / s)).astype(f32)


def _np_blur(img, sigma):
    img = img.astype(f32)
    h, w = img.shape
    f = _np_kernel(sigma)
    n = len(f)
    r = n // 2
    cols = np.array([[_reflect101(x - r + k, w) for x in range(w)] for k in range(n)])
    t = f[0] * img[:, cols[0]]
    for k in range(1, n):
        t = t + f[k] * img[:, cols[k]]
    rows_up = [np.array([_reflect101(y + k, h) for y in range(h)]) for k in range(r + 1)]
    rows_dn = [np.array([_reflect101(y - k, h) for y in range(h)]) for k in range(r + 1)]
    s = f[r] * t + f32(0)
    for k in range(1, r + 1):
        s = s + f[r + k] * (t[rows_up[k]] + t[rows_dn[k]])
    return s


def test_gauss_kernel(orc):
    for sigma in (0.7, 1.2489996, 1.2262735, 1.5450077, 1.9465878, 2.4525337, 3.0900299, 4.3):
        assert np.array_equal(orc.sift_gauss_kernel(sigma), _np_kernel(sigma)), sigma


@pytest.mark.parametrize("shape,sigma", [((37, 53), 1.6), ((96, 128), 3.09), ((5, 3), 2.45), ((3, 7), 1.22),
                                         ((1, 9), 1.5), ((8, 1), 1.9), ((64, 64), 1.2489996)])
def test_blur_bitwise(orc, shape, sigma):
    rng = np.random.default_rng(shape[0] * 7 + shape[1])
    img = (rng.random(shape) * 255).astype(f32)
    assert np.array_equal(orc.sift_blur(img, sigma), _np_blur(img, sigma))


def _np_resize_linear(src, dw, dh):
    sh, sw = src.shape
    sx_ = (1.0 / (dw / sw))
    sy_ = (1.0 / (dh / sh))
    xofs, a0, a1, xmax = [], [], [], dw
    for dx in range(dw):
        fx = f32((dx + 0.5) * sx_ - 0.5)
        sx = int(math.floor(fx))
        fx = f32(fx - f32(sx))
        if sx < 0:
            fx, sx = f32(0), 0
        if sx + 1 >= sw:
            xmax = min(xmax, dx)
            if sx >= sw - 1:
                fx, sx = f32(0), sw - 1
        xofs.append(sx)
        a0.append(f32(1) - fx)
        a1.append(fx)
    xofs, a0, a1 = np.array(xofs), np.array(a0, f32), np.array(a1, f32)
    x1 = np.minimum(xofs + 1, sw - 1)
    out = np.zeros((dh, dw), f32)
    for dy in range(dh):
        fy = f32((dy + 0.5) * sy_ - 0.5)
        sy = int(math.floor(fy))
        fy = f32(fy - f32(sy))
        S0 = src[min(max(sy, 0), sh - 1)]
        S1 = src[min(max(sy + 1, 0), sh - 1)]
        R0 = np.where(np.arange(dw) < xmax, S0[xofs] * a0 + S0[x1] * a1, S0[xofs])
        R1 = np.where(np.arange(dw) < xmax, S1[xofs] * a0 + S1[x1] * a1, S1[xofs])
        out[dy] = R0 * (f32(1) - fy) + R1 * fy
    return out


@pytest.mark.parametrize("shape,dshape", [((48, 64), (96, 128)), ((7, 5), (14, 10)), ((30, 41), (17, 23)),
                                          ((1, 6), (2, 12))])
def test_resize_linear_bitwise(orc, shape, dshape):
    rng = np.random.default_rng(3)
    src = rng.integers(0, 256, shape).astype(f32)
    assert np.array_equal(orc.sift_resize_linear(src, dshape[1], dshape[0]), _np_resize_linear(src, dshape[1], dshape[0]))


@pytest.mark.parametrize("shape", [(960, 1280), (15, 10), (7, 5), (3, 11)])
def test_resize_nn_bitwise(orc, shape):
    rng = np.random.default_rng(4)
    src = rng.random(shape).astype(f32)
    h, w = shape
    dw, dh = w // 2, h // 2
    ys = np.minimum(np.floor(np.arange(dh) * (1.0 / (dh / h))).astype(int), h - 1)
    xs = np.minimum(np.floor(np.arange(dw) * (1.0 / (dw / w))).astype(int), w - 1)
    assert np.array_equal(orc.sift_resize_nn(src, dw, dh), src[np.ix_(ys, xs)])


def test_sigmas_and_octaves(orc):
    k = 2.0 ** (1.0 / 3)
    want = [1.6] + [math.sqrt((k ** (i - 1) * 1.6 * k) ** 2 - (k ** (i - 1) * 1.6) ** 2) for i in range(1, 6)]
    assert np.array_equal(orc.sift_sigmas(3, 1.6), np.array(want))
    assert orc.sift_num_octaves(640, 480) == 9  # cvRound(log2(960) - 2) + 1
    assert orc.sift_num_octaves(640, 480, 0) == 7


# ---------------------------------------------------------------- cv::exp
TAB = np.array([float.fromhex(v) for v in """
0x1.3ce0f3e46f431p-7 0x1.40544d4d75547p-7 0x1.43d1453011896p-7 0x1.4757f65ccd1f0p-7 0x1.4ae87beef14bap-7
0x1.4e82f14d579f8p-7 0x1.5227722b3ca9dp-7 0x1.55d61a8914e9dp-7 0x1.598f06b56410cp-7 0x1.5d52534d969c3p-7
0x1.61201d3eddcf1p-7 0x1.64f881c70e0fbp-7 0x1.68db9e757fb1ap-7 0x1.6cc9912bf2329p-7 0x1.70c2781f71f03p-7
0x1.74c671d9405eep-7 0x1.78d59d37bec71p-7 0x1.7cf0196f5b91cp-7 0x1.8116060b822a4p-7 0x1.854782ef8d7c0p-7
0x1.8984b057bd157p-7 0x1.8dcdaeda2cf5ap-7 0x1.92229f67d00c5p-7 0x1.9683a34d6d757p-7 0x1.9af0dc34a0755p-7
0x1.9f6a6c24db3f1p-7 0x1.a3f075846c8c7p-7 0x1.a8831b19880ecp-7 0x1.ad22800b51c0fp-7 0x1.b1cec7e2ec22bp-7
0x1.b688168c89657p-7 0x1.bb4e90587f922p-7 0x1.c02259fc5fb16p-7 0x1.c50398940ffd7p-7 0x1.c9f271a2e9275p-7
0x1.ceef0b14d6b67p-7 0x1.d3f98b3f7a8ccp-7 0x1.d91218e353972p-7 0x1.de38db2ce7b3ep-7 0x1.e36df9b5f0d69p-7
0x1.e8b19c868d747p-7 0x1.ee03ec1674412p-7 0x1.f365114e2b44dp-7 0x1.f8d535884255fp-7 0x1.fe54829290ff9p-7
0x1.01f19157bbef2p-6 0x1.04c0a04b92bdfp-6 0x1.079783bc6f5adp-6 0x1.0a76517e255b1p-6 0x1.0d5d1fa16145cp-6
0x1.104c047452330p-6 0x1.1343168355441p-6 0x1.16426c99a2f97p-6 0x1.194a1dc1fe6bep-6 0x1.1c5a4147666e5p-6
0x1.1f72eeb5c89d0p-6 0x1.22943ddab6608p-6 0x1.25be46c61be8ep-6 0x1.28f121caf926dp-6 0x1.2c2ce7801cc88p-6
0x1.2f71b0c0e1405p-6 0x1.32bf96adebd97p-6 0x1.3616b2adede21p-6 0x1.39771e6e67ef9p-6""".split()])
A0 = float(".9670371139572337719125840413672004409288e-2")
A = [f32(float(v) / A0) for v in ("1.000000000000002438532970795181890933776", ".6931471805521448196800669615864773144641",
                                  ".2402265109513301490103372422686535526573",
                                  ".5550339366753125211915322047004666939128e-1")]  # A4, A3, A2, A1
PRE = 1.4426950408889634073599246810019 * 64


def _np_exp_sse(x):
    x = np.clip(np.asarray(x, f32), f32(-192000 / PRE), f32(192000 / PRE))
    xd = x.astype(np.float64) * PRE
    xi = np.rint(xd).astype(np.int64)
    xf = (xd - xi).astype(f32) * f32(1 / 64)
    xi = np.clip(xi, -32768, 32767)
    e = np.clip((xi >> 6) + 127, 0, 255).astype(np.uint32)
    yf = TAB[xi & 63].astype(f32) * (e << 23).view(f32)
    z = xf + A[3]
    z = z * xf + A[2]
    z = z * xf + A[1]
    z = z * xf + A[0]
    return z * yf


def _np_exp_scalar(x):
    x = np.asarray(x, f32)
    x0 = x.astype(np.float64) * PRE
    big = ((x.view(np.uint32) >> 23) & 255) > 137
    x0 = np.where(big, np.where(x < 0, -192000.0, 192000.0), x0)
    v = np.rint(x0).astype(np.int64)
    t = (v >> 6) + 127
    t = np.where((t & ~255) == 0, t, np.where(t < 0, 0, 255)).astype(np.uint32)
    x0 = (x0 - v) * (1 / 64)
    poly = (((x0 + float(A[3])) * x0 + float(A[2])) * x0 + float(A[1])) * x0 + float(A[0])
    return ((t << 23).view(f32).astype(np.float64) * TAB[v & 63] * poly).astype(f32)


def test_cv_exp_paths(orc):
    rng = np.random.default_rng(9)
    xs = np.concatenate([-rng.random(3000) * 40, rng.normal(0, 3, 2000), [0, -0.0, 1e-8, -1e-30, 20, -87, -100, -300]])
    xs = xs.astype(f32)
    sse = np.array([orc.cv_exp_at(float(x), 0, 8) for x in xs], f32)
    sca = np.array([orc.cv_exp_at(float(x), 7, 7) for x in xs], f32)
    assert np.array_equal(sse, _np_exp_sse(xs))
    assert np.array_equal(sca, _np_exp_scalar(xs))
    ref = np.exp(xs.astype(np.float64))
    ok = ref > 1e-30
    for got in (sse, sca):
        ulp = np.spacing(ref[ok].astype(f32)).astype(np.float64)
        assert np.max(np.abs(got[ok] - ref[ok]) / ulp) <= 2.0
    assert np.any(sse != sca)  # the two loops really differ: the array position matters
    # position rule: SSE2 lanes for k < 8 * floor(n / 8) when n >= 8
    x = f32(-3.3)
    assert orc.cv_exp_at(x, 15, 17) == _np_exp_sse(x) and orc.cv_exp_at(x, 16, 17) == _np_exp_scalar(x)
    assert orc.cv_exp_at(x, 3, 7) == _np_exp_scalar(x)


def test_deterministic_libm_floats_correctly_rounded(orc):
    """cosf / sinf of every float angle the descriptor sees on a 0.01-degree grid and a random
    sample, and powf(2, y) of the size exponents: the correctly rounded float (Python's double
    functions rounded to float).  This image's glibc float functions are not correctly rounded
    everywhere (cosf / sinf differ on ~1.3 % of these angles): the reference's glibc is not
    recorded, so the restatement takes the correctly rounded value."""
    import ctypes
    libm = ctypes.CDLL("libm.so.6")
    libm.cosf.restype = ctypes.c_float
    libm.cosf.argtypes = [ctypes.c_float]
    rng = np.random.default_rng(1)
    deg = np.concatenate([np.arange(0, 360, 0.01), rng.random(20000) * 360]).astype(f32)
    rad = (deg * f32(math.pi / 180)).astype(f32)
    c = np.array([orc.cv_cosf(float(v)) for v in rad], f32)
    s = np.array([orc.cv_sinf(float(v)) for v in rad], f32)
    assert np.array_equal(c, np.array([math.cos(float(v)) for v in rad]).astype(f32))
    assert np.array_equal(s, np.array([math.sin(float(v)) for v in rad]).astype(f32))
    glibc = np.array([libm.cosf(float(v)) for v in rad[:5000]], f32)
    assert np.mean(glibc != c[:5000]) < 0.03
    ys = ((np.arange(1, 4)[:, None] + (rng.random((3, 4000)) - 0.5)) / f32(3)).astype(f32).ravel()
    p = np.array([orc.cv_exp2f(float(v)) for v in ys], f32)
    assert np.array_equal(p, np.array([2.0 ** float(v) for v in ys]).astype(f32))


def test_atan2_polynomial(orc):
    for y, x in [(1, 1), (-1, 1), (1, -1), (-1, -1), (0, 1), (0, -1), (3, 0.5), (-0.2, -7), (0, 0)]:
        a = orc.cv_atan2_deg(y, x)
        assert 0 <= a < 360.0001
        if (x, y) != (0, 0):
            assert abs((a - math.degrees(math.atan2(y, x))) % 360 - 0) < 0.02 or \
                abs((a - math.degrees(math.atan2(y, x))) % 360 - 360) < 0.02


def test_solve3(orc):
    rng = np.random.default_rng(2)
    for _ in range(200):
        H = rng.normal(size=(3, 3)).astype(f32)
        H = (H + H.T) * f32(0.5) + np.eye(3, dtype=f32) * f32(6)
        b = rng.normal(size=3).astype(f32)
        x = orc.sift_solve3(H, b)
        assert np.allclose(x, np.linalg.solve(H.astype(np.float64), b.astype(np.float64)), rtol=1e-4, atol=1e-5)
    assert np.array_equal(orc.sift_solve3(np.ones((3, 3)), [1, 2, 3]), np.zeros(3, f32))


def _np_remove_duplicated(k):
    n = len(k)
    order = sorted(range(n), key=lambda i: (k["x"][i], k["y"][i], -k["size"][i], k["angle"][i], -k["response"][i],
                                            -k["octave"][i], -k["class_id"][i], i))
    mask = np.ones(n, bool)
    j = 0
    for i in range(1, n):
        a, b = k[order[i]], k[order[j]]
        if a["x"] != b["x"] or a["y"] != b["y"] or a["size"] != b["size"] or a["angle"] != b["angle"]:
            j = i
        else:
            mask[order[i]] = False
    return k[mask]


def test_remove_duplicated(orc):
    rng = np.random.default_rng(6)
    k = np.zeros(600, dtype=orc.KEYPOINT)
    k["x"] = rng.integers(0, 4, 600)
    k["y"] = rng.integers(0, 3, 600)
    k["size"] = rng.integers(1, 3, 600)
    k["angle"] = rng.integers(0, 2, 600) * 90
    k["response"] = rng.random(600)
    k["octave"] = rng.integers(0, 3, 600)
    out = orc.remove_duplicated(k)
    assert out.tobytes() == _np_remove_duplicated(k).tobytes()
    assert len(out) == len(np.unique(k[["x", "y", "size", "angle"]]))


# ---------------------------------------------------------------- whole detector
def test_pyramid_structure(orc):
    rng = np.random.default_rng(8)
    img = rng.integers(0, 256, (60, 80)).astype(np.uint8)
    g = orc.sift_pyramid(img)
    d = orc.sift_pyramid(img, dog=True)
    n = orc.sift_num_octaves(80, 60)
    assert len(g) == n * 6 and len(d) == n * 5
    base = _np_blur(_np_resize_linear(img.astype(f32), 160, 120), float(np.sqrt(max(f32(1.6) * f32(1.6) - f32(1), f32(0.01)))))
    assert np.array_equal(g[0], base.astype(f32))
    sig = orc.sift_sigmas()
    for o in range(n):
        for i in range(1, 6):
            assert np.array_equal(g[o * 6 + i], _np_blur(g[o * 6 + i - 1], sig[i]))
        for i in range(5):
            assert np.array_equal(d[o * 5 + i], g[o * 6 + i + 1] - g[o * 6 + i])
        if o:
            assert np.array_equal(g[o * 6], g[(o - 1) * 6 + 3][0:2 * (g[o * 6].shape[0]):2, 0:2 * g[o * 6].shape[1]:2])


def test_blob_centre(orc):
    """a Gaussian blob: one location, at the centre + 0.25 px (INTER_LINEAR doubling maps doubled pixel
    X to X/2 - 0.25, and the keypoint is reported at X/2)"""
    yy, xx = np.mgrid[0:240, 0:320]
    for cx, cy, s in [(160.3, 120.6, 6.0), (100.0, 80.5, 4.0), (200.7, 150.2, 9.0)]:
        b = np.rint(60 + 150 * np.exp(-((xx - cx) ** 2 + (yy - cy) ** 2) / (2 * s * s))).astype(np.uint8)
        k = orc.sift_detect(b)
        assert len(np.unique(k[["x", "y"]])) == 1, k
        assert abs(k["x"][0] - (cx + 0.25)) < 0.06 and abs(k["y"][0] - (cy + 0.25)) < 0.06
        assert 1.4 * s < k["size"][0] < 2.2 * s


def test_translation_covariance(orc, synth):
    """content shifted by 32 px: interior keypoints of octaves -1..4 move by 32 px (to float
    rounding), sizes, angles and responses identical, descriptors identical"""
    big = synth.make_frame_pair(3000, width=704, height=480, seed=11).img1
    a = np.ascontiguousarray(big[:, 0:640])
    b = np.ascontiguousarray(big[:, 32:672])
    ka, kb = orc.sift_detect(a), orc.sift_detect(b)

    def sel(k, x0):
        o = (k["octave"] & 255).astype(np.int8)
        m = (o <= 4) & (k["x"] > x0 + 140) & (k["x"] < x0 + 500) & (k["y"] > 140) & (k["y"] < 340)
        return k[m]

    sa, sb = sel(ka, 0), sel(kb, -32)
    assert len(sa) > 300 and len(sa) == len(sb)
    ia = np.lexsort((sa["angle"], sa["size"], sa["y"], np.round(sa["x"], 2)))
    ib = np.lexsort((sb["angle"], sb["size"], sb["y"], np.round(sb["x"] + 32, 2)))
    sa, sb = sa[ia], sb[ib]
    assert np.max(np.abs(sa["x"] - (sb["x"] + 32))) < 1e-3 and np.array_equal(sa["y"], sb["y"])
    for f in ("size", "angle", "response", "octave"):
        assert np.array_equal(sa[f], sb[f]), f
    _, _, da = orc.sift_compute(a, sa)
    _, _, db = orc.sift_compute(b, sb)
    assert np.mean(np.all(da == db, axis=1)) > 0.99


def test_compute_properties(orc, synth):
    img = synth.make_frame_pair(2000, seed=5).img1
    k = orc.sift_detect(img, nfeatures=800)
    assert 800 <= len(k) <= 830  # retainBest keeps ties at the boundary response
    ko, kept, d = orc.sift_compute(img, k)
    assert len(ko) == len(k) and np.array_equal(kept, np.arange(len(k)))
    assert d.dtype == f32 and np.all(d == np.rint(d)) and d.min() >= 0 and d.max() <= 255
    n = np.linalg.norm(d, axis=1)
    assert np.all((n > 400) & (n < 560))  # 512 / |clamped| scaling, then rounding
    # size-0 keypoints are removed; octave >= 0 only: the undoubled pyramid (firstOctave 0)
    k2 = k[:50].copy()
    k2["size"][::7] = 0
    ko2, kept2, _ = orc.sift_compute(img, k2)
    assert len(ko2) == 50 - len(range(0, 50, 7)) and 0 not in kept2
    k3 = k[(k["octave"] & 255) < 128][:40]
    _, _, d3 = orc.sift_compute(img, k3)
    assert len(d3) == len(k3) and np.all(np.linalg.norm(d3, axis=1) > 400)
    bad = k[:2].copy()
    bad["octave"] = 0xFE  # octave -2
    with pytest.raises(ValueError):
        orc.sift_compute(img, bad)
