"""The SURF oracle (oracle/orc_surf.c): feature detection + description of the reference's
default detector / extractor (descriptorsmatcher.cpp:110-115, 176-359; build/settings.yml:37-49).

OpenCV (nonfree) is not in this image, so the restatement is pinned by independent numpy
restatements of its pieces (integral image, INTER_AREA resize, the Gaussian weights) and by exact
properties of the algorithm (blob centres and scales, Laplacian sign, translation covariance, unit
descriptors).  Parity vs OpenCV itself is unpinned."""
import math

import numpy as np
import pytest


def _blobs(h=240, w=320, spec=((80, 60, 4.0, 1), (200, 150, 7.0, -1), (260, 60, 3.0, 1), (120, 180, 10.0, 1))):
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    img = np.full((h, w), 128.0)
    for cx, cy, sg, sign in spec:
        img += sign * 110.0 * np.exp(-((xx - cx) ** 2 + (yy - cy) ** 2) / (2 * sg * sg))
    return np.clip(np.rint(img), 0, 255).astype(np.uint8), spec


def test_integral_vs_numpy(orc):
    rng = np.random.default_rng(40)
    img = rng.integers(0, 256, (37, 53), dtype=np.uint8)
    ref = np.zeros((38, 54), dtype=np.int64)
    ref[1:, 1:] = img.astype(np.int64).cumsum(0).cumsum(1)
    assert np.array_equal(orc.integral(img), ref)


def _area_tab(ssize, dsize, scale):
    """computeResizeAreaTab (OpenCV 2.4 imgproc/resize.cpp)."""
    tab = []
    for dx in range(dsize):
        fsx1 = dx * scale
        fsx2 = fsx1 + scale
        cell = min(scale, ssize - fsx1)
        sx1, sx2 = math.ceil(fsx1), math.floor(fsx2)
        sx2 = min(sx2, ssize - 1)
        sx1 = min(sx1, sx2)
        if sx1 - fsx1 > 1e-3:
            tab.append((dx, sx1 - 1, np.float32((sx1 - fsx1) / cell)))
        for sx in range(sx1, sx2):
            tab.append((dx, sx, np.float32(1.0 / cell)))
        if fsx2 - sx2 > 1e-3:
            tab.append((dx, sx2, np.float32(min(min(fsx2 - sx2, 1.0), cell) / cell)))
    return tab


def _resize_area21_numpy(win):
    W = win.shape[0]
    scale = 1.0 / (21.0 / W)
    iscale = int(np.rint(scale))
    out = np.zeros((21, 21), dtype=np.uint8)
    if abs(scale - iscale) < np.finfo(np.float64).eps:
        for dy in range(21):
            for dx in range(21):
                blk = win[dy * iscale:(dy + 1) * iscale, dx * iscale:(dx + 1) * iscale].astype(np.int64)
                if iscale == 2 and dx < 16:
                    out[dy, dx] = (blk.sum() + 2) >> 2
                else:
                    out[dy, dx] = np.clip(np.rint(np.float32(blk.sum()) * np.float32(1.0 / (iscale * iscale))), 0, 255)
        return out
    xt, yt = _area_tab(W, 21, scale), _area_tab(W, 21, scale)
    acc = {}
    for dy, sy, beta in yt:
        buf = np.zeros(21, dtype=np.float32)
        for dx, sx, alpha in xt:
            buf[dx] = np.float32(buf[dx] + np.float32(np.float32(win[sy, sx]) * alpha))
        if dy not in acc:
            acc[dy] = np.float32(beta) * buf
        else:
            acc[dy] = np.float32(acc[dy] + np.float32(beta) * buf)
    for dy in range(21):
        out[dy] = np.clip(np.rint(acc[dy]), 0, 255)
    return out


@pytest.mark.parametrize("W", [25, 30, 42, 44, 63, 84, 101, 250])
def test_resize_area_vs_numpy(orc, W):
    """resize(win, 21x21, INTER_AREA): the general area tables and the integer-scale fast path
    (W = 42: 2x2 blocks, SSE2 rounding on the first 16 columns; W = 63 / 84: scalar)."""
    rng = np.random.default_rng(W)
    win = rng.integers(0, 256, (W, W), dtype=np.uint8)
    assert np.array_equal(orc.resize_area21(win), _resize_area21_numpy(win))


def _resize_area_up_numpy(win, D=21):
    """INTER_AREA enlarging as OpenCV 2.4.9 emulates it: bilinear with area-mode coefficients in
    11-bit fixed point, restated independently (per output pixel, numpy scalars)"""
    W = win.shape[0]
    inv = D / W
    scale = 1.0 / inv

    def coef(d):
        s = int(np.floor(d * scale))
        f = np.float32((d + 1) - (s + 1) * inv)
        f = np.float32(0) if f <= 0 else np.float32(f - np.floor(f))
        return s, f

    def q(v):  # saturate_cast<short>(float * 2048)
        return int(np.rint(np.float32(v) * np.float32(2048)))

    out = np.zeros((D, D), np.uint8)
    for dy in range(D):
        sy, fy = coef(dy)
        b0, b1 = q(np.float32(1) - fy), q(fy)
        rows = [win[min(max(sy, 0), W - 1)], win[min(max(sy + 1, 0), W - 1)]]
        for dx in range(D):
            sx, fx = coef(dx)
            interp = sx + 1 < W
            if sx >= W - 1:
                sx, fx = W - 1, np.float32(0)
            a0, a1 = q(np.float32(1) - fx), q(fx)
            h = [int(r[sx]) * a0 + int(r[sx + 1]) * a1 if interp else int(r[sx]) * 2048 for r in rows]
            if dx < 20:  # VResizeLinearVec_32s8u's columns (16 + 4 of 21)
                v = ((((h[0] >> 4) * b0) >> 16) + (((h[1] >> 4) * b1) >> 16) + 2) >> 2
            else:
                v = (b0 * h[0] + b1 * h[1] + (1 << 21)) >> 22
            out[dy, dx] = min(max(v, 0), 255)
    return out


@pytest.mark.parametrize("W", [1, 2, 3, 7, 10, 11, 14, 19, 20])
def test_resize_area_up_vs_numpy(orc, W):
    """windows narrower than the 21 x 21 patch (keypoints of size < 7.5) are enlarged"""
    rng = np.random.default_rng(100 + W)
    win = rng.integers(0, 256, (W, W), dtype=np.uint8)
    out = orc.resize_area_up(win)
    assert np.array_equal(out, _resize_area_up_numpy(win))
    flat = np.full((W, W), 173, np.uint8)
    assert (orc.resize_area_up(flat) == 173).all()
    # each output pixel lies between its two source rows' and columns' extremes
    assert out.min() >= win.min() and out.max() <= win.max()


def test_descriptor_weights_vs_numpy(orc):
    """getGaussianKernel(20, 3.3, CV_32F) outer product (SURFInvoker ctor)."""
    x = np.arange(20) - 9.5
    g = np.exp(-0.5 / (3.3 * 3.3) * x * x).astype(np.float32)
    s = 1.0 / g.astype(np.float64).sum()
    g = (g.astype(np.float64) * s).astype(np.float32)
    assert np.array_equal(orc.surf_dw(), np.outer(g, g).astype(np.float32))


def test_blob_keypoints(orc):
    """Gaussian blobs: one keypoint per blob near its centre, bright blobs Laplacian sign -1 (trace
    of the Hessian < 0 at a maximum), dark +1, and the scale grows with the blob sigma."""
    img, spec = _blobs()
    k = orc.surf_detect(img)
    assert (k["angle"] == 270).all() and np.all(np.diff(k["response"]) <= 0)
    sizes = []
    for cx, cy, sg, sign in spec:
        d = np.hypot(k["x"] - cx, k["y"] - cy)
        j = int(np.argmin(d))
        assert d[j] < 1.5, (cx, cy, d[j])
        assert k["class_id"][j] == -sign
        sizes.append(k["size"][j])
    order = np.argsort([s[2] for s in spec])
    assert np.all(np.diff(np.array(sizes)[order]) > 0), sizes


def test_translation_covariance(orc, synth):
    """Shifting the image by 16 pixels (a multiple of every octave's sample step) shifts every
    keypoint away from the borders by exactly 16 and leaves its descriptor bit-identical."""
    img = synth.make_frame_pair(300, seed=5).img1[:240, :320]
    big = np.zeros((240 + 16, 320 + 16), dtype=np.uint8)
    big[16:, 16:] = img
    big[:16, 16:] = img[:1, :]
    big[16:, :16] = img[:, :1]
    big[:16, :16] = img[0, 0]
    k0 = orc.surf_detect(img)
    k1 = orc.surf_detect(big)
    kd0, _, d0 = orc.surf_describe(img, k0)
    kd1, _, d1 = orc.surf_describe(big, k1)
    inner = lambda k: (k["x"] > 120) & (k["x"] < 200) & (k["y"] > 100) & (k["y"] < 140) & (k["size"] < 30)
    a = {(round(float(x), 3), round(float(y), 3), float(s)): i for i, (x, y, s) in
         enumerate(zip(kd0["x"], kd0["y"], kd0["size"])) if inner(kd0[i])}
    hits = 0
    for i, (x, y, s) in enumerate(zip(kd1["x"] - 16, kd1["y"] - 16, kd1["size"])):
        key = (round(float(x), 3), round(float(y), 3), float(s))
        if key in a:
            hits += 1
            assert np.array_equal(d0[a[key]], d1[i])
    assert hits >= 0.9 * len(a) and hits > 5, (hits, len(a))


def test_descriptors_unit_and_short(orc, synth):
    img = synth.make_frame_pair(300, seed=6).img1
    k = orc.surf_detect(img)[:300]
    kk, kept, d = orc.surf_describe(img, k)
    assert d.shape == (len(kk), 128) and np.array_equal(kept, np.arange(len(kk)))
    assert np.abs(np.linalg.norm(d.astype(np.float64), axis=1) - 1).max() < 1e-5
    _, _, d64 = orc.surf_describe(img, k, extended=False)
    assert d64.shape == (len(kk), 64)
    assert np.abs(np.linalg.norm(d64.astype(np.float64), axis=1) - 1).max() < 1e-5
    # extended splits each sum of dx / |dx| by the sign of dy: the pairs add back to the short sums
    # (before normalisation, so compare directions)
    big = d.reshape(-1, 16, 8).astype(np.float64)
    short = d64.reshape(-1, 16, 4).astype(np.float64)
    sx = big[:, :, 0] + big[:, :, 2]
    cos = (sx * short[:, :, 0]).sum(1) / (np.linalg.norm(sx, axis=1) * np.linalg.norm(short[:, :, 0], axis=1))
    assert (cos > 0.999).all()


# ---------------------------------------------------------------- Upright 0 (orientation)
def _fast_atan2_numpy(y, x):
    """cv::fastAtan2 of OpenCV 2.4.9+ in float32 operations (core/mathfuncs.cpp)"""
    f = np.float32
    k = f(180 / math.pi)
    p1, p3, p5, p7 = f(0.9997878412794807) * k, f(-0.3258083974640975) * k, f(0.1555786518463281) * k, \
        f(-0.04432655554792128) * k
    y, x = f(y), f(x)
    ax, ay = abs(x), abs(y)
    eps = f(np.finfo(np.float64).eps)
    if ax >= ay:
        c = ay / (ax + eps)
        c2 = c * c
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c
    else:
        c = ax / (ay + eps)
        c2 = c * c
        a = f(90) - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c
    if x < 0:
        a = f(180) - a
    if y < 0:
        a = f(360) - a
    return a


def test_fast_atan2_vs_numpy(orc):
    """the polynomial fastAtan2 (phase(..., true) and fastAtan2 of SURFInvoker): equal to a float32
    numpy restatement, within 0.01 degree of atan2, in [0, 360)"""
    rng = np.random.default_rng(11)
    vals = list(rng.normal(0, 100, (400, 2))) + [(0, 0), (0, 1), (1, 0), (-1, 0), (0, -1), (-0.0, 5), (3, 3), (-3, 3)]
    for y, x in vals:
        got = orc.fast_atan2(float(np.float32(y)), float(np.float32(x)))
        want = float(_fast_atan2_numpy(y, x))
        assert got == want, (y, x, got, want)
        assert 0 <= got < 360
        if (x, y) != (0, 0):
            exact = math.degrees(math.atan2(float(np.float32(y)), float(np.float32(x)))) % 360
            assert min(abs(got - exact), 360 - abs(got - exact)) < 0.01


def test_orientation_samples_vs_numpy(orc):
    """SURFInvoker's orientation disc: 113 samples of radius 6, x outer / y inner, Gaussian weights
    getGaussianKernel(13, 2.5, CV_32F) outer product"""
    apt, aptw = orc.surf_ori_samples()
    want = [(i, j) for i in range(-6, 7) for j in range(-6, 7) if i * i + j * j <= 36]
    assert len(apt) == 113 and [tuple(a) for a in apt] == want
    x = np.arange(13) - 6.0
    g = np.exp(-0.5 / (2.5 * 2.5) * x * x).astype(np.float32)
    g = (g.astype(np.float64) * (1.0 / g.astype(np.float64).sum())).astype(np.float32)
    assert np.array_equal(aptw, np.array([g[i + 6] * g[j + 6] for i, j in want], dtype=np.float32))


@pytest.mark.parametrize("deg", [0, 30, 100, 200, 315])
def test_orientation_of_a_ramp(orc, deg):
    """an intensity ramp rising along direction a (image axes, y down): the dx wavelet is +1 on the
    right, the dy wavelet +1 on the TOP half, so every sample is (X, Y) ~ (cos a, -sin a) and the
    dominant orientation fastAtan2(-sumY, sumX) is a; the descriptor is unit length"""
    h = w = 200
    a = math.radians(deg)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    img = np.clip(np.rint(128 + 0.5 * ((xx - 100) * math.cos(a) + (yy - 100) * math.sin(a))), 0, 255).astype(np.uint8)
    kin = np.zeros(3, dtype=orc.KEYPOINT)
    kin["x"], kin["y"], kin["size"], kin["angle"] = [100, 90.5, 110.2], [100, 105, 95.7], [20, 15, 31], -1
    k, kept, d = orc.surf_describe(img, kin, upright=False)
    assert list(kept) == [0, 1, 2]
    for ang in k["angle"]:
        diff = abs(float(ang) - deg)
        assert min(diff, 360 - diff) < 2.0, (deg, float(ang))
    assert np.abs(np.linalg.norm(d.astype(np.float64), axis=1) - 1).max() < 1e-5


def test_orientation_rotation_covariance(orc, synth):
    """rotating the image by 90 degrees (np.rot90: exact) moves keypoint (x, y) to (y, W-1-x) and a
    direction (c, s) to (s, -c): the orientation loses 90 degrees, up to the sampling grid's
    rounding; the rotation-invariant descriptors stay close"""
    img = synth.make_frame_pair(300, seed=5).img1[100:356, 100:356]
    k0 = orc.surf_detect(img, upright=False)
    r = np.ascontiguousarray(np.rot90(img))  # r[y, x] = img[x, W-1-y]
    k1 = orc.surf_detect(r, upright=False)
    _, _, d0 = orc.surf_describe(img, k0, upright=False)
    _, _, d1 = orc.surf_describe(r, k1, upright=False)
    W = img.shape[1]
    # keypoint (x, y) of img -> (y, W-1-x) in r
    pos1 = {(round(float(x), 2), round(float(y), 2), float(s)): i for i, (x, y, s) in
            enumerate(zip(k1["x"], k1["y"], k1["size"]))}
    hits, close, good = 0, 0, 0
    for i in range(len(k0)):
        key = (round(float(k0["y"][i]), 2), round(float(W - 1 - k0["x"][i]), 2), float(k0["size"][i]))
        j = pos1.get(key)
        if j is None:
            continue
        hits += 1
        diff = abs((float(k0["angle"][i]) - 90) % 360 - float(k1["angle"][j]))
        close += min(diff, 360 - diff) < 5.0
        good += float(np.dot(d0[i].astype(np.float64), d1[j].astype(np.float64))) > 0.9
    assert hits > 20 and close >= 0.9 * hits and good >= 0.8 * hits, (hits, close, good, len(k0))
