"""The ORB oracle (oracle/orc_orb.c): OpenCV 2.4.9's ORB, the detector / extractor of FeatureOptions
DetectorType / ExtractorType ORB (descriptorsmatcher.cpp:273-279, 336-341).

OpenCV is not in this image, so the restatement is pinned piece by piece:
  * std::nth_element / std::partition / std::__heap_select (KeyPointsFilter::retainBest) against
    the REAL libstdc++ of this image (tests/native/stl_select.cpp compiled here), on keypoint arrays
    full of ties -- the kept set and its order depend on exactly these algorithms;
  * resize(INTER_LINEAR) fixed point with the SSE2 vertical pass, FAST-9 + cornerScore + non-max,
    HarrisResponses, IC_Angle (umax), GaussianBlur 7x7 fixed point / SSE2 float columns, the
    makeRandomPattern cv::RNG sequence and computeOrbDescriptor: independent numpy restatements;
  * properties of the whole detector: compute() on detect()'s keypoints reproduces its descriptors,
    keypoints inside the edge border, sizes 31 * scale, per-level counts.
Parity with OpenCV's own build stays unpinned where no fixture exists; the 512-point
bit_pattern_31_ table is not in this image, so descriptors use makeRandomPattern unless a pattern is
passed."""
import ctypes
import math
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3), (-2, -2), (-3, -1),
          (-3, 0), (-3, 1), (-2, 2), (-1, 3)]
f32 = np.float32


@pytest.fixture(scope="module")
def stl(tmp_path_factory):
    so = tmp_path_factory.mktemp("stl") / "stl_select.so"
    subprocess.run(["g++", "-O2", "-shared", "-fPIC", "-o", str(so), os.path.join(ROOT, "tests", "native", "stl_select.cpp")],
                   check=True)
    return ctypes.CDLL(str(so))


def _kps(resp, seed=0):
    rng = np.random.default_rng(seed)
    k = np.zeros(len(resp), dtype=[("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                                   ("octave", "<i4"), ("class_id", "<i4")])
    k["x"] = np.arange(len(resp))  # identity of each element
    k["y"] = rng.integers(0, 100, len(resp))
    k["response"] = resp
    return k


def _cases():
    rng = np.random.default_rng(5)
    for n in (0, 1, 2, 3, 4, 5, 7, 16, 17, 100, 257, 1000, 4096):
        for kind in ("ties", "float", "sorted", "reversed", "equal", "organ"):
            if kind == "ties":
                r = rng.integers(20, 30, n).astype(np.float32)
            elif kind == "float":
                r = rng.random(n).astype(np.float32)
            elif kind == "sorted":
                r = np.arange(n, dtype=np.float32)
            elif kind == "reversed":
                r = np.arange(n, dtype=np.float32)[::-1].copy()
            elif kind == "equal":
                r = np.full(n, 7, np.float32)
            else:
                r = np.concatenate([np.arange(n // 2), np.arange(n - n // 2)[::-1]]).astype(np.float32)
            yield n, kind, r


def test_nth_element_partition_vs_libstdcxx(orc, stl):
    """orc_nth_element / orc_partition_ge / orc_retain_best reorder exactly as libstdc++'s
    std::nth_element / std::partition (whole arrays compared, element identities included)"""
    checked = 0
    for n, kind, r in _cases():
        for nth in sorted({0, 1, n // 3, n // 2, n - 1, n} & set(range(0, n + 1))):
            a = _kps(r, n)
            b = a.copy()
            stl.cxx_nth_element(b.ctypes.data_as(ctypes.c_void_p), ctypes.c_long(nth), ctypes.c_long(n))
            assert np.array_equal(orc.nth_element(a, nth).view(np.uint8), b.view(np.uint8)), (n, kind, nth)
            for keep in (nth, n // 4):
                c = a.copy()
                m = stl.cxx_retain_best(c.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(n), ctypes.c_int(keep))
                assert np.array_equal(orc.retain_best(a, keep).view(np.uint8), c[:m].view(np.uint8)), (n, kind, keep)
            if n:
                thr = float(np.median(r))
                d = a.copy()
                stl.cxx_partition_ge.restype = ctypes.c_long
                m = stl.cxx_partition_ge(d.ctypes.data_as(ctypes.c_void_p), ctypes.c_long(nth // 2), ctypes.c_long(n),
                                         ctypes.c_float(thr))
                got, gm = orc.partition_ge(a, nth // 2, n, thr)
                assert gm == m and np.array_equal(got.view(np.uint8), d.view(np.uint8)), (n, kind, nth)
            checked += 1
    assert checked > 300


def test_heap_select_vs_libstdcxx(orc, stl):
    """the introselect's depth-limit fallback (std::__heap_select) on its own"""
    import oracle as o
    for seed, (n, mid) in enumerate([(5, 2), (64, 10), (100, 99), (1000, 333), (33, 1), (2, 1)]):
        r = np.random.default_rng(seed).integers(0, 12, n).astype(np.float32)
        a, b = _kps(r, seed), _kps(r, seed)
        o.lib().orc_heap_select(a.ctypes.data_as(ctypes.c_void_p), ctypes.c_long(mid), ctypes.c_long(n))
        stl.cxx_heap_select(b.ctypes.data_as(ctypes.c_void_p), ctypes.c_long(mid), ctypes.c_long(n))
        assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), (n, mid)


# ---------------------------------------------------------------- pixel pieces vs numpy
def _resize_np(src, dw, dh):
    sh, sw = src.shape
    S = src.astype(np.int64)
    sxs = 1.0 / (dw / sw)
    fx = ((np.arange(dw) + 0.5) * sxs - 0.5).astype(np.float32)
    sx = np.floor(fx).astype(np.int64)
    fx = (fx - sx.astype(np.float32)).astype(np.float32)
    fx[sx < 0], sx[sx < 0] = 0, 0
    hi = sx + 1 >= sw
    xmax = int(np.argmax(hi)) if hi.any() else dw
    top = sx >= sw - 1
    fx[top], sx[top] = 0, sw - 1
    a0 = np.rint((f32(1) - fx) * f32(2048)).astype(np.int64)
    a1 = np.rint(fx * f32(2048)).astype(np.int64)
    sys_ = 1.0 / (dh / sh)
    fy = ((np.arange(dh) + 0.5) * sys_ - 0.5).astype(np.float32)
    sy = np.floor(fy).astype(np.int64)
    fy = (fy - sy.astype(np.float32)).astype(np.float32)
    b0 = np.rint((f32(1) - fy) * f32(2048)).astype(np.int64)
    b1 = np.rint(fy * f32(2048)).astype(np.int64)

    def hres(row):
        d = row[sx] * 2048
        m = np.arange(dw) < xmax
        d[m] = row[sx[m]] * a0[m] + row[np.minimum(sx[m] + 1, sw - 1)] * a1[m]
        return d
    # the SSE2 columns: the 16-wide loop, then 4-wide while x < width - 4
    xs = (dw // 16) * 16
    while xs < dw - 4:
        xs += 4
    out = np.zeros((dh, dw), np.uint8)
    for y in range(dh):
        D0 = hres(S[min(max(sy[y], 0), sh - 1)])
        D1 = hres(S[min(max(sy[y] + 1, 0), sh - 1)])
        v = np.where(np.arange(dw) < xs,
                     ((((D0 >> 4) * b0[y]) >> 16) + (((D1 >> 4) * b1[y]) >> 16) + 2) >> 2,
                     (b0[y] * D0 + b1[y] * D1 + (1 << 21)) >> 22)
        out[y] = np.clip(v, 0, 255)
    return out


@pytest.mark.parametrize("sw,sh,dw,dh", [(640, 480, 533, 400), (533, 400, 444, 333), (100, 77, 83, 64), (37, 29, 31, 24),
                                         (21, 20, 17, 17)])
def test_resize_linear_vs_numpy(orc, sw, sh, dw, dh):
    img = np.random.default_rng(sw).integers(0, 256, (sh, sw), dtype=np.uint8)
    assert np.array_equal(orc.orb_resize(img, dw, dh), _resize_np(img, dw, dh))


def test_level_sizes(orc):
    """getScale = (float)pow(1.2, l); cvRound(640 * (1 / scale)) ..."""
    want = [(640, 480), (533, 400), (444, 333), (370, 278), (309, 231), (257, 193), (214, 161), (179, 134)]
    assert [orc.orb_level_size(640, 480, 1.2, l) for l in range(8)] == want


def _fast_np(img, thr):
    h, w = img.shape
    I = img.astype(np.int64)
    v = I[3:h - 3, 3:w - 3]
    d = np.stack([v - I[3 + dy:h - 3 + dy, 3 + dx:w - 3 + dx] for dx, dy in CIRCLE])  # (16, H, W)
    mins = np.stack([np.min(np.stack([d[(k + j) % 16] for j in range(9)]), 0) for k in range(16)])
    maxs = np.stack([np.max(np.stack([d[(k + j) % 16] for j in range(9)]), 0) for k in range(16)])
    M = np.maximum(mins.max(0), -maxs.min(0))
    corner = np.zeros((h, w), bool)
    S = np.zeros((h, w), np.int64)
    corner[3:h - 3, 3:w - 3] = M > thr
    S[3:h - 3, 3:w - 3] = np.where(M > thr, M - 1, 0)
    pts = []
    for y in range(3, h - 3):
        for x in range(3, w - 3):
            if corner[y, x]:
                s = S[y, x]
                nb = S[y - 1:y + 2, x - 1:x + 2].copy()
                nb[1, 1] = -1
                if (s > nb).all():
                    pts.append((x, y, s))
    return pts


@pytest.mark.parametrize("thr", [20, 5, 35])
def test_fast9_vs_numpy(orc, synth, thr):
    """FAST-9: corner iff 9 contiguous circle pixels all darker than v - thr or all brighter than
    v + thr; score = the largest threshold it stays a corner at (cornerScore<16>); 3x3 non-max"""
    img = synth.make_frame_pair(300, seed=8).img1[100:190, 200:330]
    got = orc.fast9(img, thr)
    want = _fast_np(img, thr)
    assert len(want) > 5
    assert [(int(k["x"]), int(k["y"]), int(k["response"])) for k in got] == want
    assert (got["size"] == 7).all() and (got["angle"] == -1).all() and (got["class_id"] == -1).all()


def test_harris_vs_numpy(orc, synth):
    img = synth.make_frame_pair(300, seed=8).img1
    k = orc.fast9(img, 20)
    k = k[(k["x"] >= 10) & (k["x"] < 630) & (k["y"] >= 10) & (k["y"] < 470)][:200]
    got = orc.harris(img, k)
    I = img.astype(np.int64)
    Ix = (I[1:-1, 2:] - I[1:-1, :-2]) * 2 + (I[:-2, 2:] - I[:-2, :-2]) + (I[2:, 2:] - I[2:, :-2])
    Iy = (I[2:, 1:-1] - I[:-2, 1:-1]) * 2 + (I[2:, :-2] - I[:-2, :-2]) + (I[2:, 2:] - I[:-2, 2:])
    scale = f32(1) / f32(7140)
    sq = scale * scale * scale * scale
    for kp, g in zip(k, got):
        x0, y0 = int(kp["x"]) - 3, int(kp["y"]) - 3
        bx = Ix[y0 - 1:y0 + 6, x0 - 1:x0 + 6]
        by = Iy[y0 - 1:y0 + 6, x0 - 1:x0 + 6]
        a, b, c = f32((bx * bx).sum()), f32((by * by).sum()), f32((bx * by).sum())
        want = (a * b - c * c - f32(0.04) * (a + b) * (a + b)) * sq
        assert g == want


def _umax_np(half):
    u = [0] * (half + 2)
    vmax = int(np.floor(f32(half) * np.sqrt(f32(2)) / f32(2) + f32(1)))
    vmin = int(np.ceil(f32(half) * np.sqrt(f32(2)) / f32(2)))
    for v in range(vmax + 1):
        u[v] = int(np.rint(math.sqrt(half * half - v * v)))
    v0 = 0
    for v in range(half, vmin - 1, -1):
        while u[v0] == u[v0 + 1]:
            v0 += 1
        u[v] = v0
        v0 += 1
    return u


def test_umax_and_ic_angle_vs_numpy(orc, synth):
    for half in (15, 7, 10, 16):
        assert list(orc.orb_umax(half)) == _umax_np(half)
    img = synth.make_frame_pair(300, seed=8).img1
    u = _umax_np(15)
    I = img.astype(np.int64)
    rng = np.random.default_rng(2)
    for _ in range(50):
        x, y = int(rng.integers(20, 620)), int(rng.integers(20, 460))
        m10 = sum(du * I[y, x + du] for du in range(-15, 16))
        m01 = 0
        for v in range(1, 16):
            vs = 0
            for du in range(-u[v], u[v] + 1):
                vp, vm = I[y + v, x + du], I[y - v, x + du]
                vs += vp - vm
                m10 += du * (vp + vm)
            m01 += v * vs
        assert orc.ic_angle(img, 15, x, y) == orc.fast_atan2(float(f32(m01)), float(f32(m10)))


def _blur_np(src, ik):
    h, w = src.shape
    idx = lambda p, n: np.where(p < 0, -p, np.where(p >= n, 2 * n - 2 - p, p))
    S = src.astype(np.int64)
    R = sum(ik[k] * S[:, idx(np.arange(w) + k - 3, w)] for k in range(7))
    fk = [f32(ik[3 + k] * (1.0 / 65536)) for k in range(4)]
    rows = lambda o: R[idx(np.arange(h) + o, h)]
    s = R.astype(np.float32) * fk[0] + f32(0)
    for k in range(1, 4):
        s = s + (rows(k) + rows(-k)).astype(np.float32) * fk[k]
    fl = np.rint(s).astype(np.int64)
    it = ik[3] * R + sum(ik[3 + k] * (rows(k) + rows(-k)) for k in range(1, 4))
    it = (it + (1 << 15)) >> 16
    out = np.where(np.arange(w)[None, :] < (w // 4) * 4, fl, it)
    return np.clip(out, 0, 255).astype(np.uint8)


@pytest.mark.parametrize("w,h", [(640, 480), (309, 231), (37, 29), (7, 9)])
def test_blur_vs_numpy(orc, w, h):
    """GaussianBlur(7x7, 2, 2, BORDER_REFLECT_101): the kernel x256 (cvRound), int rows, the SSE2
    float columns on the first floor(w/4)*4 columns, fixed point (+2^15) >> 16 on the rest"""
    x = np.arange(7) - 3.0
    g = np.exp(-0.5 / 4.0 * x * x).astype(np.float32)
    g = (g.astype(np.float64) * (1.0 / g.astype(np.float64).sum())).astype(np.float32)
    ik = np.rint(g * f32(256)).astype(np.int64)
    assert list(orc.orb_blur_kernel()) == list(ik)
    img = np.random.default_rng(w).integers(0, 256, (h, w), dtype=np.uint8)
    assert np.array_equal(orc.orb_blur(img), _blur_np(img, ik))


def test_random_pattern_is_cv_rng(orc):
    """makeRandomPattern: cv::RNG(0x34985739), uniform(-p/2, p/2 + 1) for x then y"""
    def pattern(p, n=512):
        state, a, b, out = 0x34985739, -(p // 2), p // 2 + 1, []
        for _ in range(2 * n):
            state = ((state & 0xFFFFFFFF) * 4164903690 + (state >> 32)) & 0xFFFFFFFFFFFFFFFF
            out.append((state & 0xFFFFFFFF) % (b - a) + a)
        return np.array(out).reshape(n, 2)
    for p in (31, 25, 48):
        got = orc.orb_random_pattern(p)
        assert np.array_equal(got, pattern(p)) and got.min() >= -(p // 2) and got.max() <= p // 2


def test_descriptor_vs_numpy(orc, synth):
    """computeOrbDescriptor (WTA_K 2) of the blurred level: bit j of byte i = I(rot(p[16i+2j])) <
    I(rot(p[16i+2j+1])), rotation by the keypoint angle in float, cvRound of the coordinates"""
    img = synth.make_frame_pair(2000, seed=3).img1
    k, d = orc.orb_detect(img, nfeatures=300, nlevels=1)
    blur = orc.orb_blur(img).astype(np.int64)
    pat = orc.orb_random_pattern(31)
    for kp, row in zip(k[:60], d[:60]):
        ang = f32(kp["angle"]) * f32(math.pi / 180.0)
        a, b = f32(math.cos(float(ang))), f32(math.sin(float(ang)))
        cx, cy = int(np.rint(kp["x"])), int(np.rint(kp["y"]))
        px = pat[:, 0].astype(np.float32)
        py = pat[:, 1].astype(np.float32)
        x = np.rint(px * a - py * b).astype(np.int64)
        y = np.rint(px * b + py * a).astype(np.int64)
        t = blur[cy + y, cx + x]
        bits = (t[0::2] < t[1::2]).reshape(32, 8)
        want = (bits * (1 << np.arange(8))).sum(1)
        assert np.array_equal(row, want.astype(np.uint8))


# ---------------------------------------------------------------- the detector as a whole
def test_orb_detect_properties(orc, synth):
    img = synth.make_frame_pair(2000, seed=3).img1
    k, d = orc.orb_detect(img, nfeatures=2000)
    assert 1900 <= len(k) <= 2100 and d.shape == (len(k), 32)
    assert (np.diff(k["octave"]) >= 0).all()  # level-major
    for l in range(8):
        kl = k[k["octave"] == l]
        sf = orc.orb_scale(1.2, l)
        lw, lh = orc.orb_level_size(640, 480, 1.2, l)
        assert (kl["size"] == np.float32(31 * np.float32(sf))).all()
        lx, ly = kl["x"] / np.float32(sf), kl["y"] / np.float32(sf)
        assert (np.rint(lx) >= 31).all() and (np.rint(lx) < lw - 31).all() and (np.rint(ly) >= 31).all()
        assert ((kl["angle"] >= 0) & (kl["angle"] < 360)).all()
    # compute() on detect()'s keypoints (ORB::compute path): the same descriptors; the positions
    # go through pt * (1 / scale) * scale in float, as OpenCV's do
    ko, kept, do = orc.orb_compute(img, k)
    assert np.array_equal(kept, np.arange(len(k))) and np.array_equal(do, d)
    for f in ("size", "angle", "response", "octave", "class_id"):
        assert np.array_equal(ko[f], k[f]), f
    sf = np.array([orc.orb_scale(1.2, l) for l in range(8)], np.float32)[k["octave"]]
    inv = (np.float32(1) / sf).astype(np.float32)
    for f in ("x", "y"):
        want = np.where(k["octave"] > 0, (k[f] * inv).astype(np.float32) * sf, k[f]).astype(np.float32)
        assert np.array_equal(ko[f], want), f
    assert (ko["x"] != k["x"]).sum() > 0  # the round trip does move some


def test_orb_compute_filters_and_grouping(orc, synth):
    """ORB::compute: size < FLT_EPSILON dropped, the edge border (on rounded coordinates) dropped,
    output grouped by octave in input order, a negative octave rejected"""
    img = synth.make_frame_pair(300, seed=8).img1
    kin = np.zeros(8, dtype=orc.KEYPOINT)
    kin["x"] = [100, 30.6, 300, 608.4, 200, 320, 150, 400]
    kin["y"] = [100, 200, 40, 300, 250, 240, 449.6, 300]
    kin["size"] = [31, 31, 0, 31, 37.2, 44.64, 31, 31]
    kin["octave"] = [0, 0, 0, 0, 1, 2, 0, 1]
    kin["angle"] = [10, 20, 30, 40, 50, 60, 70, 80]
    k, kept, d = orc.orb_compute(img, kin)
    # 30.6 rounds to 31 (kept), 608.4 -> 608 < 609 (kept), 449.6 -> 450 >= 449 (dropped)
    assert list(kept) == [0, 1, 3, 4, 7, 5]
    assert np.array_equal(k["angle"], kin["angle"][kept])
    bad = kin[[0]].copy()
    bad["octave"] = -1
    with pytest.raises(ValueError):
        orc.orb_compute(img, bad)
