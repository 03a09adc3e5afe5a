"""The STAR (CenSurE) oracle (oracle/orc_star.c, OpenCV 2.4.9 StarDetector restated) against independent
numpy statements of the same definitions: the integrals as plain sums over their regions, each pattern's
box sum as the upright square plus the 45-degree diamond it covers, the responses from those sums in
float32, and the tile suppression + line test as straightforward Python loops.  OpenCV itself is not in
this image, so parity with it is unpinned beyond these definitions."""
import numpy as np
import pytest
from scipy import ndimage, signal

import oracle as orc  # tests/conftest.py puts oracle/ on the path

SIZES0 = [1, 2, 3, 4, 6, 8, 11, 12, 16, 22, 23, 32, 45, 46, 64, 90, 128]
PAIRS = [(1, 0), (3, 1), (4, 2), (5, 3), (7, 4), (8, 5), (9, 6), (11, 8), (13, 10), (14, 11), (15, 12), (16, 14)]


def _image(h, w, seed, smooth=2.0):
    """bright and dark Gaussian blobs of radius 2..12 on smoothed noise"""
    rng = np.random.default_rng(seed)
    img = ndimage.gaussian_filter(rng.normal(128, 40, (h, w)), smooth)
    yy, xx = np.mgrid[0:h, 0:w]
    for _ in range(h * w // 400):
        cy, cx, r = rng.uniform(0, h), rng.uniform(0, w), rng.uniform(2, 12)
        img += rng.choice([-1, 1]) * rng.uniform(40, 110) * np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * r * r))
    return np.clip(img, 0, 255).astype(np.uint8)


def _tri_sums(I, flat):
    h, w = I.shape
    out = np.zeros((h + 1, w + 1), np.int64)
    R = np.concatenate([np.zeros((h, 1), np.int64), I.astype(np.int64).cumsum(1)], 1)  # R[y, k] = sum I[y, :k]
    for y in range(1, h + 1):
        d = y - 1 - np.arange(y)  # rows 0..y-1
        for x in range(w + 1):
            lo = np.clip(x - 1 - d, 0, w)
            hi = np.clip(x + d + (1 if flat else 0), 0, w)  # exclusive end
            out[y, x] = (R[np.arange(y), np.maximum(hi, lo)] - R[np.arange(y), lo]).sum()
    return out


@pytest.mark.parametrize("h,w", [(7, 9), (23, 17), (31, 40)])
def test_integrals_are_region_sums(h, w):
    I = np.random.default_rng(h * w).integers(0, 256, (h, w)).astype(np.uint8)
    S, T, F = orc.star_integrals(I)
    Sd = np.zeros((h + 1, w + 1), np.int64)
    Sd[1:, 1:] = I.astype(np.int64).cumsum(0).cumsum(1)
    assert (S == Sd).all()
    assert (T == _tri_sums(I, False)).all()  # |x' - (x-1)| <= y-1-y'
    assert (F == _tri_sums(I, True)).all()   # x-1-(y-1-y') <= x' <= x+(y-1-y')


def _star_kernel(u):
    t = u + u // 2
    dy, dx = np.mgrid[-t:t + 1, -t:t + 1]
    k = (np.abs(dy) + np.abs(dx) <= t).astype(np.int64)
    k[t - u:t + u + 1, t - u:t + u + 1] += 1
    return k


def _responses_np(I, max_size):
    h, w = I.shape
    n, mi, border, sizes1, _, _ = orc.star_patterns(w, h, max_size)
    Ii = I.astype(np.int64)
    # box sums by FFT convolution with the (symmetric) pattern, rounded: exact for sums far below 2^52
    vals = [np.rint(signal.fftconvolve(Ii.astype(np.float64), _star_kernel(SIZES0[i]).astype(np.float64), "same"))
            .astype(np.int64) for i in range(mi + 1)]
    area = [int(_star_kernel(SIZES0[i]).sum()) for i in range(mi + 1)]
    R = np.zeros((h, w), np.float32)
    Z = np.zeros((h, w), np.int16)
    ys, xs = slice(border, h - border), slice(border, w - border)
    best = np.zeros((h - 2 * border, w - 2 * border), np.float32)
    bsz = np.zeros_like(best, dtype=np.int16)
    # OpenCV's SSE2 block covers the first 4*floor((w - 2*border)/4) columns and converts before
    # subtracting; the scalar tail converts the int difference (the forms differ above 2^24)
    simd = (np.arange(w - 2 * border) < 4 * ((w - 2 * border) // 4))[None, :]
    for i in range(n):
        o, q = PAIRS[i]
        inner, outer_area = vals[q][ys, xs], area[o] - area[q]
        outer = np.where(simd, vals[o][ys, xs].astype(np.float32) - inner.astype(np.float32),
                         (vals[o][ys, xs] - inner).astype(np.float32))
        r = inner.astype(np.float32) * (np.float32(1) / np.float32(area[q])) - \
            outer * (np.float32(1) / np.float32(outer_area))
        m = np.abs(r) > np.abs(best)
        best = np.where(m, r, best)
        bsz = np.where(m, sizes1[o], bsz)
    R[ys, xs], Z[ys, xs] = best, bsz
    return border, R, Z


@pytest.mark.parametrize("max_size,shape", [(45, (200, 262)), (16, (90, 130)), (23, (120, 151))])
def test_responses_match_box_sums(max_size, shape):
    I = _image(*shape, seed=max_size)
    b, R, Z = orc.star_responses(I, max_size)
    b2, R2, Z2 = _responses_np(I, max_size)
    assert b == b2
    assert np.array_equal(R.view(np.uint32), R2.view(np.uint32))
    assert (Z == Z2).all()


def test_responses_above_2p24_keep_both_column_forms():
    # MaxSize 128 on a bright image: the largest pattern's sums pass 2^24, where float(a) - float(b)
    # and float(a - b) can round differently; the oracle keeps OpenCV's form per column
    rng = np.random.default_rng(11)
    I = rng.integers(200, 256, (400, 427)).astype(np.uint8)
    b, R, Z = orc.star_responses(I, 128)
    b2, R2, Z2 = _responses_np(I, 128)
    assert b == 192
    assert np.array_equal(R.view(np.uint32), R2.view(np.uint32)) and (Z == Z2).all()


def test_pattern_set():
    # maxSize 45 (the default): pairs up to outer 46 (kept for the size rejection), border 46 + 23
    n, mi, b, sizes1, _, inv = orc.star_patterns(640, 480, 45)
    assert (n, mi, b) == (9, 13, 69)
    assert list(sizes1[:mi + 1]) == [-1, -2, 3, 4, 6, 8, 11, 12, 16, 22, 23, 32, 45, -46]
    # the StarAdjuster's detector: maxSize 16 -> pairs up to outer 16, border 24
    assert orc.star_patterns(640, 480, 16)[:3] == (6, 8, 24)
    # a small image stops the pattern set early: a pair stays while the next pair's outer border
    # (size + size/2) is below min(w, h); outer 22 (border 33) does not fit 30 rows
    assert orc.star_patterns(40, 30, 45)[:3] == (6, 8, 24)
    assert orc.star_patterns(6, 50, 45)[0] == 0 and orc.star_patterns(640, 480, 129)[0] == 0


def _lines(R, Z, x0, y0, lp, lb):
    sz = int(Z[y0, x0])
    d = sz // 4
    rad = 4 * d
    Lxx = Lyy = Lxy = np.float32(0)
    for y in range(y0 - rad, y0 + rad + 1, d):
        for x in range(x0 - rad, x0 + rad + 1, d):
            Lx = np.float32(R[y, x + 1] - R[y, x - 1])
            Ly = np.float32(R[y + 1, x] - R[y - 1, x])
            Lxx, Lyy, Lxy = np.float32(Lxx + Lx * Lx), np.float32(Lyy + Ly * Ly), np.float32(Lxy + Lx * Ly)
    if np.float32((Lxx + Lyy) * (Lxx + Lyy)) >= np.float32(np.float32(lp) * np.float32(Lxx * Lyy - Lxy * Lxy)):
        return True
    bxx = byy = bxy = 0
    for y in range(y0 - rad, y0 + rad + 1, d):
        for x in range(x0 - rad, x0 + rad + 1, d):
            bx = int(Z[y, x + 1] == sz) - int(Z[y, x - 1] == sz)
            by = int(Z[y + 1, x] == sz) - int(Z[y - 1, x] == sz)
            bxx, byy, bxy = bxx + bx * bx, byy + by * by, bxy + bx * by
    return (bxx + byy) ** 2 >= lb * (bxx * byy - bxy * bxy)


def _detect_py(I, max_size, resp, lp, lb, supp):
    h, w = I.shape
    border, R, Z = orc.star_responses(I, max_size)
    delta = supp // 2
    out = []
    for y in range(border, h - border, delta + 1):
        for x in range(border, w - border, delta + 1):
            tile = R[y:min(y + delta, h - border - 1) + 1, x:min(x + delta, w - border - 1) + 1]
            mx = mn = None
            maxr, minr = np.float32(resp), np.float32(-resp)
            for (j, i), v in np.ndenumerate(tile):
                if maxr < v:
                    maxr, mx = v, (x + i, y + j)
                elif minr > v:
                    minr, mn = v, (x + i, y + j)
            for pt, cmp in ((mx, lambda v: v >= maxr), (mn, lambda v: v <= minr)):
                if pt is None:
                    continue
                px, py = pt
                win = R[py - delta:py + delta + 1, px - delta:px + delta + 1]
                hits = [(j, i) for (j, i), v in np.ndenumerate(win) if cmp(v) and (j, i) != (delta, delta)]
                if hits:
                    continue
                if Z[py, px] >= 4 and not _lines(R, Z, px, py, lp, lb):
                    out.append((px, py, float(Z[py, px]), float(maxr)))
    return out


@pytest.mark.parametrize("params", [(45, 30, 10, 8, 5), (16, 12, 10, 8, 3), (23, 20, 6, 5, 7)])
def test_detect_matches_loops(params):
    I = _image(170, 230, seed=sum(params), smooth=1.5)
    k = orc.star_detect(I, *params)
    ref = _detect_py(I, *params)
    assert len(k) == len(ref) and len(k) > 0
    got = [(float(a["x"]), float(a["y"]), float(a["size"]), float(a["response"])) for a in k]
    assert got == ref
    assert (k["angle"] == -1).all() and (k["octave"] == 0).all() and (k["class_id"] == -1).all()


def test_undefined_inputs_refused():
    with pytest.raises(ValueError):
        orc.star_detect(np.zeros((6, 40), np.uint8))
    with pytest.raises(ValueError):
        orc.star_detect(np.zeros((300, 300), np.uint8), max_size=200)
    assert len(orc.star_detect(np.zeros((100, 100), np.uint8))) == 0  # flat: no response passes


def test_star_adjuster_walk():
    I = _image(240, 320, seed=3, smooth=1.2)
    k = orc.adaptive_detect(I, "STAR", 50, 80, 10)
    counts = []
    thresh = 30.0
    for _ in range(10):  # the same walk by hand
        kk = orc.star_detect(I, 16, int(np.rint(thresh)), 10, 8, 3)
        counts.append(len(kk))
        if len(kk) < 50:
            thresh = max(thresh * 0.9, 1.1)
        elif len(kk) > 80:
            thresh *= 1.1
        else:
            break
        if not (2 < thresh < 200) or (min(counts) < 50 and max(counts) > 80):
            break
    assert len(k) == counts[-1]
