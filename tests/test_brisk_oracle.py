"""The BRISK extractor oracle (oracle/orc_brisk.c, OpenCV 2.4.9's BRISK descriptor restated) against
independent statements of its definitions: the pattern (rings, scales, rotations, sigmas) in Python's
libm, the short pairs by distance, the keypoint scale and rotation bins, the smoothed intensity as a
fixed-point weighted box sum written with numpy slices, and the descriptor bits from those pieces.
OpenCV itself is not in this image, so parity with it is unpinned beyond these definitions
(DESIGN.md §3.13)."""
import math

import numpy as np
import pytest

import oracle as orc  # tests/conftest.py puts oracle/ on the path

f32 = np.float32
RADII = [f32(0.85 * r) for r in (0.0, 2.9, 4.9, 7.4, 10.8)]
NUM = [1, 10, 14, 15, 20]


def _scale_factor(s):
    lb = f32(math.log(30.0) / math.log(2.0))
    step = f32(lb / f32(64))
    return f32(math.pow(2.0, float(f32(s) * step)))


def _point(s, rot, i):
    ring, num = 0, i
    while num >= NUM[ring]:
        num -= NUM[ring]
        ring += 1
    sc = _scale_factor(s)
    theta = rot * 2 * math.pi / 1024
    alpha = num * 2 * math.pi / NUM[ring]
    r = f32(sc * RADII[ring])
    x = f32(float(r) * math.cos(alpha + theta))
    y = f32(float(r) * math.sin(alpha + theta))
    if ring == 0:
        sg = f32(f32(f32(1.3) * sc) * f32(0.5))
    else:
        sg = f32(float(f32(f32(1.3) * sc)) * float(RADII[ring]) * math.sin(math.pi / NUM[ring]))
    return x, y, sg, ring


@pytest.mark.parametrize("scale,rot", [(0, 0), (0, 1), (5, 300), (31, 512), (63, 1023)])
def test_pattern_points(scale, rot):
    assert orc.brisk_scale_factor(scale) == _scale_factor(scale)
    for i in range(60):
        x, y, sg, _ = _point(scale, rot, i)
        assert orc.brisk_point(scale, rot, i) == (x, y, sg), i


def test_sizes_and_pairs():
    for s in (0, 1, 17, 40, 63):
        sc = _scale_factor(s)
        want = max(math.ceil(f32(f32(sc * RADII[_point(s, 0, i)[3]]) + _point(s, 0, i)[2])) + 1 for i in range(60))
        assert orc.brisk_size(s) == want
    P = [_point(0, 0, i) for i in range(60)]
    dmin2, dmax2 = f32(8.2) * f32(8.2), f32(5.85) * f32(5.85)
    pairs = []
    for i in range(1, 60):
        for j in range(i):
            dx, dy = f32(P[j][0] - P[i][0]), f32(P[j][1] - P[i][1])
            n2 = f32(f32(dx * dx) + f32(dy * dy))
            if not n2 > dmin2 and n2 < dmax2:
                pairs.append((i, j))
    pi, pj = orc.brisk_short_pairs()
    assert len(pairs) == 512 and list(zip(pi.tolist(), pj.tolist())) == pairs


def test_keypoint_scale_and_theta():
    lb = f32(math.log(30.0)) / f32(0.693147180559945)
    for size in (1.0, 7.2, 7.2000003, 9.0, 12.0, 31.0, 44.6, 100.0, 215.9, 216.0, 1e4):
        v = f32(f32(64) / f32(lb)) * f32(f32(np.log(f32(f32(size) / f32(f32(12.0) * f32(0.6))))) / f32(0.693147180559945))
        want = min(max(int(float(v) + 0.5), 0), 63)
        assert orc.brisk_kscale(size) == want, size
    assert orc.brisk_theta(-1) == 0
    for a in (0.0, 0.17, 90.0, 179.9, 270.0, 359.9, 359.99):
        t = int(1024 * (float(f32(a)) / 360.0) + 0.5)
        assert orc.brisk_theta(a) == (t - 1024 if t >= 1024 else t), a


def _intensity(img, kx, ky, px, py, sg):
    xf, yf = f32(px + f32(kx)), f32(py + f32(ky))
    area = f32(f32(4.0) * sg * sg)
    scaling = int(4194304.0 / float(area))
    scaling2 = int(float(f32(f32(scaling) * area)) / 1024.0)
    x_1, x1, y_1, y1 = f32(xf - sg), f32(xf + sg), f32(yf - sg), f32(yf + sg)
    xl, yt, xr, yb = int(float(x_1) + 0.5), int(float(y_1) + 0.5), int(float(x1) + 0.5), int(float(y1) + 0.5)
    rx_1, ry_1 = f32(f32(f32(xl) - x_1) + f32(0.5)), f32(f32(f32(yt) - y_1) + f32(0.5))
    rx1, ry1 = f32(f32(x1 - f32(xr)) + f32(0.5)), f32(f32(y1 - f32(yb)) + f32(0.5))
    W = np.full((yb - yt + 1, xr - xl + 1), scaling, np.int64)  # interior
    W[0, :], W[-1, :] = int(f32(ry_1 * f32(scaling))), int(f32(ry1 * f32(scaling)))
    W[:, 0], W[:, -1] = int(f32(rx_1 * f32(scaling))), int(f32(rx1 * f32(scaling)))
    W[0, 0], W[0, -1] = int(f32(f32(rx_1 * ry_1) * f32(scaling))), int(f32(f32(rx1 * ry_1) * f32(scaling)))
    W[-1, -1], W[-1, 0] = int(f32(f32(rx1 * ry1) * f32(scaling))), int(f32(f32(rx_1 * ry1) * f32(scaling)))
    tot = int((W * img[yt:yb + 1, xl:xr + 1].astype(np.int64)).sum())
    assert tot + scaling2 // 2 < 2 ** 31  # OpenCV's int sum does not overflow
    return (tot + scaling2 // 2) // scaling2


def test_smoothed_intensity_is_a_weighted_box():
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (200, 240)).astype(np.uint8)
    for _ in range(300):
        s, rot, i = int(rng.integers(0, 40)), int(rng.integers(0, 1024)), int(rng.integers(0, 60))
        x, y, sg, _ = _point(s, rot, i)
        kx, ky = f32(rng.uniform(90, 150)), f32(rng.uniform(80, 120))
        assert orc.brisk_intensity(img, kx, ky, x, y, sg) == _intensity(img, kx, ky, x, y, sg)
    bright = np.full((800, 800), 255, np.uint8)  # the largest box: the int sum stays in range
    x, y, sg, _ = _point(63, 0, 59)
    assert orc.brisk_intensity(bright, 400.0, 400.0, x, y, sg) == _intensity(bright, 400.0, 400.0, x, y, sg)
    # the weights sum to ~2^22 and scaling2 is ~2^12: intensities come out x 1024 (as the bilinear branch's)
    assert abs(orc.brisk_intensity(bright, 400.0, 400.0, x, y, sg) - 255 * 1024) <= 255


def test_compute_filter_and_bits(synth):
    img = synth.make_frame_pair(300, seed=12).img1
    rng = np.random.default_rng(5)
    k = np.zeros(400, dtype=orc.KEYPOINT)
    k["x"] = rng.uniform(-5, 645, 400)
    k["y"] = rng.uniform(-5, 485, 400)
    k["size"] = rng.choice([0.0, 5.0, 7.0, 9.0, 20.0, 31.0, 44.0, 90.0], 400)
    k["angle"] = rng.choice([-1.0, 0.0, 33.3, 270.0, 359.9], 400)
    kout, kept, d = orc.brisk_compute(img, k)
    pi, pj = orc.brisk_short_pairs()
    want = []
    for q in range(400):
        kp = k[q]
        if not kp["size"] >= np.finfo(np.float32).eps:
            continue
        s = orc.brisk_kscale(float(kp["size"]))
        b = orc.brisk_size(s)
        if kp["x"] < b or kp["x"] >= 640 - b or kp["y"] < b or kp["y"] >= 480 - b:
            continue
        want.append(q)
    assert kept.tolist() == want and 50 < len(want) < 400
    for m, q in enumerate(want[:40]):
        kp = k[q]
        s, t = orc.brisk_kscale(float(kp["size"])), orc.brisk_theta(float(kp["angle"]))
        vals = [_intensity(img, kp["x"], kp["y"], *_point(s, t, i)[:3]) for i in range(60)]
        bits = np.array([vals[a] > vals[b] for a, b in zip(pi, pj)], np.uint8)
        assert np.array_equal(np.packbits(bits, bitorder="little"), d[m]), q
