"""The FREAK extractor oracle (oracle/orc_freak.c, OpenCV 2.4.9's FREAK descriptor restated) against
independent statements of its definitions: the pattern (8 circles, 64 scales, 256 orientations) in
Python's libm, the pattern sizes, the orientation weights, the keypoint scale, the integral-box mean
as a numpy slice sum, and the whole descriptor (filter, orientation, rotated intensities, the SSE2 bit
layout) rebuilt from those pieces.  OpenCV itself is not in this image, so parity with it is unpinned
beyond these definitions; FREAK::DEF_PAIRS is restated in include/fm3d_freak.h."""
import math
import os
import re

import numpy as np
import pytest

import oracle as orc  # tests/conftest.py puts oracle/ on the path

f32 = np.float32
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = [6, 6, 6, 6, 6, 6, 6, 1]
BIGR, SMALLR = 2.0 / 3.0, 2.0 / 24.0
US = (BIGR - SMALLR) / 21.0
RADIUS = [BIGR, BIGR - 6 * US, BIGR - 11 * US, BIGR - 15 * US, BIGR - 18 * US, BIGR - 20 * US, SMALLR, 0.0]
SIGMA = [r / 2.0 for r in RADIUS[:7]] + [RADIUS[6] / 2.0]


def _points(s, rot):
    sf = math.pow(math.pow(2.0, 4 / 64), s)
    theta = rot * 2 * math.pi / 256
    out = []
    for i in range(8):
        for k in range(N[i]):
            beta = math.pi / N[i] * (i % 2)
            alpha = k * 2 * math.pi / N[i] + beta + theta
            out.append((f32(RADIUS[i] * math.cos(alpha) * sf * 22.0), f32(RADIUS[i] * math.sin(alpha) * sf * 22.0),
                        f32(SIGMA[i] * sf * 22.0)))
    return out


def _tables():
    txt = open(os.path.join(ROOT, "include", "fm3d_freak.h")).read()
    def arr(name):
        body = re.search(name + r"\[[^\]]*\] = \{([^}]*)\}", txt).group(1)
        return [int(x) for x in body.replace("\n", " ").split(",") if x.strip()]
    return arr("FM3D_FREAK_DEF_PAIRS"), arr("FM3D_FREAK_ORIENT_PAIRS")


@pytest.mark.parametrize("scale,rot", [(0, 0), (0, 1), (7, 100), (33, 200), (63, 255)])
def test_pattern_points(scale, rot):
    want = _points(scale, rot)
    for i in range(43):
        assert orc.freak_point(scale, rot, i) == want[i], i


def test_sizes_weights_kscale_and_tables():
    for s in (0, 1, 20, 47, 63):
        sf = math.pow(math.pow(2.0, 4 / 64), s)
        assert orc.freak_size(s) == max(math.ceil((RADIUS[i] + SIGMA[i]) * sf * 22.0) + 1 for i in range(8))
    pairs, op = _tables()
    assert len(pairs) == 512 and len(set(pairs)) == 512 and min(pairs) >= 0 and max(pairs) < 903
    assert len(op) == 90
    P = _points(0, 0)
    wx, wy = orc.freak_weights()
    for m in range(45):
        i, j = op[2 * m], op[2 * m + 1]
        dx, dy = f32(P[i][0] - P[j][0]), f32(P[i][1] - P[j][1])
        n2 = f32(dx * dx + dy * dy)
        assert wx[m] == int(float(f32(dx / n2)) * 4096.0 + 0.5)
        assert wy[m] == int(float(f32(dy / n2)) * 4096.0 + 0.5)
    cst = f32(64 / (0.693147180559945 * 4))
    for size in (0.5, 6.9, 7.0, 7.1, 10.0, 31.0, 64.0, 128.0, 1e4):
        want = int(float(f32(np.log(f32(f32(size) / f32(7))) * cst)) + 0.5)
        assert orc.freak_kscale(size) == min(max(want, 0), 63), size


def _box_mean(img, kx, ky, px, py, r):
    xf, yf = f32(f32(px) + f32(kx)), f32(f32(py) + f32(ky))
    xl, yt = int(float(f32(xf - f32(r))) + 0.5), int(float(f32(yf - f32(r))) + 0.5)
    xr, yb = int(float(f32(xf + f32(r))) + 1.5), int(float(f32(yf + f32(r))) + 1.5)
    s = int(img[yt:yb, xl:xr].astype(np.int64).sum())  # integral(yb, xr) - ... = the pixels [yt, yb) x [xl, xr)
    return s // ((xr - xl) * (yb - yt))


def test_mean_intensity_box():
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (120, 160), dtype=np.uint8)
    for _ in range(300):
        kx, ky = rng.uniform(40, 120), rng.uniform(40, 80)
        px, py = rng.uniform(-20, 20, 2)
        r = rng.uniform(0.5, 9)
        assert orc.freak_mean_intensity(img, kx, ky, px, py, r) == _box_mean(img, kx, ky, px, py, r)


def test_descriptor_rebuilt_from_pieces(synth):
    """filter, orientation, rotated intensities and the SSE2 bit layout, restated in numpy from the
    pieces above"""
    img = synth.make_frame_pair(500, 320, 240, seed=5).img1
    rng = np.random.default_rng(6)
    n = 120
    k = np.zeros(n, dtype=orc.KEYPOINT)
    k["x"], k["y"] = rng.uniform(0, 320, n), rng.uniform(0, 240, n)
    k["size"] = rng.choice([0.0, 5.0, 7.0, 12.0, 20.0, 33.0], n)
    k["angle"] = -1
    ko, kept, d = orc.freak_compute(img, k)
    pairs, op = _tables()
    ij = []
    for p in pairs:
        a = 1
        while p >= a:
            p -= a
            a += 1
        ij.append((a, p))
    wx, wy = orc.freak_weights()
    m = 0
    for q in range(n):
        if not k["size"][q] >= np.finfo(np.float32).eps:
            continue
        s = orc.freak_kscale(k["size"][q])
        ps = f32(orc.freak_size(s))
        x, y = f32(k["x"][q]), f32(k["y"][q])
        if x <= ps or y <= ps or x >= f32(320) - ps or y >= f32(240) - ps:
            continue
        assert kept[m] == q
        v = [_box_mean(img, x, y, *pt) for pt in _points(s, 0)]
        d0 = d1 = 0
        for o in range(44, -1, -1):
            delta = v[op[2 * o]] - v[op[2 * o + 1]]
            d0 += int(delta * wx[o] / 2048)  # C division truncates toward zero
            d1 += int(delta * wy[o] / 2048)
        ang = f32(float(f32(math.atan2(float(f32(d1)), float(f32(d0))))) * (180.0 / math.pi))
        assert ko["angle"][m] == ang
        th = int(float(f32(f32(256) * ang)) * (1 / 360.0) + 0.5)
        th = th + 256 if th < 0 else (th - 256 if th >= 256 else th)
        v = [_box_mean(img, x, y, *pt) for pt in _points(s, th)]
        want = np.zeros(64, np.uint8)
        for qq in range(4):
            for t in range(8):
                for b in range(16):
                    i, j = ij[128 * qq + 16 * t + 15 - b]
                    if v[i] >= v[j]:
                        want[16 * qq + b] |= 1 << t
        assert np.array_equal(d[m], want), q
        m += 1
    assert m == len(ko) > 20


def test_rotation_invariance(synth):
    """FREAK rotates its pattern to the measured orientation: a keypoint of the image and the same
    point of the image turned by 90 degrees get mostly equal descriptor bits"""
    img = synth.make_frame_pair(500, 320, 320, seed=8).img1
    rot = np.ascontiguousarray(np.rot90(img))  # (x, y) -> (y, 319 - x)
    rng = np.random.default_rng(9)
    n = 200
    k = np.zeros(n, dtype=orc.KEYPOINT)
    k["x"], k["y"] = rng.uniform(70, 250, n).round(), rng.uniform(70, 250, n).round()
    k["size"] = 14.0
    k2 = k.copy()
    k2["x"], k2["y"] = k["y"], 319 - k["x"]
    ka, _, da = orc.freak_compute(img, k)
    kb, _, db = orc.freak_compute(rot, k2)
    assert len(ka) == len(kb) == n
    same = (np.unpackbits(da, axis=1) == np.unpackbits(db, axis=1)).mean(axis=1)
    assert np.median(same) > 0.8
