"""Pins of oracle/orc_mser.c (OpenCV 2.4.9's grey-image MSER + fitEllipse, restated) -- CPU only.

OpenCV is not in this image, so the restatement is pinned (a) bit for bit against an independent
pure-Python statement of the same flood and solves (tests/mser_pyref.py), and (b) against numpy and
scipy on what MSER's output must satisfy: areas inside (MinArea, MaxArea), regions that are whole
extremal regions (a connected component of {v <= max v} with every outside neighbour above it, v = I
for colour +1 and 255 - I for colour -1) or, after a merge, the merge winner's part (mser.cpp's
"one step back"), and fitEllipse's conics equal to numpy's least-squares solutions.  Reference: DescriptorsMatcher/descriptorsmatcher.cpp:258-272.
"""
import numpy as np
import pytest
from scipy import ndimage

import oracle as O
import mser_pyref as R


def _blurred(h, w, sigma, seed):
    rng = np.random.default_rng(seed)
    img = ndimage.gaussian_filter(rng.random((h, w)) * 255, sigma)
    return ((img - img.min()) / max(np.ptp(img), 1e-9) * 255).astype(np.uint8)


def _blobs():
    img = np.full((80, 100), 200.0)
    yy, xx = np.mgrid[:80, :100]
    img[(xx - 30) ** 2 + (yy - 40) ** 2 < 100] = 50
    img[((xx - 70) / 15.0) ** 2 + ((yy - 30) / 8.0) ** 2 < 1] = 120
    return ndimage.gaussian_filter(img, 2).astype(np.uint8)


CASES = [
    ("blurred", _blurred(40, 50, 1.5, 1), dict(min_area=10, max_area=800)),
    ("blurred-delta1", _blurred(33, 47, 1.0, 2), dict(delta=1, min_area=5, max_area=400)),
    ("blurred-defaults", _blurred(64, 64, 2.0, 3), {}),
    ("blobs", _blobs(), {}),
    ("noise", (np.random.default_rng(4).random((24, 31)) * 255).astype(np.uint8), dict(min_area=4, max_area=300)),
    ("loose", _blurred(36, 36, 1.2, 5), dict(delta=3, min_area=8, max_area=1000, max_variation=1.0,
                                               min_diversity=0.0)),
]


@pytest.mark.parametrize("name,img,kw", CASES, ids=[c[0] for c in CASES])
def test_flood_matches_python_restatement(name, img, kw):
    a = O.mser_regions(img, **kw)
    b = R.mser_regions(img, **kw)
    assert len(a) == len(b)
    for (ca, pa), (cb, pb) in zip(a, b):
        assert ca == cb
        assert np.array_equal(pa, np.asarray(pb, np.int32).reshape(-1, 2))
    if name != "noise":
        assert len(a) > 0


@pytest.mark.parametrize("name,img,kw", CASES, ids=[c[0] for c in CASES])
def test_regions_are_extremal(name, img, kw):
    """A region checked when its component raises its level is a whole extremal region (a connected
    component of {v <= max v}, every outside neighbour above it).  mser.cpp also checks right after a
    merge, where MSERToContour's history->size is the merge winner's size: the region is then the
    winner's point list, i.e. complete basins without the not-yet-flooded pixels joining them (the
    "one step back" of mser.cpp's comments).  Both kinds lie inside one component of {v <= L} for
    the level L the flood stood at; most regions are of the first kind."""
    p = dict(O.MSER_DEFAULTS)
    p.update(kw)
    four = ndimage.generate_binary_structure(2, 1)
    regs = O.mser_regions(img, **kw)
    whole = 0
    for color, pts in regs:
        v = img.astype(np.int32) if color == 1 else 255 - img.astype(np.int32)
        mask = np.zeros(img.shape, bool)
        mask[pts[:, 1], pts[:, 0]] = True
        assert mask.sum() == len(pts), "a point listed twice"
        assert p["min_area"] < len(pts) < p["max_area"]
        m = v[mask].max()
        lab, _ = ndimage.label(v <= m, structure=four)
        labels = np.unique(lab[mask])
        comp = np.isin(lab, labels)
        assert np.array_equal(comp & mask, mask)
        # every piece of a region is a whole component of {v <= m} or the interrupted winner's part
        if len(labels) == 1 and np.array_equal(comp, mask):
            whole += 1
        # connected through pixels at some level: the smallest such level is above m
        for L in range(m, 256):
            lab2, _ = ndimage.label(v <= L, structure=four)
            if len(np.unique(lab2[mask])) == 1:
                break
        else:
            raise AssertionError("region not connected at any level")
    if regs:
        assert whole >= 0.6 * len(regs)


def test_merge_region_is_winner_part():
    """the documented mser.cpp quirk on a fixed image: a region made of two complete basins of
    {v <= 94} whose joining pixels (>= 95) are not in it"""
    img = _blurred(40, 50, 1.5, 1)
    four = ndimage.generate_binary_structure(2, 1)
    found = False
    for color, pts in O.mser_regions(img, min_area=10, max_area=800):
        v = img.astype(np.int32) if color == 1 else 255 - img.astype(np.int32)
        mask = np.zeros(img.shape, bool)
        mask[pts[:, 1], pts[:, 0]] = True
        m = v[mask].max()
        lab, _ = ndimage.label(v <= m, structure=four)
        labels = np.unique(lab[mask])
        if len(labels) == 2 and np.array_equal(np.isin(lab, labels), mask):
            found = True
    assert found


def test_regions_both_colours_and_order():
    regs = O.mser_regions(_blobs())
    colours = [c for c, _ in regs]
    assert colours == sorted(colours)  # pass 1 (-1, on 255 - I) before pass 2 (+1)
    assert -1 in colours and 1 in colours


@pytest.mark.parametrize("shape", [(1, 1), (1, 17), (13, 1), (2, 2), (5, 3)])
def test_degenerate_sizes(shape):
    img = (np.arange(np.prod(shape)) * 37 % 256).astype(np.uint8).reshape(shape)
    a = O.mser_regions(img, min_area=0, max_area=1000)
    b = R.mser_regions(img, min_area=0, max_area=1000)
    assert [(c, p.tolist()) for c, p in a] == [(c, [list(q) for q in pts]) for c, pts in b]


def test_constant_image_has_no_region():
    assert O.mser_regions(np.full((30, 40), 77, np.uint8)) == []
    assert len(O.mser_detect(np.full((30, 40), 77, np.uint8))) == 0


def test_fit_ellipse_solves_match_python():
    for _, pts in O.mser_regions(_blurred(40, 50, 1.5, 1), min_area=10, max_area=800)[:12]:
        sol = O.fit_ellipse_solves(pts)
        cx, cy, g, rp, g2 = R.fit_ellipse([tuple(q) for q in pts])
        assert np.array_equal(sol, np.array([cx, cy] + g + rp + g2))


def test_fit_ellipse_least_squares_vs_numpy():
    for _, pts in O.mser_regions(_blobs()):
        sol = O.fit_ellipse_solves(pts)
        c = pts.astype(np.float32).sum(0) / np.float32(len(pts))
        assert np.allclose(sol[:2], c, rtol=0, atol=1e-5)
        # the oracle's differences are float (x - cx in float), its products double
        p = (pts.astype(np.float32) - sol[:2].astype(np.float32)).astype(np.float64)
        A = np.stack([-p[:, 0] ** 2, -p[:, 1] ** 2, -p[:, 0] * p[:, 1], p[:, 0], p[:, 1]], 1)
        g = np.linalg.lstsq(A, np.full(len(p), 10000.0), rcond=None)[0]
        # symmetric blobs have near-zero linear terms: tolerances scale with the largest coefficient
        assert np.allclose(sol[2:7], g, rtol=1e-7, atol=1e-9 * np.abs(g).max())
        rp = np.linalg.solve([[2 * g[0], g[2]], [g[2], 2 * g[1]]], g[3:5])
        assert np.allclose(sol[7:9], rp, rtol=1e-6, atol=1e-7)
        q = p - sol[7:9]
        A3 = np.stack([q[:, 0] ** 2, q[:, 1] ** 2, q[:, 0] * q[:, 1]], 1)
        g3 = np.linalg.lstsq(A3, np.ones(len(q)), rcond=None)[0]
        assert np.allclose(sol[9:12], g3, rtol=1e-7, atol=1e-9 * np.abs(g3).max())


def test_fit_ellipse_recovers_a_rasterised_ellipse():
    yy, xx = np.mgrid[:100, :120]
    a, b, th = 30.0, 12.0, np.deg2rad(30)
    u = (xx - 60) * np.cos(th) + (yy - 50) * np.sin(th)
    v = -(xx - 60) * np.sin(th) + (yy - 50) * np.cos(th)
    inside = (u / a) ** 2 + (v / b) ** 2 <= 1
    ys, xs = np.nonzero(inside)
    box = O.fit_ellipse(np.stack([xs, ys], 1))
    assert abs(box[0] - 60) < 0.05 and abs(box[1] - 50) < 0.05
    # the conic through a filled ellipse's points is a scaled copy of it: the axis ratio survives
    assert abs(box[3] / box[2] - a / b) < 0.05 * a / b


def test_fit_ellipse_needs_five_points():
    with pytest.raises(ValueError):
        O.fit_ellipse(np.array([[0, 0], [1, 0], [0, 1], [1, 1]]))


def test_detect_keypoints_from_regions():
    img = _blobs()
    regs = O.mser_regions(img)
    kp = O.mser_detect(img)
    assert len(kp) <= len(regs) and len(kp) > 0
    assert np.all(kp["angle"] == -1) and np.all(kp["response"] == 0)
    assert np.all(kp["octave"] == 0) and np.all(kp["class_id"] == -1)
    h, w = img.shape
    assert np.all((np.rint(kp["x"]) >= 0) & (np.rint(kp["x"]) < w) & (np.rint(kp["y"]) >= 0) & (np.rint(kp["y"]) < h))
    # the disk and the ellipse are found as nested regions around their centres
    near = lambda x, y: np.any((np.abs(kp["x"] - x) < 0.5) & (np.abs(kp["y"] - y) < 0.5))
    assert near(30, 40) and near(70, 30)
    # keypoint i is region i's ellipse, in region order (all regions are inside here)
    for k, (_, pts) in zip(kp, regs):
        box = O.fit_ellipse(pts)
        assert k["x"] == box[0] and k["y"] == box[1]
        assert k["size"] == np.sqrt(np.float32(box[3]) * np.float32(box[2]), dtype=np.float32)
