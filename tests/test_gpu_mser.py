"""The MSER detector on the GPU (fm3d_mser.hip: DetectorType MSER, descriptorsmatcher.cpp:258-272) bit for
bit against oracle/orc_mser.c (OpenCV 2.4.9's grey-image MSER + fitEllipse restated; pinned by
tests/test_mser_oracle.py): the regions (colour, points in list order) and the keypoints on synthetic
VGA frames and small images, the nine MSERDetector settings through fm3d_detect, the detector with
every extractor through compareWithNNDR, the degenerate cases, and OpenCV's fitEllipse throw."""
import time

import numpy as np
import pytest
from scipy import ndimage

pytestmark = pytest.mark.gpu


def _ctx(fm3d, **kw):
    s = fm3d.Settings.default()
    for k, v in kw.items():
        setattr(s, k, v)
    return fm3d.Context(s), s


def _same_kpts(a, b):
    assert len(a) == len(b), (len(a), len(b))
    for f in ("x", "y", "size", "angle", "response", "octave", "class_id"):
        assert np.array_equal(a[f], b[f]), f


def _same_regions(a, b):
    assert len(a) == len(b), (len(a), len(b))
    for (ca, pa), (cb, pb) in zip(a, b):
        assert ca == cb and np.array_equal(pa, pb)


def _blurred(h, w, sigma, seed):
    rng = np.random.default_rng(seed)
    img = ndimage.gaussian_filter(rng.random((h, w)) * 255, sigma)
    return ((img - img.min()) / max(np.ptp(img), 1e-9) * 255).astype(np.uint8)


SMALL = [
    (_blurred(40, 50, 1.5, 1), dict(min_area=10, max_area=800)),
    (_blurred(33, 47, 1.0, 2), dict(delta=1, min_area=5, max_area=400)),
    (_blurred(64, 64, 2.0, 3), {}),
    ((np.random.default_rng(4).random((24, 31)) * 255).astype(np.uint8), dict(min_area=4, max_area=300)),
    (_blurred(36, 36, 1.2, 5), dict(delta=3, min_area=8, max_area=1000, max_variation=1.0, min_diversity=0.0)),
    (np.full((30, 40), 77, np.uint8), {}),
    (np.zeros((1, 1), np.uint8), {}),
    ((np.arange(17) * 37 % 256).astype(np.uint8).reshape(1, 17), dict(min_area=0)),
    ((np.arange(13) * 37 % 256).astype(np.uint8).reshape(13, 1), dict(min_area=0)),
]


def test_mser_regions_small_bitwise(fm3d, orc):
    ctx, _ = _ctx(fm3d)
    try:
        F = fm3d.Features(ctx)
        for img, kw in SMALL:
            _same_regions(F.mser_regions(img, **kw), orc.mser_regions(img, **kw))
            if kw.get("min_area", 60) >= 4:
                _same_kpts(F.mser(img, **kw), orc.mser_detect(img, **kw))
    finally:
        ctx.close()


@pytest.mark.parametrize("seed", [71, 72])
def test_mser_vga_bitwise(fm3d, orc, synth, seed):
    img = synth.make_frame_pair(2000, seed=seed).img1
    ctx, _ = _ctx(fm3d)
    try:
        F = fm3d.Features(ctx)
        t0 = time.perf_counter()
        k = F.mser(img)
        t1 = time.perf_counter()
        r = F.mser_regions(img)
    finally:
        ctx.close()
    ko = orc.mser_detect(img)
    print(f"MSER VGA: {len(k)} keypoints, {len(r)} regions, {1e3 * (t1 - t0):.1f} ms (incl. first-call setup)")
    assert len(k) > 200
    _same_kpts(k, ko)
    _same_regions(r, orc.mser_regions(img))


def test_mser_large_image_hbm_bitmap(fm3d, orc):
    """an image past the LDS bitmap (kMserLdsBits = 983,040 pixels): the visited bits in HBM"""
    img = _blurred(1000, 1024, 3.0, 9)
    kw = dict(min_area=30, max_area=20000)
    ctx, _ = _ctx(fm3d)
    try:
        F = fm3d.Features(ctx)
        r = F.mser_regions(img, **kw)
        k = F.mser(img, **kw)
    finally:
        ctx.close()
    _same_regions(r, orc.mser_regions(img, **kw))
    _same_kpts(k, orc.mser_detect(img, **kw))
    assert len(r) > 50


def test_mser_wide_image_large_regions_centroid(fm3d, orc):
    """a wide image with large regions, where a region's coordinate sum passes 2^24 (the
    float centroid is then no longer exact in any order): the GPU sums such a region in list order,
    as OpenCV and the oracle, and the keypoints stay bit-identical"""
    img = _blurred(96, 3000, 10.0, 21)
    kw = dict(min_area=1000, max_area=60000)
    ctx, _ = _ctx(fm3d)
    try:
        k = fm3d.Features(ctx).mser(img, **kw)
    finally:
        ctx.close()
    regs = orc.mser_regions(img, **kw)
    big = [len(p) * int(p.max()) for _, p in regs]
    assert max(big) >= 1 << 24, max(big)  # the case the sequential sum exists for
    _same_kpts(k, orc.mser_detect(img, **kw))
    assert len(k) > 3


def test_mser_batch_equals_single(fm3d, orc, synth):
    """fm3d_mser_detect_batch: every image's floods side by side; each image's keypoints equal its own
    fm3d_mser_detect (and the oracle), including an image without regions in the middle"""
    imgs = [synth.make_frame_pair(2000, seed=71).img1, np.full((480, 640), 90, np.uint8),
            synth.make_frame_pair(2000, seed=72).img2, _blurred(480, 640, 2.5, 12)]
    ctx, _ = _ctx(fm3d)
    try:
        F = fm3d.Features(ctx)
        single = [F.mser(i) for i in imgs]
        batch = F.mser_batch(imgs)
        small = F.mser_batch([img for img, kw in SMALL[:3] if img.shape == (40, 50)] * 3, min_area=10,
                             max_area=800)
    finally:
        ctx.close()
    assert len(batch) == len(imgs)
    for a, b in zip(batch, single):
        _same_kpts(a, b)
    assert len(batch[1]) == 0 and len(batch[0]) > 100
    _same_kpts(batch[2], orc.mser_detect(imgs[2]))
    want = orc.mser_detect(SMALL[0][0], min_area=10, max_area=800)
    assert len(small) == 3
    for k in small:
        _same_kpts(k, want)


def test_mser_batch_hbm_bitmap(fm3d, orc):
    """a batch of images past the LDS bitmap: every slot's visited bits at its own offset in HBM"""
    imgs = [_blurred(1000, 1024, 3.0, 9), _blurred(1000, 1024, 2.0, 10)]
    kw = dict(min_area=30, max_area=20000)
    ctx, _ = _ctx(fm3d)
    try:
        batch = fm3d.Features(ctx).mser_batch(imgs, **kw)
    finally:
        ctx.close()
    for img, k in zip(imgs, batch):
        _same_kpts(k, orc.mser_detect(img, **kw))
    assert len(batch[0]) > 50 and len(batch[1]) > 50


def test_mser_settings_through_detect(fm3d, orc, synth):
    """DetectorType MSER with the nine MSERDetector keys (the last four do not steer grey images)"""
    img = synth.make_frame_pair(1500, seed=75).img2
    kw = dict(mserDelta=3, mserMinArea=30, mserMaxArea=5000, mserMaxVariation=0.4, mserMinDiversity=0.1,
              mserMaxEvolution=100, mserAreaThreshold=1.2, mserMinMargin=0.01, mserEdgeBlurSize=3)
    ctx, s = _ctx(fm3d, detectorType=fm3d.FEAT_MSER, **kw)
    try:
        k = fm3d.Features(ctx).detect(img)
    finally:
        ctx.close()
    ko = orc.mser_detect(img, delta=3, min_area=30, max_area=5000, max_variation=0.4, min_diversity=0.1)
    _same_kpts(k, ko)
    assert len(k) > 100


def test_mser_throws_like_fit_ellipse(fm3d, orc):
    """MinArea < 4 lets a region of under 5 points through, where OpenCV's fitEllipse throws"""
    img = (np.random.default_rng(8).random((20, 20)) * 255).astype(np.uint8)  # a 4-point region
    with pytest.raises(ValueError):
        orc.mser_detect(img, min_area=0, max_area=400, max_variation=10.0, min_diversity=0.0)
    ctx, _ = _ctx(fm3d)
    try:
        with pytest.raises(fm3d.Fm3dError):
            fm3d.Features(ctx).mser(img, min_area=0, max_area=400, max_variation=10.0, min_diversity=0.0)
        # the regions themselves are still defined
        _same_regions(fm3d.Features(ctx).mser_regions(img, min_area=0, max_area=400, max_variation=10.0,
                                                      min_diversity=0.0),
                      orc.mser_regions(img, min_area=0, max_area=400, max_variation=10.0, min_diversity=0.0))
    finally:
        ctx.close()


@pytest.mark.parametrize("ext", ["BRISK", "ORB", "FREAK"])
def test_mser_detector_with_extractor(fm3d, orc, synth, ext):
    """the reference's two calls: MSER keypoints, then the settings' extractor, matched by NNDR"""
    fp = synth.make_frame_pair(3000, seed=71)
    T = {"BRISK": fm3d.FEAT_BRISK, "ORB": fm3d.FEAT_ORB, "FREAK": fm3d.FEAT_FREAK}
    ctx, s = _ctx(fm3d, detectorType=fm3d.FEAT_MSER, extractorType=T[ext])
    try:
        m, ka, kb, da, db = fm3d.DescriptorsMatcher(ctx).compareWithNNDRImages(0.8, fp.img1, fp.img2)
    finally:
        ctx.close()
    oa, ob = orc.mser_detect(fp.img1), orc.mser_detect(fp.img2)
    f = {"BRISK": orc.brisk_compute, "ORB": orc.orb_compute, "FREAK": orc.freak_compute}[ext]
    ra, rb = f(fp.img1, oa), f(fp.img2, ob)
    kind = orc.BITS
    _same_kpts(ka, ra[0])
    _same_kpts(kb, rb[0])
    assert np.array_equal(da, ra[-1]) and np.array_equal(db, rb[-1])
    q, t, dist = orc.match_nndr(ra[-1], rb[-1], kind, 0.8)
    assert len(m) == len(q) > 5
    assert np.array_equal(m["queryIdx"], q) and np.array_equal(m["trainIdx"], t)
