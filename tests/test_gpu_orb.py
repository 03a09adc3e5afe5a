"""GPU ORB (csrc/fm3d_orb.hip + the host's retainBest) against the ORB oracle (oracle/orc_orb.c), bit
for bit: keypoints (position, size, angle, Harris response, octave, class_id) in ORB's level-major
order and their 32-byte descriptors; compute on given keypoints; a caller pattern; compareWithNNDR
from the images with the settings' ORB (FeatureOptions DetectorType / ExtractorType ORB,
descriptorsmatcher.cpp:273-279, 336-341)."""
import numpy as np
import pytest

from conftest import oracle_threads

pytestmark = pytest.mark.gpu


def _ctx(fm3d, **kw):
    s = fm3d.Settings.default()
    s.detectorType = s.extractorType = fm3d.FEAT_ORB
    for k, v in kw.items():
        setattr(s, k, v)
    return fm3d.Context(s), s


def _same_kpts(a, b):
    assert len(a) == len(b), (len(a), len(b))
    for f in ("x", "y", "size", "angle", "response", "octave", "class_id"):
        assert np.array_equal(a[f], b[f]), f


def _orc_kw(s):
    return dict(nfeatures=s.orbNumFeatures, scaleFactor=s.orbScaleFactor, nlevels=s.orbNumLevels,
                edgeThreshold=s.orbEdgeThreshold, patchSize=s.orbPatchSize, fastThreshold=s.orbFastThreshold)


@pytest.mark.parametrize("nfeatures", [500, 2000, 10_000])
def test_orb_detect_describe_vga_bitwise(fm3d, orc, synth, nfeatures):
    """the reference's ORB construction cv::ORB(NumFeatures, 1.2, 8) on the synthetic VGA frames"""
    img = synth.make_frame_pair(4000, seed=3).img1
    ctx, s = _ctx(fm3d, orbNumFeatures=nfeatures)
    try:
        k, d = fm3d.ORB(ctx).detect(img, with_descriptors=True)
        k2 = fm3d.ORB(ctx).detect(img)
    finally:
        ctx.close()
    ko, do = orc.orb_detect(img, **_orc_kw(s))
    assert len(ko) > min(nfeatures, 3000) * 0.8
    _same_kpts(k, ko)
    _same_kpts(k2, ko)
    assert np.array_equal(d, do)


@pytest.mark.parametrize("shape,sf,nl,nf,thr", [((333, 257), 1.5, 4, 800, 20), ((480, 640), 1.1, 10, 3000, 12),
                                                 ((100, 90), 1.2, 8, 500, 20), ((64, 64), 1.2, 3, 100, 10)])
def test_orb_shapes_and_settings(fm3d, orc, shape, sf, nl, nf, thr):
    """odd sizes (the SSE/scalar column splits of resize and blur), other scale factors and level
    counts, levels smaller than the edge border (empty), another FAST threshold"""
    h, w = shape
    rng = np.random.default_rng(h * w)
    yy, xx = np.mgrid[0:h, 0:w]
    img = np.clip(128 + 80 * np.sin(xx * 0.21 + yy * 0.13) * np.cos(yy * 0.17 - xx * 0.05) + rng.normal(0, 25, shape),
                  0, 255).astype(np.uint8)
    ctx, s = _ctx(fm3d, orbScaleFactor=sf, orbNumLevels=nl, orbNumFeatures=nf, orbFastThreshold=thr)
    try:
        k, d = fm3d.ORB(ctx).detect(img, with_descriptors=True)
    finally:
        ctx.close()
    ko, do = orc.orb_detect(img, **_orc_kw(s))
    _same_kpts(k, ko)
    assert np.array_equal(d, do)


def test_orb_compute_given_keypoints(fm3d, orc, synth):
    """compute on detect()'s keypoints (the reference's detect-then-compute), on keypoints cut by the
    border / size filters, and the negative-octave error"""
    img = synth.make_frame_pair(4000, seed=5).img2
    ctx, s = _ctx(fm3d, orbNumFeatures=3000)
    try:
        orb = fm3d.ORB(ctx)
        k = orb.detect(img)
        kc, kept, d = orb.compute(img, k)
        kin = np.zeros(8, dtype=fm3d.KEYPOINT)
        kin["x"] = [100, 30.6, 300, 608.4, 200, 320, 150, 400]
        kin["y"] = [100, 200, 40, 300, 250, 240, 449.6, 300]
        kin["size"] = [31, 31, 0, 31, 37.2, 44.64, 31, 31]
        kin["octave"] = [0, 0, 0, 0, 1, 2, 0, 1]
        kin["angle"] = [10, 20, 30, 40, 50, 60, 70, 80]
        k2, kept2, d2 = orb.compute(img, kin)
        bad = kin[[0]].copy()
        bad["octave"] = -1
        with pytest.raises(fm3d.Fm3dError):
            orb.compute(img, bad)
    finally:
        ctx.close()
    ko, kepto, do = orc.orb_compute(img, k)
    _same_kpts(kc, ko)
    assert np.array_equal(kept, kepto) and np.array_equal(d, do) and len(kc) == len(k)
    ko2, kepto2, do2 = orc.orb_compute(img, kin)
    assert list(kept2) == [0, 1, 3, 4, 7, 5] and np.array_equal(kept2, kepto2)
    _same_kpts(k2, ko2)
    assert np.array_equal(d2, do2)


def test_orb_caller_pattern(fm3d, orc, synth):
    """fm3d_orb_set_pattern: the 512 points are data (OpenCV's bit_pattern_31_ when the caller has
    it); None restores makeRandomPattern"""
    img = synth.make_frame_pair(3000, seed=6).img1
    pat = np.random.default_rng(77).integers(-13, 14, (512, 2)).astype(np.int32)
    ctx, s = _ctx(fm3d, orbNumFeatures=1000)
    try:
        orb = fm3d.ORB(ctx)
        orb.set_pattern(pat)
        k, d = orb.detect(img, with_descriptors=True)
        orb.set_pattern(None)
        _, d0 = orb.detect(img, with_descriptors=True)
    finally:
        ctx.close()
    ko, do = orc.orb_detect(img, **_orc_kw(s), pattern=pat)
    _same_kpts(k, ko)
    assert np.array_equal(d, do) and not np.array_equal(d, d0)
    assert np.array_equal(d0, orc.orb_detect(img, **_orc_kw(s))[1])


def test_compare_with_nndr_from_images_orb(fm3d, orc, synth):
    """compareWithNNDR from the images with DetectorType / ExtractorType ORB: detect, compute on the
    detected keypoints, Hamming knnMatch (the binary extractor type, descriptorsmatcher.cpp:64), NNDR
    -- the same matches, keypoints and descriptors as the oracle chain"""
    pair = synth.make_frame_pair(4000, seed=4)
    ctx, s = _ctx(fm3d, orbNumFeatures=2000)
    try:
        m, ka, kb, da, db = fm3d.DescriptorsMatcher(ctx).compareWithNNDRImages(0.8, pair.img1, pair.img2)
    finally:
        ctx.close()
    out = []
    for img in (pair.img1, pair.img2):
        kd, _ = orc.orb_detect(img, **_orc_kw(s), descriptors=False)
        kc, _, dc = orc.orb_compute(img, kd)
        out.append((kc, dc))
    _same_kpts(ka, out[0][0])
    _same_kpts(kb, out[1][0])
    assert np.array_equal(da, out[0][1]) and np.array_equal(db, out[1][1])
    idx, dist = orc.knn2(out[0][1], out[1][1], orc.BITS, oracle_threads())
    q, t, dd = orc.nndr(idx, dist, 0.8)
    assert np.array_equal(m["queryIdx"], q) and np.array_equal(m["trainIdx"], t) and np.array_equal(m["distance"], dd)
    assert len(m) > 100
