"""The settings' detector / extractor pairs beyond one detector type (descriptorsmatcher.cpp:176-359):
FAST (cv::FastFeatureDetector(Threshold, NonMaxSuppression), :215-222), the ADAPTIVE mode with the
FAST and SURF adjusters (cv::DynamicAdaptedFeatureDetector, :185-201), and mixed detector /
extractor pairs through fm3d_detect / fm3d_compute -- bit for bit against the oracles (FAST and SURF
restated in oracle/orc_orb.c and orc_surf.c; the adjusters' threshold walk in oracle.adaptive_detect)."""
import numpy as np
import pytest

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


@pytest.mark.parametrize("thr,nonmax", [(10, True), (25, True), (10, False), (40, False)])
def test_fast_detector_bitwise(fm3d, orc, synth, thr, nonmax):
    img = synth.make_frame_pair(3000, seed=31).img1
    ctx, s = _ctx(fm3d, detectorType=fm3d.FEAT_FAST, fastThreshold=thr, fastNonmax=int(nonmax))
    try:
        k = fm3d.Features(ctx).detect(img)
        k2 = fm3d.Features(ctx).fast(img, thr, nonmax)
    finally:
        ctx.close()
    ko = orc.fast_detect(img, thr, nonmax)
    assert len(ko) > 100
    _same_kpts(k, ko)
    _same_kpts(k2, ko)


@pytest.mark.parametrize("kind,lo,hi", [("FAST", 400, 500), ("FAST", 3000, 3500), ("SURF", 400, 500),
                                        ("SURF", 100, 120)])
def test_adaptive_detector_bitwise(fm3d, orc, synth, kind, lo, hi):
    """DynamicAdaptedFeatureDetector: the threshold walk ends on the same call, the keypoints equal"""
    img = synth.make_frame_pair(3000, seed=32).img1
    typ = fm3d.FEAT_FAST if kind == "FAST" else fm3d.FEAT_SURF
    ctx, s = _ctx(fm3d, detectorType=typ, detectorMode=1, adaptiveMinFeatures=lo, adaptiveMaxFeatures=hi,
                  adaptiveMaxIters=30)
    try:
        k = fm3d.Features(ctx).detect(img)
    finally:
        ctx.close()
    ko = orc.adaptive_detect(img, kind, lo, hi, 30)
    _same_kpts(k, ko)


@pytest.mark.parametrize("det,ex", [("FAST", "SIFT"), ("SURF", "SIFT"), ("ORB", "SIFT"), ("FAST", "ORB"),
                                    ("STAR", "SIFT"), ("STAR", "ORB"), ("FAST", "SURF"), ("STAR", "SURF")])
def test_mixed_detector_extractor(fm3d, orc, synth, det, ex):
    """feature_detector_ and descriptor_extractor_ of different types (the reference builds them
    independently): detect with one, compute with the other, as compareWithNNDR's two calls"""
    fp = synth.make_frame_pair(3000, seed=33)
    T = {"FAST": fm3d.FEAT_FAST, "SURF": fm3d.FEAT_SURF, "SIFT": fm3d.FEAT_SIFT, "ORB": fm3d.FEAT_ORB,
         "STAR": fm3d.FEAT_STAR}
    ctx, s = _ctx(fm3d, detectorType=T[det], extractorType=T[ex])
    try:
        m, ka, kb, da, db = fm3d.DescriptorsMatcher(ctx).compareWithNNDRImages(0.8, fp.img1, fp.img2)
    finally:
        ctx.close()

    def detect(img):
        if det == "FAST":
            return orc.fast_detect(img, s.fastThreshold, bool(s.fastNonmax))
        if det == "SURF":
            return orc.surf_detect(img, s.surfHessianThreshold, s.surfOctaves, s.surfOctaveLayers, upright=bool(s.surfUpright))
        if det == "STAR":
            return orc.star_detect(img, s.starMaxSize, s.starResponse, s.starLineThreshold, s.starLineBinarized,
                                   s.starSuppression)
        if det == "ORB":
            return orc.orb_detect(img, s.orbNumFeatures, s.orbScaleFactor, s.orbNumLevels, s.orbEdgeThreshold,
                                  s.orbPatchSize, s.orbFastThreshold, descriptors=False)[0]
        return orc.sift_detect(img)

    def compute(img, k):
        if ex == "SIFT":
            return orc.sift_compute(img, k)
        if ex == "SURF":  # FAST's size 7 and STAR's 4..6 take the enlarged-window path
            return orc.surf_describe(img, k, extended=bool(s.surfExtended), upright=bool(s.surfUpright))
        return orc.orb_compute(img, k)

    oa, ob = compute(fp.img1, detect(fp.img1)), compute(fp.img2, detect(fp.img2))
    _same_kpts(ka, oa[0])
    _same_kpts(kb, ob[0])
    assert np.array_equal(da, oa[2]) and np.array_equal(db, ob[2])
    if ex == "ORB":
        q, t, dist = orc.match_nndr(oa[2], ob[2], orc.BITS, 0.8)
    elif ex == "SURF":
        q, t, dist = orc.match_nndr(oa[2], ob[2], orc.F32, 0.8)
    else:
        q, t, dist = orc.match_nndr(oa[2].astype(np.uint8), ob[2].astype(np.uint8), orc.U8, 0.8)
    assert len(m) == len(q) > 5
    assert np.array_equal(m["queryIdx"], q) and np.array_equal(m["trainIdx"], t) and np.array_equal(m["distance"], dist)


def test_unsupported_types_fail_loudly(fm3d, synth):
    """a detector type with no GPU implementation; and SIFT keypoints into the ORB extractor, whose
    compute indexes its pyramid by KeyPoint::octave (SIFT's packed octave code: OpenCV's ORB would
    build millions of levels and assert)"""
    img = synth.make_frame_pair(500, seed=34).img1
    ctx, s = _ctx(fm3d, detectorType=fm3d.FEAT_OTHER)
    try:
        with pytest.raises(fm3d.Fm3dError):
            fm3d.Features(ctx).detect(img)
    finally:
        ctx.close()
    ctx, s = _ctx(fm3d, detectorType=fm3d.FEAT_SIFT, extractorType=fm3d.FEAT_ORB)
    try:
        f = fm3d.Features(ctx)
        with pytest.raises(fm3d.Fm3dError):
            f.compute(img, f.detect(img))
    finally:
        ctx.close()
