"""The BRISK extractor on the GPU (fm3d_brisk.hip: ExtractorType BRISK, descriptorsmatcher.cpp:343-348)
bit for bit against oracle/orc_brisk.c (OpenCV 2.4.9's BRISK descriptor restated): caller keypoints of
every scale, rotation and border position, the settings-driven fm3d_compute, and the reference's
detector + BRISK extractor pairs matched by Hamming distance through compareWithNNDR."""
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


@pytest.mark.parametrize("seed", [1, 2])
def test_brisk_compute_bitwise(fm3d, orc, synth, seed):
    img = synth.make_frame_pair(2000, seed=60 + seed).img1
    rng = np.random.default_rng(seed)
    n = 3000
    k = np.zeros(n, dtype=fm3d.KEYPOINT)
    k["x"] = rng.uniform(-5, 645, n)
    k["y"] = rng.uniform(-5, 485, n)
    k["size"] = rng.choice([0.0, 1e-9, 3.0, 7.0, 7.2, 9.0, 12.5, 20.0, 31.0, 44.6, 64.0, 90.0, 140.0], n)
    k["angle"] = np.where(rng.random(n) < 0.3, -1.0, rng.uniform(0, 360, n))
    k["response"] = rng.random(n)
    ctx, _ = _ctx(fm3d, extractorType=fm3d.FEAT_BRISK)
    try:
        kc, kept, d = fm3d.Features(ctx).compute(img, k)
    finally:
        ctx.close()
    ko, kepto, do = orc.brisk_compute(img, k)
    assert len(ko) > n // 3
    assert np.array_equal(kept, kepto)
    _same_kpts(kc, ko)
    assert d.dtype == np.uint8 and d.shape == (len(ko), 64) and np.array_equal(d, do)


@pytest.mark.parametrize("det", ["SURF", "FAST", "ORB"])
def test_detector_with_brisk_extractor(fm3d, orc, synth, det):
    """the settings' detector, then BRISK on its keypoints (the reference's two calls), matched with
    the Hamming distance as the reference's binary extractor types select (descriptorsmatcher.cpp:64)"""
    fp = synth.make_frame_pair(3000, seed=71)
    T = {"SURF": fm3d.FEAT_SURF, "FAST": fm3d.FEAT_FAST, "ORB": fm3d.FEAT_ORB}
    ctx, s = _ctx(fm3d, detectorType=T[det], extractorType=fm3d.FEAT_BRISK)
    try:
        m, ka, kb, da, db = fm3d.DescriptorsMatcher(ctx).compareWithNNDRImages(0.8, fp.img1, fp.img2)
    finally:
        ctx.close()

    def detect(img):
        if det == "SURF":
            return orc.surf_detect(img, s.surfHessianThreshold, s.surfOctaves, s.surfOctaveLayers, upright=bool(s.surfUpright))
        if det == "FAST":
            return orc.fast_detect(img, s.fastThreshold, bool(s.fastNonmax))
        return orc.orb_detect(img, s.orbNumFeatures, s.orbScaleFactor, s.orbNumLevels, s.orbEdgeThreshold,
                              s.orbPatchSize, s.orbFastThreshold, descriptors=False)[0]

    oa, ob = orc.brisk_compute(fp.img1, detect(fp.img1)), orc.brisk_compute(fp.img2, detect(fp.img2))
    _same_kpts(ka, oa[0])
    _same_kpts(kb, ob[0])
    assert np.array_equal(da, oa[2]) and np.array_equal(db, ob[2])
    q, t, dist = orc.match_nndr(oa[2], ob[2], orc.BITS, 0.8)
    assert len(m) == len(q) > 5
    assert np.array_equal(m["queryIdx"], q) and np.array_equal(m["trainIdx"], t) and np.array_equal(m["distance"], dist)
