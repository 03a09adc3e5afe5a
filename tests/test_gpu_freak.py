"""The FREAK extractor on the GPU (fm3d_freak.hip: ExtractorType FREAK, descriptorsmatcher.cpp:350-353)
bit for bit against oracle/orc_freak.c (OpenCV 2.4.9's FREAK descriptor restated): caller keypoints of
every scale and border position (angles set by FREAK's orientation), a caller pair table, the
settings-driven fm3d_compute, extractDescriptorsFromPatches, and the reference's detector + FREAK
extractor pairs matched by Hamming distance through compareWithNNDR."""
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


def _kpts(fm3d, rng, n, w, h):
    k = np.zeros(n, dtype=fm3d.KEYPOINT)
    k["x"] = rng.uniform(-5, w + 5, n)
    k["y"] = rng.uniform(-5, h + 5, n)
    k["size"] = rng.choice([0.0, 1e-9, 3.0, 7.0, 7.2, 9.0, 12.5, 20.0, 31.0, 44.6, 64.0, 90.0, np.nan], n)
    k["angle"] = np.where(rng.random(n) < 0.3, -1.0, rng.uniform(0, 360, n))
    k["response"] = rng.random(n)
    return k


@pytest.mark.parametrize("seed", [1, 2])
def test_freak_compute_bitwise(fm3d, orc, synth, seed):
    img = synth.make_frame_pair(2000, seed=80 + seed).img1
    k = _kpts(fm3d, np.random.default_rng(seed), 3000, 640, 480)
    ctx, _ = _ctx(fm3d, extractorType=fm3d.FEAT_FREAK)
    try:
        kc, kept, d = fm3d.Features(ctx).compute(img, k)
    finally:
        ctx.close()
    ko, kepto, do = orc.freak_compute(img, k)
    assert len(ko) > 3000 // 4
    assert np.array_equal(kept, kepto)
    _same_kpts(kc, ko)
    assert d.dtype == np.uint8 and d.shape == (len(ko), 64) and np.array_equal(d, do)
    assert 0.3 < np.unpackbits(d).mean() < 0.7


def test_freak_custom_pairs_small_images(fm3d, orc, synth):
    """fm3d_freak_set_pairs with another valid table, then the default again; tiny and odd images (every
    keypoint filtered, or a few); no keypoints at all"""
    img = synth.make_frame_pair(500, seed=90).img1
    rng = np.random.default_rng(4)
    table = rng.permutation(903)[:512].astype(np.int32)
    k = _kpts(fm3d, rng, 800, 640, 480)
    ctx, _ = _ctx(fm3d, extractorType=fm3d.FEAT_FREAK)
    try:
        F = fm3d.Features(ctx)
        F.set_freak_pairs(table)
        kc, kept, d = F.compute(img, k)
        ko, kepto, do = orc.freak_compute(img, k, pairs=table)
        assert np.array_equal(kept, kepto) and np.array_equal(d, do) and len(ko) > 100
        F.set_freak_pairs(None)
        kc, kept, d = F.compute(img, k)
        assert np.array_equal(d, orc.freak_compute(img, k)[2])
        with pytest.raises(fm3d.Fm3dError):
            F.set_freak_pairs(np.arange(511, dtype=np.int32))
        for h, w in ((37, 53), (60, 61), (200, 90)):
            sub = np.ascontiguousarray(img[:h, :w])
            kk = _kpts(fm3d, rng, 300, w, h)
            kc, kept, d = F.compute(sub, kk)
            ko, kepto, do = orc.freak_compute(sub, kk)
            assert np.array_equal(kept, kepto) and np.array_equal(d, do)
            _same_kpts(kc, ko)
        kc, kept, d = F.compute(img, np.zeros(0, dtype=fm3d.KEYPOINT))
        assert len(kc) == 0
    finally:
        ctx.close()


@pytest.mark.parametrize("det", ["SURF", "FAST", "ORB"])
def test_detector_with_freak_extractor(fm3d, orc, synth, det):
    """the settings' detector, then FREAK on its keypoints (the reference's two calls), matched with
    the Hamming distance as the reference's binary extractor types select (descriptorsmatcher.cpp:64)"""
    fp = synth.make_frame_pair(3000, seed=71)
    T = {"SURF": fm3d.FEAT_SURF, "FAST": fm3d.FEAT_FAST, "ORB": fm3d.FEAT_ORB}
    ctx, s = _ctx(fm3d, detectorType=T[det], extractorType=fm3d.FEAT_FREAK)
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

    oa, ob = orc.freak_compute(fp.img1, detect(fp.img1)), orc.freak_compute(fp.img2, detect(fp.img2))
    _same_kpts(ka, oa[0])
    _same_kpts(kb, ob[0])
    assert np.array_equal(da, oa[2]) and np.array_equal(db, ob[2])
    q, t, dist = orc.match_nndr(oa[2], ob[2], orc.BITS, 0.8)
    assert len(m) == len(q) > 5
    assert np.array_equal(m["queryIdx"], q) and np.array_equal(m["trainIdx"], t) and np.array_equal(m["distance"], dist)


def test_freak_patches(fm3d, orc, synth):
    """extractDescriptorsFromPatches with the FREAK extractor: the centred keypoint of size = patch edge
    needs a pattern larger than the patch, so every row stays zero, as the reference's Mat::zeros rows
    (the BRISK case, descriptorsmatcher.cpp:142-172); a small keypoint size on a large patch survives"""
    img = synth.make_frame_pair(500, seed=92).img1
    P = np.stack([np.ascontiguousarray(img[y:y + 128, x:x + 128]) for y, x in ((10, 10), (200, 300), (300, 100))])
    ctx, s = _ctx(fm3d, extractorType=fm3d.FEAT_FREAK)
    try:
        d = fm3d.Features(ctx).extractDescriptorsFromPatches(P)
    finally:
        ctx.close()
    assert d.shape == (3, 64) and d.dtype == np.uint8 and not d.any()
    k = np.zeros(1, dtype=fm3d.KEYPOINT)
    k["x"] = k["y"] = 64.0
    k["size"] = 7.0
    ko, _, do = orc.freak_compute(P[1], k)
    assert len(ko) == 1 and do.any()
