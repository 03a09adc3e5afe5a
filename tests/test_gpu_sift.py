"""GPU SIFT (csrc/fm3d_sift.hip + the host's removeDuplicated / retainBest) against the SIFT oracle
(oracle/orc_sift.c), bit for bit: the Gaussian and DoG pyramids, keypoints (position, size, angle,
response, octave code, class_id) in the reference's order and their 128-float descriptors; compute on
given keypoints (removed sizes, the undoubled pyramid, the assertion cases); compareWithNNDR from the
images with the settings' SIFT (FeatureOptions DetectorType / ExtractorType SIFT,
descriptorsmatcher.cpp:243-257, 302-315)."""
import numpy as np
import pytest

from conftest import oracle_threads

pytestmark = pytest.mark.gpu


def _ctx(fm3d, **kw):
    s = fm3d.Settings.default()
    s.detectorType = s.extractorType = fm3d.FEAT_SIFT
    for k, v in kw.items():
        setattr(s, k, v)
    return fm3d.Context(s), s


def _orc_kw(s):
    return dict(nfeatures=s.siftNumFeatures, nOctaveLayers=s.siftOctaveLayers, contrastThreshold=s.siftContrastThreshold,
                edgeThreshold=s.siftEdgeThreshold, sigma=s.siftSigma)


def _same_kpts(a, b):
    assert len(a) == len(b), (len(a), len(b))
    for f in ("x", "y", "size", "angle", "response", "octave", "class_id"):
        assert np.array_equal(a[f], b[f]), f


def test_sift_pyramids_bitwise(fm3d, orc, synth):
    img = synth.make_frame_pair(2000, seed=4).img1
    ctx, s = _ctx(fm3d)
    try:
        sift = fm3d.SIFT(ctx)
        for first, dog in ((-1, False), (-1, True), (0, False)):
            g = sift.pyramid(img, first, dog=dog)
            o = orc.sift_pyramid(img, first, dog=dog)
            assert len(g) == len(o)
            for i, (a, b) in enumerate(zip(g, o)):
                assert a.shape == b.shape and np.array_equal(a, b), (first, dog, i)
    finally:
        ctx.close()


@pytest.mark.parametrize("nfeatures", [0, 500])
def test_sift_detect_describe_vga_bitwise(fm3d, orc, synth, nfeatures):
    """cv::SIFT(NumFeatures, 3, 0.04, 10, 1.6) on the synthetic VGA frames"""
    img = synth.make_frame_pair(4000, seed=3).img1
    ctx, s = _ctx(fm3d, siftNumFeatures=nfeatures)
    try:
        k, d = fm3d.SIFT(ctx).detect(img, with_descriptors=True)
        k2 = fm3d.SIFT(ctx).detect(img)
    finally:
        ctx.close()
    ko = orc.sift_detect(img, **_orc_kw(s))
    assert len(ko) > (400 if nfeatures else 3000)
    _same_kpts(k, ko)
    _same_kpts(k2, ko)
    _, _, do = orc.sift_compute(img, ko)
    assert d.shape == do.shape and np.array_equal(d, do)


@pytest.mark.parametrize("shape,kw", [
    ((257, 333), dict(siftOctaveLayers=2)),
    ((240, 320), dict(siftOctaveLayers=4, siftContrastThreshold=0.02)),
    ((200, 301), dict(siftEdgeThreshold=5.0, siftContrastThreshold=0.08)),
    ((180, 240), dict(siftSigma=1.2)),
    ((160, 200), dict(siftSigma=2.0, siftOctaveLayers=3)),
    ((30, 40), dict()),
])
def test_sift_settings_and_sizes_bitwise(fm3d, orc, synth, shape, kw):
    img = np.ascontiguousarray(synth.make_frame_pair(3000, seed=6).img1[:shape[0], :shape[1]])
    ctx, s = _ctx(fm3d, **kw)
    try:
        k, d = fm3d.SIFT(ctx).detect(img, with_descriptors=True)
    finally:
        ctx.close()
    ko = orc.sift_detect(img, **_orc_kw(s))
    _same_kpts(k, ko)
    if len(ko):
        _, _, do = orc.sift_compute(img, ko, nOctaveLayers=s.siftOctaveLayers, sigma=s.siftSigma)
        assert np.array_equal(d, do)


def test_sift_compute_given_keypoints(fm3d, orc, synth):
    """compute on edited keypoints: sizes 0 removed in order, octave >= 0 only (the undoubled
    pyramid of firstOctave 0), keypoints of another detector (octave = level, no layer byte), and
    OpenCV's assertion cases as FM3D_ERR_INVALID"""
    img = synth.make_frame_pair(3000, seed=8).img1
    ctx, s = _ctx(fm3d)
    try:
        sift = fm3d.SIFT(ctx)
        kall = sift.detect(img)
        k = kall[:400].copy()
        k["size"][::9] = 0
        ko, kept, d = sift.compute(img, k)
        oo, okept, od = orc.sift_compute(img, k)
        _same_kpts(ko, oo)
        assert np.array_equal(kept, okept) and np.array_equal(d, od)
        k0 = kall[(kall["octave"] & 255) < 128][:200]
        assert len(k0) > 50
        _, _, d0 = sift.compute(img, k0)
        assert np.array_equal(d0, orc.sift_compute(img, k0)[2])
        ks = np.zeros(64, dtype=fm3d.KEYPOINT)  # SURF-like: octave = 0..3, layer byte 0
        rng = np.random.default_rng(2)
        ks["x"] = rng.uniform(20, 620, 64)
        ks["y"] = rng.uniform(20, 460, 64)
        ks["size"] = rng.uniform(8, 40, 64)
        ks["angle"] = rng.uniform(0, 360, 64)
        ks["octave"] = rng.integers(0, 4, 64)
        _, _, ds = sift.compute(img, ks)
        assert np.array_equal(ds, orc.sift_compute(img, ks)[2])
        bad = k[:3].copy()
        bad["size"] = 5
        bad["octave"] = 0xFE
        with pytest.raises(fm3d.Fm3dError):
            sift.compute(img, bad)
    finally:
        ctx.close()


def test_sift_blob(fm3d, orc):
    yy, xx = np.mgrid[0:240, 0:320]
    b = np.rint(60 + 150 * np.exp(-((xx - 160.3) ** 2 + (yy - 120.6) ** 2) / (2 * 36.0))).astype(np.uint8)
    ctx, s = _ctx(fm3d)
    try:
        k, d = fm3d.SIFT(ctx).detect(b, with_descriptors=True)
    finally:
        ctx.close()
    ko = orc.sift_detect(b)
    _same_kpts(k, ko)
    assert np.array_equal(d, orc.sift_compute(b, ko)[2])
    assert abs(k["x"][0] - 160.55) < 0.06


def test_sift_compare_with_nndr_images(fm3d, orc, synth):
    """compareWithNNDR from the images with the settings' SIFT: detect + compute on both frames,
    then the exact integer matcher (SIFT's descriptors are integers 0..255) and NNDR"""
    fp = synth.make_frame_pair(4000, seed=12)
    ctx, s = _ctx(fm3d)
    try:
        m, ka, kb, da, db = fm3d.DescriptorsMatcher(ctx).compareWithNNDRImages(0.8, fp.img1, fp.img2)
    finally:
        ctx.close()
    oa, ob = orc.sift_detect(fp.img1), orc.sift_detect(fp.img2)
    _same_kpts(ka, oa)
    _same_kpts(kb, ob)
    _, _, oda = orc.sift_compute(fp.img1, oa)
    _, _, odb = orc.sift_compute(fp.img2, ob)
    assert np.array_equal(da, oda) and np.array_equal(db, odb)
    qi, ti, dist = orc.match_nndr(oda.astype(np.uint8), odb.astype(np.uint8), orc.U8, 0.8)
    assert len(m) == len(qi) > 100
    assert np.array_equal(m["queryIdx"], qi) and np.array_equal(m["trainIdx"], ti)
    assert np.array_equal(m["distance"], dist)


def test_sift_patches_bitwise(fm3d, orc):
    """extractDescriptorsFromPatches with the SIFT extractor (descriptorsmatcher.cpp:133-174): per patch
    SIFT::operator() with the centred keypoint (size = the edge, angle -1, octave 0), equal to the
    oracle's compute on each patch; odd patch sizes too"""
    rng = np.random.default_rng(13)
    ctx, s = _ctx(fm3d)
    try:
        for size, P in ((128, 40), (65, 12)):
            yy, xx = np.mgrid[0:size, 0:size]
            patches = np.stack([np.clip(128 + 60 * np.sin(xx * rng.uniform(0.05, 0.3) + yy * rng.uniform(0.05, 0.3))
                                        + rng.normal(0, 20, (size, size)), 0, 255).astype(np.uint8) for _ in range(P)])
            d = fm3d.SIFT(ctx).extractDescriptorsFromPatches(patches)
            kp = np.zeros(1, dtype=fm3d.KEYPOINT)
            kp["x"] = kp["y"] = size // 2
            kp["size"] = size
            kp["angle"] = -1
            kp["response"] = 1
            ref = np.stack([orc.sift_compute(p, kp)[2][0] for p in patches])
            assert d.shape == (P, 128) and np.array_equal(d, ref), size
    finally:
        ctx.close()


@pytest.mark.parametrize("nfeat", [3_500])
def test_c2_sift_from_images_full_pipeline(fm3d, orc, synth, nfeat):
    """BASELINE configs[1] (C2: SIFT-128 per 640x480 frame, match + DLT) starting from the images, as
    the reference does with DetectorType / ExtractorType SIFT: SIFT detection and description on the
    GPU (ContrastThreshold 0.02; the synthetic frame pair holds 7.8k / 3.9k such keypoints, so
    retainBest(NumFeatures 3,500) trims both -- C2's 10k rows per frame are matched from the
    generated descriptors in test_c2_sift10k_match_and_dlt), then the
    device-resident pipeline (match + NNDR on the integer-valued float rows, DLT, LM).  Keypoints,
    descriptors, matches, inliers and points are checked in full against the oracle chain; the LM on
    a seeded 96-point sample bit-exact against the oracle's DETMATH mode."""
    fp = synth.make_frame_pair(10_000, seed=101)
    s = fm3d.Settings.default()
    s.set_camera(fp.cam)
    s.detectorType = s.extractorType = fm3d.FEAT_SIFT
    s.siftNumFeatures, s.siftContrastThreshold = nfeat, 0.02
    ctx = fm3d.Context(s)
    try:
        sift = fm3d.SIFT(ctx)
        ka, _, da = sift.compute(fp.img1, sift.detect(fp.img1))
        kb, _, db = sift.compute(fp.img2, sift.detect(fp.img2))
        sct = fm3d.SingleCameraTriangulator(ctx)
        sct.set_g12(fp.g12)
        R2, t2 = sct.camera2()
        xy = lambda k: np.stack([k["x"], k["y"]], axis=1).astype(np.float32)
        pipe = fm3d.Pipeline(ctx)
        pipe.upload(da, db, xy(ka), xy(kb), fp.img1, fp.img2)
        n, stats = pipe.run()
        rec = pipe.records(n)
    finally:
        ctx.close()
    kw = dict(nfeatures=nfeat, contrastThreshold=0.02)
    oa, ob = orc.sift_detect(fp.img1, **kw), orc.sift_detect(fp.img2, **kw)
    _same_kpts(ka, oa)
    _same_kpts(kb, ob)
    assert nfeat <= len(oa) < nfeat * 1.01 and nfeat <= len(ob) < nfeat * 1.01
    oda, odb = orc.sift_compute(fp.img1, oa)[2], orc.sift_compute(fp.img2, ob)[2]
    assert np.array_equal(da, oda) and np.array_equal(db, odb)
    q, t, d = orc.match_nndr(oda.astype(np.uint8), odb.astype(np.uint8), orc.U8, s.nndrEpsilon)
    assert stats["matches"] == len(q) > 500
    pts, mask = orc.triangulate(fp.cam, fp.g12, 1.5, 2.4, xy(oa), xy(ob), q, t)
    assert stats["inliers"] == len(pts)
    pos = np.searchsorted(q[mask], rec["queryIdx"])
    assert np.array_equal(q[mask][pos], rec["queryIdx"]) and np.array_equal(rec["trainIdx"], t[mask][pos])
    assert np.array_equal(rec["distance"], d[mask][pos]) and np.array_equal(rec["point"], pts[pos])
    sel = np.sort(np.random.default_rng(1101).choice(len(pts), min(96, len(pts)), replace=False))
    ref = orc.optimize_normals(fp.cam, R2, t2, fp.img1, fp.img2, s.pyramids, pts[sel], s.pixelsRay, mode=orc.DETMATH,
                               nthreads=oracle_threads())
    ok = ref["status"] == 0
    assert np.array_equal(np.isin(sel, pos), ok)
    assert np.array_equal(rec[np.isin(pos, sel)]["normal"], ref["normals"][ok])
