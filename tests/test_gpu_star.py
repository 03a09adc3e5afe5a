"""The STAR detector on the GPU (fm3d_star.hip: DetectorType STAR, descriptorsmatcher.cpp:204-213, and the
StarAdjuster of the ADAPTIVE mode, :185-200) bit for bit against oracle/orc_star.c (OpenCV 2.4.9's
StarDetector restated): the response and size maps, the keypoints in tile order, the settings-driven
fm3d_detect, the adjuster walk, and the inputs OpenCV leaves undefined."""
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


def _blobs(h, w, seed):
    rng = np.random.default_rng(seed)
    img = rng.normal(128, 20, (h, w))
    yy, xx = np.mgrid[0:h, 0:w]
    for _ in range(h * w // 500):
        cy, cx, r = rng.uniform(0, h), rng.uniform(0, w), rng.uniform(2, 14)
        img += rng.choice([-1, 1]) * rng.uniform(40, 110) * np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * r * r))
    return np.clip(img, 0, 255).astype(np.uint8)


def _images(synth):
    fp = synth.make_frame_pair(3000, seed=41)
    bright = np.random.default_rng(11).integers(200, 256, (400, 427)).astype(np.uint8)
    return {"vga": fp.img1, "vga2": fp.img2, "blobs": _blobs(333, 517, 5), "bright": bright}


@pytest.mark.parametrize("tilt", ["diag", "rows"])
@pytest.mark.parametrize("name,max_size", [("vga", 45), ("vga", 16), ("blobs", 23), ("blobs", 90), ("bright", 128),
                                           ("vga2", 8)])
def test_star_responses_bitwise(fm3d, orc, synth, name, max_size, tilt, monkeypatch):
    """both forms of the tilted integrals: the diagonal scans (default) and the row walk"""
    if tilt == "rows":
        monkeypatch.setenv("FM3D_STAR_TILT", "rows")
    img = _images(synth)[name]
    ctx, _ = _ctx(fm3d)
    try:
        b, R, Z = fm3d.Features(ctx).star_responses(img, max_size)
    finally:
        ctx.close()
    bo, Ro, Zo = orc.star_responses(img, max_size)
    assert b == bo
    assert np.array_equal(R.view(np.uint32), Ro.view(np.uint32))
    assert np.array_equal(Z, Zo)
    assert np.count_nonzero(R) > 0


@pytest.mark.parametrize("h,w", [(1080, 1920), (300, 4100), (61, 6000), (2000, 40)])
def test_star_responses_image_shapes(fm3d, orc, synth, h, w):
    """wide images take fewer staged rows per block in the tilted-integral kernel (and more than
    64 KiB of LDS), tall narrow ones many blocks"""
    base = _images(synth)["vga"]
    img = np.ascontiguousarray(np.tile(base, (h // 480 + 1, w // 640 + 1))[:h, :w])
    ctx, _ = _ctx(fm3d)
    try:
        b, R, Z = fm3d.Features(ctx).star_responses(img, 16)
        k = fm3d.Features(ctx).star(img, 16, 30, 10, 8, 3)
    finally:
        ctx.close()
    bo, Ro, Zo = orc.star_responses(img, 16)
    assert b == bo and np.array_equal(R.view(np.uint32), Ro.view(np.uint32)) and np.array_equal(Z, Zo)
    _same_kpts(k, orc.star_detect(img, 16, 30, 10, 8, 3))


@pytest.mark.parametrize("name,params", [("vga", (45, 30, 10, 8, 5)), ("vga", (16, 30, 10, 8, 3)),
                                         ("vga2", (45, 10, 10, 8, 5)), ("blobs", (23, 20, 6, 5, 7)),
                                         ("blobs", (64, 15, 10, 8, 1)), ("bright", (128, 0, 100, 100, 3)),
                                         ("bright", (128, 0, 1000, 1000, 1))])
def test_star_detect_bitwise(fm3d, orc, synth, name, params):
    img = _images(synth)[name]
    ctx, _ = _ctx(fm3d)
    try:
        k = fm3d.Features(ctx).star(img, *params)
    finally:
        ctx.close()
    ko = orc.star_detect(img, *params)
    assert len(ko) > 0
    _same_kpts(k, ko)


def test_star_settings_static_and_adaptive(fm3d, orc, synth):
    img = _images(synth)["vga"]
    ctx, s = _ctx(fm3d, detectorType=fm3d.FEAT_STAR, starMaxSize=32, starResponse=25, starLineThreshold=9,
                  starLineBinarized=7, starSuppression=4)
    try:
        k = fm3d.Features(ctx).detect(img)
    finally:
        ctx.close()
    _same_kpts(k, orc.star_detect(img, 32, 25, 9, 7, 4))
    for lo, hi in ((400, 500), (100, 120), (2000, 2500)):
        ctx, s = _ctx(fm3d, detectorType=fm3d.FEAT_STAR, detectorMode=1, adaptiveMinFeatures=lo,
                      adaptiveMaxFeatures=hi, adaptiveMaxIters=30)
        try:
            k = fm3d.Features(ctx).detect(img)
        finally:
            ctx.close()
        _same_kpts(k, orc.adaptive_detect(img, "STAR", lo, hi, 30))


def test_star_undefined_inputs_fail_loudly(fm3d):
    ctx, _ = _ctx(fm3d)
    try:
        f = fm3d.Features(ctx)
        with pytest.raises(fm3d.Fm3dError):
            f.star(np.zeros((6, 50), np.uint8))            # OpenCV reads pairs[-1]
        with pytest.raises(fm3d.Fm3dError):
            f.star(np.zeros((400, 400), np.uint8), 129)    # OpenCV reads sizes0[-1]
        with pytest.raises(fm3d.Fm3dError):
            f.star(np.zeros((100, 100), np.uint8), 8, 30, 10, 8, 40)  # window beyond the border
        assert len(f.star(np.full((120, 160), 77, np.uint8))) == 0   # flat
        assert len(f.star(np.zeros((30, 40), np.uint8))) == 0        # border 24: no interior
    finally:
        ctx.close()
