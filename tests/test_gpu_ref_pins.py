"""The GPU kernels against the REFERENCE'S OWN OUTPUT FILES (tests/golden/ref_pins.npz; the CPU
side of the same checks, on the oracle, is tests/test_ref_pins.py -- see there for what the files
are).  Through the C ABI on the device:
  * fm3d_plane_to_image2 (extractPixelsContour + get3dPointsFromImage1Pixels +
    projectPointsToImage2 at scale 1, singlecameratriangulator.cpp:341-397, 530-644): bit-exact
    against the oracle, and painted in drawing order it reproduces image1pixels.pgm and
    image2pixels.pgm pixel for pixel (rounding ties tolerated);
  * fm3d_features_frames (normaloptimizer.cpp:454-504) bit-exact against the oracle, then
    fm3d_export_patches (projectReferencePointsToImageWithFrames, :769-849) on the unpainted image-1
    background against results/<run>_img1/patch_<i>.pgm (the reference wrote those through
    projectPointsToImage on the square neighbourhoods, :667-767, the same projection composed in
    another order): >= 99 % of the eligible patch pixels equal, every one within 1, >= 93 % per patch
    (the 64px4l1c.64e run held out of the fit)."""
import os

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu
PINS = os.path.join(ROOT, "tests", "golden", "ref_pins.npz")
W, H, RAY = 1024, 768, 64


class Cam:
    def __init__(self, c):
        self.fx, self.fy, self.cx, self.cy = c[:4]
        self.k = tuple(c[4:9])


@pytest.fixture(scope="module")
def pins():
    if not os.path.exists(PINS):
        pytest.skip("tests/golden/ref_pins.npz not generated yet")
    with np.load(PINS, allow_pickle=False) as z:
        d = {k: z[k] for k in z.files}
    d["cam"] = Cam(d["camera"])
    return d


def _ctx(fm3d, pins, **kw):
    s = fm3d.Settings.default()
    s.set_camera(pins["cam"])
    s.pixelsRay, s.boundWidth, s.boundHeight, s.zThresholdMax = RAY, W, H, 2.4
    for i in range(3):
        s.rodriguesIC[i] = pins["rIC"][i]
        s.translationIC[i] = pins["tIC"][i]
    for k, v in kw.items():
        setattr(s, k, v)
    ctx = fm3d.Context(s)
    sct = fm3d.SingleCameraTriangulator(ctx)
    g = sct.setg12(pins["pos1"][:3], pins["pos2"][:3], pins["pos1"][3:], pins["pos2"][3:])
    assert np.array_equal(g, pins["g12"])  # setg12 of the GPU library == the oracle's
    no = fm3d.NormalOptimizer(ctx, sct)
    no.setImages(pins["bg1"], pins["bg2"])
    return ctx, sct, no


def _paint(lists):
    lab = np.zeros((H, W), np.uint8)
    for r, uv in enumerate(lists):
        px = np.floor(uv + 0.5).astype(np.int64)
        ok = (px[:, 0] >= 0) & (px[:, 1] >= 0) & (px[:, 0] < W) & (px[:, 1] < H)
        lab[px[ok, 1], px[ok, 0]] = r + 1
    return lab


def test_gpu_plane_projection_paints_the_reference_images(fm3d, orc, pins):
    ctx, sct, _ = _ctx(fm3d, pins)
    try:
        got = [sct.plane_to_image2(X, n) for X, n in zip(pins["X"], pins["n"])]
    finally:
        ctx.close()
    R2, t2 = orc.camera2_from_g12(pins["g12"])
    for (xy, uv, st), X, n in zip(got, pins["X"], pins["n"]):
        pix = orc.neighborhood(pins["cam"], X, RAY, W, H)
        ruv, rst = orc.plane_to_image2(pins["cam"], R2, t2, X, n, pix, 2.4, size=(W, H))
        assert np.array_equal(xy, pix) and np.array_equal(uv, ruv) and np.array_equal(st, rst)
        assert (st == 0).all() and len(xy) == 12_853
    assert np.array_equal(_paint([g[0] for g in got]), pins["lab1"])
    from test_ref_pins import check_image2
    check_image2(pins["lab2"], _paint([g[1] for g in got]), [g[1] for g in got])


@pytest.mark.parametrize("run,eps,cmpp", [("64px4l.5c.32e", 0.32, 0.5), ("64px4l1c.64e", 0.64, 1.0)])
def test_gpu_frames_and_patch_export_against_reference_patches(fm3d, orc, pins, run, eps, cmpp):
    ctx, sct, no = _ctx(fm3d, pins, neighEpsilon=eps, cmPerPixel=cmpp)
    try:
        frames = no.computeFeaturesFrames(pins["X"], pins["n"])
        patches, uv = sct.projectReferencePointsToImageWithFrames(None, frames, image_points=True)
    finally:
        ctx.close()
    assert np.array_equal(frames, orc.features_frames(pins["X"], pins["n"], orc.gravity(pins["rIC"])))
    ref = pins["patch_" + f"{run}_img1".replace(".", "_")]
    lab = pins["lab1"]
    tot_eq = tot = 0
    for i in range(len(frames)):
        u = uv[i].astype(np.float32)
        x0, y0 = np.floor(u[:, 0]).astype(np.int64), np.floor(u[:, 1]).astype(np.int64)
        ok = (x0 >= 0) & (y0 >= 0) & (x0 + 1 < W) & (y0 + 1 < H)
        e = np.zeros(len(u), bool)
        k = np.nonzero(ok)[0]
        e[k] = ((lab[y0[k], x0[k]] == 0) & (lab[y0[k] + 1, x0[k]] == 0) & (lab[y0[k], x0[k] + 1] == 0)
                & (lab[y0[k] + 1, x0[k] + 1] == 0))
        # point order i*size + j -> patch[j][i] (the reference's transposed write)
        size = patches.shape[1]
        got = patches[i].T.reshape(-1)
        want = ref[i].T.reshape(-1)
        d = np.abs(got[e].astype(int) - want[e].astype(int))
        assert e.sum() > 40 and d.max() <= 1 and (d == 0).mean() >= 0.93, (i, int(d.max()), float((d == 0).mean()))
        tot_eq += int((d == 0).sum())
        tot += int(e.sum())
        assert size == 128
    print(f"{run}: {tot_eq} of {tot} eligible patch pixels equal")
    assert tot_eq >= 0.99 * tot
