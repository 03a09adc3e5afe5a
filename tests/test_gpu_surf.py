"""GPU SURF (csrc/fm3d_surf.hip) against the SURF oracle (oracle/orc_surf.c), bit for bit:
keypoints (position, size, angle, response, octave, Laplacian sign) in KeypointGreater order and
their descriptors; compute on given keypoints; extractDescriptorsFromPatches; compareWithNNDR
starting from the images (descriptorsmatcher.cpp:107-174); the same with Upright 0 (the settings'
SURF Upright key, descriptorsmatcher.cpp:176-359: dominant orientation + rotated window)."""
import numpy as np
import pytest

from conftest import oracle_threads

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


@pytest.mark.parametrize("which", ["img1", "img2"])
def test_surf_detect_describe_vga_bitwise(fm3d, orc, synth, which):
    """The reference's settings (threshold 400, 4 octaves, 2 layers, extended, upright) on the
    synthetic VGA frames."""
    pair = synth.make_frame_pair(2000, seed=3)
    img = getattr(pair, which)
    ctx, s = _ctx(fm3d)
    try:
        k, d = fm3d.SURF(ctx).detect(img, with_descriptors=True)
    finally:
        ctx.close()
    ko = orc.surf_detect(img, s.surfHessianThreshold, s.surfOctaves, s.surfOctaveLayers)
    kd, kept, do = orc.surf_describe(img, ko, extended=True)
    assert len(ko) > 500
    _same_kpts(k, ko)
    assert np.array_equal(kept, np.arange(len(ko)))
    assert np.array_equal(d, do)


@pytest.mark.parametrize("shape,thr,octaves,layers,extended", [
    ((77, 100), 100.0, 4, 2, 1), ((29, 33), 10.0, 2, 3, 0), ((480, 64), 200.0, 5, 1, 1), ((8, 8), 1.0, 1, 1, 1)])
def test_surf_shapes_and_settings(fm3d, orc, shape, thr, octaves, layers, extended):
    """Odd and tiny images, layers that do not fit (skipped), other octave / layer counts, the 64-D
    descriptor."""
    rng = np.random.default_rng(sum(shape))
    h, w = shape
    yy, xx = np.mgrid[0:h, 0:w]
    img = np.clip(128 + 90 * np.sin(xx * 0.31 + yy * 0.17) * np.cos(yy * 0.23) + rng.normal(0, 8, shape), 0,
                  255).astype(np.uint8)
    ctx, s = _ctx(fm3d, surfHessianThreshold=thr, surfOctaves=octaves, surfOctaveLayers=layers,
                  surfExtended=extended)
    try:
        k, d = fm3d.SURF(ctx).detect(img, with_descriptors=True)
    finally:
        ctx.close()
    ko = orc.surf_detect(img, thr, octaves, layers)
    _, _, do = orc.surf_describe(img, ko, extended=bool(extended))
    _same_kpts(k, ko)
    assert d.shape == (len(ko), 128 if extended else 64) and np.array_equal(d, do)


def test_surf_compute_given_keypoints(fm3d, orc, synth):
    """compute on caller keypoints: a keypoint whose wavelet exceeds the image is removed (the
    others keep their order, angle 270), windows cut by every border."""
    img = synth.make_frame_pair(300, seed=8).img1
    kin = np.zeros(7, dtype=fm3d.KEYPOINT)
    kin["x"] = [0.0, 639.4, 320.5, 5.0, 100.0, 600.0, 2.5]
    kin["y"] = [0.0, 479.9, 240.2, 470.0, 3.0, 10.0, 2.5]
    kin["size"] = [9, 20, 4000, 31, 77, 150, 15]
    kin["angle"] = -1
    ctx, _ = _ctx(fm3d)
    try:
        k, kept, d = fm3d.SURF(ctx).compute(img, kin)
    finally:
        ctx.close()
    ko, kepto, do = orc.surf_describe(img, kin, extended=True)
    assert list(kept) == [0, 1, 3, 4, 5, 6] and np.array_equal(kept, kepto)
    _same_kpts(k, ko)
    assert np.array_equal(d, do)


def test_surf_compute_size_filter_and_outside_centres(fm3d, orc, synth):
    """DescriptorExtractor::compute first drops keypoints of size < FLT_EPSILON
    (KeyPointsFilter::runByKeypointSize; runByImageBorder with border 0 removes nothing), so size 0
    and negative sizes disappear; centres outside the image keep their border-replicated window;
    a kept keypoint of size < 0.36 (an empty window: OpenCV's resize asserts) is FM3D_ERR_INVALID on
    the GPU and an error in the oracle, not a silent wrong descriptor."""
    img = synth.make_frame_pair(300, seed=8).img1
    kin = np.zeros(6, dtype=fm3d.KEYPOINT)
    kin["x"] = [100.0, -20.0, 700.0, 320.0, 50.0, 320.0]
    kin["y"] = [100.0, 240.0, 500.0, -5.5, 60.0, 240.0]
    kin["size"] = [0.0, 24.0, 31.0, 18.0, -3.0, 1e-9]
    kin["angle"] = -1
    ctx, _ = _ctx(fm3d)
    try:
        k, kept, d = fm3d.SURF(ctx).compute(img, kin)
        small = kin[[1]].copy()
        small["size"] = 0.3
        with pytest.raises(fm3d.Fm3dError) as e:
            fm3d.SURF(ctx).compute(img, small)
        assert e.value.code == fm3d.ERR_INVALID
    finally:
        ctx.close()
    ko, kepto, do = orc.surf_describe(img, kin, extended=True)
    assert list(kept) == [1, 2, 3] and np.array_equal(kept, kepto)
    _same_kpts(k, ko)
    assert np.array_equal(d, do)
    with pytest.raises(ValueError):
        orc.surf_describe(img, small, extended=True)


@pytest.mark.parametrize("upright", [1, 0])
def test_surf_compute_small_keypoints_enlarge_the_window(fm3d, orc, synth, upright):
    """keypoints of size < 7.5 (FAST's 7, STAR's 4..6, ...): the window is narrower than the 21 x 21
    patch and OpenCV's INTER_AREA enlarges it by its linear emulation (oracle orc_resize_area_up);
    windows of 1 to 20 pixels, inside the image and cut by its borders, upright and oriented."""
    img = synth.make_frame_pair(300, seed=18).img1
    sizes = [0.4, 1.0, 2.2, 3.0, 4.0, 5.0, 6.0, 6.9, 7.0, 7.1, 7.4, 7.5, 8.0, 12.0]
    rng = np.random.default_rng(4)
    kin = np.zeros(3 * len(sizes), dtype=fm3d.KEYPOINT)
    kin["size"] = sizes * 3
    kin["x"] = np.concatenate([rng.uniform(20, 620, len(sizes)), rng.uniform(-3, 3, len(sizes)),
                               rng.uniform(636, 642, len(sizes))])
    kin["y"] = np.concatenate([rng.uniform(20, 460, len(sizes)), rng.uniform(0, 479, len(sizes)),
                               rng.uniform(-2, 481, len(sizes))])
    kin["angle"] = -1
    ctx, _ = _ctx(fm3d, surfUpright=upright)
    try:
        k, kept, d = fm3d.SURF(ctx).compute(img, kin)
    finally:
        ctx.close()
    ko, kepto, do = orc.surf_describe(img, kin, extended=True, upright=bool(upright))
    assert len(ko) > len(kin) // 2 and np.array_equal(kept, kepto)
    _same_kpts(k, ko)
    assert np.array_equal(d, do)


def test_extract_descriptors_from_patches(fm3d, orc, synth):
    """extractDescriptorsFromPatches (descriptorsmatcher.cpp:133-174) on the exported 128x128
    normal-rectified patches: one keypoint at (64, 64) of size 128 per patch."""
    rng = np.random.default_rng(9)
    patches = rng.integers(0, 256, (40, 128, 128), dtype=np.uint8)
    patches[:, 32:96, 32:96] //= 3
    ctx, _ = _ctx(fm3d)
    try:
        d = fm3d.SURF(ctx).extractDescriptorsFromPatches(patches)
    finally:
        ctx.close()
    kp = np.zeros(1, dtype=fm3d.KEYPOINT)
    kp["x"] = kp["y"] = 64
    kp["size"] = 128
    kp["angle"] = -1
    kp["response"] = 1
    ref = np.stack([orc.surf_describe(p, kp, extended=True)[2][0] for p in patches])
    assert d.shape == (40, 128) and np.array_equal(d, ref)


def test_compare_with_nndr_from_images(fm3d, orc, synth):
    """compareWithNNDR from the images: SURF on both frames, FLANN-order L2 knnMatch, NNDR -- the
    same matches, keypoints and descriptors as the oracle chain."""
    pair = synth.make_frame_pair(2000, seed=4)
    ctx, s = _ctx(fm3d)
    try:
        dm = fm3d.DescriptorsMatcher(ctx)
        m, ka, kb, da, db = dm.compareWithNNDRImages(0.55, pair.img1, pair.img2)
    finally:
        ctx.close()
    koa = orc.surf_detect(pair.img1)
    kob = orc.surf_detect(pair.img2)
    _, _, doa = orc.surf_describe(pair.img1, koa)
    _, _, dob = orc.surf_describe(pair.img2, kob)
    _same_kpts(ka, koa)
    _same_kpts(kb, kob)
    assert np.array_equal(da, doa) and np.array_equal(db, dob)
    idx, dist = orc.knn2(doa, dob, orc.F32, oracle_threads())
    q, t, dd = orc.nndr(idx, dist, 0.55)
    assert np.array_equal(m["queryIdx"], q) and np.array_equal(m["trainIdx"], t) and np.array_equal(m["distance"], dd)
    assert len(m) > 50


# ---------------------------------------------------------------- Upright 0 (SURFInvoker orientation)
@pytest.mark.parametrize("extended", [1, 0])
def test_surf_oriented_detect_describe_bitwise(fm3d, orc, synth, extended):
    """Upright 0: every keypoint's dominant orientation (orient_kernel) and its descriptor of the
    rotated, bilinear window (describe_kernel) equal the oracle's, keypoints without an orientation
    sample removed in both"""
    img = synth.make_frame_pair(2000, seed=3).img1
    ctx, s = _ctx(fm3d, surfUpright=0, surfExtended=extended)
    try:
        k, d = fm3d.SURF(ctx).detect(img, with_descriptors=True)
    finally:
        ctx.close()
    ko = orc.surf_detect(img, s.surfHessianThreshold, s.surfOctaves, s.surfOctaveLayers, upright=False)
    _, kept, do = orc.surf_describe(img, ko, extended=bool(extended), upright=False)
    assert len(ko) > 500 and len(np.unique(ko["angle"])) > 100
    _same_kpts(k, ko)
    assert np.array_equal(kept, np.arange(len(ko))) and np.array_equal(d, do)


def test_surf_oriented_compute_borders_and_axis_angles(fm3d, orc, synth):
    """Upright 0 on caller keypoints: windows cut by every border (the nearest-pixel branch), a
    keypoint whose orientation disc misses the integral image (removed), and images whose gradients
    are exactly horizontal / vertical, so angles 0 / 90 / 180 / 270 whose cos or sin is ~1e-8 --
    row positions that are not closed-form exact, the kernel's sequential fallback"""
    img = synth.make_frame_pair(300, seed=8).img1
    kin = np.zeros(9, dtype=fm3d.KEYPOINT)
    kin["x"] = [0.0, 639.4, 320.5, 5.0, 100.0, 600.0, 2.5, -300.0, 320.0]
    kin["y"] = [0.0, 479.9, 240.2, 470.0, 3.0, 10.0, 2.5, -300.0, 240.0]
    kin["size"] = [9, 20, 4000, 31, 77, 150, 15, 12, 0.0]
    kin["angle"] = -1
    xx = np.arange(640)
    stripes_x = np.tile((128 + 100 * np.sin(xx * 0.05)).astype(np.uint8), (480, 1))
    ramp_y = np.tile(np.clip(np.arange(480) // 2, 0, 255).astype(np.uint8)[:, None], (1, 640))
    ctx, _ = _ctx(fm3d, surfUpright=0)
    try:
        for im in (img, stripes_x, ramp_y, np.ascontiguousarray(255 - ramp_y)):
            k, kept, d = fm3d.SURF(ctx).compute(im, kin)
            ko, kepto, do = orc.surf_describe(im, kin, extended=True, upright=False)
            assert np.array_equal(kept, kepto) and 7 not in list(kept) and 8 not in list(kept)
            _same_kpts(k, ko)
            assert np.array_equal(d, do)
        angles = set(np.round(orc.surf_describe(stripes_x, kin, upright=False)[0]["angle"], 3)) | set(
            np.round(orc.surf_describe(ramp_y, kin, upright=False)[0]["angle"], 3))
        assert angles & {0.0, 90.0, 180.0, 270.0}, angles
    finally:
        ctx.close()


def test_surf_oriented_patches(fm3d, orc):
    """extractDescriptorsFromPatches with Upright 0: each patch's keypoint oriented on that patch's
    own integral image (launch_integral_batch), then its rotated window"""
    rng = np.random.default_rng(19)
    patches = rng.integers(0, 256, (24, 128, 128), dtype=np.uint8)
    yy, xx = np.mgrid[0:128, 0:128]
    for i in range(24):
        a = i * 15 * np.pi / 180
        patches[i] = np.clip(patches[i] // 4 + 96 + 0.6 * ((xx - 64) * np.cos(a) + (yy - 64) * np.sin(a)), 0, 255)
    ctx, _ = _ctx(fm3d, surfUpright=0)
    try:
        d = fm3d.SURF(ctx).extractDescriptorsFromPatches(patches)
    finally:
        ctx.close()
    kp = np.zeros(1, dtype=fm3d.KEYPOINT)
    kp["x"] = kp["y"] = 64
    kp["size"] = 128
    kp["angle"] = -1
    kp["response"] = 1
    ref = np.stack([orc.surf_describe(p, kp, extended=True, upright=False)[2][0] for p in patches])
    assert d.shape == (24, 128) and np.array_equal(d, ref)
