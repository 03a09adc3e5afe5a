"""The SURF oracle (oracle/orc_surf.c): feature detection + description of the reference's
default detector / extractor (descriptorsmatcher.cpp:110-115, 176-359; build/settings.yml:37-49).

OpenCV (nonfree) is not in this image, so the restatement is pinned by independent numpy
restatements of its pieces (integral image, INTER_AREA resize, the Gaussian weights) and by exact
properties of the algorithm (blob centres and scales, Laplacian sign, translation covariance, unit
descriptors).  Parity vs OpenCV itself is unpinned."""
import math

import numpy as np
import pytest


def _blobs(h=240, w=320, spec=((80, 60, 4.0, 1), (200, 150, 7.0, -1), (260, 60, 3.0, 1), (120, 180, 10.0, 1))):
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    img = np.full((h, w), 128.0)
    for cx, cy, sg, sign in spec:
        img += sign * 110.0 * np.exp(-((xx - cx) ** 2 + (yy - cy) ** 2) / (2 * sg * sg))
    return np.clip(np.rint(img), 0, 255).astype(np.uint8), spec


def test_integral_vs_numpy(orc):
    rng = np.random.default_rng(40)
    img = rng.integers(0, 256, (37, 53), dtype=np.uint8)
    ref = np.zeros((38, 54), dtype=np.int64)
    ref[1:, 1:] = img.astype(np.int64).cumsum(0).cumsum(1)
    assert np.array_equal(orc.integral(img), ref)


def _area_tab(ssize, dsize, scale):
    """computeResizeAreaTab (OpenCV 2.4 imgproc/resize.cpp)."""
    tab = []
    for dx in range(dsize):
        fsx1 = dx * scale
        fsx2 = fsx1 + scale
        cell = min(scale, ssize - fsx1)
        sx1, sx2 = math.ceil(fsx1), math.floor(fsx2)
        sx2 = min(sx2, ssize - 1)
        sx1 = min(sx1, sx2)
        if sx1 - fsx1 > 1e-3:
            tab.append((dx, sx1 - 1, np.float32((sx1 - fsx1) / cell)))
        for sx in range(sx1, sx2):
            tab.append((dx, sx, np.float32(1.0 / cell)))
        if fsx2 - sx2 > 1e-3:
            tab.append((dx, sx2, np.float32(min(min(fsx2 - sx2, 1.0), cell) / cell)))
    return tab


def _resize_area21_numpy(win):
    W = win.shape[0]
    scale = 1.0 / (21.0 / W)
    iscale = int(np.rint(scale))
    out = np.zeros((21, 21), dtype=np.uint8)
    if abs(scale - iscale) < np.finfo(np.float64).eps:
        for dy in range(21):
            for dx in range(21):
                blk = win[dy * iscale:(dy + 1) * iscale, dx * iscale:(dx + 1) * iscale].astype(np.int64)
                if iscale == 2 and dx < 16:
                    out[dy, dx] = (blk.sum() + 2) >> 2
                else:
                    out[dy, dx] = np.clip(np.rint(np.float32(blk.sum()) * np.float32(1.0 / (iscale * iscale))), 0, 255)
        return out
    xt, yt = _area_tab(W, 21, scale), _area_tab(W, 21, scale)
    acc = {}
    for dy, sy, beta in yt:
        buf = np.zeros(21, dtype=np.float32)
        for dx, sx, alpha in xt:
            buf[dx] = np.float32(buf[dx] + np.float32(np.float32(win[sy, sx]) * alpha))
        if dy not in acc:
            acc[dy] = np.float32(beta) * buf
        else:
            acc[dy] = np.float32(acc[dy] + np.float32(beta) * buf)
    for dy in range(21):
        out[dy] = np.clip(np.rint(acc[dy]), 0, 255)
    return out


@pytest.mark.parametrize("W", [25, 30, 42, 44, 63, 84, 101, 250])
def test_resize_area_vs_numpy(orc, W):
    """resize(win, 21x21, INTER_AREA): the general area tables and the integer-scale fast path
    (W = 42: 2x2 blocks, SSE2 rounding on the first 16 columns; W = 63 / 84: scalar)."""
    rng = np.random.default_rng(W)
    win = rng.integers(0, 256, (W, W), dtype=np.uint8)
    assert np.array_equal(orc.resize_area21(win), _resize_area21_numpy(win))


def test_descriptor_weights_vs_numpy(orc):
    """getGaussianKernel(20, 3.3, CV_32F) outer product (SURFInvoker ctor)."""
    x = np.arange(20) - 9.5
    g = np.exp(-0.5 / (3.3 * 3.3) * x * x).astype(np.float32)
    s = 1.0 / g.astype(np.float64).sum()
    g = (g.astype(np.float64) * s).astype(np.float32)
    assert np.array_equal(orc.surf_dw(), np.outer(g, g).astype(np.float32))


def test_blob_keypoints(orc):
    """Gaussian blobs: one keypoint per blob near its centre, bright blobs Laplacian sign -1 (trace
    of the Hessian < 0 at a maximum), dark +1, and the scale grows with the blob sigma."""
    img, spec = _blobs()
    k = orc.surf_detect(img)
    assert (k["angle"] == 270).all() and np.all(np.diff(k["response"]) <= 0)
    sizes = []
    for cx, cy, sg, sign in spec:
        d = np.hypot(k["x"] - cx, k["y"] - cy)
        j = int(np.argmin(d))
        assert d[j] < 1.5, (cx, cy, d[j])
        assert k["class_id"][j] == -sign
        sizes.append(k["size"][j])
    order = np.argsort([s[2] for s in spec])
    assert np.all(np.diff(np.array(sizes)[order]) > 0), sizes


def test_translation_covariance(orc, synth):
    """Shifting the image by 16 pixels (a multiple of every octave's sample step) shifts every
    keypoint away from the borders by exactly 16 and leaves its descriptor bit-identical."""
    img = synth.make_frame_pair(300, seed=5).img1[:240, :320]
    big = np.zeros((240 + 16, 320 + 16), dtype=np.uint8)
    big[16:, 16:] = img
    big[:16, 16:] = img[:1, :]
    big[16:, :16] = img[:, :1]
    big[:16, :16] = img[0, 0]
    k0 = orc.surf_detect(img)
    k1 = orc.surf_detect(big)
    kd0, _, d0 = orc.surf_describe(img, k0)
    kd1, _, d1 = orc.surf_describe(big, k1)
    inner = lambda k: (k["x"] > 120) & (k["x"] < 200) & (k["y"] > 100) & (k["y"] < 140) & (k["size"] < 30)
    a = {(round(float(x), 3), round(float(y), 3), float(s)): i for i, (x, y, s) in
         enumerate(zip(kd0["x"], kd0["y"], kd0["size"])) if inner(kd0[i])}
    hits = 0
    for i, (x, y, s) in enumerate(zip(kd1["x"] - 16, kd1["y"] - 16, kd1["size"])):
        key = (round(float(x), 3), round(float(y), 3), float(s))
        if key in a:
            hits += 1
            assert np.array_equal(d0[a[key]], d1[i])
    assert hits >= 0.9 * len(a) and hits > 5, (hits, len(a))


def test_descriptors_unit_and_short(orc, synth):
    img = synth.make_frame_pair(300, seed=6).img1
    k = orc.surf_detect(img)[:300]
    kk, kept, d = orc.surf_describe(img, k)
    assert d.shape == (len(kk), 128) and np.array_equal(kept, np.arange(len(kk)))
    assert np.abs(np.linalg.norm(d.astype(np.float64), axis=1) - 1).max() < 1e-5
    _, _, d64 = orc.surf_describe(img, k, extended=False)
    assert d64.shape == (len(kk), 64)
    assert np.abs(np.linalg.norm(d64.astype(np.float64), axis=1) - 1).max() < 1e-5
    # extended splits each sum of dx / |dx| by the sign of dy: the pairs add back to the short sums
    # (before normalisation, so compare directions)
    big = d.reshape(-1, 16, 8).astype(np.float64)
    short = d64.reshape(-1, 16, 4).astype(np.float64)
    sx = big[:, :, 0] + big[:, :, 2]
    cos = (sx * short[:, :, 0]).sum(1) / (np.linalg.norm(sx, axis=1) * np.linalg.norm(short[:, :, 0], axis=1))
    assert (cos > 0.999).all()
