"""Pin the CPU oracle to the golden fixtures (numpy / scipy restatements, see
tests/golden/make_golden.py).  CPU only."""
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


class Cam:
    def __init__(self, arr):
        self.fx, self.fy, self.cx, self.cy = arr[:4]
        self.k = tuple(arr[4:9])


@pytest.mark.parametrize("kind", ["u8", "f32", "bits"])
def test_knn2_and_nndr_match_numpy(orc, kind):
    g = load("match.npz")
    dtype = {"u8": orc.U8, "f32": orc.F32, "bits": orc.BITS}[kind]
    eps = {"u8": 0.55, "f32": 0.6, "bits": 0.8}[kind]
    idx, dist = orc.knn2(g[f"{kind}_A"], g[f"{kind}_B"], dtype, 2)
    assert np.array_equal(idx, g[f"{kind}_idx"])
    assert np.array_equal(dist, g[f"{kind}_dist"])
    q, t, d = orc.nndr(idx, dist, eps)
    assert np.array_equal(q, g[f"{kind}_q"]) and np.array_equal(t, g[f"{kind}_t"]) and np.array_equal(d, g[f"{kind}_d"])


def test_u8_duplicate_row_tie(orc):
    g = load("match.npz")
    B = g["u8_B"]
    dup = np.nonzero((B == B[np.argmax((B[:, None, :] == B[None]).all(-1).sum(1) > 1)]).all(1))[0]
    assert len(dup) == 2
    idx, _ = orc.knn2(B[dup[:1]], B, orc.U8, 1)
    assert list(idx[0]) == list(dup)  # equal distance -> lowest trainIdx first


def test_undistort_project_bitwise(orc):
    g = load("camera.npz")
    cam = Cam(g["cam"])
    assert np.array_equal(orc.undistort(cam, g["uv"]), g["und"])
    assert np.array_equal(orc.project(cam, np.eye(3), np.zeros(3), g["P"]), g["proj_id"])
    assert np.array_equal(orc.project(cam, g["R2"], g["t2"], g["P"]), g["proj2"])


def test_setg12_vs_numpy_inverse(orc):
    g = load("camera.npz")
    g12 = orc.setg12(g["rIC"], g["tIC"], g["pos1"][:3], g["pos2"][:3], g["pos1"][3:], g["pos2"][3:])
    assert np.abs(g12 - g["g12"]).max() < 1e-13


def test_rodrigues_roundtrip(orc):
    rng = np.random.default_rng(4)
    for r in rng.normal(0, 1, (50, 3)):
        R = orc.rodrigues_v2m(r)
        assert np.abs(R @ R.T - np.eye(3)).max() < 1e-14
        assert np.abs(orc.rodrigues_m2v(R) - r).max() < 1e-12 or np.linalg.norm(r) > np.pi


def test_dlt_vs_numpy_svd(orc):
    g = load("dlt.npz")
    cam = Cam(g["cam"])
    pts, mask = orc.triangulate(cam, g["g12"], 1.5, 2.4, g["kp1"], g["kp2"], g["q"], g["t"])
    assert np.array_equal(mask, g["mask"])
    rel = np.abs(pts - g["pts"]) / np.maximum(1.0, np.abs(g["pts"]))
    assert rel.max() < 1e-9


def test_pyrdown_vs_scipy(orc):
    g = load("pyr.npz")
    for i in range(5):
        assert np.array_equal(orc.pyrdown(g[f"img{i}"]), g[f"down{i}"]), i


def test_lm_normals_vs_scipy_leastsq(orc):
    """computeOptimizedNormals with MINPACK lmdif: the oracle's restatement against
    scipy.optimize.leastsq driving an independent numpy evaluateNormal."""
    g = load("lm.npz")
    cam = Cam(g["cam"])
    h, w = g["img1"].shape
    r = orc.optimize_normals(cam, g["R2"], g["t2"], g["img1"], g["img2"], int(g["levels"]), g["points"],
                             int(g["ray"]), w, h, mode=orc.STRICT, nthreads=2)
    assert np.array_equal(r["status"], g["status"])
    L = int(g["levels"]) + 1
    assert np.array_equal(r["nfev"][:, :L], g["nfev"])
    assert np.array_equal(r["info"][:, :L], g["info"])
    ok = g["status"] == 0
    assert ok.sum() >= 10
    assert np.abs(r["normals"][ok] - g["normals"][ok]).max() < 1e-12


def test_detmath_does_not_move_lm(orc):
    """The kernel's deterministic sin/cos/atan2/exp replace libm: on the golden
    scene the LM result moves by < 1e-12 (in practice by ulps)."""
    g = load("lm.npz")
    cam = Cam(g["cam"])
    h, w = g["img1"].shape
    args = (cam, g["R2"], g["t2"], g["img1"], g["img2"], int(g["levels"]), g["points"], int(g["ray"]), w, h)
    a = orc.optimize_normals(*args, mode=orc.STRICT, nthreads=2)
    b = orc.optimize_normals(*args, mode=orc.DETMATH, nthreads=2)
    assert np.array_equal(a["status"], b["status"])
    ok = a["status"] == 0
    assert np.abs(a["normals"][ok] - b["normals"][ok]).max() < 1e-12


def test_features_frames_and_patches_vs_numpy(orc):
    """computeFeaturesFrames + patch export: the oracle against the numpy restatement
    (tests/golden/make_golden.py make_patches): frames bit for bit (same scalar operations),
    gravity to 1e-15 (numpy inverts by LU), patches allowing the rare 1-level truncation flip
    that the SVD-vs-Newton polar factor and libm ulps can cause."""
    g = load("patches.npz")
    cam = Cam(g["cam"])
    assert np.abs(orc.gravity(g["rIC"]) - g["g"]).max() < 1e-15
    frames = orc.features_frames(g["points"], g["normals"], g["g"])
    assert np.array_equal(frames, g["frames"])
    eps, cmpp = float(g["eps"]), float(g["cmpp"])
    assert orc.patch_size(eps, cmpp) == int(g["size"])
    patches, pts = orc.export_patches(cam, g["img1"], frames, eps, cmpp, mode=orc.STRICT, image_points=True)
    assert np.abs(pts - g["image_points"]).max() < 1e-9
    d = np.abs(patches.astype(int) - g["patches"].astype(int))
    assert d.max() <= 1 and (d == 0).mean() > 0.99
    # DETMATH (the GPU's transcendentals) moves nothing here beyond the same truncation flips
    p2 = orc.export_patches(cam, g["img1"], frames, eps, cmpp, mode=orc.DETMATH)
    assert np.abs(p2.astype(int) - patches.astype(int)).max() <= 1


def test_square_neighborhoods_vs_numpy(orc):
    """computeSquareNeighborhoodsByNormals (neighborhoodsgenerator.cpp:76-132): the oracle against
    a numpy restatement with the same scalar operations (Matx44d * Vec4d summed from 0 in k order),
    on the golden frames plus a non-rigid frame (w != 1: scaled by 1/w)."""
    g = load("patches.npz")
    frames = np.concatenate([g["frames"].reshape(-1, 16), [[1, 0.5, 0.25, 0.1, 0, 1, 0, 0.2, 0.3, 0, 1, 2.0,
                                                              0.01, -0.02, 0.5, 0.9]]])
    eps, cmpp = 0.016, 0.025
    size = orc.patch_size(eps, cmpp)
    out = orc.square_neighborhoods(frames, eps, cmpp)
    assert out.shape == (len(frames), size * size, 3)
    inc = cmpp * 0.01
    i, j = np.meshgrid(np.arange(size), np.arange(size), indexing="ij")
    v = [(-eps + inc * i.astype(np.float64)).ravel(), (-eps + inc * j.astype(np.float64)).ravel(),
         np.zeros(size * size), np.ones(size * size)]
    for p, F in enumerate(frames):
        h = [(((0.0 + F[4 * r] * v[0]) + F[4 * r + 1] * v[1]) + F[4 * r + 2] * v[2]) + F[4 * r + 3] * v[3]
             for r in range(4)]
        a = np.where(h[3] != 1, 1.0 / h[3], 1.0)
        ref = np.stack([np.where(h[3] != 1, h[k] * a, h[k]) for k in range(3)], axis=1)
        assert np.array_equal(out[p], ref), p
    assert not np.array_equal(out[-1][:, :3], out[-1][:, :3] * 0)  # the w != 1 frame produced points


def test_reference_patch_size():
    """build/settings.yml (Neighborhoods epsilon 0.16, cmPerPixel 0.25) gives the 128x128 patches
    of the reference's results/*/patch_*.pgm (P5 128 128)."""
    import oracle
    assert oracle.patch_size(0.16, 0.25) == 128
