"""Synthetic frame pairs for the 3DFeatureMatcher hot path.

The reference's inputs (``build/settings.yml:8-9``, images under /home/mpp/...)
are not shipped, so tests and the bench use ray-cast renders of a known
piecewise-planar scene:

* camera: ``build/settings.yml`` intrinsics scaled to the image width
  (0.625 for VGA), same distortion (k0,k1,p1,p2,k2);
* pose: ``g12`` from ``IMAGES.pos1/pos2`` and the IMU calibration, exactly as
  ``SingleCameraTriangulator::setg12`` builds it (0.66 m forward motion, 6 deg);
* scene: an 8x8 grid of planar facets at depths in [1.6, 2.3] m with normals
  within 40 deg of the optical axis, value-noise texture on each facet;
* keypoints: sub-pixel image-1 positions on surfaces visible in both views,
  image-2 positions = their projections;
* descriptors: SIFT-like uint8 (``min(255,|N(0,40)|)``), frame-2 copy with
  +-8 uniform noise, 10 % distractors, frame 2 permuted; or ORB-like 256-bit
  strings with 5 % of the bits flipped.

Everything is seeded (numpy PCG64) so a config is reproducible.
"""
from __future__ import annotations

import dataclasses
import math

import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

_BLOCK = 65536


def _workers() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))

# build/settings.yml (CameraSettings, IMAGES) -- reference defaults
REF_CAMERA = dict(Fx=572.4765, Fy=572.69354, Cx=549.75189, Cy=411.68039,
                  p1=-6.6e-05, p2=0.000567, k0=-0.299957, k1=0.124129, k2=-0.028357)
REF_RODRIGUES_IC = (-1.2005, 1.1981, -1.2041)
REF_TRANSLATION_IC = (0.0, 0.015, -0.051)
REF_POS1 = (5.301099, 8.031408, 1.977258, 0.153433, 0.149941, -2.658648)
REF_POS2 = (4.735536, 7.691893, 1.913166, 0.252828, 0.048977, -2.676886)
REF_WIDTH = 1024  # images the reference was run on (results/*/projectedPatches.pgm)


@dataclasses.dataclass
class Camera:
    fx: float
    fy: float
    cx: float
    cy: float
    k: tuple  # OpenCV order (k1, k2, p1, p2, k3) == settings (k0, k1, p1, p2, k2)

    @staticmethod
    def reference(width: int = 640) -> "Camera":
        s = width / REF_WIDTH
        c = REF_CAMERA
        return Camera(c["Fx"] * s, c["Fy"] * s, c["Cx"] * s, c["Cy"] * s,
                      (c["k0"], c["k1"], c["p1"], c["p2"], c["k2"]))


def rodrigues(r):
    r = np.asarray(r, dtype=np.float64)
    th = math.sqrt(float(r @ r))
    if th < np.finfo(float).eps:
        return np.eye(3)
    k = r / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return math.cos(th) * np.eye(3) + (1 - math.cos(th)) * np.outer(k, k) + math.sin(th) * K


def reference_g12() -> np.ndarray:
    """g12 = gIC^-1 g2^-1 g1 gIC (singlecameratriangulator.cpp:123-143)."""
    def g(R, t):
        G = np.eye(4)
        G[:3, :3] = R
        G[:3, 3] = t
        return G
    gIC = g(rodrigues(REF_RODRIGUES_IC), REF_TRANSLATION_IC)
    g1 = g(rodrigues(REF_POS1[3:]), REF_POS1[:3])
    g2 = g(rodrigues(REF_POS2[3:]), REF_POS2[:3])
    return np.linalg.inv(gIC) @ np.linalg.inv(g2) @ g1 @ gIC


def project(cam: Camera, P: np.ndarray, R=None, t=None) -> np.ndarray:
    """OpenCV 2.4 projectPoints (vectorised, float64)."""
    P = np.asarray(P, dtype=np.float64)
    if R is not None:
        P = P @ np.asarray(R).T + np.asarray(t)
    z = P[:, 2]
    x = P[:, 0] / z
    y = P[:, 1] / z
    k1, k2, p1, p2, k3 = cam.k
    r2 = x * x + y * y
    cd = 1 + k1 * r2 + k2 * r2 * r2 + k3 * r2 * r2 * r2
    xd = x * cd + 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
    yd = y * cd + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
    return np.stack([xd * cam.fx + cam.cx, yd * cam.fy + cam.cy], axis=1)


def undistort(cam: Camera, uv: np.ndarray) -> np.ndarray:
    """OpenCV 2.4 undistortPoints, 5 iterations (vectorised)."""
    k1, k2, p1, p2, k3 = cam.k
    x0 = (uv[:, 0] - cam.cx) * (1.0 / cam.fx)
    y0 = (uv[:, 1] - cam.cy) * (1.0 / cam.fy)
    x, y = x0.copy(), y0.copy()
    for _ in range(5):
        r2 = x * x + y * y
        icd = 1.0 / (1 + ((k3 * r2 + k2) * r2 + k1) * r2)
        dx = 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
        dy = p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
        x = (x0 - dx) * icd
        y = (y0 - dy) * icd
    return np.stack([x, y], axis=1)


class FacetScene:
    """An 8x8 grid of textured planar facets seen by camera 1."""

    def __init__(self, rng: np.random.Generator, cells: int = 8, fov: float = 2.6,
                 zmin: float = 1.6, zmax: float = 2.3, max_tilt_deg: float = 40.0):
        self.cells = cells
        self.edges = np.linspace(-fov / 2, fov / 2, cells + 1)
        n = cells * cells
        depth = rng.uniform(zmin + 0.08, zmax - 0.08, n)
        cxy = (self.edges[:-1] + self.edges[1:]) / 2
        xc, yc = np.meshgrid(cxy, cxy, indexing="ij")  # [a][b] -> x index a, y index b
        self.Q = np.stack([xc.ravel() * depth, yc.ravel() * depth, depth], axis=1)
        # normal facing the camera, tilted by <= max_tilt from -z; tilt kept small
        # enough that the facet stays inside [zmin, zmax] over its cell
        tilt = np.radians(rng.uniform(0, max_tilt_deg, n))
        az = rng.uniform(0, 2 * np.pi, n)
        nrm = np.stack([np.sin(tilt) * np.cos(az), np.sin(tilt) * np.sin(az), -np.cos(tilt)], axis=1)
        self.N = nrm
        # in-plane orthonormal basis for the texture coordinates
        ref = np.where(np.abs(nrm[:, 0:1]) < 0.9, np.array([[1.0, 0, 0]]), np.array([[0, 1.0, 0]]))
        e1 = np.cross(nrm, ref)
        e1 /= np.linalg.norm(e1, axis=1, keepdims=True)
        self.E1 = e1
        self.E2 = np.cross(nrm, e1)
        self.tex_offset = rng.uniform(0, 1000, (n, 2))
        # value-noise lattices, shared by all facets (offset differs per facet)
        self.lattices = [rng.uniform(0, 1, (257, 257)) for _ in range(3)]
        self.wavelengths = (0.03, 0.08, 0.2)  # metres (~5, 14, 36 px at 2 m in VGA)
        self.weights = (0.45, 0.35, 0.20)
        self.zmin, self.zmax = zmin, zmax

    def intersect(self, C: np.ndarray, D: np.ndarray):
        """Nearest facet hit for rays C + s D (C: (3,) or (n,3); D: (n,3)).
        Returns (s, facet id, point); id -1 where no facet is hit.

        Large ray sets run in fixed 64k-ray blocks on a thread pool (numpy releases the
        GIL): every ray's arithmetic is the same, so the output is byte-identical to one
        block (checked for the bench and test configurations)."""
        n = D.shape[0]
        if n > _BLOCK:
            Cb = np.asarray(C, dtype=np.float64)
            with ThreadPoolExecutor(_workers()) as ex:
                parts = list(ex.map(lambda a: self._intersect(Cb if Cb.ndim == 1 else Cb[a:a + _BLOCK],
                                                              D[a:a + _BLOCK]), range(0, n, _BLOCK)))
            return tuple(np.concatenate([q[k] for q in parts]) for k in range(3))
        return self._intersect(C, D)

    def _intersect(self, C: np.ndarray, D: np.ndarray):
        n = D.shape[0]
        best_s = np.full(n, np.inf)
        best_j = np.full(n, -1, dtype=np.int64)
        C = np.broadcast_to(np.asarray(C, dtype=np.float64), D.shape)
        for j in range(self.Q.shape[0]):
            nj = self.N[j]
            den = D @ nj
            num = (self.Q[j] - C) @ nj
            with np.errstate(divide="ignore", invalid="ignore"):
                s = num / den
            P = C + s[:, None] * D
            with np.errstate(divide="ignore", invalid="ignore"):
                ax = P[:, 0] / P[:, 2]
                ay = P[:, 1] / P[:, 2]
            a, b = divmod(j, self.cells)
            ok = (s > 1e-9) & (P[:, 2] > 0) & (ax >= self.edges[a]) & (ax < self.edges[a + 1]) \
                & (ay >= self.edges[b]) & (ay < self.edges[b + 1]) & (s < best_s)
            best_s = np.where(ok, s, best_s)
            best_j = np.where(ok, j, best_j)
        P = C + np.where(np.isfinite(best_s), best_s, 0)[:, None] * D
        return best_s, best_j, P

    def texture(self, P: np.ndarray, j: np.ndarray) -> np.ndarray:
        jj = np.maximum(j, 0)
        d = P - self.Q[jj]
        a = np.einsum("ij,ij->i", d, self.E1[jj]) + self.tex_offset[jj, 0]
        b = np.einsum("ij,ij->i", d, self.E2[jj]) + self.tex_offset[jj, 1]
        val = np.zeros(P.shape[0])
        for lat, wl, wt in zip(self.lattices, self.wavelengths, self.weights):
            u = a / wl
            v = b / wl
            iu = np.floor(u)
            iv = np.floor(v)
            fu = u - iu
            fv = v - iv
            fu = fu * fu * (3 - 2 * fu)
            fv = fv * fv * (3 - 2 * fv)
            i0 = iu.astype(np.int64) % 256
            k0 = iv.astype(np.int64) % 256
            v00 = lat[i0, k0]
            v10 = lat[i0 + 1, k0]
            v01 = lat[i0, k0 + 1]
            v11 = lat[i0 + 1, k0 + 1]
            val += wt * ((v00 * (1 - fu) + v10 * fu) * (1 - fv) + (v01 * (1 - fu) + v11 * fu) * fv)
        img = np.clip(20 + 215 * val, 0, 255)
        return np.where(j >= 0, img, 40.0)


@dataclasses.dataclass
class FramePair:
    cam: Camera
    g12: np.ndarray
    img1: np.ndarray          # (H, W) uint8
    img2: np.ndarray
    kp1: np.ndarray           # (N1, 2) float32
    kp2: np.ndarray           # (N2, 2) float32
    desc1: np.ndarray         # (N1, D) uint8
    desc2: np.ndarray         # (N2, D) uint8
    true_train: np.ndarray    # (N1,) frame-2 index of the true match, -1 if none
    points: np.ndarray        # (N1, 3) ground-truth 3D points (camera-1 frame)
    normals: np.ndarray       # (N1, 3) ground-truth surface normals (facing camera 1)


def render(scene: FacetScene, cam: Camera, g12: np.ndarray, width: int, height: int, which: int) -> np.ndarray:
    u, v = np.meshgrid(np.arange(width, dtype=np.float64), np.arange(height, dtype=np.float64))
    uv = np.stack([u.ravel(), v.ravel()], axis=1)
    xy = undistort(cam, uv)
    d = np.concatenate([xy, np.ones((xy.shape[0], 1))], axis=1)
    if which == 1:
        C = np.zeros(3)
        D = d
    else:
        R = g12[:3, :3]
        t = g12[:3, 3]
        C = -R.T @ t
        D = d @ R  # R^T d for each row
    _, j, P = scene.intersect(C, D)
    return np.round(scene.texture(P, j)).astype(np.uint8).reshape(height, width)


def make_frame_pair(n_kp: int, width: int = 640, height: int = 480, seed: int = 0, desc: str = "sift",
                    distractor_frac: float = 0.1, desc_noise: int = 8, g12=None, cam=None) -> FramePair:
    rng = np.random.default_rng(seed)
    cam = cam or Camera.reference(width)
    g12 = reference_g12() if g12 is None else np.asarray(g12, dtype=np.float64)
    scene = FacetScene(rng)
    img1 = render(scene, cam, g12, width, height, 1)
    img2 = render(scene, cam, g12, width, height, 2)
    R = g12[:3, :3]
    t = g12[:3, 3]
    C2 = -R.T @ t
    # keypoints on surfaces visible in both frames
    pts, kps1, kps2, fac = [], [], [], []
    need = n_kp
    while need > 0:
        m = int(need * 1.8) + 64
        uv = np.stack([rng.uniform(0, width, m), rng.uniform(0, height, m)], axis=1).astype(np.float32)
        xy = undistort(cam, uv.astype(np.float64))
        D = np.concatenate([xy, np.ones((m, 1))], axis=1)
        s, j, P = scene.intersect(np.zeros(3), D)
        ok = j >= 0
        uv2 = project(cam, P, R, t)
        ok &= (uv2[:, 0] >= 0) & (uv2[:, 0] < width) & (uv2[:, 1] >= 0) & (uv2[:, 1] < height)
        ok &= (P @ R.T + t)[:, 2] > 0.1
        # occlusion test along the camera-2 ray
        D2 = P - C2
        s2, j2, _ = scene.intersect(C2, D2)
        ok &= (j2 == j) & (np.abs(s2 - 1.0) < 1e-7)
        idx = np.nonzero(ok)[0][:need]
        pts.append(P[idx])
        kps1.append(uv[idx])
        kps2.append(uv2[idx].astype(np.float32))
        fac.append(j[idx])
        need -= idx.size
    P = np.concatenate(pts)
    kp1 = np.concatenate(kps1)
    kp2_true = np.concatenate(kps2)
    facet = np.concatenate(fac)
    normals = -scene.N[facet]  # orientation is irrelevant for a plane; report the camera-facing side flipped
    n1 = n_kp
    n_true = int(round(n1 * (1 - distractor_frac)))
    n_distr = n1 - n_true
    if desc == "sift":
        dim = 128
        base = np.minimum(255, np.abs(rng.normal(0, 40, (n1, dim)))).astype(np.int32)
        d1 = base.astype(np.uint8)
        noisy = np.clip(base[:n_true] + rng.integers(-desc_noise, desc_noise + 1, (n_true, dim)), 0, 255)
        distr = np.minimum(255, np.abs(rng.normal(0, 40, (n_distr, dim)))).astype(np.int32)
        d2 = np.concatenate([noisy, distr]).astype(np.uint8)
    elif desc == "orb":
        dim = 32
        d1 = rng.integers(0, 256, (n1, dim), dtype=np.uint8)
        flips = (rng.random((n_true, dim * 8)) < 0.05).astype(np.uint8)
        fb = np.packbits(flips, axis=1)
        d2 = np.concatenate([d1[:n_true] ^ fb, rng.integers(0, 256, (n_distr, dim), dtype=np.uint8)])
    else:
        raise ValueError(desc)
    kp2 = np.concatenate([kp2_true[:n_true],
                          np.stack([rng.uniform(0, width, n_distr), rng.uniform(0, height, n_distr)],
                                   axis=1).astype(np.float32)])
    perm = rng.permutation(n1)            # frame 2 order: position perm[i] holds original i
    inv = np.empty_like(perm)
    inv[perm] = np.arange(n1)
    d2p = np.empty_like(d2)
    kp2p = np.empty_like(kp2)
    d2p[perm] = d2
    kp2p[perm] = kp2
    true_train = np.where(np.arange(n1) < n_true, perm, -1)
    return FramePair(cam, g12, img1, img2, kp1.astype(np.float32), kp2p.astype(np.float32),
                     d1, d2p, true_train, P, normals)
