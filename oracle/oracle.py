"""ctypes wrapper of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py.  The product never imports it.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

F32, U8, BITS = 0, 1, 2
STRICT, DETMATH = 0, 2  # libm transcendentals / fm3d_crmath.h (the GPU contract)
TREE, GRAM = 64, 128    # fm3d_oracle.c ORC_LM_TREE / ORC_LM_GRAM: the LM kernel's lmReduction = 1 is DETMATH|TREE|GRAM
LIBM_SIN, LIBM_COS, LIBM_ATAN2, LIBM_EXP, DET_1ULP = 256, 512, 1024, 2048, 4096  # ORC_LIBM_* / ORC_DET_1ULP


def tree_stats(reset=False):
    """orc_tree_stats: [Gram-form QRs, Householder-form QRs, sequential-enorm fallbacks, Householder-form
    QRs of a zero Jacobian] of the tree
    mode since the last reset (test infrastructure)."""
    arr = (ctypes.c_longlong * 4).in_dll(lib(), "orc_tree_stats")
    out = [int(v) for v in arr]
    if reset:
        for i in range(4):
            arr[i] = 0
    return out

def math_eval(fn, x, y=None, mode=DETMATH):
    """orc_math_eval: fn "sin", "cos", "exp" of x, or "atan2" / "hypot" of (x, y), elementwise,
    in an oracle mode (DETMATH: include/fm3d_crmath.h's correctly rounded functions; DETMATH |
    DET_1ULP: fm3d_detmath.h's; 0: libm)."""
    f = {"sin": 0, "cos": 1, "atan2": 2, "exp": 3, "hypot": 4}[fn]
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = x if y is None else np.ascontiguousarray(y, dtype=np.float64)
    out = np.empty_like(x)
    dp = ctypes.POINTER(ctypes.c_double)
    lib().orc_math_eval(ctypes.c_int(f), ctypes.c_int(mode), x.ctypes.data_as(dp), y.ctypes.data_as(dp),
                        ctypes.c_int(x.size), out.ctypes.data_as(dp))
    return out


ST_OK, ST_NO_PIXELS, ST_ABORT_BBOX, ST_ABORT_PIX1, ST_ABORT_PIX2, ST_NAN_PLANE, ST_NAN_NORMAL = range(7)


class OrcCamera(ctypes.Structure):
    _fields_ = [("fx", ctypes.c_double), ("fy", ctypes.c_double), ("cx", ctypes.c_double),
                ("cy", ctypes.c_double), ("k", ctypes.c_double * 5)]

    @staticmethod
    def from_cam(cam) -> "OrcCamera":
        c = OrcCamera()
        c.fx, c.fy, c.cx, c.cy = cam.fx, cam.fy, cam.cx, cam.cy
        for i in range(5):
            c.k[i] = cam.k[i]
        return c


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle/liboracle.so missing: run `make -C oracle` (or __graft_entry__.build())")
        _LIB = ctypes.CDLL(path)
    return _LIB


def _p(a, t=ctypes.c_double):
    return a.ctypes.data_as(ctypes.POINTER(t))


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def setg12(rIC, tIC, T1, T2, r1, r2):
    g = np.zeros(16)
    lib().orc_setg12(_p(_f64(rIC)), _p(_f64(tIC)), _p(_f64(T1)), _p(_f64(T2)), _p(_f64(r1)), _p(_f64(r2)), _p(g))
    return g.reshape(4, 4)


def camera2_from_g12(g12):
    R2 = np.zeros(9)
    t2 = np.zeros(3)
    lib().orc_camera2_from_g12(_p(_f64(np.asarray(g12).ravel())), _p(R2), _p(t2))
    return R2.reshape(3, 3), t2


# orc_set_geometry_mode switches (fm3d_oracle.c ORC_GEOM_*; measurement only, tools/dlt_parity.py):
# the rounds 1-5 DLT (4-row system, round-robin Jacobi), the rounds 1-5 Newton polar factor,
# JacobiSVDImpl_'s SSE2 two-lane dot / givensx accumulation, libm's hypot in the SVD rotation
GEOM_DLT_LEGACY, GEOM_POLAR_NEWTON, GEOM_SVD_LANES, GEOM_LIBM_HYPOT = 1, 2, 4, 8


def set_geometry_mode(mode: int) -> int:
    """set the oracle's geometry mode (0 = OpenCV 2.4's cvSVD everywhere, the product contract);
    returns the previous mode"""
    prev = int(lib().orc_get_geometry_mode())
    lib().orc_set_geometry_mode(ctypes.c_int(mode))
    return prev


class geometry_mode:
    """with orc.geometry_mode(orc.GEOM_DLT_LEGACY): ... -- restores the previous mode"""

    def __init__(self, mode: int):
        self.mode = mode

    def __enter__(self):
        self.prev = set_geometry_mode(self.mode)
        return self

    def __exit__(self, *exc):
        set_geometry_mode(self.prev)


def cv_svd(A):
    """cv::SVD::compute of an m x n (m >= n, both <= 8) double matrix as OpenCV 2.4's JacobiSVD does it:
    w (n, descending), u (m x n), vt (n x n)"""
    A = _f64(A)
    m, n = A.shape
    w, u, vt = np.zeros(n), np.zeros((m, n)), np.zeros((n, n))
    rc = lib().orc_cv_svd_eval(_p(A), ctypes.c_int(m), ctypes.c_int(n), _p(w), _p(u), _p(vt))
    if rc != 0:
        raise ValueError("orc_cv_svd_eval: m >= n, n, m <= 8")
    return w, u, vt


def cv_polar3(R):
    """cvRodrigues2's orthonormalisation U V^T of a 3 x 3 matrix"""
    out = np.zeros(9)
    lib().orc_cv_polar3(_p(_f64(np.asarray(R).ravel())), _p(out))
    return out.reshape(3, 3)


def rodrigues_v2m(r):
    R = np.zeros(9)
    lib().orc_rodrigues_v2m(_p(_f64(r)), _p(R))
    return R.reshape(3, 3)


def rodrigues_m2v(R):
    r = np.zeros(3)
    lib().orc_rodrigues_m2v(_p(_f64(np.asarray(R).ravel())), _p(r))
    return r


def undistort(cam, xy):
    xy = _f64(xy).reshape(-1, 2)
    out = np.zeros_like(xy)
    c = OrcCamera.from_cam(cam)
    lib().orc_undistort(ctypes.byref(c), _p(xy), ctypes.c_int(xy.shape[0]), _p(out))
    return out


def project(cam, R, t, P):
    P = _f64(P).reshape(-1, 3)
    out = np.zeros((P.shape[0], 2))
    c = OrcCamera.from_cam(cam)
    lib().orc_project(ctypes.byref(c), _p(_f64(np.asarray(R).ravel())), _p(_f64(t)), _p(P),
                      ctypes.c_int(P.shape[0]), _p(out))
    return out


def knn2(desc_a, desc_b, dtype: int, nthreads: int = 0):
    a = np.ascontiguousarray(desc_a)
    b = np.ascontiguousarray(desc_b)
    n_a, dim = a.shape
    idx = np.zeros((n_a, 2), dtype=np.int32)
    dist = np.zeros((n_a, 2), dtype=np.float32)
    lib().orc_knn2(ctypes.c_int(dtype), a.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(n_a),
                   b.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(b.shape[0]), ctypes.c_int(dim),
                   _p(idx, ctypes.c_int), _p(dist, ctypes.c_float), ctypes.c_int(nthreads))
    return idx, dist


def nndr(idx, dist, eps: float):
    n_a = idx.shape[0]
    q = np.zeros(n_a, dtype=np.int32)
    t = np.zeros(n_a, dtype=np.int32)
    d = np.zeros(n_a, dtype=np.float32)
    n = lib().orc_nndr(_p(np.ascontiguousarray(idx, dtype=np.int32), ctypes.c_int),
                       _p(np.ascontiguousarray(dist, dtype=np.float32), ctypes.c_float), ctypes.c_int(n_a),
                       ctypes.c_double(eps), _p(q, ctypes.c_int), _p(t, ctypes.c_int), _p(d, ctypes.c_float))
    return q[:n], t[:n], d[:n]


def match_nndr(desc_a, desc_b, dtype: int, eps: float, nthreads: int = 0):
    idx, dist = knn2(desc_a, desc_b, dtype, nthreads)
    return nndr(idx, dist, eps)


def triangulate(cam, g12, zmin, zmax, kp1, kp2, query, train):
    K = len(query)
    mask = np.zeros(K, dtype=np.uint8)
    pts = np.zeros((max(K, 1), 3))
    c = OrcCamera.from_cam(cam)
    n = lib().orc_triangulate(ctypes.byref(c), _p(_f64(np.asarray(g12).ravel())), ctypes.c_double(zmin),
                              ctypes.c_double(zmax), _p(np.ascontiguousarray(kp1, dtype=np.float32), ctypes.c_float),
                              _p(np.ascontiguousarray(kp2, dtype=np.float32), ctypes.c_float),
                              _p(np.ascontiguousarray(query, dtype=np.int32), ctypes.c_int),
                              _p(np.ascontiguousarray(train, dtype=np.int32), ctypes.c_int), ctypes.c_int(K),
                              _p(mask, ctypes.c_uint8), _p(pts))
    return pts[:n].copy(), mask.astype(bool)


def triangulate1(g12, u1, u2):
    X = np.zeros(4)
    lib().orc_triangulate1(_p(_f64(np.asarray(g12).ravel())), _p(_f64(u1)), _p(_f64(u2)), _p(X))
    return X


def pyrdown(img):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    out = np.zeros(((h + 1) // 2, (w + 1) // 2), dtype=np.uint8)
    lib().orc_pyrdown(_p(img, ctypes.c_uint8), ctypes.c_int(w), ctypes.c_int(h), _p(out, ctypes.c_uint8))
    return out


def bilinear(img, x, y):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    f = lib().orc_bilinear_sample
    f.restype = ctypes.c_float
    return f(_p(img, ctypes.c_uint8), ctypes.c_int(w), ctypes.c_int(h), ctypes.c_float(x), ctypes.c_float(y))


def neighborhood(cam, X, ray, bound_w=1024, bound_h=768):
    cap = (2 * ray + 1) ** 2
    out = np.zeros((cap, 2))
    c = OrcCamera.from_cam(cam)
    n = lib().orc_neighborhood(ctypes.byref(c), _p(_f64(X)), ctypes.c_int(ray), ctypes.c_int(bound_w),
                               ctypes.c_int(bound_h), _p(out), ctypes.c_int(cap))
    return out[:n].copy()


def plane_to_image2(cam, R2, t2, X, n, pix, zmax=2.4, size=None):
    """orc_plane_to_image2: image-1 pixels through the plane (X, n) into image 2 at level 0
    (get3dPointsFromImage1Pixels + projectPointsToImage2): (uv (m, 2), status (m,))."""
    pix = _f64(pix).reshape(-1, 2)
    m = pix.shape[0]
    uv = np.zeros((max(m, 1), 2))
    st = np.zeros(max(m, 1), dtype=np.int32)
    w, h = size if size is not None else (0, 0)
    c = OrcCamera.from_cam(cam)
    lib().orc_plane_to_image2(ctypes.byref(c), _p(_f64(np.asarray(R2).ravel())), _p(_f64(t2)), _p(_f64(X)), _p(_f64(n)),
                              _p(pix), ctypes.c_int(m), ctypes.c_double(zmax), ctypes.c_int(w), ctypes.c_int(h), _p(uv),
                              _p(st, ctypes.c_int))
    return uv[:m], st[:m]


def sample_points(img, uv):
    """orc_sample_points: the (uchar) bilinear patch sample at each uv (0 where isPixelGood fails)."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    uv = _f64(uv).reshape(-1, 2)
    out = np.zeros(max(len(uv), 1), dtype=np.uint8)
    lib().orc_sample_points(_p(img, ctypes.c_uint8), ctypes.c_int(w), ctypes.c_int(h), _p(uv), ctypes.c_int(len(uv)),
                            _p(out, ctypes.c_uint8))
    return out[:len(uv)]


def optimize_normals(cam, R2, t2, img1, img2, levels, points, ray, bound_w=1024, bound_h=768,
                     epsfcn=1e-10, zmax=2.4, mode=STRICT, nthreads=0):
    img1 = np.ascontiguousarray(img1, dtype=np.uint8)
    img2 = np.ascontiguousarray(img2, dtype=np.uint8)
    h, w = img1.shape
    P = _f64(points).reshape(-1, 3)
    n = P.shape[0]
    normals = np.zeros((n, 3))
    status = np.zeros(n, dtype=np.int32)
    info = np.zeros((n, 8), dtype=np.int32)
    nfev = np.zeros((n, 8), dtype=np.int32)
    mdat = np.zeros(n, dtype=np.int32)
    c = OrcCamera.from_cam(cam)
    lib().orc_optimize_normals(ctypes.byref(c), _p(_f64(np.asarray(R2).ravel())), _p(_f64(t2)),
                               _p(img1, ctypes.c_uint8), _p(img2, ctypes.c_uint8), ctypes.c_int(w), ctypes.c_int(h),
                               ctypes.c_int(levels), _p(P), ctypes.c_int(n), ctypes.c_int(ray), ctypes.c_int(bound_w),
                               ctypes.c_int(bound_h), ctypes.c_double(epsfcn), ctypes.c_double(zmax),
                               ctypes.c_int(mode), _p(normals), _p(status, ctypes.c_int),
                               _p(info, ctypes.c_int), _p(nfev, ctypes.c_int), _p(mdat, ctypes.c_int),
                               ctypes.c_int(nthreads))
    return dict(normals=normals, status=status, info=info, nfev=nfev, mdat=mdat)


def eval_residual(cam, R2, t2, img1, img2, X, pix, par, zmax=2.4, mode=STRICT):
    img1 = np.ascontiguousarray(img1, dtype=np.uint8)
    img2 = np.ascontiguousarray(img2, dtype=np.uint8)
    h, w = img1.shape
    pix = _f64(pix).reshape(-1, 2)
    f = np.zeros(pix.shape[0])
    c = OrcCamera.from_cam(cam)
    st = lib().orc_eval_residual(ctypes.byref(c), _p(_f64(np.asarray(R2).ravel())), _p(_f64(t2)),
                                 _p(img1, ctypes.c_uint8), _p(img2, ctypes.c_uint8), ctypes.c_int(w), ctypes.c_int(h),
                                 _p(_f64(X)), _p(pix), ctypes.c_int(pix.shape[0]), ctypes.c_double(zmax),
                                 ctypes.c_int(mode), _p(_f64(par)), _p(f))
    return st, f


def lm_single_level(cam, R2, t2, img1, img2, X, pix, par0, epsfcn=1e-10, zmax=2.4, mode=STRICT):
    img1 = np.ascontiguousarray(img1, dtype=np.uint8)
    img2 = np.ascontiguousarray(img2, dtype=np.uint8)
    h, w = img1.shape
    pix = _f64(pix).reshape(-1, 2)
    par = _f64(par0).copy()
    nfev = ctypes.c_int(0)
    c = OrcCamera.from_cam(cam)
    info = lib().orc_lm_single_level(ctypes.byref(c), _p(_f64(np.asarray(R2).ravel())), _p(_f64(t2)),
                                     _p(img1, ctypes.c_uint8), _p(img2, ctypes.c_uint8), ctypes.c_int(w),
                                     ctypes.c_int(h), _p(_f64(X)), _p(pix), ctypes.c_int(pix.shape[0]),
                                     ctypes.c_double(epsfcn), ctypes.c_double(zmax), ctypes.c_int(mode),
                                     _p(par), ctypes.byref(nfev))
    return info, par, nfev.value


def gravity(rIC):
    g = np.zeros(3)
    lib().orc_gravity(_p(_f64(rIC)), _p(g))
    return g


def features_frames(points, normals, g):
    P = _f64(points).reshape(-1, 3)
    N = _f64(normals).reshape(-1, 3)
    frames = np.zeros((P.shape[0], 4, 4))
    lib().orc_features_frames(_p(P), _p(N), ctypes.c_int(P.shape[0]), _p(_f64(g)), _p(frames))
    return frames


def patch_size(eps, cmpp):
    return lib().orc_patch_size(ctypes.c_double(eps), ctypes.c_double(cmpp))


def square_neighborhoods(frames, eps=0.16, cmpp=0.25):
    """computeSquareNeighborhoodsByNormals (neighborhoodsgenerator.cpp:76-132): (P, size*size, 3)."""
    F = _f64(frames).reshape(-1, 16)
    n = F.shape[0]
    size = patch_size(eps, cmpp)
    out = np.zeros((n, max(size, 0) ** 2, 3))
    lib().orc_square_neighborhoods(_p(F), ctypes.c_int(n), ctypes.c_double(eps), ctypes.c_double(cmpp), _p(out))
    return out


def circular_neighborhoods(points, normals=None, eps=0.16, thetas=15, rays=5):
    """computeCircularNeighborhoodsByNormals (neighborhoodsgenerator.cpp:160-224): (P, thetas*rays, 3);
    normals None -> the initial guess X/|X|."""
    X = _f64(points).reshape(-1, 3)
    n = X.shape[0]
    N = _f64(normals).reshape(-1, 3) if normals is not None else None
    out = np.zeros((n, thetas * rays, 3))
    lib().orc_circular_neighborhoods(_p(X), _p(N) if N is not None else None, ctypes.c_int(n), ctypes.c_double(eps),
                                     ctypes.c_int(thetas), ctypes.c_int(rays), _p(out))
    return out


def ncc_hypotheses(cam, R2, t2, img1, img2, points, ray, hphi=4, htheta=4, span=0.4, bound=(1024, 768), zmax=2.4):
    """NCC scoring of hphi x htheta candidate normals per point (the GPU's fm3d_ncc_hypotheses):
    (scores (P, H), best normals (P, 3), best index (P,))."""
    X = _f64(points).reshape(-1, 3)
    n = X.shape[0]
    img1 = np.ascontiguousarray(img1, dtype=np.uint8)
    img2 = np.ascontiguousarray(img2, dtype=np.uint8)
    h, w = img1.shape
    H = hphi * htheta
    scores = np.zeros((max(n, 1), H))
    normals = np.zeros((max(n, 1), 3))
    best = np.zeros(max(n, 1), dtype=np.int32)
    c = OrcCamera.from_cam(cam)
    lib().orc_ncc_hypotheses(ctypes.byref(c), _p(_f64(R2)), _p(_f64(t2)), _p(img1, ctypes.c_uint8),
                             _p(img2, ctypes.c_uint8), ctypes.c_int(w), ctypes.c_int(h), _p(X), ctypes.c_int(n),
                             ctypes.c_int(ray), ctypes.c_int(bound[0]), ctypes.c_int(bound[1]), ctypes.c_double(zmax),
                             ctypes.c_int(hphi), ctypes.c_int(htheta), ctypes.c_double(span), _p(scores), _p(normals),
                             _p(best, ctypes.c_int))
    return scores[:n], normals[:n], best[:n]


def export_patches(cam, img1, frames, eps=0.16, cmpp=0.25, mode=STRICT, image_points=False):
    img1 = np.ascontiguousarray(img1, dtype=np.uint8)
    h, w = img1.shape
    F = _f64(frames).reshape(-1, 16)
    n = F.shape[0]
    size = patch_size(eps, cmpp)
    patches = np.zeros((n, size, size), dtype=np.uint8)
    pts = np.zeros((n, size * size, 2)) if image_points else None
    c = OrcCamera.from_cam(cam)
    lib().orc_export_patches(ctypes.byref(c), _p(img1, ctypes.c_uint8), ctypes.c_int(w), ctypes.c_int(h), _p(F),
                             ctypes.c_int(n), ctypes.c_double(eps), ctypes.c_double(cmpp), ctypes.c_int(mode),
                             _p(patches, ctypes.c_uint8), _p(pts) if pts is not None else None)
    return (patches, pts) if image_points else patches


# ---------------------------------------------------------------- SURF (orc_surf.c)
KEYPOINT = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                     ("octave", "<i4"), ("class_id", "<i4")])  # cv::KeyPoint


def integral(img):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    out = np.zeros((h + 1, w + 1), dtype=np.int32)
    lib().orc_integral(_p(img, ctypes.c_uint8), ctypes.c_int(w), ctypes.c_int(h), _p(out, ctypes.c_int))
    return out


def surf_detect(img, thr=400.0, octaves=4, layers=2, upright=True):
    """SURF detect (fastHessianDetector + the detect pass of SURFInvoker: upright angle, or the
    dominant orientation with upright False): cv::KeyPoint records, sorted."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    f = lib().orc_surf_detect2
    f.restype = ctypes.c_int
    args = (_p(img, ctypes.c_uint8), ctypes.c_int(w), ctypes.c_int(h), ctypes.c_float(thr), ctypes.c_int(octaves),
            ctypes.c_int(layers), ctypes.c_int(1 if upright else 0))
    n = f(*args, None, ctypes.c_int(0))
    out = np.zeros(max(n, 1), dtype=KEYPOINT)
    f(*args, out.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(n))
    return out[:n]


def surf_describe(img, kpts, extended=True, upright=True):
    """SURF compute (upright, or oriented with upright False): (kept keypoints, input index of each,
    descriptors n x 128|64 float32)."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    kin = np.ascontiguousarray(kpts, dtype=KEYPOINT)
    n = len(kin)
    kout = np.zeros(max(n, 1), dtype=KEYPOINT)
    kept = np.zeros(max(n, 1), dtype=np.int32)
    desc = np.zeros((max(n, 1), 128 if extended else 64), dtype=np.float32)
    f = lib().orc_surf_describe2
    f.restype = ctypes.c_int
    m = f(_p(img, ctypes.c_uint8), ctypes.c_int(w), ctypes.c_int(h), kin.ctypes.data_as(ctypes.c_void_p),
          ctypes.c_int(n), ctypes.c_int(1 if extended else 0), ctypes.c_int(1 if upright else 0),
          kout.ctypes.data_as(ctypes.c_void_p),
          _p(kept, ctypes.c_int), _p(desc, ctypes.c_float))
    if m < 0:
        raise ValueError("SURF describe: a keypoint of size < 0.36 (an empty window; OpenCV's resize asserts)")
    return kout[:m], kept[:m], desc[:m]


def resize_area_up(win, D=21):
    """resize(win, (D, D), INTER_AREA) of a W x W window with W < D: OpenCV's linear emulation"""
    win = np.ascontiguousarray(win, dtype=np.uint8)
    W = win.shape[0]
    out = np.zeros((D, D), np.uint8)
    lib().orc_resize_area_up(_p(win, ctypes.c_uint8), ctypes.c_int(W), ctypes.c_int(D), _p(out, ctypes.c_uint8))
    return out


def fast_atan2(y, x):
    f = lib().orc_fast_atan2
    f.restype = ctypes.c_float
    return f(ctypes.c_float(y), ctypes.c_float(x))


def surf_ori_samples():
    """SURFInvoker's orientation disc: (apt (n, 2) int, aptw (n,) float32)"""
    apt = np.zeros((169, 2), dtype=np.int32)
    aptw = np.zeros(169, dtype=np.float32)
    n = lib().orc_surf_ori_samples(_p(apt, ctypes.c_int), _p(aptw, ctypes.c_float))
    return apt[:n], aptw[:n]


def surf_dw():
    dw = np.zeros(400, dtype=np.float32)
    lib().orc_surf_dw(_p(dw, ctypes.c_float))
    return dw.reshape(20, 20)


def resize_area21(win):
    win = np.ascontiguousarray(win, dtype=np.uint8)
    out = np.zeros((21, 21), dtype=np.uint8)
    lib().orc_resize_area21(_p(win, ctypes.c_uint8), ctypes.c_int(win.shape[0]), _p(out, ctypes.c_uint8))
    return out


# ---------------------------------------------------------------- ORB (orc_orb.c)
ORB_DEFAULTS = dict(nfeatures=500, scaleFactor=1.2, nlevels=8, edgeThreshold=31, patchSize=31, fastThreshold=20)


def _kp(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def orb_scale(scaleFactor, level):
    f = lib().orc_orb_scale
    f.restype = ctypes.c_float
    return f(ctypes.c_double(scaleFactor), ctypes.c_int(level))


def orb_level_size(w, h, scaleFactor, level):
    lw, lh = ctypes.c_int(0), ctypes.c_int(0)
    lib().orc_orb_level_size(ctypes.c_int(w), ctypes.c_int(h), ctypes.c_double(scaleFactor), ctypes.c_int(level),
                             ctypes.byref(lw), ctypes.byref(lh))
    return lw.value, lh.value


def orb_resize(src, dw, dh):
    src = np.ascontiguousarray(src, dtype=np.uint8)
    out = np.zeros((dh, dw), dtype=np.uint8)
    lib().orc_orb_resize(_p(src, ctypes.c_uint8), ctypes.c_int(src.shape[1]), ctypes.c_int(src.shape[0]),
                         _p(out, ctypes.c_uint8), ctypes.c_int(dw), ctypes.c_int(dh))
    return out


def vresize_sse_end(width):
    return lib().orc_vresize_sse_end(ctypes.c_int(width))


def fast9(img, thr=20):
    """FAST(img, kpts, thr, true): KEYPOINT records in raster order"""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    n = lib().orc_fast9(_p(img, ctypes.c_uint8), ctypes.c_int(w), ctypes.c_int(h), ctypes.c_int(thr), None, 0)
    out = np.zeros(max(n, 1), dtype=KEYPOINT)
    lib().orc_fast9(_p(img, ctypes.c_uint8), ctypes.c_int(w), ctypes.c_int(h), ctypes.c_int(thr), _kp(out),
                    ctypes.c_int(n))
    return out[:n]


def fast_detect(img, thr=10, nonmax=True):
    """FastFeatureDetector(thr, nonmax).detect(img): KEYPOINT records in raster order"""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    args = (_p(img, ctypes.c_uint8), ctypes.c_int(w), ctypes.c_int(h), ctypes.c_int(thr), ctypes.c_int(1 if nonmax else 0))
    n = lib().orc_fast_detect(*args, None, 0)
    out = np.zeros(max(n, 1), dtype=KEYPOINT)
    lib().orc_fast_detect(*args, _kp(out), ctypes.c_int(n))
    return out[:n]


def nth_element(kpts, nth):
    """std::nth_element(k, k + nth, k + n, KeypointResponseGreater()) on a copy"""
    k = np.ascontiguousarray(kpts, dtype=KEYPOINT).copy()
    lib().orc_nth_element(_kp(k), ctypes.c_long(nth), ctypes.c_long(len(k)))
    return k


def partition_ge(kpts, lo, hi, thr):
    """std::partition(k + lo, k + hi, response >= thr) on a copy: (array, split index)"""
    k = np.ascontiguousarray(kpts, dtype=KEYPOINT).copy()
    f = lib().orc_partition_ge
    f.restype = ctypes.c_long
    m = f(_kp(k), ctypes.c_long(lo), ctypes.c_long(hi), ctypes.c_float(thr))
    return k, int(m)


def retain_best(kpts, npts):
    k = np.ascontiguousarray(kpts, dtype=KEYPOINT).copy()
    m = lib().orc_retain_best(_kp(k), ctypes.c_int(len(k)), ctypes.c_int(npts))
    return k[:m]


def harris(img, kpts, block=7, k=0.04):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    kk = np.ascontiguousarray(kpts, dtype=KEYPOINT).copy()
    lib().orc_harris(_p(img, ctypes.c_uint8), ctypes.c_int(img.shape[1]), _kp(kk), ctypes.c_int(len(kk)),
                     ctypes.c_int(block), ctypes.c_float(k))
    return kk["response"]


def orb_umax(half):
    u = np.zeros(half + 2, dtype=np.int32)
    lib().orc_orb_umax(ctypes.c_int(half), _p(u, ctypes.c_int))
    return u


def ic_angle(img, half, x, y):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    u = orb_umax(half)
    f = lib().orc_ic_angle
    f.restype = ctypes.c_float
    return f(_p(img, ctypes.c_uint8), ctypes.c_int(img.shape[1]), ctypes.c_int(half), ctypes.c_float(x),
             ctypes.c_float(y), _p(u, ctypes.c_int))


def orb_blur_kernel():
    k = np.zeros(7, dtype=np.int32)
    lib().orc_orb_blur_kernel(_p(k, ctypes.c_int))
    return k


def orb_blur(img):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    out = np.zeros_like(img)
    lib().orc_orb_blur(_p(img, ctypes.c_uint8), ctypes.c_int(img.shape[1]), ctypes.c_int(img.shape[0]),
                       _p(out, ctypes.c_uint8))
    return out


def orb_random_pattern(patchSize=31, npoints=512):
    xy = np.zeros((npoints, 2), dtype=np.int32)
    lib().orc_orb_random_pattern(ctypes.c_int(patchSize), _p(xy, ctypes.c_int), ctypes.c_int(npoints))
    return xy


def _pattern(pattern, patchSize):
    if pattern is None:
        return orb_random_pattern(patchSize)
    p = np.ascontiguousarray(pattern, dtype=np.int32).reshape(512, 2)
    return p


def orb_detect(img, nfeatures=500, scaleFactor=1.2, nlevels=8, edgeThreshold=31, patchSize=31, fastThreshold=20,
               pattern=None, descriptors=True):
    """ORB::operator()(img, noArray(), kpts, desc): (KEYPOINT records level-major, (n, 32) uint8
    descriptors or None)"""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    pat = _pattern(pattern, patchSize)
    args = (_p(img, ctypes.c_uint8), ctypes.c_int(w), ctypes.c_int(h), ctypes.c_int(nfeatures),
            ctypes.c_double(scaleFactor), ctypes.c_int(nlevels), ctypes.c_int(edgeThreshold), ctypes.c_int(patchSize),
            ctypes.c_int(fastThreshold), _p(pat, ctypes.c_int))
    n = lib().orc_orb_detect(*args, None, None, ctypes.c_int(0))
    out = np.zeros(max(n, 1), dtype=KEYPOINT)
    d = np.zeros((max(n, 1), 32), dtype=np.uint8)
    lib().orc_orb_detect(*args, _kp(out), _p(d, ctypes.c_uint8) if descriptors else None, ctypes.c_int(n))
    return out[:n], (d[:n] if descriptors else None)


def orb_compute(img, kpts, scaleFactor=1.2, edgeThreshold=31, patchSize=31, pattern=None):
    """ORB::compute on given keypoints: (kept keypoints level-major, input index of each, (m, 32)
    uint8 descriptors)"""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    kin = np.ascontiguousarray(kpts, dtype=KEYPOINT)
    n = len(kin)
    kout = np.zeros(max(n, 1), dtype=KEYPOINT)
    kept = np.zeros(max(n, 1), dtype=np.int32)
    d = np.zeros((max(n, 1), 32), dtype=np.uint8)
    pat = _pattern(pattern, patchSize)
    m = lib().orc_orb_compute(_p(img, ctypes.c_uint8), ctypes.c_int(w), ctypes.c_int(h), _kp(kin), ctypes.c_int(n),
                              ctypes.c_double(scaleFactor), ctypes.c_int(edgeThreshold), ctypes.c_int(patchSize),
                              _p(pat, ctypes.c_int), _kp(kout), _p(kept, ctypes.c_int), _p(d, ctypes.c_uint8))
    if m < 0:
        raise ValueError("ORB compute: a keypoint with a negative octave (OpenCV indexes allKeypoints[-1])")
    return kout[:m], kept[:m], d[:m]


# ---------------------------------------------------------------- SIFT (orc_sift.c)
SIFT_DEFAULTS = dict(nfeatures=0, nOctaveLayers=3, contrastThreshold=0.04, edgeThreshold=10.0, sigma=1.6)


def _fn(name, restype):
    f = getattr(lib(), name)
    f.restype = restype
    return f


def cv_exp_at(x, k, n):
    """element k of cv::exp over an array of n floats (SSE2 loop or scalar loop by position)"""
    return _fn("orc_cv_exp_at", ctypes.c_float)(ctypes.c_float(x), ctypes.c_int(k), ctypes.c_int(n))


def cv_exp2f(y):
    return _fn("orc_cv_exp2f", ctypes.c_float)(ctypes.c_float(y))


def cv_cosf(x):
    return _fn("orc_cv_cosf", ctypes.c_float)(ctypes.c_float(x))


def cv_sinf(x):
    return _fn("orc_cv_sinf", ctypes.c_float)(ctypes.c_float(x))


def cv_atan2_deg(y, x):
    return _fn("orc_cv_atan2_deg", ctypes.c_float)(ctypes.c_float(y), ctypes.c_float(x))


def sift_gauss_kernel(sigma):
    n = lib().orc_sift_gauss_ksize(ctypes.c_double(sigma))
    k = np.zeros(n, dtype=np.float32)
    lib().orc_sift_gauss_kernel(ctypes.c_double(sigma), _p(k, ctypes.c_float))
    return k


def sift_blur(img, sigma):
    """GaussianBlur(img, Size(), sigma) of a float32 image"""
    img = np.ascontiguousarray(img, dtype=np.float32)
    out = np.zeros_like(img)
    lib().orc_sift_blur(_p(img, ctypes.c_float), _p(out, ctypes.c_float), ctypes.c_int(img.shape[1]),
                        ctypes.c_int(img.shape[0]), ctypes.c_double(sigma))
    return out


def sift_resize_linear(img, dw, dh):
    img = np.ascontiguousarray(img, dtype=np.float32)
    out = np.zeros((dh, dw), dtype=np.float32)
    lib().orc_sift_resize_linear(_p(img, ctypes.c_float), ctypes.c_int(img.shape[1]), ctypes.c_int(img.shape[0]),
                                 _p(out, ctypes.c_float), ctypes.c_int(dw), ctypes.c_int(dh))
    return out


def sift_resize_nn(img, dw, dh):
    img = np.ascontiguousarray(img, dtype=np.float32)
    out = np.zeros((dh, dw), dtype=np.float32)
    lib().orc_sift_resize_nn(_p(img, ctypes.c_float), ctypes.c_int(img.shape[1]), ctypes.c_int(img.shape[0]),
                             _p(out, ctypes.c_float), ctypes.c_int(dw), ctypes.c_int(dh))
    return out


def sift_num_octaves(w, h, first_octave=-1):
    return lib().orc_sift_num_octaves(ctypes.c_int(w), ctypes.c_int(h), ctypes.c_int(first_octave))


def sift_sigmas(layers=3, sigma=1.6):
    s = np.zeros(layers + 3)
    lib().orc_sift_sigmas(ctypes.c_int(layers), ctypes.c_double(sigma), _p(s))
    return s


def sift_pyramid(img, first_octave=-1, octaves=None, layers=3, sigma=1.6, dog=False):
    """the Gaussian (or DoG) pyramid levels, octave-major: a list of float32 images"""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    if octaves is None:
        octaves = sift_num_octaves(w, h, first_octave)
    f = _fn("orc_sift_pyramid", ctypes.c_long)
    args = (_p(img, ctypes.c_uint8), ctypes.c_int(w), ctypes.c_int(h), ctypes.c_int(first_octave),
            ctypes.c_int(octaves), ctypes.c_int(layers), ctypes.c_double(sigma), ctypes.c_int(1 if dog else 0))
    tot = f(*args, None, None)
    if tot < 0:
        raise ValueError("SIFT pyramid: an octave would be empty")
    nl = octaves * (layers + 2 if dog else layers + 3)
    out = np.zeros(max(tot, 1), dtype=np.float32)
    sizes = np.zeros(2 * nl, dtype=np.int32)
    f(*args, _p(out, ctypes.c_float), _p(sizes, ctypes.c_int))
    levels, o = [], 0
    for i in range(nl):
        lw, lh = int(sizes[2 * i]), int(sizes[2 * i + 1])
        levels.append(out[o:o + lw * lh].reshape(lh, lw))
        o += lw * lh
    return levels


def sift_solve3(H, b):
    H = np.ascontiguousarray(H, dtype=np.float32).ravel()
    b = np.ascontiguousarray(b, dtype=np.float32)
    x = np.zeros(3, dtype=np.float32)
    lib().orc_sift_solve3(_p(H, ctypes.c_float), _p(b, ctypes.c_float), _p(x, ctypes.c_float))
    return x


def sift_ori_hist(level, x, y, radius, sigma, n=36):
    level = np.ascontiguousarray(level, dtype=np.float32)
    hist = np.zeros(n, dtype=np.float32)
    f = _fn("orc_sift_ori_hist", ctypes.c_float)
    m = f(_p(level, ctypes.c_float), ctypes.c_int(level.shape[1]), ctypes.c_int(level.shape[0]), ctypes.c_int(x),
          ctypes.c_int(y), ctypes.c_int(radius), ctypes.c_float(sigma), _p(hist, ctypes.c_float), ctypes.c_int(n))
    return m, hist


def sift_descriptor(level, x, y, ori, scl):
    level = np.ascontiguousarray(level, dtype=np.float32)
    d = np.zeros(128, dtype=np.float32)
    lib().orc_sift_descriptor(_p(level, ctypes.c_float), ctypes.c_int(level.shape[1]), ctypes.c_int(level.shape[0]),
                              ctypes.c_float(x), ctypes.c_float(y), ctypes.c_float(ori), ctypes.c_float(scl),
                              _p(d, ctypes.c_float))
    return d


def remove_duplicated(kpts):
    k = np.ascontiguousarray(kpts, dtype=KEYPOINT).copy()
    m = lib().orc_remove_duplicated(_kp(k), ctypes.c_int(len(k)))
    return k[:m]


def sift_detect(img, nfeatures=0, nOctaveLayers=3, contrastThreshold=0.04, edgeThreshold=10.0, sigma=1.6, raw=False):
    """FeatureDetector::detect with cv::SIFT: KEYPOINT records (raw: the findScaleSpaceExtrema list in
    doubled-image coordinates, before removeDuplicated / retainBest)"""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    args = (_p(img, ctypes.c_uint8), ctypes.c_int(w), ctypes.c_int(h), ctypes.c_int(nfeatures),
            ctypes.c_int(nOctaveLayers), ctypes.c_double(contrastThreshold), ctypes.c_double(edgeThreshold),
            ctypes.c_double(sigma), ctypes.c_int(1 if raw else 0))
    n = lib().orc_sift_detect(*args, None, ctypes.c_int(0))
    if n < 0:
        raise ValueError("SIFT detect: an octave would be empty")
    out = np.zeros(max(n, 1), dtype=KEYPOINT)
    lib().orc_sift_detect(*args, _kp(out), ctypes.c_int(n))
    return out[:n]


def sift_compute(img, kpts, nOctaveLayers=3, sigma=1.6):
    """DescriptorExtractor::compute with cv::SIFT: (kept keypoints, input index of each, (m, 128)
    float32 descriptors holding integers 0..255)"""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    kin = np.ascontiguousarray(kpts, dtype=KEYPOINT)
    n = len(kin)
    kout = np.zeros(max(n, 1), dtype=KEYPOINT)
    kept = np.zeros(max(n, 1), dtype=np.int32)
    d = np.zeros((max(n, 1), 128), dtype=np.float32)
    m = lib().orc_sift_compute(_p(img, ctypes.c_uint8), ctypes.c_int(w), ctypes.c_int(h), ctypes.c_int(nOctaveLayers),
                               ctypes.c_double(sigma), _kp(kin), ctypes.c_int(n), _kp(kout), _p(kept, ctypes.c_int),
                               _p(d, ctypes.c_float))
    if m < 0:
        raise ValueError("SIFT compute: OpenCV asserts (octave < -1, layer > nOctaveLayers + 2, or an empty octave)")
    return kout[:m], kept[:m], d[:m]


# ---------------------------------------------------------------- DynamicAdaptedFeatureDetector
def adaptive_detect(img, kind, min_features=400, max_features=500, max_iters=5):
    """DynamicAdaptedFeatureDetector(AdjusterAdapter::create(kind), min, max, iters)::detect
    (OpenCV 2.4 features2d/src/dynamic.cpp): FastAdjuster(20, true, 1, 200) steps the FAST threshold by
    one; SurfAdjuster(400, 2, 1000) runs the default SURF (4 octaves, 2 layers, not upright) and scales
    its Hessian threshold by 0.9 (floored at 1.1) / 1.1; StarAdjuster(30, 2, 200) runs
    StarFeatureDetector(16, cvRound(thresh), 10, 8, 3) with the same scaling.  Returns the last call's
    keypoints."""
    fast = kind == "FAST"
    thresh, lo, hi = {"FAST": (20, 1, 200), "SURF": (400.0, 2, 1000), "STAR": (30.0, 2, 200)}[kind]
    down = up = good = False
    it = max_iters
    k = np.zeros(0, dtype=KEYPOINT)
    while it > 0 and not (down and up) and not good and lo < thresh < hi:
        if fast:
            k = fast_detect(img, int(thresh), True)
        elif kind == "SURF":
            k = surf_detect(img, float(thresh), 4, 2, upright=False)
        else:  # StarAdjuster: StarFeatureDetector(16, cvRound(thresh), 10, 8, 3)
            k = star_detect(img, 16, int(np.rint(thresh)), 10, 8, 3)
        if len(k) < min_features:
            down = True
            if fast:
                thresh -= 1
            else:
                thresh *= 0.9
                if thresh < 1.1:
                    thresh = 1.1
        elif len(k) > max_features:
            up = True
            if fast:
                thresh += 1
            else:
                thresh *= 1.1
        else:
            good = True
        it -= 1
    return k


def star_integrals(img):
    """computeIntegralImages (stardetector.cpp): (S, T, F), (h+1, w+1) int32 each"""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    S, T, F = (np.zeros((h + 1, w + 1), np.int32) for _ in range(3))
    lib().orc_star_integrals(_p(img, ctypes.c_uint8), ctypes.c_int(w), ctypes.c_int(h), _p(S, ctypes.c_int),
                             _p(T, ctypes.c_int), _p(F, ctypes.c_int))
    return S, T, F


def star_patterns(w, h, max_size=45):
    """(npairs, maxIdx, border, signed sizes, (17, 8) integral offsets, (12, 2) reciprocal areas)"""
    mi, b = ctypes.c_int(0), ctypes.c_int(0)
    sz = np.zeros(17, np.int32)
    ofs = np.zeros((17, 8), np.int32)
    inv = np.zeros((12, 2), np.float32)
    n = lib().orc_star_patterns(ctypes.c_int(w), ctypes.c_int(h), ctypes.c_int(max_size), ctypes.byref(mi),
                                ctypes.byref(b), _p(sz, ctypes.c_int), _p(ofs, ctypes.c_int), _p(inv, ctypes.c_float))
    return n, mi.value, b.value, sz, ofs, inv


def star_responses(img, max_size=45):
    """StarDetectorComputeResponses: (border, float32 responses, int16 sizes); border -1 if undefined"""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    R = np.zeros((h, w), np.float32)
    Z = np.zeros((h, w), np.int16)
    b = lib().orc_star_responses(_p(img, ctypes.c_uint8), ctypes.c_int(w), ctypes.c_int(h), ctypes.c_int(max_size),
                                 _p(R, ctypes.c_float), _p(Z, ctypes.c_short))
    return b, R, Z


def star_detect(img, max_size=45, response=30, line_proj=10, line_bin=8, suppression=5):
    """StarFeatureDetector(maxSize, responseThreshold, lineThresholdProjected, lineThresholdBinarized,
    suppressNonmaxSize).detect(img): KEYPOINT records in tile order"""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    args = (_p(img, ctypes.c_uint8), ctypes.c_int(w), ctypes.c_int(h), ctypes.c_int(max_size), ctypes.c_int(response),
            ctypes.c_int(line_proj), ctypes.c_int(line_bin), ctypes.c_int(suppression))
    n = lib().orc_star_detect(*args, None, ctypes.c_int(0))
    if n < 0:
        raise ValueError("STAR detect: undefined for this image size / MaxSize / Suppression")
    out = np.zeros(max(n, 1), dtype=KEYPOINT)
    lib().orc_star_detect(*args, _kp(out), ctypes.c_int(n))
    return out[:n]


def brisk_point(scale, rot, i):
    """BRISK generateKernel's point i at (scale, rotation): (x, y, sigma) float32"""
    x, y, s = ctypes.c_float(0), ctypes.c_float(0), ctypes.c_float(0)
    lib().orc_brisk_point(ctypes.c_int(scale), ctypes.c_int(rot), ctypes.c_int(i), ctypes.byref(x), ctypes.byref(y),
                          ctypes.byref(s))
    return np.float32(x.value), np.float32(y.value), np.float32(s.value)


def brisk_scale_factor(scale):
    return np.float32(_fn("orc_brisk_scale_factor", ctypes.c_float)(ctypes.c_int(scale)))


def brisk_size(scale):
    return int(lib().orc_brisk_size(ctypes.c_int(scale)))


def brisk_short_pairs():
    """(i, j) of the short pairs in generation order"""
    pi = np.zeros(1770, np.int32)
    pj = np.zeros(1770, np.int32)
    n = lib().orc_brisk_short_pairs(_p(pi, ctypes.c_int), _p(pj, ctypes.c_int))
    return pi[:n], pj[:n]


def brisk_kscale(size):
    return int(lib().orc_brisk_kscale(ctypes.c_float(size)))


def brisk_theta(angle):
    return int(lib().orc_brisk_theta(ctypes.c_float(angle)))


def brisk_intensity(img, kx, ky, px, py, sigma):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    return int(lib().orc_brisk_intensity(_p(img, ctypes.c_uint8), None, ctypes.c_int(img.shape[1]), ctypes.c_float(kx),
                                         ctypes.c_float(ky), ctypes.c_float(px), ctypes.c_float(py),
                                         ctypes.c_float(sigma)))


def brisk_compute(img, kpts):
    """DescriptorExtractor::compute with cv::BRISK (provided keypoints): (kept keypoints, input index of
    each, (m, 64) uint8 descriptors)"""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    kin = np.ascontiguousarray(kpts, dtype=KEYPOINT)
    n = len(kin)
    kout = np.zeros(max(n, 1), dtype=KEYPOINT)
    kept = np.zeros(max(n, 1), dtype=np.int32)
    desc = np.zeros((max(n, 1), 64), dtype=np.uint8)
    m = lib().orc_brisk_compute(_p(img, ctypes.c_uint8), ctypes.c_int(w), ctypes.c_int(h), _kp(kin), ctypes.c_int(n),
                                _kp(kout), _p(kept, ctypes.c_int), _p(desc, ctypes.c_uint8))
    return kout[:m], kept[:m], desc[:m]


# ---------------------------------------------------------------- FREAK (orc_freak.c)
def freak_point(scale, rot, i):
    """FREAK buildPattern's point i at (scale, orientation) of the default pattern: (x, y, sigma) float32"""
    x, y, s = ctypes.c_float(0), ctypes.c_float(0), ctypes.c_float(0)
    lib().orc_freak_point(ctypes.c_int(scale), ctypes.c_int(rot), ctypes.c_int(i), ctypes.byref(x), ctypes.byref(y),
                          ctypes.byref(s))
    return np.float32(x.value), np.float32(y.value), np.float32(s.value)


def freak_size(scale):
    return int(lib().orc_freak_size(ctypes.c_int(scale)))


def freak_kscale(size, octaves=4):
    return int(lib().orc_freak_kscale(ctypes.c_float(size), ctypes.c_int(octaves)))


def freak_weights():
    """the 45 orientation pairs' (weight_dx, weight_dy) of the default pattern"""
    lut = np.zeros(64 * 256 * 43 * 3, np.float32)
    sizes = np.zeros(64, np.int32)
    lib().orc_freak_pattern(ctypes.c_float(22.0), ctypes.c_int(4), _p(lut, ctypes.c_float), _p(sizes, ctypes.c_int))
    wx = np.zeros(45, np.int32)
    wy = np.zeros(45, np.int32)
    lib().orc_freak_weights(_p(lut, ctypes.c_float), _p(wx, ctypes.c_int), _p(wy, ctypes.c_int))
    return wx, wy


def freak_mean_intensity(img, kx, ky, px, py, sigma):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    s = np.zeros((h + 1) * (w + 1), np.int32)
    lib().orc_freak_integral(_p(img, ctypes.c_uint8), ctypes.c_int(w), ctypes.c_int(h), _p(s, ctypes.c_int))
    return int(lib().orc_freak_mean_intensity(_p(img, ctypes.c_uint8), _p(s, ctypes.c_int), ctypes.c_int(w),
                                              ctypes.c_float(kx), ctypes.c_float(ky), ctypes.c_float(px),
                                              ctypes.c_float(py), ctypes.c_float(sigma)))


def freak_compute(img, kpts, pairs=None):
    """DescriptorExtractor::compute with cv::FREAK() (defaults): (kept keypoints with their angles, input
    index of each, (m, 64) uint8 descriptors); pairs: 512 pair indices (None: the default table)"""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    kin = np.ascontiguousarray(kpts, dtype=KEYPOINT)
    n = len(kin)
    kout = np.zeros(max(n, 1), dtype=KEYPOINT)
    kept = np.zeros(max(n, 1), dtype=np.int32)
    desc = np.zeros((max(n, 1), 64), dtype=np.uint8)
    pp = None if pairs is None else _p(np.ascontiguousarray(pairs, dtype=np.int32), ctypes.c_int)
    m = lib().orc_freak_compute(_p(img, ctypes.c_uint8), ctypes.c_int(w), ctypes.c_int(h), _kp(kin), ctypes.c_int(n),
                                pp, _kp(kout), _p(kept, ctypes.c_int), _p(desc, ctypes.c_uint8))
    return kout[:m], kept[:m], desc[:m]


# ---------------------------------------------------------------- MSER (orc_mser.c)
MSER_DEFAULTS = dict(delta=5, min_area=60, max_area=14400, max_variation=0.25, min_diversity=0.2)


def _mser_args(img, delta, min_area, max_area, max_variation, min_diversity):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    return img, (_p(img, ctypes.c_uint8), ctypes.c_int(w), ctypes.c_int(h), ctypes.c_int(delta), ctypes.c_int(min_area),
                 ctypes.c_int(max_area), ctypes.c_double(max_variation), ctypes.c_double(min_diversity))


def mser_regions(img, delta=5, min_area=60, max_area=14400, max_variation=0.25, min_diversity=0.2):
    """MSER::operator()(img, msers): [(colour -1 | +1, (k, 2) int32 points (x, y) in region-list order)]"""
    img, a = _mser_args(img, delta, min_area, max_area, max_variation, min_diversity)
    npts = ctypes.c_longlong(0)
    n = lib().orc_mser_regions(*a, None, None, ctypes.c_int(0), None, ctypes.c_longlong(0), ctypes.byref(npts))
    if n < 0:
        raise ValueError("MSER: bad input")
    color = np.zeros(max(n, 1), np.int32)
    count = np.zeros(max(n, 1), np.int32)
    pts = np.zeros((max(npts.value, 1), 2), np.int32)
    lib().orc_mser_regions(*a, _p(color, ctypes.c_int), _p(count, ctypes.c_int), ctypes.c_int(n), _p(pts, ctypes.c_int),
                           ctypes.c_longlong(npts.value), ctypes.byref(npts))
    out, off = [], 0
    for i in range(n):
        out.append((int(color[i]), pts[off:off + count[i]].copy()))
        off += int(count[i])
    return out


def fit_ellipse(points):
    """cvFitEllipse2 on integer points: (cx, cy, width, height, angle) float32"""
    p = np.ascontiguousarray(points, dtype=np.int32).reshape(-1, 2)
    box = np.zeros(5, np.float32)
    if lib().orc_fit_ellipse(_p(p, ctypes.c_int), ctypes.c_int(len(p)), _p(box, ctypes.c_float)) < 0:
        raise ValueError("fitEllipse: fewer than 5 points")
    return box


def mser_detect(img, delta=5, min_area=60, max_area=14400, max_variation=0.25, min_diversity=0.2):
    """MserFeatureDetector(...).detect(img): KEYPOINT records in region order"""
    img, a = _mser_args(img, delta, min_area, max_area, max_variation, min_diversity)
    n = lib().orc_mser_detect(*a, None, ctypes.c_int(0))
    if n < 0:
        raise ValueError("MSER: a region below 5 points (fitEllipse throws) or bad input")
    out = np.zeros(max(n, 1), dtype=KEYPOINT)
    lib().orc_mser_detect(*a, _kp(out), ctypes.c_int(n))
    return out[:n]


def fit_ellipse_solves(points):
    """cvFitEllipse2's solves: (cx, cy, conic A..E (5), centre (2), re-fit A..C (3)) float64"""
    p = np.ascontiguousarray(points, dtype=np.int32).reshape(-1, 2)
    sol = np.zeros(12, np.float64)
    if lib().orc_fit_ellipse_solves(_p(p, ctypes.c_int), ctypes.c_int(len(p)), _p(sol)) < 0:
        raise ValueError("fitEllipse: fewer than 5 points")
    return sol
