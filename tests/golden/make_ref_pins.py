"""Pins of the oracle against the REFERENCE'S OWN OUTPUT FILES (tests/golden/ref_pins.npz).

TEST INFRASTRUCTURE, run here in the container (reads /root/reference, which the GPU box lacks):

    python tests/golden/make_ref_pins.py [--threads 8]

The reference ships no tests and no inputs, but its results/ tree holds output images of one real
run (the image pair img_750 / img_770 whose poses main.cpp:25-26 records; build/settings.yml's
camera):
  * results/*/image1pixels.pgm (identical in every results dir): image 1 with the kept
    neighbourhood of every surviving point painted in its colour -- the drawing code of an earlier
    revision of computeOptimizedNormals (normaloptimizer.cpp:404-419: round(x_), round(y_) of every
    extractPixelsContour pixel, :341-397);
  * results/*/image2pixels.pgm: image 2 with the same pixels pushed through the plane of the
    optimised normal into camera 2 (:421-445: get3dPointsFromImage1Pixels +
    projectPointsToImage2(pointGroup, 1.0), singlecameratriangulator.cpp:530-644);
  * results/64px4l{.5c.32e,1c.64e}_img{1,2}/patch_<i>.pgm: the 128x128 patches of the square
    neighbourhoods (neighborhoodsgenerator.cpp:76-132) of the features frames
    (normaloptimizer.cpp:454-504), projected into image 1 / image 2 and sampled
    (projectPointsToImage, singlecameratriangulator.cpp:667-767; the call main.cpp:179 keeps
    commented out).
The colours are drawMatches' cv::RNG(0xFFF0FF0F) sequence (tools.cpp:116-120, 159-167): colour i
belongs to inlier i, which identifies the 15 survivors (inliers 2, 5, 6, ..., 22) and the order in
which they were drawn (later survivors paint over earlier ones).

What this script extracts (data, no reference text): per image a label map (0 = unpainted,
1 + survivor rank) and the grey background where unpainted, the patches, and per survivor the
image-1 centre and the (X, n) of its plane fitted to the painted image-2 pixels WITH THE ORACLE'S
OWN GEOMETRY (orc_neighborhood, orc_plane_to_image2, orc_setg12 / orc_camera2_from_g12 under the
main.cpp:25-26 poses).  Fitting 5 numbers (sub-pixel centre, depth, two normal angles) to ~13k
painted pixels per survivor cannot absorb a wrong camera model, g12 composition, distortion order
or projection: the painted set is the ROUNDED image of the whole neighbourhood, so any model error
above ~0.01 px flips pixels.  A held-out check fits on the even neighbourhood entries only and
counts the odd ones.  tests/test_ref_pins.py then re-derives everything from the fixture.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
REF = "/root/reference"
OUT = os.path.join(HERE, "ref_pins.npz")
W, H = 1024, 768
RAY = 64


class Cam:
    """build/settings.yml CameraSettings (OpenCV order k1, k2, p1, p2, k3 = k0, k1, p1, p2, k2)."""
    fx, fy, cx, cy = 572.4765, 572.69354, 549.75189, 411.68039
    k = (-0.299957, 0.124129, -6.6e-05, 0.000567, -0.028357)


RIC = np.array([-1.2005, 1.1981, -1.2041])        # build/settings.yml:53
TIC = np.array([0.0, 0.015, -0.051])              # build/settings.yml:54
# main.cpp:25-26: "IMG_1 pose: ... POS : 4.467813 3.420069 0.806258 0.074931 -0.160281 0.563678" (T, then r)
POS1 = np.array([4.467813, 3.420069, 0.806258, 0.074931, -0.160281, 0.563678])
POS2 = np.array([5.034858, 3.667427, 0.833424, 0.014587, -0.248119, 0.523502])
ZMAX = 2.4
PATCH_DIRS = ("64px4l.5c.32e_img1", "64px4l.5c.32e_img2", "64px4l1c.64e_img1", "64px4l1c.64e_img2",
              "64px4l.25c.16e_img1", "64px4l.25c.16e_img2")
PATCH_PARAMS = {"64px4l.5c.32e": (0.32, 0.5), "64px4l1c.64e": (0.64, 1.0), "64px4l.25c.16e": (0.16, 0.25)}


def read_pnm(path):
    b = open(path, "rb").read()
    toks, i = [], 0
    while len(toks) < 4:
        while b[i:i + 1].isspace():
            i += 1
        if b[i:i + 1] == b"#":
            while b[i:i + 1] not in (b"\n", b""):
                i += 1
            continue
        j = i
        while not b[j:j + 1].isspace():
            j += 1
        toks.append(b[i:j])
        i = j
    i += 1
    w, h = int(toks[1]), int(toks[2])
    c = 3 if toks[0] == b"P6" else 1
    a = np.frombuffer(b[i:i + w * h * c], np.uint8)
    return a.reshape(h, w, c) if c == 3 else a.reshape(h, w)


def rng_colours(n):
    """cv::RNG(0xFFF0FF0F).next() -> random_color -> CV_RGB: file (R, G, B) = (c & 255, c >> 8 & 255, c >> 16 & 255)"""
    st, out = 0xFFF0FF0F, []
    for _ in range(n):
        st = ((st & 0xFFFFFFFF) * 4164903690 + (st >> 32)) & 0xFFFFFFFFFFFFFFFF
        c = st & 0xFFFFFFFF
        out.append((c & 255, (c >> 8) & 255, (c >> 16) & 255))
    return out


def labels(img, colours):
    """label map (0 unpainted, 1 + rank of the survivor in drawing order), grey background, survivors"""
    found = []
    lab = np.zeros(img.shape[:2], np.uint8)
    for k, c in enumerate(colours):
        m = (img[..., 0] == c[0]) & (img[..., 1] == c[1]) & (img[..., 2] == c[2])
        if m.any():
            found.append(k)
            lab[m] = len(found)
    grey = (img[..., 0] == img[..., 1]) & (img[..., 1] == img[..., 2])
    assert ((lab > 0) == ~grey).all(), "a painted pixel of an unexpected colour"
    bg = np.where(lab == 0, img[..., 0], 0).astype(np.uint8)
    return lab, bg, found


def round_px(uv):
    """the drawing code's cv::Point2i(round(x), round(y)) (half away from zero; coordinates are >= 0)"""
    return np.floor(uv + 0.5).astype(np.int64)


class Geometry:
    def __init__(self):
        import oracle as orc
        self.orc = orc
        g12 = orc.setg12(RIC, TIC, POS1[:3], POS2[:3], POS1[3:], POS2[3:])
        self.g12 = g12
        self.R2, self.t2 = orc.camera2_from_g12(g12)

    @staticmethod
    def normal(phi, theta):
        return np.array([np.cos(theta) * np.cos(phi), np.cos(theta) * np.sin(phi), np.sin(theta)])

    def point(self, cx, cy, d):
        u = self.orc.undistort(Cam, np.array([[cx, cy]]))[0]
        return d * np.array([u[0], u[1], 1.0])

    def predict(self, par):
        """par = (cx, cy, depth, phi, theta) -> X, n, image-1 pixels, image-2 uv"""
        X = self.point(*par[:3])
        n = self.normal(par[3], par[4])
        pix = self.orc.neighborhood(Cam, X, RAY, W, H)
        uv, _ = self.orc.plane_to_image2(Cam, self.R2, self.t2, X, n, pix, ZMAX)
        return X, n, pix, uv


def paint(lab_shape, pts_list):
    """the drawing loop: survivor after survivor, later colours over earlier ones"""
    lab = np.zeros(lab_shape, np.uint8)
    for r, px in enumerate(pts_list):
        ok = (px[:, 0] >= 0) & (px[:, 1] >= 0) & (px[:, 0] < lab_shape[1]) & (px[:, 1] < lab_shape[0])
        lab[px[ok, 1], px[ok, 0]] = r + 1
    return lab


def centre_of(lab1, rank, later_circles):
    """integer centre (round(c.x), round(c.y)) of survivor `rank`'s image-1 circle: every painted
    pixel inside the circle, every circle pixel painted or under a later survivor's circle"""
    m = lab1 == rank + 1
    ys, xs = np.nonzero(m)
    off = np.array([(i, j) for i in range(-RAY, RAY + 1) for j in range(-RAY, RAY + 1) if i * i + j * j <= RAY * RAY])
    best = None
    for a in range(xs.max() - RAY, xs.min() + RAY + 1):
        for b in range(ys.max() - RAY, ys.min() + RAY + 1):
            if ((xs - a) ** 2 + (ys - b) ** 2 > RAY * RAY).any():
                continue
            px = off + (a, b)
            ok = (px[:, 0] >= 0) & (px[:, 1] >= 0) & (px[:, 0] < W) & (px[:, 1] < H)
            extra = int((~m[px[ok, 1], px[ok, 0]] & ~later_circles[px[ok, 1], px[ok, 0]]).sum())
            if best is None or extra < best[0]:
                best = (extra, a, b)
    return best


def mismatch(geo, par, M, later, ab, entries=None):
    a, b = ab
    if not (a - 0.5 <= par[0] < a + 0.5 and b - 0.5 <= par[1] < b + 0.5) or par[2] <= 0:
        return 10 ** 9, None
    _, _, _, uv = geo.predict(par)
    if not np.isfinite(uv).all():
        return 10 ** 9, None
    r = round_px(uv)
    ok = (r[:, 0] >= 0) & (r[:, 1] >= 0) & (r[:, 0] < W) & (r[:, 1] < H)
    hit = np.zeros(len(uv), bool)
    hit[ok] = M[r[ok, 1], r[ok, 0]] | later[r[ok, 1], r[ok, 0]]
    if entries is not None:  # forward count on a subset of neighbourhood entries
        return int((~hit[entries]).sum()), hit
    P = np.zeros((H, W), bool)
    P[r[ok, 1], r[ok, 0]] = True
    return int((M & ~P).sum() + (P & ~M & ~later).sum()), hit


def cmaes(f, x0, sd, iters=400, lam=14, seed=0):
    """minimal CMA-ES (N. Hansen's tutorial formulation) minimising f(x0 + sd * y)"""
    rng = np.random.default_rng(seed)
    n = len(x0)
    sd = np.asarray(sd, float)
    mu = lam // 2
    w = np.log(mu + 0.5) - np.log(np.arange(1, mu + 1))
    w /= w.sum()
    mueff = 1 / np.sum(w ** 2)
    cc = (4 + mueff / n) / (n + 4 + 2 * mueff / n)
    cs = (mueff + 2) / (n + mueff + 5)
    c1 = 2 / ((n + 1.3) ** 2 + mueff)
    cmu = min(1 - c1, 2 * (mueff - 2 + 1 / mueff) / ((n + 2) ** 2 + mueff))
    damps = 1 + 2 * max(0, np.sqrt((mueff - 1) / (n + 1)) - 1) + cs
    chin = np.sqrt(n) * (1 - 1 / (4 * n) + 1 / (21 * n * n))
    m, sigma, pc, ps, C = np.zeros(n), 1.0, np.zeros(n), np.zeros(n), np.eye(n)
    best = (f(np.asarray(x0, float)), np.asarray(x0, float))
    for g in range(iters):
        if best[0] == 0:
            break
        dg, B = np.linalg.eigh(C)
        dg = np.sqrt(np.maximum(dg, 1e-20))
        y = rng.normal(size=(lam, n)) @ np.diag(dg) @ B.T
        fs = np.array([f(x0 + sd * (m + sigma * yy)) for yy in y])
        idx = np.argsort(fs, kind="stable")
        if fs[idx[0]] < best[0]:
            best = (fs[idx[0]], x0 + sd * (m + sigma * y[idx[0]]))
        yw = w @ y[idx[:mu]]
        m = m + sigma * yw
        ps = (1 - cs) * ps + np.sqrt(cs * (2 - cs) * mueff) * (B @ np.diag(1 / dg) @ B.T) @ yw
        hs = np.linalg.norm(ps) / np.sqrt(1 - (1 - cs) ** (2 * (g + 1))) < (1.4 + 2 / (n + 1)) * chin
        pc = (1 - cc) * pc + hs * np.sqrt(cc * (2 - cc) * mueff) * yw
        C = ((1 - c1 - cmu) * C + c1 * (np.outer(pc, pc) + (1 - hs) * cc * (2 - cc) * C)
             + cmu * (y[idx[:mu]].T @ np.diag(w) @ y[idx[:mu]]))
        sigma *= np.exp((cs / damps) * (np.linalg.norm(ps) / chin - 1))
    return best[1], int(best[0])


def fit(geo, M, later, ab, entries=None, log=print, extra_starts=()):
    """(cx, cy, depth, phi, theta) of one survivor: blob moments (multi-start) -> density
    registration of the predicted points against the painted pixels (Gaussian blur 4 -> 0.6 px)
    -> CMA-ES on the exact mismatch count (entries given: forward count on those entries only)."""
    from scipy.ndimage import gaussian_filter
    from scipy.optimize import least_squares
    a, b = ab
    lo = [a - 0.5, b - 0.5, 0.5, -np.inf, -np.inf]
    hi = [a + 0.4999, b + 0.4999, 5.0, np.inf, np.inf]
    ys, xs = np.nonzero(M)
    pc = np.stack([xs, ys], 1).astype(float)

    def visible(uv):
        r = round_px(uv)
        ok = (r[:, 0] >= 0) & (r[:, 1] >= 0) & (r[:, 0] < W) & (r[:, 1] < H)
        keep = ok.copy()
        keep[ok] = ~later[r[ok, 1], r[ok, 0]]
        return keep

    def moments(p):
        m = p.mean(0)
        C = np.cov(p.T)
        return np.array([m[0], m[1], np.sqrt(C[0, 0]), np.sqrt(C[1, 1]), C[0, 1] / np.sqrt(C[0, 0] * C[1, 1])])

    tgt = moments(pc)

    def res_m(q):
        _, _, _, uv = geo.predict((a, b, *q))
        if not np.isfinite(uv).all():
            return np.full(5, 1e3)
        keep = visible(uv)
        if keep.sum() < 10:
            return np.full(5, 1e3)
        return (moments(uv[keep]) - tgt) * np.array([1, 1, 1, 1, 50])

    grid = [(d, p, t) for d in (1.6, 2.0, 2.4, 3.0) for p in np.radians([-150, -90, -30, 30, 90, 150])
            for t in np.radians([-60, -20, 20, 60])]
    grid.sort(key=lambda q: float(np.sum(res_m(q) ** 2)))
    starts = []
    for q0 in grid[:6]:
        try:
            r = least_squares(res_m, q0, method="lm")
            starts.append(np.array([a, b, *r.x]))
        except Exception:
            continue

    def render(uv, box):
        x0, y0, w, h = box
        u, v = uv[:, 0] - x0, uv[:, 1] - y0
        ok = (u >= 0) & (v >= 0) & (u < w - 1) & (v < h - 1)
        u, v = u[ok], v[ok]
        iu, iv = np.floor(u).astype(int), np.floor(v).astype(int)
        fu, fv = u - iu, v - iv
        D = np.zeros((h, w))
        np.add.at(D, (iv, iu), (1 - fu) * (1 - fv))
        np.add.at(D, (iv, iu + 1), fu * (1 - fv))
        np.add.at(D, (iv + 1, iu), (1 - fu) * fv)
        np.add.at(D, (iv + 1, iu + 1), fu * fv)
        return D

    def register(par):
        _, _, _, uv = geo.predict(par)
        if not np.isfinite(uv).all():
            return par
        x0 = max(int(min(xs.min(), uv[:, 0].min())) - 30, 0)
        y0 = max(int(min(ys.min(), uv[:, 1].min())) - 30, 0)
        x1 = min(int(max(xs.max(), uv[:, 0].max())) + 30, W)
        y1 = min(int(max(ys.max(), uv[:, 1].max())) + 30, H)
        box = (x0, y0, x1 - x0, y1 - y0)
        Mc = M[y0:y1, x0:x1].astype(float)
        free = (~later[y0:y1, x0:x1]).astype(float)
        for sg in (4, 2, 1, 0.6):
            Mb = gaussian_filter(Mc, sg)
            wgt = gaussian_filter(free, sg) > 0.999

            def res(p):
                _, _, _, uv = geo.predict(p)
                if not np.isfinite(uv).all():
                    return np.full(int(wgt.sum()), 10.0)
                return (gaussian_filter(render(uv, box), sg) - Mb)[wgt]
            try:
                par = least_squares(res, np.clip(par, lo, hi), x_scale=[0.1, 0.1, 1e-3, 1e-3, 1e-3], diff_step=1e-6,
                                    max_nfev=100, bounds=(lo, hi)).x
            except Exception:
                break
        return par

    cand = []
    for p0 in starts[:3]:
        p1 = register(p0)
        cand.append((mismatch(geo, p1, M, later, ab, entries)[0], p1))
    for p0 in extra_starts:
        cand.append((mismatch(geo, p0, M, later, ab, entries)[0], np.asarray(p0, float)))
    cand.sort(key=lambda t: t[0])
    f, par = cand[0]
    log(f"    moments + registration: {f}")
    obj = lambda p: mismatch(geo, p, M, later, ab, entries)[0]
    for restart in range(10):
        sd = [0.05, 0.05, 1e-4, 1e-4, 1e-4] if restart % 2 == 0 else [0.01, 0.01, 2e-5, 2e-5, 2e-5]
        par, f = cmaes(obj, par, sd, iters=400, seed=restart)
        log(f"    CMA-ES ({restart}): {f}")
        if f == 0:
            break
    return par, f


FIT_RUN = "64px4l.5c.32e"


def patch_l1(geo, X, n, rk, lab1, lab2, bg1, bg2, patches, g, run):
    """sum over both images of |oracle sample - reference patch| on the eligible pixels (four
    bilinear taps unpainted) of run `run`'s patch_<rk>.pgm"""
    orc = geo.orc
    F = orc.features_frames(X[None], n[None], g)
    eps, cmpp = PATCH_PARAMS[run]
    pts = orc.square_neighborhoods(F, eps, cmpp)[0]
    tot = 0
    for image, R, t, lab, bg in ((1, np.eye(3), np.zeros(3), lab1, bg1), (2, geo.R2, geo.t2, lab2, bg2)):
        uv = orc.project(Cam, R, t, pts)
        x0 = np.floor(uv[:, 0].astype(np.float32)).astype(np.int64)
        y0 = np.floor(uv[:, 1].astype(np.float32)).astype(np.int64)
        ok = (x0 >= 0) & (y0 >= 0) & (x0 + 1 < W) & (y0 + 1 < H)
        e = np.zeros(len(uv), bool)
        i = np.nonzero(ok)[0]
        e[i] = (lab[y0[i], x0[i]] == 0) & (lab[y0[i] + 1, x0[i]] == 0) & (lab[y0[i], x0[i] + 1] == 0) & (
            lab[y0[i] + 1, x0[i] + 1] == 0)
        want = patches[f"{run}_img{image}"][rk].T.reshape(-1)
        tot += int(np.abs(orc.sample_points(bg, uv)[e].astype(np.int64) - want[e]).sum())
    return tot


def refine_on_patches(geo, p0, sg, rk, lab1, lab2, bg1, bg2, patches, ab, g):
    """Nelder-Mead on the FIT_RUN patch L1 from the label fit, three simplex scales"""
    from scipy.optimize import minimize
    Mk, later = lab2 == rk + 1, lab2 > rk + 1
    m0, _ = mismatch(geo, p0, Mk, later, ab)

    def f(p):
        m, _ = mismatch(geo, p, Mk, later, ab)
        if m > m0:
            return 1e12 + m
        return patch_l1(geo, geo.point(*p[:3]), sg * geo.normal(p[3], p[4]), rk, lab1, lab2, bg1, bg2, patches, g,
                        FIT_RUN)

    best, fb = p0.copy(), f(p0)
    step = np.array([1.0, 1.0, 0.05, 1.0, 1.0])
    for sc in (1e-2, 3e-3, 1e-3):
        simplex = np.vstack([best] + [best + sc * step[i] * np.eye(5)[i] for i in range(5)])
        r = minimize(f, best, method="Nelder-Mead",
                     options=dict(initial_simplex=simplex, maxfev=600, xatol=1e-7, fatol=0.5))
        if r.fun < fb:
            best, fb = r.x, r.fun
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=1)
    ap.parse_args()
    import oracle as orc
    geo = Geometry()
    cols = rng_colours(64)
    img1 = read_pnm(os.path.join(REF, "results/64px4l.25c.16e_img1/image1pixels.pgm"))
    img2 = read_pnm(os.path.join(REF, "results/64px4l.25c.16e_img1/image2pixels.pgm"))
    lab1, bg1, surv1 = labels(img1, cols)
    lab2, bg2, surv2 = labels(img2, cols)
    assert surv1 == surv2
    surv = surv1
    print("survivors (inlier index = colour index):", surv, flush=True)
    S = len(surv)
    # image-1 centres, last drawn first (its circle is whole)
    centres = [None] * S
    later1 = np.zeros((H, W), bool)
    off = np.array([(i, j) for i in range(-RAY, RAY + 1) for j in range(-RAY, RAY + 1) if i * i + j * j <= RAY * RAY])
    for rk in reversed(range(S)):
        extra, a, b = centre_of(lab1, rk, later1)
        assert extra == 0, (rk, extra)
        centres[rk] = (a, b)
        px = off + (a, b)
        ok = (px[:, 0] >= 0) & (px[:, 1] >= 0) & (px[:, 0] < W) & (px[:, 1] < H)
        later1[px[ok, 1], px[ok, 0]] = True
    print("image-1 centres:", centres, flush=True)
    params, fit_mis, held = np.zeros((S, 5)), np.zeros(S, np.int64), np.zeros((S, 2), np.int64)
    cache_path = "/tmp/ref_pins_cache.npz"  # resume a killed run (per-survivor results)
    cache = dict(np.load(cache_path)) if os.path.exists(cache_path) else {}
    for rk in range(S):
        t0 = time.time()
        if f"par{rk}" in cache and int(cache[f"mis{rk}"]) == 0:
            params[rk], fit_mis[rk], held[rk] = cache[f"par{rk}"], 0, cache[f"held{rk}"]
            print(f"survivor {rk}: cached, held-out {held[rk].tolist()}", flush=True)
            continue
        M = lab2 == rk + 1
        later = lab2 > rk + 1
        print(f"survivor {rk} (inlier {surv[rk]}): {int(M.sum())} painted image-2 pixels", flush=True)
        # held-out: fit the even neighbourhood entries, count the odd ones
        n_ent = len(geo.predict((centres[rk][0], centres[rk][1], 2.0, 0.0, 1.0))[2])
        even = np.arange(0, n_ent, 2)
        p_even, _ = fit(geo, M, later, centres[rk], entries=even, log=lambda s: print(s, flush=True))
        _, hit = mismatch(geo, p_even, M, later, centres[rk], np.arange(n_ent))
        odd = np.arange(1, n_ent, 2)
        held[rk] = (int(hit[odd].sum()), len(odd))
        print(f"    held-out: {held[rk][0]} of {held[rk][1]} odd entries on painted pixels", flush=True)
        starts = [p_even] + ([cache[f"par{rk}"]] if f"par{rk}" in cache else [])
        par, f = fit(geo, M, later, centres[rk], log=lambda s: print(s, flush=True), extra_starts=starts)
        params[rk], fit_mis[rk] = par, f
        cache.update({f"par{rk}": par, f"mis{rk}": np.array(f), f"held{rk}": held[rk]})
        np.savez(cache_path, **cache)
        print(f"  survivor {rk}: mismatch {f}, par {par.tolist()} ({time.time() - t0:.0f} s)", flush=True)
    X = np.stack([geo.point(*p[:3]) for p in params])
    n = np.stack([geo.normal(p[3], p[4]) for p in params])
    # the LM's normal keeps the initial guess X/|X|'s side of the plane only by continuity; the
    # patches (frames z = n) decide the sign: compare both against patch_<i>.pgm
    patches = {}
    for d in PATCH_DIRS:
        patches[d] = np.stack([read_pnm(os.path.join(REF, "results", d, f"patch_{i}.pgm")) for i in range(S)])
    g = orc.gravity(RIC)
    sign = np.ones(S)
    for rk in range(S):
        score = []
        for sg in (1.0, -1.0):
            F = orc.features_frames(X[rk:rk + 1], sg * n[rk:rk + 1], g)
            eq = 0
            for d in ("64px4l.5c.32e_img1", "64px4l1c.64e_img1"):
                eps, cmpp = PATCH_PARAMS[d[:-5]]
                pts = orc.square_neighborhoods(F, eps, cmpp)[0]
                uv = orc.project(Cam, np.eye(3), np.zeros(3), pts)
                got = orc.sample_points(bg1, uv).reshape(128, 128).T  # patch.at<uchar>(col = j, row = i)
                eq += int((got == patches[d][rk]).sum())
            score.append(eq)
        sign[rk] = 1.0 if score[0] >= score[1] else -1.0
        print(f"  survivor {rk}: normal sign {sign[rk]:+.0f} (patch pixels equal {score})", flush=True)
    n = n * sign[:, None]
    # sub-pixel refinement: the label images pin the 5 numbers to integer rounding only; the
    # patches are bilinear samples at sub-pixel positions.  Fit on the FIT_RUN patches (both
    # images), the label mismatch never above the label fit's; the other runs are held out.
    refined = np.zeros((S, 5))
    for rk in range(S):
        t0 = time.time()
        if f"ref{rk}" in cache:
            refined[rk] = cache[f"ref{rk}"]
        else:
            refined[rk] = refine_on_patches(geo, params[rk], sign[rk], rk, lab1, lab2, bg1, bg2, patches,
                                            centres[rk], g)
            cache[f"ref{rk}"] = refined[rk]
            np.savez(cache_path, **cache)
        print(f"  survivor {rk}: refined {(refined[rk] - params[rk]).tolist()} ({time.time() - t0:.0f} s)", flush=True)
    X = np.stack([geo.point(*p[:3]) for p in refined])
    n = np.stack([geo.normal(p[3], p[4]) for p in refined]) * sign[:, None]
    fit_mis = np.array([mismatch(geo, refined[rk], lab2 == rk + 1, lab2 > rk + 1, centres[rk])[0] for rk in range(S)])
    np.savez_compressed(
        OUT, lab1=lab1, lab2=lab2, bg1=bg1, bg2=bg2, survivors=np.array(surv), colours=np.array(cols[:max(surv) + 1]),
        centres=np.array(centres), params=refined, label_params=params, fit_run=FIT_RUN, X=X, n=n, fit_mismatch=fit_mis, heldout=held,
        camera=np.array([Cam.fx, Cam.fy, Cam.cx, Cam.cy, *Cam.k]), rIC=RIC, tIC=TIC, pos1=POS1, pos2=POS2,
        g12=geo.g12, **{"patch_" + d.replace(".", "_"): patches[d] for d in PATCH_DIRS})
    print("wrote", OUT, flush=True)


if __name__ == "__main__":
    main()
