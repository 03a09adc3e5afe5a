"""How meaningful is "normals within 1e-4 of the reference" when lmfit and OpenCV are unpinned?

CPU only, oracle only (test infrastructure; no GPU).  At the C4 settings (VGA, pixelsRay 64,
pyramids 3) the LM normals of a seeded random sample of triangulated points are recomputed
with the libm oracle (STRICT) under input perturbations that an unpinned OpenCV / libm could
plausibly introduce, and compared with the unperturbed run:

  * R2 from an SVD polar factor (numpy SVD: OpenCV's cvRodrigues2 orthonormalises R by
    cvSVD, U V^T) instead of the three Newton polar steps of fm3d_host.cpp rodrigues_m2v;
  * t2 moved by one ulp (each component up; each component down);
  * fx moved by one ulp (undistortion of the neighbourhood pixels and the camera-2
    projection: the inputs of every bilinear sample coordinate);
  * the deterministic transcendentals of the GPU (DETMATH) instead of libm;
  * lmfit 3.x's lmmin where it is recalled to differ from the MINPACK lmdif the oracle restates
    (oracle/fm3d_oracle.c ORC_LMV_*): the forward-difference step floor
    MAX(eps^2, eps|x|), lm_enorm's sqrt(DBL_MIN) / sqrt(DBL_MAX) thresholds, the early return on a
    starting fnorm <= DBL_MIN, all three together (the lmfit 3.x set), and the 1e-14 tolerances of
    lmfit builds with the hard-coded "x86" constants.

For each variant: the fraction of points whose keep/drop status changes, and among the points
kept by both, the fraction whose normal moves by more than 1e-4 (and 1e-6), plus the largest
move.  Writes a JSON summary (default profiles/r02_parity_risk.json).

    python tools/parity_risk.py [--points 1000] [--threads 8] [--out ...]
"""
from __future__ import annotations

import argparse
import importlib
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as orc  # noqa: E402  (checker)


def m2v_no_polar(R):
    """cvRodrigues2 matrix -> vector after the orthonormalisation (OpenCV 2.4 calibration.cpp),
    the same branch structure as fm3d_host.cpp rodrigues_m2v."""
    rx, ry, rz = R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]
    s = math.sqrt((rx * rx + ry * ry + rz * rz) * 0.25)
    c = (R[0, 0] + R[1, 1] + R[2, 2] - 1) * 0.5
    c = min(1.0, max(-1.0, c))
    theta = math.acos(c)
    if s < 1e-5:
        raise ValueError("near-identity / half-turn rotation: not exercised by the C4 pose")
    vth = 1 / (2 * s) * theta
    return np.array([rx * vth, ry * vth, rz * vth])


def compare(base, other):
    kb, ko = base["status"] == 0, other["status"] == 0
    both = kb & ko
    d = np.abs(base["normals"][both] - other["normals"][both]).max(axis=1) if both.any() else np.zeros(0)
    return {
        "status_changed": float(np.mean(base["status"] != other["status"])),
        "kept_both": int(both.sum()),
        "moved_gt_1e-4": float(np.mean(d > 1e-4)) if d.size else 0.0,
        "moved_gt_1e-6": float(np.mean(d > 1e-6)) if d.size else 0.0,
        "max_move": float(d.max()) if d.size else 0.0,
        "median_move": float(np.median(d)) if d.size else 0.0,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=1000)
    ap.add_argument("--threads", type=int, default=len(os.sched_getaffinity(0)))
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r03_parity_risk.json"))
    args = ap.parse_args()
    synth = importlib.import_module("3dfeaturematcher_amd.synth")
    pair = synth.make_frame_pair(100_000, 640, 480, seed=args.seed)  # the C4 bench frame pair
    rng = np.random.default_rng(1234)
    qs = np.sort(rng.choice(len(pair.desc1), 4 * args.points, replace=False))
    q, t, _ = orc.match_nndr(pair.desc1[qs], pair.desc2, orc.U8, 0.55, args.threads)
    pts, _ = orc.triangulate(pair.cam, pair.g12, 1.5, 2.4, pair.kp1[qs], pair.kp2, q, t)
    sel = np.sort(rng.choice(len(pts), min(args.points, len(pts)), replace=False))
    P = pts[sel]
    R2, t2 = orc.camera2_from_g12(pair.g12)

    # R2 through an SVD polar factor (OpenCV) instead of the Newton polar
    R = np.asarray(pair.g12)[:3, :3]
    U, _, Vt = np.linalg.svd(R)
    R2svd = orc.rodrigues_v2m(m2v_no_polar(U @ Vt))

    LMV_FDFLOOR, LMV_ENORM, LMV_DWARFEXIT, LMV_TOL1E14 = 4, 8, 16, 32  # fm3d_oracle.c ORC_LMV_*

    def run(cam=pair.cam, R2_=R2, t2_=t2, mode=orc.STRICT):
        return orc.optimize_normals(cam, R2_, t2_, pair.img1, pair.img2, 3, P, 64, mode=mode,
                                    nthreads=args.threads)

    cam_fx = synth.Camera(np.nextafter(pair.cam.fx, np.inf), pair.cam.fy, pair.cam.cx, pair.cam.cy, pair.cam.k)
    t0 = time.time()
    base = run()
    variants = {
        "R2_svd_polar": run(R2_=R2svd),
        "t2_plus_1ulp": run(t2_=np.nextafter(t2, np.inf)),
        "t2_minus_1ulp": run(t2_=np.nextafter(t2, -np.inf)),
        "fx_plus_1ulp": run(cam=cam_fx),
        "detmath_vs_libm": run(mode=orc.DETMATH),
        "lmfit_fd_step_floor": run(mode=orc.STRICT | LMV_FDFLOOR),
        "lmfit_enorm_thresholds": run(mode=orc.STRICT | LMV_ENORM),
        "lmfit_dwarf_exit": run(mode=orc.STRICT | LMV_DWARFEXIT),
        "lmfit3_all_three": run(mode=orc.STRICT | LMV_FDFLOOR | LMV_ENORM | LMV_DWARFEXIT),
        "lmfit_tol_1e-14": run(mode=orc.STRICT | LMV_TOL1E14),
    }
    out = {
        "workload": "C4 frame pair (100k SIFT, 640x480, seed %d), pixelsRay 64, pyramids 3, oracle STRICT" % args.seed,
        "points": int(len(P)),
        "kept_base": int((base["status"] == 0).sum()),
        "R2_svd_minus_newton_max_abs": float(np.abs(R2svd - R2).max()),
        "R2_svd_equals_newton_bitwise": bool(np.array_equal(R2svd, R2)),
        "variants": {k: compare(base, v) for k, v in variants.items()},
        "cpu_seconds": round(time.time() - t0, 1),
        "threads": args.threads,
    }
    print(json.dumps(out, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
