"""How much of the C4 result the unpinnable last bits of OpenCV's SVD can move.

CPU only, oracle only.  The DLT and the polar factor follow OpenCV 2.4.9's JacobiSVDImpl_
(include/fm3d_cvsvd.h, oracle orc_cv_jacobi_svd) with a correctly rounded hypot.  Two details of
the reference's build are not recorded: which glibc hypot it linked (this image's is not correctly
rounded everywhere), and whether its OpenCV 2.4.x accumulated the rotation's dot product and norms in
VBLAS's two SSE2 lanes (the releases that kept W in _Tp) or in scalar doubles (2.4.9).  Over every
C4 inlier this runs the LM (DETMATH) on the points and R2 of each variant (oracle geometry modes
GEOM_LIBM_HYPOT, GEOM_SVD_LANES) and compares with the contract's run (tests/golden/full_c4.npz and
the per-match statuses of tests/golden/dlt_parity_c4.npz).  Adds "sensitivity" to
profiles/r06_dlt_parity.json.

    python tools/dlt_sensitivity.py [--threads 8]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import oracle as orc  # noqa: E402  (checker)
import make_full_fixtures as mff  # noqa: E402
from full_parity import diff  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=len(os.sched_getaffinity(0)))
    ap.add_argument("--table", default=os.path.join(ROOT, "profiles", "r06_dlt_parity.json"))
    args = ap.parse_args()
    wl = mff.WORKLOADS["c4"]
    fp = mff.make_pair(wl)
    q, tr, _ = orc.match_nndr(fp.desc1, fp.desc2, orc.U8, wl["eps"], args.threads)
    pts, mask = orc.triangulate(fp.cam, fp.g12, 1.5, 2.4, fp.kp1, fp.kp2, q, tr)
    fx = mff.load_fixture("c4")
    dp = np.load(os.path.join(ROOT, "tests", "golden", "dlt_parity_c4.npz"), allow_pickle=False)
    st = dp["status_opencv"].astype(np.int32)[mask]
    assert np.array_equal(pts[st == 0], fx["records"]["point"]), "the contract's points != full_c4.npz"
    normals = np.zeros((len(pts), 3))
    normals[st == 0] = fx["records"]["normal"]
    base = dict(status=st, normals=normals, nfev=np.ones(1))
    out = {}
    for name, mode in (("libm_hypot", orc.GEOM_LIBM_HYPOT), ("sse2_lanes", orc.GEOM_SVD_LANES)):
        with orc.geometry_mode(mode):
            p2, m2 = orc.triangulate(fp.cam, fp.g12, 1.5, 2.4, fp.kp1, fp.kp2, q, tr)
            R2, t2 = orc.camera2_from_g12(fp.g12)
        assert np.array_equal(m2, mask)
        t = time.time()
        r = orc.optimize_normals(fp.cam, R2, t2, fp.img1, fp.img2, wl["levels"], p2, wl["ray"], mode=orc.DETMATH,
                                 nthreads=args.threads)
        r["nfev"] = np.ones(1)
        _, tab = diff(base, r)
        tab.pop("evals_ratio", None)
        tab["points_bit_equal"] = int((np.abs(p2 - pts).max(axis=1) == 0).sum())
        tab["seconds"] = time.time() - t
        out[name] = tab
        print(name, json.dumps(tab), flush=True)
    with open(args.table) as f:
        table = json.load(f)
    table["sensitivity"] = out
    with open(args.table, "w") as f:
        json.dump(table, f, indent=1)
    print("->", args.table)


if __name__ == "__main__":
    main()
