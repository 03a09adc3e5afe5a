"""What the rounds 1-5 geometry stand-ins did to the C4 results.

CPU only, oracle only (test infrastructure; no GPU).  Rounds 1-5 computed two OpenCV primitives on
the hot path with stand-ins:

  * the DLT null vector (cv::triangulatePoints, Triangulator/singlecameratriangulator.cpp:186) from
    a 4-row system with a round-robin one-sided Jacobi -- OpenCV 2.4's cvTriangulatePoints builds a
    6 x 4 system (a third row x P.row1 - y P.row0 per view) and runs JacobiSVD on it;
  * the polar factor of cvRodrigues2 (decomposeTransformation, tools.cpp:110) by three Newton steps
    -- OpenCV takes U V^T of the same JacobiSVD.

Round 6 restates both (oracle orc_cv_jacobi_svd, product include/fm3d_cvsvd.h).  Over every match of
the C4 frame pair (100k SIFT-128, 640x480, seed 7; exact knn + NNDR), this tool:

  1. triangulates with each geometry mode (oracle orc_set_geometry_mode): OpenCV (the contract),
     the legacy DLT, the legacy polar factor, both legacy (= rounds 1-5), and two sensitivity
     variants of the SVD itself (VBLAS's two-lane SSE2 dot / givensx sums; libm's hypot) -- and
     tabulates inlier-mask changes and point differences against OpenCV and against numpy's SVD of
     the 6 x 4 system;
  2. runs the LM (DETMATH, the GPU contract) over every inlier with the OpenCV geometry and writes
     the new tests/golden/full_c4.npz (the same format as make_full_fixtures.py);
  3. compares it point by point with the rounds 1-5 contract: the old per-inlier statuses
     (--old-status: full_parity_c4.npz's status_detmath) and kept normals (--old-records: the old
     full_c4.npz), after checking that the "both legacy" mode reproduces the old kept points bit for
     bit;
  4. with --attribution, runs the LM with one stand-in at a time (legacy DLT only, legacy polar only)
     to split the difference.

Writes profiles/r06_dlt_parity.json and tests/golden/dlt_parity_c4.npz (per-inlier statuses and
differences, and a pinned subset that tests/test_dlt_parity.py re-runs through the oracle).

    cp tests/golden/full_c4.npz /tmp/full_c4_r05.npz   # before: the tool overwrites it
    python tools/dlt_parity.py --old-records /tmp/full_c4_r05.npz --old-status tests/golden/full_parity_c4.npz
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

MODES = {
    "opencv": 0,
    "legacy_dlt": orc.GEOM_DLT_LEGACY,
    "legacy_polar": orc.GEOM_POLAR_NEWTON,
    "legacy_both": orc.GEOM_DLT_LEGACY | orc.GEOM_POLAR_NEWTON,
    "sse2_lanes": orc.GEOM_SVD_LANES,
    "libm_hypot": orc.GEOM_LIBM_HYPOT,
}


def numpy_dlt(g12, u1, u2):
    P1, P2 = np.eye(4)[:3], g12[:3]
    A = np.stack([u1[:, :1] * P1[2] - P1[0], u1[:, 1:] * P1[2] - P1[1], u1[:, :1] * P1[1] - u1[:, 1:] * P1[0],
                  u2[:, :1] * P2[2] - P2[0], u2[:, 1:] * P2[2] - P2[1], u2[:, :1] * P2[1] - u2[:, 1:] * P2[0]], 1)
    X = np.linalg.svd(A)[2][:, -1]
    return X[:, :3] / X[:, 3:]


def rel(a, b):
    return np.abs(a - b).max(axis=1) / np.maximum(1.0, np.abs(b).max(axis=1))


def point_table(pts, mask, base_pts, base_mask):
    both = mask & base_mask
    # positions of the common inliers in each compacted list
    ia = np.cumsum(mask) - 1
    ib = np.cumsum(base_mask) - 1
    r = rel(pts[ia[both]], base_pts[ib[both]])
    return r, {
        "inliers": int(mask.sum()),
        "mask_changed": int((mask != base_mask).sum()),
        "points_bit_equal": int((r == 0).sum()),
        "max_rel": float(r.max()),
        "median_rel": float(np.median(r)),
        "p99_rel": float(np.quantile(r, 0.99)),
        "beyond_1e-9": int((r > 1e-9).sum()),
        "beyond_1e-6": int((r > 1e-6).sum()),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=len(os.sched_getaffinity(0)))
    ap.add_argument("--old-records", default="/tmp/full_c4_r05.npz")
    ap.add_argument("--old-status", default=os.path.join(ROOT, "tests", "golden", "full_parity_c4.npz"))
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r06_dlt_parity.json"))
    ap.add_argument("--fixture", default=os.path.join(ROOT, "tests", "golden", "dlt_parity_c4.npz"))
    ap.add_argument("--attribution", action="store_true")
    ap.add_argument("--no-write-c4", action="store_true", help="do not overwrite tests/golden/full_c4.npz")
    args = ap.parse_args()
    wl = mff.WORKLOADS["c4"]
    t0 = time.time()
    fp = mff.make_pair(wl)
    dig = mff.input_digests(fp)
    q, tr, d = orc.match_nndr(fp.desc1, fp.desc2, orc.U8, wl["eps"], args.threads)
    print(f"{len(q)} matches ({time.time() - t0:.0f} s)", flush=True)

    geo = {}
    for name, mode in MODES.items():
        with orc.geometry_mode(mode):
            pts, mask = orc.triangulate(fp.cam, fp.g12, 1.5, 2.4, fp.kp1, fp.kp2, q, tr)
            R2, t2 = orc.camera2_from_g12(fp.g12)
        geo[name] = dict(pts=pts, mask=mask, R2=R2, t2=t2)
        print(f"  {name}: {int(mask.sum())} inliers", flush=True)
    base = geo["opencv"]
    u1 = orc.undistort(fp.cam, fp.kp1[q].astype(np.float64))
    u2 = orc.undistort(fp.cam, fp.kp2[tr].astype(np.float64))
    np_pts = numpy_dlt(fp.g12, u1, u2)
    np_mask = ~((np_pts[:, 2] < 1.5) | (np_pts[:, 2] >= 2.4))
    r_np, t_np = point_table(base["pts"], base["mask"], np_pts[np_mask], np_mask)
    tables = {"opencv_vs_numpy_svd_6x4": t_np}
    r_legacy = None
    for name in MODES:
        if name == "opencv":
            continue
        r, t = point_table(geo[name]["pts"], geo[name]["mask"], base["pts"], base["mask"])
        t["R2_max_abs_diff"] = float(np.abs(geo[name]["R2"] - base["R2"]).max())
        tables[f"{name}_vs_opencv"] = t
        if name == "legacy_both":
            r_legacy = r
    print(json.dumps(tables, indent=1), flush=True)

    # the rounds 1-5 contract, reproduced: the legacy modes give the old fixture's kept points
    old = np.load(args.old_records, allow_pickle=False)
    old_status = np.load(args.old_status, allow_pickle=False)["status_detmath"].astype(np.int32)
    lg = geo["legacy_both"]
    assert len(old_status) == int(lg["mask"].sum()), "old statuses are not over the legacy inliers"
    assert np.array_equal(lg["pts"][old_status == 0], old["records"]["point"]), "legacy mode != rounds 1-5 points"
    old_normals = np.zeros((len(old_status), 3))
    old_normals[old_status == 0] = old["records"]["normal"]
    print("legacy mode reproduces the rounds 1-5 kept points bit for bit", flush=True)

    def run(g, P=None, tag=""):
        t = time.time()
        P = g["pts"] if P is None else P
        r = orc.optimize_normals(fp.cam, g["R2"], g["t2"], fp.img1, fp.img2, wl["levels"], P, wl["ray"],
                                 mode=orc.DETMATH, nthreads=args.threads)
        r["seconds"] = time.time() - t
        print(f"  LM {tag}: {int((r['status'] == 0).sum())} kept of {len(P)} ({r['seconds']:.0f} s)", flush=True)
        return r

    new = run(base, tag="opencv")
    ok = new["status"] == 0
    K = len(q)

    def by_match(g, r):
        """per-match arrays (-1: not a DLT inlier under g's geometry)"""
        st = np.full(K, -1, dtype=np.int32)
        nr = np.zeros((K, 3))
        st[g["mask"]] = r["status"]
        nr[g["mask"]] = r["normals"]
        return st, nr

    def compare(g_other, r_other):
        s_new, n_new = by_match(base, new)
        s_oth, n_oth = by_match(g_other, r_other)
        both = (s_new >= 0) & (s_oth >= 0)
        d_all, t = diff(dict(status=s_new[both], normals=n_new[both], nfev=np.ones(1)),
                        dict(status=s_oth[both], normals=n_oth[both], nfev=np.ones(1)))
        t.pop("evals_ratio", None)
        t["inlier_only_opencv"] = int(((s_new >= 0) & (s_oth < 0)).sum())
        t["inlier_only_opencv_kept"] = int(((s_new == 0) & (s_oth < 0)).sum())
        t["inlier_only_other"] = int(((s_new < 0) & (s_oth >= 0)).sum())
        t["inlier_only_other_kept"] = int(((s_new < 0) & (s_oth == 0)).sum())
        t["survivors_opencv"] = int((s_new == 0).sum())
        t["survivors_other"] = int((s_oth == 0).sum())
        d = np.full(K, np.nan)
        d[both] = d_all
        return d, t, s_oth

    oldr = dict(status=old_status, normals=old_normals)
    d_old, t_old, s_old_m = compare(lg, oldr)
    tables["legacy_both_vs_opencv_lm"] = t_old
    print(json.dumps(t_old, indent=1), flush=True)

    # the new full_c4 fixture (make_full_fixtures.py's format)
    rec = np.zeros(int(ok.sum()), dtype=mff.RECORD)
    rec["queryIdx"] = q[base["mask"]][ok]
    rec["trainIdx"] = tr[base["mask"]][ok]
    rec["distance"] = d[base["mask"]][ok]
    rec["point"] = base["pts"][ok]
    rec["normal"] = new["normals"][ok]
    counts = [len(fp.desc1), len(q), int(base["mask"].sum()), int(ok.sum())]
    if not args.no_write_c4:
        keys = sorted(dig)
        np.savez_compressed(mff.fixture_path("c4"), records=rec, digest_keys=np.array(keys),
                            digest_vals=np.array([dig[k] for k in keys]), counts=np.array(counts),
                            drops=np.array(np.bincount(new["status"], minlength=8).tolist()),
                            records_sha256=np.array(mff.records_digest(rec)), workload=np.array(repr(wl)))
        print(f"-> {mff.fixture_path('c4')} ({counts}, sha {mff.records_digest(rec)})", flush=True)

    attribution = {}
    d_attr = {}
    if args.attribution:
        for name in ("legacy_dlt", "legacy_polar"):
            r = run(geo[name], tag=name)
            dd, t, sm = compare(geo[name], r)
            attribution[f"{name}_vs_opencv_lm"] = t
            d_attr[name] = (sm, dd)
            print(json.dumps(t, indent=1), flush=True)

    # the pinned subset (indices into the OpenCV inliers): the 16 largest normal moves, 16 status
    # changes, 32 seeded points
    s_new_m, _ = by_match(base, new)
    inl = np.flatnonzero(base["mask"])  # match index of each OpenCV inlier
    d_in = np.nan_to_num(d_old[inl], nan=-1.0)
    changed = np.flatnonzero((s_old_m[inl] >= 0) & (s_old_m[inl] != new["status"]))
    rng = np.random.default_rng(6)
    pin = np.unique(np.concatenate([np.argsort(-d_in)[:16], changed[:16],
                                    rng.choice(len(inl), 32, replace=False)]))
    out = {
        "workload": "C4 frame pair (100k SIFT-128, 640x480, seed 7), pixelsRay 64, pyramids 3, every match / DLT inlier",
        "matches": int(len(q)),
        "inliers": int(base["mask"].sum()),
        "kept": int(ok.sum()),
        "records_sha256": mff.records_digest(rec),
        "threads": args.threads,
        "lm_seconds": new["seconds"],
        "points": tables,
        "attribution": attribution,
        "pinned_subset": pin.tolist(),
    }
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    extra = {}
    for name, (sm, dd) in d_attr.items():
        extra[f"status_{name}"] = sm.astype(np.int8)
        extra[f"dn_{name}"] = dd
    # per match (K entries; status -1 / dn NaN where a geometry has no inlier)
    np.savez_compressed(
        args.fixture, status_opencv=s_new_m.astype(np.int8), status_legacy=s_old_m.astype(np.int8),
        dn_legacy=d_old, rel_points_legacy=r_legacy, rel_points_numpy=r_np,
        pin_index=pin, pin_points=base["pts"][pin],
        pin_normals=new["normals"][pin], pin_status=new["status"][pin],
        R2=base["R2"], t2=base["t2"], R2_legacy=lg["R2"], img1=fp.img1, img2=fp.img2,
        cam=np.array([fp.cam.fx, fp.cam.fy, fp.cam.cx, fp.cam.cy, *fp.cam.k]), **extra)
    print(f"-> {args.out}, {args.fixture} ({time.time() - t0:.0f} s)")


if __name__ == "__main__":
    main()
