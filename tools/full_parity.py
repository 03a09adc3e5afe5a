"""Full-set LM parity measurements on the C4 frame pair.

CPU only, oracle only (test infrastructure; no GPU).  Over EVERY DLT inlier of the C4 frame pair
(100k SIFT-128, 640x480, seed 7, pixelsRay 64, pyramids 3; 71,238 inliers) the LM is run by the
oracle (oracle/fm3d_oracle.c) in

  * DETMATH            -- the GPU contract (the records of tests/golden/full_c4.npz);
  * STRICT             -- libm transcendentals, the reference's (normals "within 1e-4");
  * DETMATH|TREE|GRAM  -- every m_dat-long sum as a fixed blocked tree and the 2-column QR from the
                          Jacobian sweep's tree sums (the reduction mode VERDICT r04 item 1 asks to
                          gate);

and compared point by point with DETMATH: status agreement, and over the points both keep the
max-abs difference of the normals.  The points where STRICT and DETMATH differ at all are then
re-run with libm for ONE transcendental at a time (sin, cos, atan2, exp) to attribute the
difference.

Writes profiles/r06_full_parity.json (the tables; round 5's, over the rounds 1-5 DLT, stay in
profiles/r05_full_parity.json) and tests/golden/full_parity_c4.npz (per-point
statuses and differences, plus the inputs and expected outputs of a small pinned subset that
tests/test_full_parity.py re-runs through the oracle).

    python tools/full_parity.py [--threads 8]
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
import oracle as orc  # noqa: E402  (checker)
import make_full_fixtures as mff  # noqa: E402

TREE, GRAM = 64, 128  # fm3d_oracle.c ORC_LM_TREE / ORC_LM_GRAM
LIBM = {"sin": 256, "cos": 512, "atan2": 1024, "exp": 2048}  # ORC_LIBM_*


def diff(base, other):
    """status agreement and normal differences of other vs base (both dicts of optimize_normals)"""
    sb, so = base["status"], other["status"]
    both = (sb == 0) & (so == 0)
    d = np.zeros(len(sb))
    d[both] = np.abs(base["normals"][both] - other["normals"][both]).max(axis=1)
    kb = int((sb == 0).sum())
    dk = d[both]
    hist_edges = [0, 1e-15, 1e-12, 1e-9, 1e-6, 1e-4, 1e-3, 1e-2, 1e-1, 10]
    return d, {
        "points": int(len(sb)),
        "status_equal": int((sb == so).sum()),
        "status_changed": int((sb != so).sum()),
        "keep_drop_changed": int(((sb == 0) != (so == 0)).sum()),
        "kept_base": kb,
        "kept_other": int((so == 0).sum()),
        "kept_both": int(both.sum()),
        "normals_bit_equal": int((dk == 0).sum()),
        "within_1e-4": int((dk <= 1e-4).sum()),
        "beyond_1e-4": int((dk > 1e-4).sum()),
        "frac_within_1e-4": float((dk <= 1e-4).mean()) if dk.size else 1.0,
        "max": float(dk.max()) if dk.size else 0.0,
        "p99": float(np.quantile(dk, 0.99)) if dk.size else 0.0,
        "p999": float(np.quantile(dk, 0.999)) if dk.size else 0.0,
        "median": float(np.median(dk)) if dk.size else 0.0,
        "histogram": {"edges": hist_edges, "counts": np.histogram(dk, bins=hist_edges)[0].tolist()},
        "evals_ratio": float(other["nfev"].sum() / max(1, base["nfev"].sum())),
    }


def attribute(run, pts, base, strict, d_strict):
    """libm for one function at a time, on the points where STRICT and DETMATH differ by more than 1e-9
    or in status ("large"), and on 2,000 seeded points among those that differ at all (a status, or
    the normal of a point both keep)"""
    anyd = (base["status"] != strict["status"]) | (d_strict != 0)
    large = np.flatnonzero((base["status"] != strict["status"]) | (d_strict > 1e-9))
    rng0 = np.random.default_rng(11)
    some = np.flatnonzero(anyd)
    some = np.sort(rng0.choice(some, min(2000, len(some)), replace=False)) if len(some) else some
    attribution = {"points_differing_at_all": int(anyd.sum()), "large_points": int(len(large)),
                   "sample_points": int(len(some))}
    for tag, sel in (("large", large), ("sample", some)):
        if not len(sel):
            continue
        sub = pts[sel]
        bsub = {k: base[k][sel] for k in ("status", "normals", "nfev")}
        ssub = {k: strict[k][sel] for k in ("status", "normals", "nfev")}
        for name, bit in list(LIBM.items()) + [("sin+cos", LIBM["sin"] | LIBM["cos"])]:
            r = run(orc.DETMATH | bit, sub)
            attribution[f"{tag}:{name}"] = {"vs_detmath": diff(bsub, r)[1], "vs_strict": diff(ssub, r)[1]}
    return attribution


def attribution_only(args, fp, wl, pts, R2, t2, t0):
    """the attribution again from the saved per-point arrays: DETMATH and STRICT re-run on the chosen
    points only (they are deterministic), then the libm variants"""
    fx = np.load(args.fixture, allow_pickle=False)
    sb, ss, d_strict = fx["status_detmath"].astype(np.int32), fx["status_strict"].astype(np.int32), fx["dn_strict"]
    assert len(sb) == len(pts)

    def run(mode, P):
        t = time.time()
        r = orc.optimize_normals(fp.cam, R2, t2, fp.img1, fp.img2, wl["levels"], P, wl["ray"], mode=mode,
                                 nthreads=args.threads)
        print(f"  mode {mode}: {len(P)} points ({time.time() - t:.0f} s)", flush=True)
        return r

    anyd = (sb != ss) | (d_strict != 0)
    cand = np.flatnonzero(anyd)
    rb, rs = run(orc.DETMATH, pts[cand]), run(orc.STRICT, pts[cand])
    assert np.array_equal(rb["status"], sb[cand]) and np.array_equal(rs["status"], ss[cand])
    nb = np.zeros((len(pts), 3))
    ns = np.zeros((len(pts), 3))
    nb[cand], ns[cand] = rb["normals"], rs["normals"]
    fb = np.ones((len(pts), 8), dtype=np.int32)
    base = dict(status=sb, normals=nb, nfev=fb)
    strict = dict(status=ss, normals=ns, nfev=fb)
    attribution = attribute(lambda mode, P: run(mode, P), pts, base, strict, d_strict)
    with open(args.out) as f:
        out = json.load(f)
    out["attribution"] = attribution
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(attribution, indent=1)[:3000])
    print(f"-> {args.out} ({time.time() - t0:.0f} s)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=len(os.sched_getaffinity(0)))
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r06_full_parity.json"))
    ap.add_argument("--fixture", default=os.path.join(ROOT, "tests", "golden", "full_parity_c4.npz"))
    ap.add_argument("--limit", type=int, default=0, help="first N inliers only (a dry run)")
    ap.add_argument("--reuse-base", action="store_true",
                    help="take the DETMATH run from full_c4.npz + dlt_parity_c4.npz instead of running it")
    ap.add_argument("--attribution-only", action="store_true",
                    help="redo only the attribution runs, from the per-point arrays of --fixture and the table of --out")
    args = ap.parse_args()
    wl = mff.WORKLOADS["c4"]
    t0 = time.time()
    fp = mff.make_pair(wl)
    q, tr, _ = orc.match_nndr(fp.desc1, fp.desc2, orc.U8, wl["eps"], args.threads)
    pts, _ = orc.triangulate(fp.cam, fp.g12, 1.5, 2.4, fp.kp1, fp.kp2, q, tr)
    if args.limit:
        pts = pts[: args.limit]
    R2, t2 = orc.camera2_from_g12(fp.g12)
    print(f"{len(pts)} inliers ({time.time() - t0:.0f} s)", flush=True)

    def run(mode, P=pts):
        t = time.time()
        r = orc.optimize_normals(fp.cam, R2, t2, fp.img1, fp.img2, wl["levels"], P, wl["ray"], mode=mode,
                                 nthreads=args.threads)
        r["seconds"] = time.time() - t
        print(f"  mode {mode}: {int((r['status'] == 0).sum())} kept ({r['seconds']:.0f} s)", flush=True)
        return r

    if args.attribution_only:
        return attribution_only(args, fp, wl, pts, R2, t2, t0)
    dlt_par = os.path.join(ROOT, "tests", "golden", "dlt_parity_c4.npz")
    if args.reuse_base and not args.limit and os.path.exists(dlt_par):
        # the DETMATH run over every inlier is tools/dlt_parity.py's (its per-match statuses and the
        # survivors' normals of full_c4.npz): not run again
        fx = mff.load_fixture("c4")
        _, mask = orc.triangulate(fp.cam, fp.g12, 1.5, 2.4, fp.kp1, fp.kp2, q, tr)
        st = np.load(dlt_par, allow_pickle=False)["status_opencv"].astype(np.int32)[mask]
        assert np.array_equal(pts[st == 0], fx["records"]["point"]), "dlt_parity_c4.npz / full_c4.npz != this geometry"
        nrm = np.zeros((len(pts), 3))
        nrm[st == 0] = fx["records"]["normal"]
        base = dict(status=st, normals=nrm, nfev=np.ones((len(pts), 8), dtype=np.int32), seconds=0.0)
        print(f"  DETMATH: from full_c4.npz + dlt_parity_c4.npz ({int((st == 0).sum())} kept)", flush=True)
    else:
        base = run(orc.DETMATH)
    if not args.limit:
        fx = mff.load_fixture("c4")
        assert int((base["status"] == 0).sum()) == len(fx["records"]), "DETMATH run != full_c4.npz"
        assert np.array_equal(base["normals"][base["status"] == 0], fx["records"]["normal"]), "DETMATH != fixture"
    strict = run(orc.STRICT)
    tree = run(orc.DETMATH | TREE | GRAM)
    d_strict, t_strict = diff(base, strict)
    d_tree, t_tree = diff(base, tree)
    _, t_tree_strict = diff(strict, tree)

    attribution = attribute(run, pts, base, strict, d_strict)

    # the pinned subset: the 16 largest STRICT moves, the 16 largest tree moves, 32 seeded random
    rng = np.random.default_rng(5)
    pin = np.unique(np.concatenate([np.argsort(-d_strict)[:16], np.argsort(-d_tree)[:16],
                                    rng.choice(len(pts), 32, replace=False)]))
    out = {
        "workload": "C4 frame pair (100k SIFT-128, 640x480, seed 7), pixelsRay 64, pyramids 3, every DLT inlier",
        "inliers": int(len(pts)),
        "threads": args.threads,
        "seconds": {"detmath": base["seconds"], "strict": strict["seconds"], "tree_gram": tree["seconds"]},
        "strict_vs_detmath": t_strict,
        "tree_gram_vs_detmath": t_tree,
        "tree_gram_vs_strict": t_tree_strict,
        "attribution": attribution,
        "pinned_subset": pin.tolist(),
    }
    print(json.dumps({k: v for k, v in out.items() if k != "pinned_subset"}, indent=1))
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    np.savez_compressed(
        args.fixture,
        status_detmath=base["status"].astype(np.int8), status_strict=strict["status"].astype(np.int8),
        status_tree=tree["status"].astype(np.int8),
        dn_strict=d_strict, dn_tree=d_tree,
        pin_index=pin, pin_points=pts[pin],
        pin_normals_detmath=base["normals"][pin], pin_normals_strict=strict["normals"][pin],
        pin_normals_tree=tree["normals"][pin],
        pin_status_detmath=base["status"][pin], pin_status_strict=strict["status"][pin],
        pin_status_tree=tree["status"][pin],
        R2=R2, t2=t2, img1=fp.img1, img2=fp.img2,
        records_sha256=np.array(mff.load_fixture("c4")["records_sha256"]) if not args.limit else np.array(""),
        cam=np.array([fp.cam.fx, fp.cam.fy, fp.cam.cx, fp.cam.cy, *fp.cam.k]),
    )
    print(f"-> {args.out}, {args.fixture} ({time.time() - t0:.0f} s)")


if __name__ == "__main__":
    main()
