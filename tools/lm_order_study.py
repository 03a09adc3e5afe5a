"""How much of the LM launch is the end-of-queue tail, and how much a better point order would
recover: the C4 frame pair's inliers through computeOptimizedNormals in index order, then in
longest-first order of their measured cost (evaluations x m_dat of the first run: an upper bound
for any cost predictor), then in a random order.  The per-point results do not depend on the
order (checked); only the schedule changes.

    python tools/lm_order_study.py [--keypoints 100000] [--reps 2] [--out gpurun_out/order.json]
"""
import argparse
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keypoints", type=int, default=100000)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--ray", type=int, default=64)
    ap.add_argument("--levels", type=int, default=3)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    fm3d = importlib.import_module("3dfeaturematcher_amd")
    synth = importlib.import_module("3dfeaturematcher_amd.synth")
    pair = synth.make_frame_pair(a.keypoints, 640, 480, seed=a.seed)
    s = fm3d.Settings.default()
    s.set_camera(pair.cam)
    s.pixelsRay = a.ray
    s.pyramids = a.levels
    ctx = fm3d.Context(s)
    dm = fm3d.DescriptorsMatcher(ctx)
    m = dm.compareWithNNDR(s.nndrEpsilon, pair.desc1, pair.desc2)
    sct = fm3d.SingleCameraTriangulator(ctx)
    sct.set_g12(pair.g12)
    sct.setKeypoints(pair.kp1, pair.kp2, m)
    pts, _ = sct.triangulate()
    no = fm3d.NormalOptimizer(ctx, sct)
    no.setImages(pair.img1, pair.img2)
    print(f"points {len(pts)}", flush=True)

    def run(order, tag):
        res = []
        for _ in range(a.reps):
            kept, normals = no.computeOptimizedNormals(pts[order])
            st = no.last_stats
            khz = max(st["wall_clock_khz"], 1)
            r = {"order": tag, "kernel_ms": st["kernel_ms"], "last_end_ms": st["last_group_end_ticks"] / khz,
                 "queue_empty_ms": st["queue_empty_ticks"] / khz,
                 "group_life_mean_over_max": st["wall_ticks_sum"] / max(st["groups"], 1) / max(st["wall_ticks_max"], 1)}
            res.append(r)
            print(json.dumps(r), flush=True)
        inv = np.empty_like(order)
        inv[order] = np.arange(len(order))
        return res, no.last_status[inv].copy(), no.last_nfev[inv].copy()

    out = {"points": int(len(pts))}
    idx = np.arange(len(pts))
    out["index"], st0, nf0 = run(idx, "index")
    # m_dat is not returned per point; the oracle study shows cost ~ evaluations (m barely varies)
    cost = nf0.sum(1).astype(np.float64)
    lpt = np.argsort(-cost, kind="stable")
    out["lpt"], st1, nf1 = run(lpt, "longest-first (measured cost)")
    assert np.array_equal(st0, st1) and np.array_equal(nf0, nf1), "order changed per-point results"
    rnd = np.random.default_rng(1).permutation(len(pts))
    out["random"], _, _ = run(rnd, "random")
    out["cost_percentiles"] = {str(q): float(np.percentile(cost, q)) for q in (10, 50, 90, 99, 100)}
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    ctx.close()


if __name__ == "__main__":
    main()
