"""Which quantity known before the LM runs predicts a point's LM cost (evaluations x neighbourhood
size)?  Reads tools/lm_cost_features.py's output (the C4 frame pair's per-point nfev from the GPU) and
prints Spearman correlations and the share of the total cost a longest-first order by each predictor
puts in its first 10 % (the oracle order's share is the bound), as one JSON line.

    python tools/lm_cost_predictors.py gpurun_out/lm_cost.npz
"""
import importlib
import json
import os
import sys

import numpy as np
from scipy.spatial import cKDTree
from scipy.stats import spearmanr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    d = np.load(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/lm_cost.npz")
    synth = importlib.import_module("3dfeaturematcher_amd.synth")
    pair = synth.make_frame_pair(100000, 640, 480, seed=7)
    pts, nfev = d["pts"], d["nfev"]
    uv = synth.project(pair.cam, pts)
    u, v = uv[:, 0], uv[:, 1]
    ev = nfev[:, :4].sum(1).astype(float)
    R = 64
    mdat = ((np.minimum(u + R, 639) - np.maximum(u - R, 0) + 1).clip(0) *
            (np.minimum(v + R, 479) - np.maximum(v - R, 0) + 1).clip(0) * np.pi / 4)
    cost = ev * mdat
    rng = np.random.default_rng(0)
    idx = rng.choice(len(pts), 8000, replace=False)
    img = pair.img1.astype(np.float64)
    gy, gx = np.gradient(img)
    g = np.hypot(gx, gy)
    std = np.zeros(len(idx))
    grad = np.zeros(len(idx))
    for k, i in enumerate(idx):
        y, x = int(np.clip(round(v[i]), 0, 479)), int(np.clip(round(u[i]), 0, 639))
        w = img[max(y - 32, 0):y + 33, max(x - 32, 0):x + 33]
        std[k] = w.std()
        grad[k] = g[max(y - 32, 0):y + 33, max(x - 32, 0):x + 33].mean()
    tree = cKDTree(uv)
    _, nn = tree.query(uv[idx], k=12)
    ang = np.zeros(len(idx))
    for k, i in enumerate(idx):
        Q = pts[nn[k]]
        n = np.linalg.svd(Q - Q.mean(0))[2][2]
        ang[k] = np.degrees(np.arccos(min(1.0, abs(n @ (pts[i] / np.linalg.norm(pts[i]))))))
    neigh = np.array([np.median(cost[nn[k, 1:6]]) for k in range(len(idx))])
    feats = {"m_dat": mdat[idx], "depth_z": pts[idx, 2], "image_std_65px": std, "image_grad_65px": grad,
             "u": u[idx], "v": v[idx], "local_plane_angle": ang, "coarsest_level_evals (needs a run)": nfev[idx, 0],
             "neighbours_measured_cost (needs their runs)": neigh}
    c = cost[idx]
    top = np.sort(c)[::-1][: len(c) // 10].sum() / c.sum()
    out = {"points": int(len(pts)), "evals_mean": float(ev.mean()), "evals_p99": float(np.percentile(ev, 99)),
           "oracle_first10pct_share": round(float(top), 3), "predictors": {}}
    for k, f in feats.items():
        o = np.argsort(-f)
        out["predictors"][k] = {"spearman": round(float(spearmanr(f, c).correlation), 3),
                                "first10pct_share": round(float(c[o][: len(c) // 10].sum() / c.sum()), 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
