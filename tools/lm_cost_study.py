"""Per-point LM cost distribution on a bench scene, from the CPU oracle (identical
evaluation counts to the GPU kernel).  Used to reason about the LM kernel's tail.

    python tools/lm_cost_study.py --keypoints 20000 [--threads 8]
"""
import argparse
import importlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keypoints", type=int, default=20000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    ap.add_argument("--limit", type=int, default=0)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import oracle as orc
    synth = importlib.import_module("3dfeaturematcher_amd.synth")
    fm3d = importlib.import_module("3dfeaturematcher_amd")
    pair = synth.make_frame_pair(a.keypoints, 640, 480, seed=a.seed)
    s = fm3d.Settings.default()
    q, tr, _ = orc.match_nndr(pair.desc1, pair.desc2, orc.U8, s.nndrEpsilon, a.threads)
    pts, _ = orc.triangulate(pair.cam, pair.g12, s.zThresholdMin, s.zThresholdMax, pair.kp1, pair.kp2, q, tr)
    if a.limit:
        pts = pts[:a.limit]
    R2, t2 = fm3d.camera2_from_g12(pair.g12)
    t = time.perf_counter()
    r = orc.optimize_normals(pair.cam, R2, t2, pair.img1, pair.img2, s.pyramids, pts, s.pixelsRay,
                             mode=orc.DETMATH, nthreads=a.threads)
    dt = time.perf_counter() - t
    nf = r["nfev"].sum(1)
    m = r["mdat"]
    print(f"points {len(pts)}  oracle {dt:.1f} s  evals {nf.sum()}  pixel-evals {(nf * m).sum():.4g}")
    for qq in (50, 90, 99, 99.9, 100):
        print(f"  evals/point p{qq}: {np.percentile(nf, qq):.0f}")
    print("  status counts:", np.bincount(r["status"], minlength=8).tolist())
    if a.out:
        np.savez_compressed(a.out, nfev=r["nfev"], info=r["info"], status=r["status"], mdat=m)


if __name__ == "__main__":
    main()
