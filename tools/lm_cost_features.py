"""Per-point LM cost of the C4 frame pair on the GPU (evaluations per pyramid level from
computeOptimizedNormals' nfev) saved with the points, for an offline search for a cost predictor
(the end-of-queue tail: a longest-first order recovers up to ~8 %).

    python tools/lm_cost_features.py --out gpurun_out/lm_cost.npz
"""
import argparse
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/lm_cost.npz")
    a = ap.parse_args()
    fm3d = importlib.import_module("3dfeaturematcher_amd")
    synth = importlib.import_module("3dfeaturematcher_amd.synth")
    pair = synth.make_frame_pair(100000, 640, 480, seed=7)
    s = fm3d.Settings.default()
    s.set_camera(pair.cam)
    s.pixelsRay, s.pyramids = 64, 3
    ctx = fm3d.Context(s)
    m = fm3d.DescriptorsMatcher(ctx).compareWithNNDR(s.nndrEpsilon, pair.desc1, pair.desc2)
    sct = fm3d.SingleCameraTriangulator(ctx)
    sct.set_g12(pair.g12)
    sct.setKeypoints(pair.kp1, pair.kp2, m)
    pts, mask = sct.triangulate()
    no = fm3d.NormalOptimizer(ctx, sct)
    no.setImages(pair.img1, pair.img2)
    kept, normals = no.computeOptimizedNormals(pts)
    np.savez_compressed(a.out, pts=pts, matches=m, mask=mask, status=no.last_status, info=no.last_info,
                        nfev=no.last_nfev)
    ctx.close()
    print("saved", a.out, len(pts), flush=True)


if __name__ == "__main__":
    main()
