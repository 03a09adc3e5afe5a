"""Times the widened rows on the GPU: SURF detect + describe on both VGA frames of a C4-style pair,
extractDescriptorsFromPatches on exported 128x128 patches, circular neighbourhoods, and NCC
hypothesis scoring (16 and 32 normals).  Run under rocprofv3 --kernel-trace --stats for the
kernels' own times (the calls include host copies).

    python tools/time_front.py [--patches 1300] [--points 20000] [--reps 3]
"""
import argparse
import importlib
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
fm3d = importlib.import_module("3dfeaturematcher_amd")
synth = importlib.import_module("3dfeaturematcher_amd.synth")


def timed(label, fn, reps):
    out = None
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        print(f"{label}: call {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--patches", type=int, default=1300)
    ap.add_argument("--points", type=int, default=20000)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    pair = synth.make_frame_pair(a.points, 640, 480, seed=7)
    s = fm3d.Settings.default()
    s.set_camera(pair.cam)
    ctx = fm3d.Context(s)
    try:
        surf = fm3d.SURF(ctx)
        k, d = timed("SURF detect+describe img1", lambda: surf.detect(pair.img1, with_descriptors=True), a.reps)
        print(f"  {len(k)} keypoints, descriptors {d.shape}", flush=True)
        timed("SURF detect+describe img2", lambda: surf.detect(pair.img2, with_descriptors=True), a.reps)
        rng = np.random.default_rng(2)
        patches = rng.integers(0, 256, (a.patches, 128, 128), dtype=np.uint8)
        timed(f"extractDescriptorsFromPatches x{a.patches}", lambda: surf.extractDescriptorsFromPatches(patches), a.reps)
        sc = fm3d.Settings.default()
        sc.neighMethod = 1  # circular
        ng = fm3d.NeighborhoodsGenerator(sc)
        pts = pair.points[:a.points] if hasattr(pair, "points") else rng.normal([0, 0, 2], [0.4, 0.3, 0.1], (a.points, 3))
        nrm = np.tile([0.0, 0.0, -1.0], (len(pts), 1))
        ctx2 = fm3d.Context(sc)  # the method is checked against the context's settings
        try:
            out = timed(f"circular neighbourhoods x{len(pts)}",
                        lambda: ng.computeCircularNeighborhoodsByNormals(ctx2, pts, nrm), a.reps)
        finally:
            ctx2.close()
        print(f"  output {out.shape} {out.nbytes / 1e6:.0f} MB", flush=True)
        sct = fm3d.SingleCameraTriangulator(ctx)
        sct.set_g12(pair.g12)
        no = fm3d.NormalOptimizer(ctx, sct)
        no.setImages(pair.img1, pair.img2)
        for hp, ht in ((4, 4), (8, 4)):
            timed(f"NCC {hp * ht} hypotheses x{len(pts)}", lambda: no.nccHypotheses(pts, hp, ht), a.reps)
    finally:
        ctx.close()


if __name__ == "__main__":
    main()
