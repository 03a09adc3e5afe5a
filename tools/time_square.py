"""Times computeSquareNeighborhoodsByNormals and the patch export on the GPU (build/settings.yml grid: 128 x 128 points
per frame, 24 B written per point).  Run under rocprofv3 --kernel-trace --stats for the kernel's
own time (the call itself includes the D2H copy of the host output buffer).

    python tools/time_square.py [--frames 1300] [--reps 3]
"""
import argparse
import importlib
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
fm3d = importlib.import_module("3dfeaturematcher_amd")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1300)  # 1300 x 16384 x 24 B = 511 MB: one chunk
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    rng = np.random.default_rng(1)
    frames = np.zeros((args.frames, 4, 4))
    frames[:, :3, :3] = np.linalg.qr(rng.normal(size=(args.frames, 3, 3)))[0]
    frames[:, :3, 3] = rng.normal(0, 1, (args.frames, 3))
    frames[:, 3, 3] = 1
    s = fm3d.Settings.default()
    ctx = fm3d.Context(s)
    try:
        ng = fm3d.NeighborhoodsGenerator(s)
        for _ in range(args.reps):
            t0 = time.perf_counter()
            out = ng.computeSquareNeighborhoodsByNormals(ctx, frames)
            dt = time.perf_counter() - t0
            print(f"frames {args.frames}: {out.shape[1]} points each, {out.nbytes / 1e6:.0f} MB, "
                  f"call {1e3 * dt:.1f} ms (incl. D2H)", flush=True)
        # projectReferencePointsToImageWithFrames on a synthetic image (128x128 8-bit patches)
        no = fm3d.NormalOptimizer(ctx)
        img = rng.integers(0, 256, (480, 640), dtype=np.uint8)
        no.setImages(img, img)
        sct = fm3d.SingleCameraTriangulator(ctx)
        fr = frames.copy()
        fr[:, :3, 3] = np.array([0.0, 0.0, 2.0]) + rng.normal(0, 0.3, (args.frames, 3))
        for _ in range(args.reps):
            t0 = time.perf_counter()
            patches = sct.projectReferencePointsToImageWithFrames(None, fr)
            dt = time.perf_counter() - t0
            print(f"patches {args.frames}: {patches.nbytes / 1e6:.0f} MB, call {1e3 * dt:.1f} ms", flush=True)
    finally:
        ctx.close()


if __name__ == "__main__":
    main()
