"""Times knnMatch(k=2) on the GPU for each descriptor type at a given size (wall clock of the
C-ABI call, H2D/D2H included; run under rocprofv3 --kernel-trace --stats for kernel times).

    python tools/time_match.py [--n 100000] [--reps 3]
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
    ap.add_argument("--n", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--kinds", default="surf64_f32,sift128_f32,sift128_u8,orb256_bits")
    args = ap.parse_args()
    rng = np.random.default_rng(3)
    n = args.n
    cases = {
        "surf64_f32": rng.random((2, n, 64), dtype=np.float32) * 0.25,
        "sift128_f32": rng.random((2, n, 128), dtype=np.float32) * 100.3,
        "sift128_u8": rng.integers(0, 256, (2, n, 128), dtype=np.uint8),
        "orb256_bits": rng.integers(0, 256, (2, n, 32), dtype=np.uint8),
    }
    ctx = fm3d.Context(fm3d.Settings.default())
    try:
        for name, d in cases.items():
            if name not in args.kinds.split(","):
                continue
            m = fm3d.DescriptorsMatcher(ctx, binary=name.endswith("bits"))
            ts = []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                m.knn_match(d[0], d[1])
                ts.append(time.perf_counter() - t0)
            print(f"{name}: n={n} wall ms " + " ".join(f"{1e3 * t:.1f}" for t in ts), flush=True)
    finally:
        ctx.close()


if __name__ == "__main__":
    main()
