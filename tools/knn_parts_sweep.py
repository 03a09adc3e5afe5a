"""knnMatch(k=2) of random u8 SIFT-128 rows at n x n under several FM3D_I8_PARTS settings, in
launch order (run under rocprofv3 --kernel-trace; tools/kstats.py-style per-dispatch durations
are read from the trace in the same order).

    python tools/knn_parts_sweep.py [--n 100000] [--parts auto,1,2,4,8,16] [--reps 3]
"""
import argparse
import importlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
fm3d = importlib.import_module("3dfeaturematcher_amd")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000)
    ap.add_argument("--parts", default="1,2,4,8,16")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--binary", action="store_true")
    args = ap.parse_args()
    rng = np.random.default_rng(3)
    w = 32 if args.binary else 128
    d = rng.integers(0, 256, (2, args.n, w), dtype=np.uint8)
    ctx = fm3d.Context(fm3d.Settings.default())
    try:
        m = fm3d.DescriptorsMatcher(ctx, binary=args.binary)
        ref = None
        for p in args.parts.split(","):
            if p == "auto":
                os.environ.pop("FM3D_I8_PARTS", None)
            else:
                os.environ["FM3D_I8_PARTS"] = p
            for _ in range(args.reps):
                r = m.knn_match(d[0], d[1])
                if ref is None:
                    ref = r
                else:
                    assert np.array_equal(r, ref), p
            print(f"parts {p}: {args.reps} calls, results equal", flush=True)
    finally:
        ctx.close()


if __name__ == "__main__":
    main()
