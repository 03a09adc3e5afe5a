"""Times knnMatch(k = 2) of float descriptors on one GPU: the bf16 MFMA prefilter (default) against
the exact VALU scan (FM3D_F32_MFMA=0), on SURF-128 descriptors of synthetic frame pairs (real SURF
rows: unit length, neighbours with margin) pooled to N per side, and on uniform noise (the no-margin
case that falls back to the full scan).  Checks that both give byte-identical results; prints one
JSON line.  Run under rocprofv3 --kernel-trace --stats for the kernel times.

    python tools/time_f32.py [--n 100000] [--reps 3]
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
fm3d = importlib.import_module("3dfeaturematcher_amd")
synth = importlib.import_module("3dfeaturematcher_amd.synth")


def surf_pool(n, ctx):
    a, b, seed = [], [], 100
    while sum(len(x) for x in a) < n or sum(len(x) for x in b) < n:
        fp = synth.make_frame_pair(200, seed=seed)
        seed += 1
        _, da = fm3d.SURF(ctx).detect(fp.img1, with_descriptors=True)
        _, db = fm3d.SURF(ctx).detect(fp.img2, with_descriptors=True)
        a.append(da)
        b.append(db)
    return np.concatenate(a)[:n], np.concatenate(b)[:n], seed - 100


def timed(f, reps):
    f()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        out = f()
        ts.append((time.perf_counter() - t0) * 1e3)
    return out, min(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    ctx = fm3d.Context(fm3d.Settings.default())
    res = {}
    try:
        t0 = time.perf_counter()
        A, B, frames = surf_pool(args.n, ctx)
        res["surf_pool"] = {"frames": frames, "s": round(time.perf_counter() - t0, 1)}
        rng = np.random.default_rng(3)
        cases = {"surf128": (A, B), "uniform128": (rng.random((args.n // 4, 128), dtype=np.float32),
                                                   rng.random((args.n // 4, 128), dtype=np.float32))}
        m = fm3d.DescriptorsMatcher(ctx)
        for name, (a, b) in cases.items():
            got, t_mfma = timed(lambda: m.knn_match(a, b), args.reps)
            os.environ["FM3D_F32_FUSED"] = "0"
            try:
                two, t_two = timed(lambda: m.knn_match(a, b), args.reps)
            finally:
                del os.environ["FM3D_F32_FUSED"]
            os.environ["FM3D_F32_MFMA"] = "0"
            try:
                ref, t_valu = timed(lambda: m.knn_match(a, b), args.reps)
            finally:
                del os.environ["FM3D_F32_MFMA"]
            res[name] = {"nA": len(a), "nB": len(b), "mfma_fused_ms": round(t_mfma, 2),
                         "mfma_two_pass_ms": round(t_two, 2), "valu_ms": round(t_valu, 2),
                         "identical": bool(got.tobytes() == ref.tobytes() == two.tobytes())}
            print(name, res[name], flush=True)
    finally:
        ctx.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
