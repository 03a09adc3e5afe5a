"""Load balance of C5's query shares (bench.py --gpus N): the 1M-keypoint frame pair on ONE GPU,
share by share as rank r of N would run it, with each share's step time, LM time and survivors.
The max over shares is what bench.py's max-over-ranks clock sees at N GPUs.  --contiguous: the
contiguous blocks of shard.partition (queryOffset); default: the block-cyclic shares of
shard.query_blocks that bench.py runs.

    python tools/c5_balance.py [--ranks 2 4 8] [--contiguous] [--out gpurun_out/c5_balance.json]
"""
import argparse
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--keypoints", type=int, default=1_000_000)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--contiguous", action="store_true")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    fm3d = importlib.import_module("3dfeaturematcher_amd")
    synth = importlib.import_module("3dfeaturematcher_amd.synth")
    shard = importlib.import_module("3dfeaturematcher_amd.shard")
    t = time.time()
    pair = synth.make_frame_pair(a.keypoints, 640, 480, seed=a.seed)
    print(f"pair {a.keypoints} in {time.time() - t:.1f} s", flush=True)
    s = fm3d.Settings.default()
    s.set_camera(pair.cam)
    s.pixelsRay = 64
    s.pyramids = 3
    ctx = fm3d.Context(s)
    sct = fm3d.SingleCameraTriangulator(ctx)
    sct.set_g12(pair.g12)
    pipe = fm3d.Pipeline(ctx)
    out = {"keypoints": a.keypoints, "partition": "contiguous" if a.contiguous else f"block-cyclic ({shard.BLOCK})",
           "blocks": {}}
    n = len(pair.desc1)
    for N in a.ranks:
        rows = []
        for r in range(N):
            if a.contiguous:
                lo, hi = shard.partition(n, N, r)
                pipe.upload(pair.desc1[lo:hi], pair.desc2, pair.kp1[lo:hi], pair.kp2, pair.img1, pair.img2,
                            query_offset=lo)
                nq = hi - lo
            else:
                q = shard.query_blocks(n, N, r)
                pipe.upload(pair.desc1[q], pair.desc2, pair.kp1[q], pair.kp2, pair.img1, pair.img2, query_offset=0)
                nq = len(q)
            k, st = pipe.run()
            rows.append({"rank": r, "queries": nq, "inliers": st["inliers"], "kept": k,
                         "total_ms": st["total_ms"], "lm_ms": st["lm_ms"], "match_ms": st["match_ms"]})
            print(json.dumps({"N": N, **rows[-1]}), flush=True)
        tmax = max(x["total_ms"] for x in rows)
        tmean = sum(x["total_ms"] for x in rows) / N
        kept = sum(x["kept"] for x in rows)
        out["blocks"][str(N)] = {"rows": rows, "max_ms": tmax, "mean_ms": tmean, "balance": tmean / tmax,
                                 "kept": kept, "kept_per_s_at_max": kept / (tmax / 1e3)}
        print(f"N={N}: max {tmax:.0f} ms, mean {tmean:.0f} ms, balance {tmean / tmax:.3f}, "
              f"{kept / (tmax / 1e3):.0f} kept/s if ranks were these blocks", flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    ctx.close()


if __name__ == "__main__":
    main()
