"""bench.py -- headline benchmark of the 3DFeatureMatcher hot path on MI355X.

Metric (BASELINE.json): matched + triangulated + normal-optimised keypoints/s.
Workload (BASELINE.json configs[3], "C4"): 100k SIFT-128 keypoints per 640x480
frame pair, full pipeline (exact brute-force match + NNDR -> DLT triangulation ->
LM normal refinement with pixelsRay 64 over 3+1 pyramid levels), synthetic data
(3dfeaturematcher_amd/synth.py).  One step = one frame pair through the whole
path with its inputs already resident in HBM.

Multi-GPU (one process per GPU, launched by torch.distributed.run): every rank
processes its own frame pair (weak scaling) and the per-rank survivor records
(queryIdx, trainIdx, distance, 3D point, normal) are all-gathered over RCCL.
value = keypoints kept by all ranks / max-over-ranks time.

Rank 0 at N=1 also times the CPU oracle (the reference algorithm restated in C,
OpenMP over queries/points) on a bounded sample and extrapolates (cpu_baseline).
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "matched+triangulated+normal-optimised keypoints/sec; HBM GB/s vs roofline"
FLOPS_PER_PIXEL_EVAL = 91   # restated evaluateNormal per pixel
FP64_PEAK_TFLOPS = 78.6     # MI355X fp64 (vector == matrix) peak
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--keypoints", type=int, default=100_000)
    ap.add_argument("--ray", type=int, default=64)
    ap.add_argument("--levels", type=int, default=3)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--lm-waves", type=int, default=0)
    ap.add_argument("--cpu-budget-s", type=float, default=20.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--out", type=str, default="")
    ap.add_argument("--pmc-json", type=str, default=os.path.join(ROOT, "profiles", "r01_pmc_c4_final.json"),
                    help="rocprofv3 PMC summary of the same command (HBM bytes per LM launch)")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl")  # RCCL over xGMI
        dist = tdist

    fm3d = importlib.import_module("3dfeaturematcher_amd")
    synth = importlib.import_module("3dfeaturematcher_amd.synth")

    t_gen = time.time()
    pair = synth.make_frame_pair(args.keypoints, args.width, args.height, seed=args.seed + 1000 * rank)
    t_gen = time.time() - t_gen
    s = fm3d.Settings.default()
    s.set_camera(pair.cam)
    s.pixelsRay = args.ray
    s.pyramids = args.levels
    s.lmWaves = args.lm_waves
    ctx = fm3d.Context(s, device=local if world > 1 else 0)
    sct = fm3d.SingleCameraTriangulator(ctx)
    sct.set_g12(pair.g12)
    pipe = fm3d.Pipeline(ctx)
    pipe.upload(pair.desc1, pair.desc2, pair.kp1, pair.kp2, pair.img1, pair.img2)

    rec_buf = None
    if dist is not None:
        import torch
        rec_buf = torch.empty((args.keypoints, 64), dtype=torch.uint8, device=f"cuda:{local}")
        gathered = torch.empty((world, args.keypoints, 64), dtype=torch.uint8, device=f"cuda:{local}")
        counts = torch.zeros(world, dtype=torch.int32, device=f"cuda:{local}")

    def step():
        n, st = pipe.run(rec_buf.data_ptr() if rec_buf is not None else None)
        if dist is not None:
            import torch
            mine = torch.tensor([n], dtype=torch.int32, device=rec_buf.device)
            dist.all_gather_into_tensor(counts, mine)
            dist.all_gather_into_tensor(gathered.view(-1), rec_buf.view(-1))
        return n, st

    for _ in range(args.warmup):
        step()

    def sync():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()
            torch.cuda.synchronize()

    sync()
    t0 = time.perf_counter()
    kept_total = 0
    stats = []
    for _ in range(args.steps):
        n, st = step()
        kept_total += n
        stats.append(st)
    sync()
    elapsed = time.perf_counter() - t0

    all_kept = kept_total
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device=rec_buf.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        k = torch.tensor([kept_total], dtype=torch.int64, device=rec_buf.device)
        dist.all_reduce(k, op=dist.ReduceOp.SUM)
        all_kept = int(k.item())

    lm_ms = float(np.mean([st["lm_ms"] for st in stats]))
    traffic = pmc_traffic(args)
    pix = float(np.mean([st["lm"]["pixel_evaluations"] for st in stats]))
    evals = float(np.mean([st["lm"]["evaluations"] for st in stats]))
    last = stats[-1]
    achieved_tflops = FLOPS_PER_PIXEL_EVAL * pix / (lm_ms * 1e-3) / 1e12 if lm_ms > 0 else 0.0

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(pair, s, last, args)

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": all_kept / elapsed,
            "unit": "keypoints/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (ray-cast facet scene, seeded; 3dfeaturematcher_amd/synth.py)",
            "config": {
                "workload": f"C4: {args.keypoints // 1000}k SIFT-128 (u8) keypoints per {args.width}x{args.height} "
                            f"frame pair, full pipeline, pixelsRay {args.ray}, pyramids {args.levels}",
                "keypoints_per_frame": args.keypoints, "pixelsRay": args.ray, "pyramids": args.levels,
                "parallelism": f"dp{world}: one frame pair per rank, RCCL all-gather of survivor records",
            },
            "roofline": {
                "kernel": "fm3d::lm2_kernel (LM normal refinement)",
                "bound": "mfma",
                "compute": "fp64 (issued on the VALU; MI355X fp64 matrix and vector peaks coincide at 78.6 TFLOP/s)",
                "achieved": achieved_tflops,
                "peak": FP64_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": achieved_tflops / FP64_PEAK_TFLOPS,
                "traffic": traffic["bytes"] if traffic else None,
                "traffic_unit": "bytes per launch (HBM, rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)",
                "traffic_GBps": traffic["bytes"] / (lm_ms * 1e6) if traffic and lm_ms > 0 else None,
                "traffic_source": traffic["source"] if traffic else None,
                "algorithmic": f"{FLOPS_PER_PIXEL_EVAL} flop per pixel evaluation x {pix:.4g} pixel evaluations "
                               f"({evals:.4g} residual evaluations) per launch",
                "avg_launch_ms": lm_ms,
            },
            "cpu_baseline": cpu,
            "stages_ms": {k: last[k] for k in ("match_ms", "nndr_ms", "triangulate_ms", "lm_ms", "total_ms")},
            "counts": {k: last[k] for k in ("queries", "matches", "inliers", "kept")},
            "lm_profile": lm_profile(last["lm"]),
            "setup_s": {"synthetic_generation": round(t_gen, 2)},
        }
        line = json.dumps(out)
        print(line, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(line + "\n")
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def pmc_traffic(args):
    """HBM bytes per LM launch from the committed rocprofv3 PMC summary of this workload
    (separate --pmc passes; rocprofv3 cannot run inside the timed process)."""
    try:
        with open(args.pmc_json) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    w = d.get("workload", {})
    if (w.get("keypoints"), w.get("ray"), w.get("levels")) != (args.keypoints, args.ray, args.levels):
        return None
    return {"bytes": d["hbm_bytes_per_launch"], "source": os.path.relpath(args.pmc_json, ROOT)}


def lm_profile(lm):
    """Where the LM kernel's time goes (in-kernel clock counters, fm3d_lm_stats)."""
    tot = lm["cycles_total"]
    return {
        "groups": lm["groups"], "passes": lm["passes"],
        "chain_busy": lm["cycles_chain"] / tot if tot else None,    # chain wave adding / group lifetime
        "control_over_terms": lm["cycles_control"] / max(lm["cycles_terms"], 1),  # lmdif bookkeeping
        "wait_over_terms": lm["cycles_wait"] / max(lm["cycles_terms"], 1),        # term waves waiting on the chain
        # mean number of term waves inside a pass over the lifetime of a workgroup's first wave
        "busy_slots_per_group": lm["cycles_terms"] / tot if tot else None,
        "group_life_mean_over_max": lm["wall_ticks_sum"] / max(lm["groups"], 1) / max(lm["wall_ticks_max"], 1),
        "clock_ghz": lm["cycles_total"] / max(lm["wall_ticks_sum"], 1) * lm["wall_clock_khz"] * 1e-6,
        "kcycles_per_pass_by_class": {n: round(cy / max(c, 1) / 1e3, 1) for n, c, cy in
                                      zip(("jac", "eval", "qr", "once"), lm["class_passes"], lm["class_cycles"])},
        "passes_by_class": dict(zip(("jac", "eval", "qr", "once"), lm["class_passes"])),
        "last_group_end_ms": lm["last_group_end_ticks"] / max(lm["wall_clock_khz"], 1),
    }


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(pair, s, gpu_stats, args):
    """Time the CPU oracle (reference algorithm, C + OpenMP) on a bounded sample of the
    same workload and extrapolate to the full frame pair."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    budget = args.cpu_budget_s
    nA = len(pair.desc1)
    # match: sample of queries against the full train set
    qs = 64
    while True:
        t = time.perf_counter()
        orc.knn2(pair.desc1[:qs], pair.desc2, orc.U8, threads)
        dt = time.perf_counter() - t
        if dt > 0.15 * budget or qs >= nA:
            break
        qs = min(nA, qs * 4)
    t_match = dt / qs * nA
    # triangulation on the GPU's matches (full set)
    q, tr, _ = orc.match_nndr(pair.desc1[:2000], pair.desc2, orc.U8, s.nndrEpsilon, threads)
    t = time.perf_counter()
    pts, _ = orc.triangulate(pair.cam, pair.g12, s.zThresholdMin, s.zThresholdMax, pair.kp1, pair.kp2, q, tr)
    t_tri = (time.perf_counter() - t) / max(len(q), 1) * gpu_stats["matches"]
    # LM normals: sample of points
    fm3d = importlib.import_module("3dfeaturematcher_amd")
    R2, t2 = fm3d.camera2_from_g12(pair.g12)
    # a seeded random subset (per-point LM cost varies by orders of magnitude), 16 points per
    # thread so the dynamic schedule balances
    sub = np.random.default_rng(7).permutation(len(pts))
    npts = min(len(pts), 16 * threads)
    t = time.perf_counter()
    r = orc.optimize_normals(pair.cam, R2, t2, pair.img1, pair.img2, s.pyramids, pts[sub[:npts]], s.pixelsRay,
                             mode=orc.STRICT, nthreads=threads)
    dt = time.perf_counter() - t
    t_lm = dt / npts * gpu_stats["inliers"]
    total = t_match + t_tri + t_lm
    # the same stages on one core (both 1-thread and all-cores figures)
    t = time.perf_counter()
    orc.knn2(pair.desc1[:256], pair.desc2, orc.U8, 1)
    t1_match = (time.perf_counter() - t) / 256 * nA
    t = time.perf_counter()
    n1 = min(len(pts), 16)
    orc.optimize_normals(pair.cam, R2, t2, pair.img1, pair.img2, s.pyramids, pts[sub[:n1]], s.pixelsRay,
                         mode=orc.STRICT, nthreads=1)
    t1_lm = (time.perf_counter() - t) / n1 * gpu_stats["inliers"]
    total1 = t1_match + t_tri + t1_lm
    return {
        "value": gpu_stats["kept"] / total,
        "unit": "keypoints/s",
        "cores": threads,
        "kind": "port",
        "cpu_model": cpu_model(),
        "single_thread": {"value": gpu_stats["kept"] / total1, "unit": "keypoints/s", "cores": 1,
                          "sample": f"knn2 of 256 queries, LM normals of {n1} points, 1 thread (est. {total1:.0f} s "
                                    f"per frame pair: match {t1_match:.1f}, LM {t1_lm:.1f})"},
        "sample": f"oracle (C, OpenMP {threads} threads): knn2 of {qs} queries x {len(pair.desc2)} train, "
                  f"DLT of {len(q)} matches, LM normals of {npts} random points (pixelsRay {s.pixelsRay}); "
                  f"extrapolated to {nA} queries / {gpu_stats['matches']} matches / {gpu_stats['inliers']} points "
                  f"(est. {total:.1f} s per frame pair: match {t_match:.1f}, DLT {t_tri:.3f}, LM {t_lm:.1f})",
    }


if __name__ == "__main__":
    main()
