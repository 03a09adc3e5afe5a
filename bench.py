"""bench.py -- headline benchmark of the 3DFeatureMatcher hot path on MI355X.

Metric (BASELINE.json): matched + triangulated + normal-optimised keypoints/s.

Workloads (BASELINE.json configs):
  * C4 (configs[3], the default at one GPU): 100k SIFT-128 keypoints per 640x480 frame
    pair, full pipeline (exact brute-force match + NNDR -> DLT triangulation -> LM normal
    refinement with pixelsRay 64 over 3+1 pyramid levels).
  * C5 (configs[4], the default at N > 1 GPUs): ONE 1M-keypoint frame pair (the C4 scene and
    settings, 1M sub-pixel keypoints per 640x480 frame), sharded over the N
    ranks: rank r takes the query blocks shard.query_blocks(1M, N, r) (4,096
    queries each, dealt round-robin so every rank gets the same mix: contiguous blocks left the
    last rank the synthetic frame's distractor tail, a fifth of the others' work) against all
    of frame B (replicated), runs the whole path on its GPU, and the per-rank survivor records
    (queryIdx, trainIdx, distance, 3D point, normal) are all-gathered over RCCL (counts, then
    fixed-capacity record buffers) every step.  value = kept keypoints of the frame pair /
    max-over-ranks time (strong scaling).  After the timed steps rank 0 runs the same frame
    pair unsharded on its GPU and checks that the merge of the gathered records (local query
    indices mapped back, in query order) is byte-identical to it.
  * --weak: the round-1 mode, every rank its own C4 frame pair (weak scaling), labelled weak.

One step = one frame pair (or one shard of it) through the path with its inputs already
resident in HBM: descriptors, keypoints and the image pyramids are uploaded / built before
the timed region (upload_ms in the line), the survivor records stay in HBM (or go to the
all-gather).  Synthetic data: 3dfeaturematcher_amd/synth.py (seeded ray-cast facet scene).

Rank 0 at N=1 also times the CPU oracle (the reference algorithm restated in C, OpenMP over
queries/points, on every CPU the process may run on) on a bounded sample and extrapolates
(cpu_baseline).
"""
from __future__ import annotations

import argparse
import hashlib
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
FP64_PEAK_TFLOPS = 78.6     # MI355X fp64 vector peak, an FMA counted as 2 flops
FP64_PEAK_NO_FMA = 39.3     # the same issue rate for 1-flop instructions (-ffp-contract=off: no FMA)
HBM_PEAK_GBS = 8000.0
WORKLOADS = {"c4": dict(keypoints=100_000, width=640, height=480),
             "c5": dict(keypoints=1_000_000, width=640, height=480),
             "c2": dict(keypoints=10_000, width=640, height=480),
             "c3": dict(keypoints=10_000, width=640, height=480)}
INT8_PEAK_TOPS = 5000.0      # MI355X dense int8 MFMA (2x the ~2.5 PFLOP/s dense bf16; MI355X_MICROARCH.md)


WORKLOAD_DEFAULTS = {
    "c4": {"ray": 64, "nndr": 0.55, "seed": 7, "inflight": 2},
    "c5": {"ray": 64, "nndr": 0.55, "seed": 7, "inflight": 2},
    # C2: three contexts in flight (one box, 400 steps each: 2 -> 0.070, 3 -> 0.055, 4 -> 0.060 ms)
    "c2": {"ray": 64, "nndr": 0.55, "seed": 7, "inflight": 3},
    # C3's ORB rows: the 0.8 ratio and the 64 x 64 neighbourhood of BASELINE's wording; four contexts
    # in flight (one box, 60 steps each: 1 -> 1.66, 2 -> 1.52, 3 -> 1.49, 4 -> 1.47 ms per frame pair)
    "c3": {"ray": 32, "nndr": 0.8, "seed": 102, "inflight": 4},
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=("auto", "c4", "c5", "c2", "c3"), default="auto",
                    help="auto: C4 at one GPU, C5 (one sharded 1M-keypoint frame pair) at N > 1; c2: BASELINE's "
                         "C2 (10k SIFT per frame, match + DLT triangulate only, one GPU); c3: BASELINE's C3 as "
                         "worded (10k ORB, Hamming match + DLT + 64x64-patch NCC over 16 normal hypotheses)")
    ap.add_argument("--weak", action="store_true", help="every rank its own C4 frame pair (weak scaling)")
    ap.add_argument("--keypoints", type=int, default=0)
    ap.add_argument("--width", type=int, default=0)
    ap.add_argument("--height", type=int, default=0)
    # None: the workload's own value (C2 / C4 / C5: pixelsRay 64, NNDR 0.55, seed 7; C3: 32, 0.8, 102)
    ap.add_argument("--ray", type=int, default=None)
    ap.add_argument("--levels", type=int, default=3)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--desc", choices=("sift", "orb"), default="sift",
                    help="descriptor kind of the synthetic pair (orb: 256-bit, Hamming; BASELINE C3 with "
                         "--keypoints 10000 --seed 102 --nndr 0.8 --ray 32|64)")
    ap.add_argument("--nndr", type=float, default=None)
    ap.add_argument("--desc-dtype", choices=("u8", "f32"), default="u8",
                    help="SIFT rows as u8, or as the float cv::Mat rows the reference's knnMatch receives "
                         "(descriptorsmatcher.cpp:114-117; checked and packed to u8 on the device)")
    ap.add_argument("--io", choices=("resident", "host"), default="resident",
                    help="C2: resident -- inputs uploaded once, steps on HBM-resident inputs; host -- every step "
                         "one frame pair's descriptors and keypoints from host memory and its matches and "
                         "inlier points back to host memory")
    ap.add_argument("--lm-waves", type=int, default=0)
    ap.add_argument("--lm-tree", action="store_true",
                    help="settings.lmReduction = 1: the opt-in tree-reduction LM (fails the parity gate; A/B only)")
    ap.add_argument("--mode", choices=("stream", "resident"), default="stream",
                    help="stream (C4 headline): every step a frame pair from host memory to host memory, "
                         "--inflight pairs in flight; resident: inputs uploaded once, one step in flight")
    ap.add_argument("--inflight", type=int, default=None,
                    help="LM launches in flight in the stream mode (C4 / C5: 2); contexts in flight for C2 (3) / C3 (4)")
    ap.add_argument("--lm-pairs", type=int, default=2,
                    help="frame pairs per LM launch in the stream mode (2-4: fm3d_pipeline_link)")
    ap.add_argument("--mgpu", action="store_true",
                    help="the one-process multi-GPU path (fm3d_mgpu, C5) also at --gpus 1 (its reference point)")
    ap.add_argument("--alias-devices", action="store_true",
                    help="diagnostic, not a bench line: --gpus N --mgpu with device 0 listed N times "
                         "(fm3d_mgpu's test mode FM3D_DEBUG_MGPU_ALIAS): the N-device host path on one GPU")
    ap.add_argument("--cpu-budget-s", type=float, default=20.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-check", action="store_true", help="skip the C5 byte-identity check against one GPU")
    ap.add_argument("--ref-steps", type=int, default=2,
                    help="--gpus N > 1: frame pairs of the same C5 stream on device 0 alone after the timed steps "
                         "(value_one_gpu, efficiency); 0 skips")
    ap.add_argument("--out", type=str, default="")
    ap.add_argument("--dump-records", type=str, default="",
                    help="torchrun C5: rank 0 saves the last step's merged survivor records (.npy)")
    ap.add_argument("--pmc-json", type=str, default=next(
        (p for p in (os.path.join(ROOT, "profiles", f"r0{r}_pmc_c4.json") for r in (6, 5, 4, 3, 2)) if os.path.exists(p)),
        os.path.join(ROOT, "profiles", "r02_pmc_c4.json")),
                    help="rocprofv3 PMC summary of the same command (HBM bytes per LM launch)")
    return ap.parse_args()


def desc_rows(args, a):
    """the descriptor rows as the caller hands them (--desc-dtype): u8, or SIFT's float cv::Mat rows"""
    return a.astype(np.float32) if getattr(args, "desc_dtype", "u8") == "f32" and a.dtype == np.uint8 and \
        args.desc != "orb" else a


def records_digest(rec_bytes: bytes) -> str:
    return hashlib.sha256(rec_bytes).hexdigest()[:16]


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    workload = args.workload
    if workload == "auto":
        workload = "c5" if (world > 1 or args.gpus > 1 or args.mgpu) and not args.weak else "c4"
    if args.weak:
        workload = "c4"
    for k, v in WORKLOAD_DEFAULTS.get(workload, WORKLOAD_DEFAULTS["c4"]).items():
        if getattr(args, k) is None:  # only what the command line left open
            setattr(args, k, v)
    if world == 1 and (args.gpus > 1 or args.mgpu):
        # the driver's `bench.py --gpus N` without a torchrun environment: this one process drives
        # N GPUs through the C ABI's multi-GPU host (fm3d_mgpu)
        return run_mgpu(args, workload)
    if workload == "c2":
        return run_c2(args)
    if workload == "c3":
        return run_c3(args)
    if world == 1 and workload == "c4" and args.mode == "stream":
        return run_c4_stream(args)
    if world > 1 and not args.weak and args.mode == "stream":
        return run_torchrun_stream(args, workload)
    return run_resident(args, workload)


def emit(out, args):
    line = json.dumps(out)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


def lm_workload(args):
    return {"pixelsRay": args.ray, "pyramids": args.levels}


def c4_settings(fm3d, pair, args):
    s = fm3d.Settings.default()
    s.set_camera(pair.cam)
    s.nndrEpsilon = args.nndr
    s.pixelsRay = args.ray
    s.pyramids = args.levels
    s.lmWaves = args.lm_waves
    s.lmReduction = 1 if getattr(args, "lm_tree", False) else 0
    return s


def run_c4_stream(args):
    """The headline (BASELINE configs[3], C4) as a stream of frame pairs, SURVEY.md §8(d)'s timed
    region: every step takes one frame pair from host memory through the whole path and back --
    H2D of descriptors, keypoints and both images (pinned staging), the a6 pyramids, match -> NNDR
    -> DLT -> LM normals -> survivor records, D2H of the records -- with `inflight` frame pairs in
    flight on as many contexts (one HIP stream each; fm3d_pipeline_submit / fm3d_pipeline_wait).
    The next pair's front half and LM workgroups take the CUs the previous LM launch frees in its
    tail, which a single launch leaves idle.  value = kept keypoints of the K timed
    pairs / the host wall time of the K steps (fill and drain of the pipeline included)."""
    import torch
    fm3d = importlib.import_module("3dfeaturematcher_amd")
    synth = importlib.import_module("3dfeaturematcher_amd.synth")
    wl = dict(WORKLOADS["c4"])
    for k in ("keypoints", "width", "height"):
        if getattr(args, k):
            wl[k] = getattr(args, k)
    t_gen = time.time()
    pair = synth.make_frame_pair(wl["keypoints"], wl["width"], wl["height"], seed=args.seed, desc=args.desc)
    t_gen = time.time() - t_gen
    s = c4_settings(fm3d, pair, args)
    nl = max(1, args.lm_pairs)
    nf = max(1, args.inflight) * nl  # contexts: `inflight` LM launches of `lm_pairs` frame pairs each
    streams = [torch.cuda.Stream(device=0) for _ in range(nf)]
    ctxs, pipes = [], []
    for st in streams:
        ctx = fm3d.Context(s, device=0)
        ctx.set_stream(st.cuda_stream)
        fm3d.SingleCameraTriangulator(ctx).set_g12(pair.g12)
        ctxs.append(ctx)
        pipes.append(fm3d.Pipeline(ctx))
    if not 1 <= nl <= 4:
        raise SystemExit("--lm-pairs: 1 to 4")
    # contexts nl*i .. nl*i + nl - 2 join the LM launches of context nl*i + nl - 1 (fm3d_pipeline_link)
    for i in range(0, nf, nl):
        for j in range(i, i + nl - 1):
            pipes[j].link(pipes[i + nl - 1])
    binary = args.desc == "orb"
    bufs = [np.zeros(len(pair.desc1), dtype=fm3d.RECORD) for _ in range(nf)]
    inputs = (desc_rows(args, pair.desc1), desc_rows(args, pair.desc2), pair.kp1, pair.kp2, pair.img1, pair.img2)

    def stream_run(n_steps, timed):
        """n_steps frame pairs through the pipeline; returns per-pair (kept, stats, latency s, digest)."""
        res = []
        pend = [None] * nf
        ends = [None] * nf
        t_sub = [0.0] * nf

        def drain(j):
            rec, st = pipes[j].wait(bufs[j])
            res.append((len(rec), st, time.perf_counter() - t_sub[j], records_digest(rec.tobytes())))
            pend[j] = None
            return rec

        last = None
        for k in range(n_steps):
            j = k % nf
            if pend[j] is not None:
                last = drain(j)
            t_sub[j] = time.perf_counter()
            pipes[j].submit(*inputs, binary=binary)
            if timed:
                ends[j] = torch.cuda.Event(enable_timing=True)
                ends[j].record(streams[j])
            pend[j] = True
        for k in range(n_steps, n_steps + nf):  # drain in submission order
            j = k % nf
            if pend[j] is not None:
                last = drain(j)
        return res, ends, last

    stream_run(args.warmup, False)
    torch.cuda.synchronize()
    start = torch.cuda.Event(enable_timing=True)
    start.record(streams[0])
    for st in streams[1:]:
        st.wait_stream(streams[0])
    t0 = time.perf_counter()
    res, ends, last_rec = stream_run(args.steps, True)
    elapsed = time.perf_counter() - t0
    torch.cuda.synchronize()
    span_ms = max(start.elapsed_time(e) for e in ends if e is not None)
    kept_total = sum(r[0] for r in res)
    stats = [r[1] for r in res]
    lat = [r[2] * 1e3 for r in res]
    digests = sorted(set(r[3] for r in res))
    last_st = stats[-1]
    # the same frame pair HBM-resident, one launch at a time (the pre-round-4 headline): inputs
    # uploaded once, pipe.run() per step -- the per-launch roofline of lm2_kernel
    res_steps = max(1, min(3, args.steps))
    pipes[0].upload(*inputs, binary=binary)
    pipes[0].run()
    t1 = time.perf_counter()
    rstats = [pipes[0].run()[1] for _ in range(res_steps)]
    res_elapsed = time.perf_counter() - t1
    for c in ctxs:
        c.close()
    pix = float(np.mean([st["lm"]["pixel_evaluations"] for st in stats]))
    evals = float(np.mean([st["lm"]["evaluations"] for st in stats]))
    cpu = None
    if not args.no_cpu and args.desc == "sift":
        cpu = cpu_baseline(pair, s, last_st, args)
    rlm_ms = float(np.mean([st["lm_ms"] for st in rstats]))
    roof = roofline(stats, span_ms / args.steps, pix, evals, args, pair, s)
    roof.update({
        "kernel": "fm3d::lm2_kernel (LM normal refinement), launches overlapped two at a time",
        "avg_launch_ms": span_ms / args.steps,
        "achieved_basis": (f"{FLOPS_PER_PIXEL_EVAL} flop x the pixel evaluations of the {args.steps} timed LM launches / "
                           f"the device span of the timed region ({span_ms:.1f} ms, HIP events on the context "
                           f"streams: first submit -> last pair's records); avg_launch_ms = that span / launches"),
        "overlapped_launch_ms_each": float(np.mean([st["lm_ms"] for st in stats])),
        # PMC bytes are measured on one resident launch: divide by that launch's time, not the span
        "traffic_GBps": roof["traffic"] / (rlm_ms * 1e6) if roof.get("traffic") and rlm_ms > 0 else None,
        "traffic_GBps_basis": ("HBM bytes of one resident launch (rocprofv3 PMC, traffic_source) / the resident "
                               "launch's HIP-event time (single_launch.avg_launch_ms): both one launch at a time"),
        "single_launch": {
            "avg_launch_ms": rlm_ms,
            "achieved": FLOPS_PER_PIXEL_EVAL * pix / (rlm_ms * 1e-3) / 1e12,
            "frac": FLOPS_PER_PIXEL_EVAL * pix / (rlm_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
            "note": "one launch in flight (HBM-resident inputs, fm3d_pipeline_run), HIP events on its stream",
        },
    })
    kp_k = wl["keypoints"] // 1000
    rows = "float" if getattr(args, "desc_dtype", "u8") == "f32" else "u8"
    desc = (f"C4: {kp_k}k SIFT-128 ({rows}) keypoints per {wl['width']}x{wl['height']} frame pair, full pipeline, "
            f"pixelsRay {args.ray}, pyramids {args.levels}") if args.desc == "sift" else (
            f"C3-like: {kp_k}k ORB-256 (Hamming) keypoints per {wl['width']}x{wl['height']} frame pair, NNDR "
            f"{args.nndr}, full pipeline, pixelsRay {args.ray}, pyramids {args.levels}")
    frame_s = elapsed / args.steps
    out = {
        "metric": METRIC,
        "value": kept_total / elapsed,
        "unit": "keypoints/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": frame_s * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (ray-cast facet scene, seeded; 3dfeaturematcher_amd/synth.py)",
        "config": {
            "workload": desc,
            "keypoints_per_frame": wl["keypoints"], "width": wl["width"], "height": wl["height"],
            "pixelsRay": args.ray, "pyramids": args.levels, "parallelism": "1 GPU",
            "mode": (f"stream: {nf} frame pairs in flight (one context + HIP stream each, fm3d_pipeline_submit/wait), "
                     f"{nl} frame pair(s) per LM launch" + (" (fm3d_pipeline_link)" if nl > 1 else "")),
            "timed": ("per step, from host memory to host memory: H2D of descriptors, keypoints and images (pinned "
                      "staging), pyramids (a6), match -> NNDR -> DLT -> LM normals -> survivor records, D2H of the "
                      "records; the K steps' wall time includes filling and draining the pipeline"),
        },
        "latency_ms": {"mean": float(np.mean(lat)), "max": float(np.max(lat)),
                       "note": "per frame pair, submit call -> its records on the host"},
        "device_resident_value": sum(st["kept"] for st in rstats) / res_elapsed,
        "device_resident_note": (f"the same pair, inputs HBM-resident, one step in flight ({res_steps} steps of "
                                 f"fm3d_pipeline_run, {res_elapsed / res_steps * 1e3:.1f} ms each)"),
        "input_keypoints_per_s": wl["keypoints"] / frame_s,
        "roofline": roof,
        "cpu_baseline": cpu,
        # stage costs from the resident run (one pair in flight); in the stream every stage's HIP events
        # also take the time its launches wait behind the other pairs' LM launches
        "stages_ms": {k: rstats[-1][k] for k in ("match_ms", "nndr_ms", "triangulate_ms", "lm_ms", "total_ms")},
        "stages_note": ("stages_ms: the device-resident run's last step (one pair in flight: stage costs; nndr_ms "
                        "is folded into match_ms); stages_ms_queued_and_run: the stream's last pair, whose stage "
                        "events also span the time its launches queue behind the other pairs' LM launches"),
        "stages_ms_queued_and_run": {k: last_st[k] for k in ("match_ms", "triangulate_ms", "pyramid_ms", "lm_ms",
                                                              "total_ms")},
        "counts": {k: last_st[k] for k in ("queries", "matches", "inliers", "kept")},
        "lm_profile": lm_profile(rstats[-1]["lm"]),
        "lm_profile_overlapped": lm_profile(last_st["lm"]),
        "setup_s": {"synthetic_generation": round(t_gen, 2)},
        "records_sha256": digests[0] if len(digests) == 1 else digests,
        "records_identical_across_steps": len(digests) == 1,
    }
    out.update(verify_against_fixture(args, wl, "c4", pair, last_rec))
    if len(digests) != 1:
        out["verified"] = False
    emit(out, args)


def run_mgpu(args, workload):
    """`bench.py --gpus N` without a torchrun environment (the driver's command shape): this one
    process drives N GPUs through the C ABI's multi-GPU host (fm3d_mgpu, csrc/fm3d_mgpu.cpp).  C5
    (BASELINE configs[4]): ONE 1M-keypoint frame pair per step, its 4,096-query blocks dealt
    round-robin over the N devices, one replica of frame B and the images per device and one pass
    (one LM launch) per device, RCCL all-gather of the survivor records over xGMI, merged in query
    order on the host; two frame pairs in flight (fm3d_mgpu_submit / fm3d_mgpu_wait), every step
    from host memory to host memory as at one GPU.  Strong scaling: value = kept keypoints of the K
    pairs / wall time.  Exits non-zero when fewer than N GPUs are visible.

    The same workload on ONE GPU is measured after the timed steps (--ref-steps pairs through
    fm3d_mgpu on device 0 alone, the same stream shape): `value_one_gpu` and
    `efficiency = value / (N * value_one_gpu)` in the line, so the 1 -> N curve of C5 has its own
    one-GPU point (the driver's `--gpus 1` line is C4, the headline).  torch is never imported on
    this route: the visible-device count comes from libfm3d (hipGetDeviceCount), so the only RCCL in
    the process is the one fm3d_mgpu loads."""
    fm3d = importlib.import_module("3dfeaturematcher_amd")
    n = args.gpus
    vis = fm3d.device_count()
    alias = bool(getattr(args, "alias_devices", False))
    if alias:
        os.environ["FM3D_DEBUG_MGPU_ALIAS"] = "1"
    if vis < (1 if alias else n):
        print(f"bench.py --gpus {n}: only {vis} GPU(s) visible", file=sys.stderr, flush=True)
        raise SystemExit(2)
    if workload != "c5":
        print(f"bench.py --gpus {n}: the one-process multi-GPU run is C5 (--workload auto / c5); use torchrun "
              f"for --weak or other workloads", file=sys.stderr, flush=True)
        raise SystemExit(2)
    synth = importlib.import_module("3dfeaturematcher_amd.synth")
    wl = dict(WORKLOADS["c5"])
    for k in ("keypoints", "width", "height"):
        if getattr(args, k):
            wl[k] = getattr(args, k)
    t_gen = time.time()
    pair = synth.make_frame_pair(wl["keypoints"], wl["width"], wl["height"], seed=args.seed, desc=args.desc)
    t_gen = time.time() - t_gen
    s = c4_settings(fm3d, pair, args)
    torch_at_create = "torch" in sys.modules
    mg = fm3d.MultiGPU(s, devices=[0] * n if alias else list(range(n)), shares=n)
    mg.set_g12(pair.g12)
    binary = args.desc == "orb"
    inputs = (desc_rows(args, pair.desc1), desc_rows(args, pair.desc2), pair.kp1, pair.kp2, pair.img1, pair.img2)
    bufs = [np.zeros(len(pair.desc1), dtype=fm3d.RECORD) for _ in range(2)]  # the last two waits' records

    def stream_run(n_steps, mg=mg):
        res, pend, last = [], 0, None
        t_sub = []
        for k in range(n_steps):
            if pend == 4:  # fm3d_mgpu's four context sets: two LM launches of two frame pairs each
                rec, st = mg.wait(bufs[len(res) % 2])
                res.append((len(rec), st, time.perf_counter() - t_sub[len(res)], records_digest(rec.tobytes())))
                last, pend = rec, pend - 1
            t_sub.append(time.perf_counter())
            mg.submit(*inputs, binary=binary)
            pend += 1
        while pend:
            rec, st = mg.wait(bufs[len(res) % 2])
            res.append((len(rec), st, time.perf_counter() - t_sub[len(res)], records_digest(rec.tobytes())))
            last, pend = rec, pend - 1
        return res, last

    stream_run(args.warmup)
    t0 = time.perf_counter()
    res, last_rec = stream_run(args.steps)
    elapsed = time.perf_counter() - t0
    # one pair alone after the stream (untimed): its stage events are stage costs, not time queued
    # behind the other pairs' LM launches
    iso_st = stream_run(1)[0][0][1]
    mg.close()
    kept_total = sum(r[0] for r in res)
    value = kept_total / elapsed
    # the same C5 stream on device 0 alone (untimed by the metric): the curve's one-GPU point
    one = {"value_one_gpu": value, "efficiency": 1.0, "one_gpu_steps": args.steps,
           "one_gpu_note": "this run is one GPU: value_one_gpu = value"}
    if n > 1 and args.ref_steps > 0:
        m1 = fm3d.MultiGPU(s, devices=[0], shares=1)
        try:
            m1.set_g12(pair.g12)
            stream_run(1, m1)
            t1 = time.perf_counter()
            r1, rec1 = stream_run(args.ref_steps, m1)
            v1 = sum(r[0] for r in r1) / (time.perf_counter() - t1)
        finally:
            m1.close()
        one = {"value_one_gpu": v1, "efficiency": value / (n * v1), "one_gpu_steps": args.ref_steps,
               "one_gpu_records_equal": bool(rec1.tobytes() == last_rec.tobytes()),
               "one_gpu_note": (f"the same C5 frame pair through fm3d_mgpu on device 0 alone, {args.ref_steps} "
                                f"pairs after 1 warmup pair, same stream shape; efficiency = value / "
                                f"({n} x value_one_gpu)")}
    stats = [r[1] for r in res]
    lat = [r[2] * 1e3 for r in res]
    digests = sorted(set(r[3] for r in res))
    last_st = stats[-1]
    frame_s = elapsed / args.steps
    pix = float(np.mean([st["lm"]["pixel_evaluations"] for st in stats]))
    kp_k = wl["keypoints"] // 1000
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "keypoints/s",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": frame_s * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (ray-cast facet scene, seeded; 3dfeaturematcher_amd/synth.py)",
        "config": {
            "workload": (f"C5: one {kp_k}k-keypoint SIFT-128 (u8) frame pair ({wl['width']}x{wl['height']}, sub-pixel "
                         f"keypoints) per step, full pipeline, pixelsRay {args.ray}, pyramids {args.levels}, query "
                         f"blocks over {n} GPUs, RCCL all-gather of survivor records"),
            "keypoints_per_frame": wl["keypoints"], "width": wl["width"], "height": wl["height"],
            "pixelsRay": args.ray, "pyramids": args.levels,
            "parallelism": (f"dp{n} in one process (fm3d_mgpu): 4,096-query blocks dealt round-robin over the "
                            f"devices, one replica of frame B + images and one LM launch per device, RCCL "
                            f"all-gather of counts + 64-B survivor records every step"),
            "mode": ("stream: 4 frame pairs in flight, 2 per LM launch on every device (fm3d_mgpu_submit / "
                     "fm3d_mgpu_wait, context sets linked by fm3d_pipeline_link)"),
            "timed": ("per step, from host memory to host memory: per-device query gather + H2D (pinned), pyramids, "
                      "match -> NNDR -> DLT -> LM -> records, RCCL all-gather, D2H of device 0's gathered "
                      "records, host merge in query order"),
        },
        "latency_ms": {"mean": float(np.mean(lat)), "max": float(np.max(lat)),
                       "note": "per frame pair, submit call -> merged records on the host"},
        "input_keypoints_per_s": wl["keypoints"] / frame_s,
        "roofline": {
            "kernel": "fm3d::lm2_kernel on every device, two frame pairs per launch, launches overlapped",
            "bound": "fp64-valu",
            "achieved": FLOPS_PER_PIXEL_EVAL * pix / frame_s / 1e12,
            "peak": FP64_PEAK_TFLOPS * n, "unit": "TFLOP/s",
            "frac": FLOPS_PER_PIXEL_EVAL * pix / frame_s / 1e12 / (FP64_PEAK_TFLOPS * n),
            "traffic": None,
            "algorithmic": f"{FLOPS_PER_PIXEL_EVAL} flop x {pix:.4g} pixel evaluations per frame pair (all devices) "
                           f"/ the wall time per step; peak = {n} x {FP64_PEAK_TFLOPS}",
            "avg_launch_ms": frame_s * 1e3,
        },
        "cpu_baseline": None,
        "stages_ms": {k: iso_st[k] for k in ("match_ms", "lm_ms", "total_ms", "pyramid_ms")},
        "stages_ms_queued_and_run": {k: last_st[k] for k in ("match_ms", "lm_ms", "total_ms", "pyramid_ms")},
        "stages_note": ("stages_ms: one frame pair alone after the timed stream (device 0's stage events: stage "
                        "costs); stages_ms_queued_and_run: the stream's last pair, whose events also span the time "
                        "its launches and copies wait behind the other pairs' LM launches"),
        "counts": {k: last_st[k] for k in ("queries", "matches", "inliers", "kept")},
        "setup_s": {"synthetic_generation": round(t_gen, 2)},
        "records_sha256": digests[0] if len(digests) == 1 else digests,
        "records_identical_across_steps": len(digests) == 1,
        "torch_imported_at_mgpu_create": torch_at_create,
        **one,
    }
    out.update(verify_against_fixture(args, wl, "c5", pair, last_rec))
    if len(digests) != 1:
        out["verified"] = False
    if alias:
        out["alias_devices"] = {
            "note": (f"diagnostic, not a scaling point: device 0 listed {n} times (FM3D_DEBUG_MGPU_ALIAS=1), so "
                     f"all {n} shares, their {4 * n} context sets and {n} concurrent LM launches share ONE GPU and "
                     f"the all-gather is restated as device copies; value / value_one_gpu is the {n}-way host "
                     f"path's cost on one GPU"),
            "value_over_one_device": value / out["value_one_gpu"]}
        out["efficiency"] = None
        out["n_gpus"] = 1
    emit(out, args)


def run_torchrun_stream(args, workload):
    """The torchrun route (WORLD_SIZE > 1, one process per GPU), C5 as north_star states it: ONE 1M-
    keypoint frame pair per step, the same on every rank; rank r takes the 4,096-query blocks
    shard.query_blocks(1M, N, r) (frame B and both images replicated) and keeps frame pairs in flight
    as at one GPU (`inflight` LM launches of `lm_pairs` linked pairs, fm3d_pipeline_submit / wait, one
    context + HIP stream each); every finished step's survivor records are all-gathered over RCCL
    (torch.distributed, backend nccl) and rank 0 merges the last one in query order and checks it
    against the committed fixture.  Each step runs from host memory to host memory as at one GPU.
    Strong scaling: value = kept keypoints of the K frame pairs (all ranks) / the max-over-ranks wall
    time.  FM3D_BENCH_BACKEND=gloo with FM3D_BENCH_SHARE_DEVICE=1 runs the ranks on one GPU with a CPU
    all-gather (the multi-rank logic on a one-GPU box; tests/test_gpu_parity.py)."""
    import torch
    import torch.distributed as tdist
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("FM3D_BENCH_BACKEND", "nccl")
    vis = torch.cuda.device_count()
    dev = 0 if os.environ.get("FM3D_BENCH_SHARE_DEVICE") == "1" else local
    if dev >= vis:
        print(f"bench.py rank {rank}: device {dev} not visible ({vis} GPU(s))", file=sys.stderr, flush=True)
        raise SystemExit(2)
    torch.cuda.set_device(dev)
    tdist.init_process_group(backend)  # nccl: RCCL over xGMI
    fm3d = importlib.import_module("3dfeaturematcher_amd")
    synth = importlib.import_module("3dfeaturematcher_amd.synth")
    shard = importlib.import_module("3dfeaturematcher_amd.shard")
    wl = dict(WORKLOADS[workload])
    for k in ("keypoints", "width", "height"):
        if getattr(args, k):
            wl[k] = getattr(args, k)
    t_gen = time.time()
    pair = synth.make_frame_pair(wl["keypoints"], wl["width"], wl["height"], seed=args.seed, desc=args.desc)
    t_gen = time.time() - t_gen
    s = c4_settings(fm3d, pair, args)
    n = len(pair.desc1)
    qidx = shard.query_blocks(n, world, rank)
    inputs = (desc_rows(args, pair.desc1[qidx]), desc_rows(args, pair.desc2), pair.kp1[qidx], pair.kp2, pair.img1,
              pair.img2)
    nl = max(1, args.lm_pairs)
    nf = max(1, args.inflight) * nl
    streams = [torch.cuda.Stream(device=dev) for _ in range(nf)]
    ctxs, pipes = [], []
    for st in streams:
        ctx = fm3d.Context(s, device=dev)
        ctx.set_stream(st.cuda_stream)
        fm3d.SingleCameraTriangulator(ctx).set_g12(pair.g12)
        ctxs.append(ctx)
        pipes.append(fm3d.Pipeline(ctx))
    for i in range(0, nf, nl):
        for j in range(i, i + nl - 1):
            pipes[j].link(pipes[i + nl - 1])
    binary = args.desc == "orb"
    bufs = [np.zeros(len(qidx), dtype=fm3d.RECORD) for _ in range(nf)]
    cap = shard.blocks_capacity(n, world)
    rec_t = torch.zeros((cap, shard.RECORD_BYTES), dtype=torch.uint8,
                        device="cpu" if backend == "gloo" else f"cuda:{dev}")

    def gather(rec):
        k = len(rec)
        if k:
            rec_t[:k].copy_(torch.from_numpy(rec.view(np.uint8).reshape(k, shard.RECORD_BYTES)))
        return shard.all_gather_device(rec_t, k)

    def stream_run(n_steps):
        res, pend, t_sub, last = [], [None] * nf, [0.0] * nf, None

        def drain(j):
            rec, st = pipes[j].wait(bufs[j])
            g = gather(rec)
            res.append((len(rec), st, time.perf_counter() - t_sub[j]))
            pend[j] = None
            return g

        for k in range(n_steps):
            j = k % nf
            if pend[j] is not None:
                last = drain(j)
            t_sub[j] = time.perf_counter()
            pipes[j].submit(*inputs, binary=binary)
            pend[j] = True
        for k in range(n_steps, n_steps + nf):
            j = k % nf
            if pend[j] is not None:
                last = drain(j)
        return res, last

    def sync():
        torch.cuda.synchronize()
        tdist.barrier()
        torch.cuda.synchronize()

    stream_run(args.warmup)
    sync()
    t0 = time.perf_counter()
    res, last = stream_run(args.steps)
    sync()
    elapsed = time.perf_counter() - t0
    for c in ctxs:
        c.close()
    red = torch.tensor([elapsed, float(sum(r[0] for r in res))], dtype=torch.float64, device=rec_t.device)
    t_max = red[:1].clone()
    tdist.all_reduce(t_max, op=tdist.ReduceOp.MAX)
    kept = red[1:].clone()
    tdist.all_reduce(kept, op=tdist.ReduceOp.SUM)
    elapsed, all_kept = float(t_max.item()), int(kept.item())
    stats = [r[1] for r in res]
    lat = [r[2] * 1e3 for r in res]
    if rank == 0:
        merged = shard.merge_gathered_shares(last[0], last[1], n)
        frame_s = elapsed / args.steps
        pix_local = float(np.mean([st["lm"]["pixel_evaluations"] for st in stats]))
        kp_k = wl["keypoints"] // 1000
        last_st = stats[-1]
        out = {
            "metric": METRIC,
            "value": all_kept / elapsed,
            "unit": "keypoints/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": frame_s * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (ray-cast facet scene, seeded; 3dfeaturematcher_amd/synth.py)",
            "config": {
                "workload": (f"C5: one {kp_k}k-keypoint SIFT-128 (u8) frame pair ({wl['width']}x{wl['height']}, "
                             f"sub-pixel keypoints) per step, full pipeline, pixelsRay {args.ray}, pyramids "
                             f"{args.levels}, query blocks over {world} GPUs, RCCL all-gather of survivor records"),
                "keypoints_per_frame": wl["keypoints"], "width": wl["width"], "height": wl["height"],
                "pixelsRay": args.ray, "pyramids": args.levels,
                "parallelism": (f"dp{world}: one process per GPU (torchrun), 4,096-query blocks of one frame pair "
                                f"dealt round-robin over the ranks, frame B + images replicated, RCCL all-gather "
                                f"of counts + 64-B survivor records every step ({backend})"),
                "mode": (f"stream: {nf} frame pairs in flight per rank, {nl} per LM launch (fm3d_pipeline_submit / "
                         f"wait / link)"),
                "timed": ("per step on every rank, from host memory to host memory: its query share's H2D (pinned), "
                          "pyramids, match -> NNDR -> DLT -> LM -> records, D2H, the all-gather; barrier + "
                          "synchronize on both sides, max over ranks"),
            },
            "latency_ms": {"mean": float(np.mean(lat)), "max": float(np.max(lat)),
                           "note": "rank 0, per frame pair, submit call -> its gathered records"},
            "input_keypoints_per_s": wl["keypoints"] / frame_s,
            "roofline": {
                "kernel": "fm3d::lm2_kernel on every rank's GPU, launches overlapped",
                "bound": "fp64-valu",
                "achieved": FLOPS_PER_PIXEL_EVAL * pix_local / frame_s / 1e12,
                "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": FLOPS_PER_PIXEL_EVAL * pix_local / frame_s / 1e12 / FP64_PEAK_TFLOPS,
                "traffic": None,
                "algorithmic": (f"{FLOPS_PER_PIXEL_EVAL} flop x rank 0's {pix_local:.4g} pixel evaluations per frame "
                                f"pair / the wall time per step, against one GPU's peak"),
                "avg_launch_ms": frame_s * 1e3,
            },
            "cpu_baseline": None,
            "stages_ms_queued_and_run": {k: last_st[k] for k in ("match_ms", "lm_ms", "total_ms", "pyramid_ms")},
            "stages_note": ("rank 0's last pair of the stream: its stage events also span the time its launches "
                            "and copies wait behind the other pairs' LM launches"),
            "counts_rank0": {k: last_st[k] for k in ("queries", "matches", "inliers", "kept")},
            "kept_per_frame_pair": int(len(merged)),
            "setup_s": {"synthetic_generation": round(t_gen, 2)},
        }
        out.update(verify_against_fixture(args, wl, "c5", pair, merged))
        if args.dump_records:
            np.save(args.dump_records, merged)
        emit(out, args)
    tdist.barrier()
    tdist.destroy_process_group()


def run_resident(args, workload):
    """Inputs uploaded once, one step in flight (fm3d_pipeline_run): --mode resident at one GPU, and
    the torchrun route (WORLD_SIZE > 1: one process per GPU, C5 sharded or --weak)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    wl = dict(WORKLOADS[workload])
    for k in ("keypoints", "width", "height"):
        if getattr(args, k):
            wl[k] = getattr(args, k)
    sharded = not args.weak and world > 1
    dist = torch = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl")  # RCCL over xGMI
        dist = tdist

    fm3d = importlib.import_module("3dfeaturematcher_amd")
    synth = importlib.import_module("3dfeaturematcher_amd.synth")
    shard = importlib.import_module("3dfeaturematcher_amd.shard")

    t_gen = time.time()
    seed = args.seed + (1000 * rank if args.weak else 0)
    pair = synth.make_frame_pair(wl["keypoints"], wl["width"], wl["height"], seed=seed, desc=args.desc)
    t_gen = time.time() - t_gen
    s = fm3d.Settings.default()
    s.set_camera(pair.cam)
    s.nndrEpsilon = args.nndr
    s.pixelsRay = args.ray
    s.pyramids = args.levels
    s.lmWaves = args.lm_waves
    n = len(pair.desc1)
    # this rank's queries (block-cyclic over the ranks), gathered into one array: local queryIdx
    qidx = shard.query_blocks(n, world, rank) if sharded else None
    ctx = fm3d.Context(s, device=local if world > 1 else 0)
    sct = fm3d.SingleCameraTriangulator(ctx)
    sct.set_g12(pair.g12)
    pipe = fm3d.Pipeline(ctx)
    d1, k1 = (pair.desc1, pair.kp1) if qidx is None else (pair.desc1[qidx], pair.kp1[qidx])
    t_up = time.perf_counter()
    pipe.upload(d1, pair.desc2, k1, pair.kp2, pair.img1, pair.img2, query_offset=0, binary=args.desc == "orb")
    upload_ms = (time.perf_counter() - t_up) * 1e3

    rec_buf = None
    if dist is not None:
        cap = shard.blocks_capacity(n, world) if sharded else n
        rec_buf = torch.empty((cap, shard.RECORD_BYTES), dtype=torch.uint8, device=f"cuda:{local}")
    last = {}

    def step():
        k, st = pipe.run(rec_buf.data_ptr() if rec_buf is not None else None)
        if dist is not None:
            last["gathered"], last["counts"] = shard.all_gather_device(rec_buf, k)
        return k, st

    for _ in range(args.warmup):
        step()

    def sync():
        if dist is not None:
            torch.cuda.synchronize()
            dist.barrier()
            torch.cuda.synchronize()

    sync()
    t0 = time.perf_counter()
    kept_total = 0
    stats = []
    for _ in range(args.steps):
        k, st = step()
        kept_total += k
        stats.append(st)
    sync()
    elapsed = time.perf_counter() - t0

    all_kept = kept_total
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=rec_buf.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        kk = torch.tensor([kept_total], dtype=torch.int64, device=rec_buf.device)
        dist.all_reduce(kk, op=dist.ReduceOp.SUM)
        all_kept = int(kk.item())

    # D2H of the survivor records (outside the timed region; reported beside it)
    t_dl = time.perf_counter()
    if dist is None:
        mine = pipe.records(stats[-1]["kept"])
    else:
        # the C++ merge of the C ABI (fm3d_merge_shares, as fm3d_mgpu_pipeline_run merges)
        merged = (shard.merge_gathered_shares(last["gathered"], last["counts"], n) if sharded else
                  shard.merge_gathered(last["gathered"], last["counts"]))
    download_ms = (time.perf_counter() - t_dl) * 1e3

    check = None
    if sharded:
        check = check_against_one_gpu(args, fm3d, pair, s, merged, local, rank, dist, torch)

    lm_ms = float(np.mean([st["lm_ms"] for st in stats]))
    pix = float(np.mean([st["lm"]["pixel_evaluations"] for st in stats]))
    evals = float(np.mean([st["lm"]["evaluations"] for st in stats]))
    last_st = stats[-1]
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and args.desc == "sift":
        cpu = cpu_baseline(pair, s, last_st, args)

    if rank == 0:
        kp_k = wl["keypoints"] // 1000
        if workload == "c5":
            desc = (f"C5: one {kp_k}k-keypoint SIFT-128 (u8) frame pair ({wl['width']}x{wl['height']}, sub-pixel "
                    f"keypoints), full pipeline, pixelsRay {args.ray}, pyramids {args.levels}, " +
                    (f"query blocks sharded over {world} GPUs, RCCL all-gather of survivor records" if sharded else
                     "whole on one GPU (the reference point of the N-GPU strong-scaling runs)"))
        elif args.desc == "orb":
            desc = (f"C3-like: {kp_k}k ORB-256 (Hamming) keypoints per {wl['width']}x{wl['height']} frame pair, "
                    f"NNDR {args.nndr}, full pipeline, pixelsRay {args.ray}, pyramids {args.levels}")
        else:
            desc = (f"C4: {kp_k}k SIFT-128 (u8) keypoints per {wl['width']}x{wl['height']} frame pair, full "
                    f"pipeline, pixelsRay {args.ray}, pyramids {args.levels}")
        frame_s = elapsed / args.steps
        out = {
            "metric": METRIC,
            "value": all_kept / elapsed,
            "unit": "keypoints/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": frame_s * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if sharded else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (ray-cast facet scene, seeded; 3dfeaturematcher_amd/synth.py)",
            "config": {
                "workload": desc,
                "keypoints_per_frame": wl["keypoints"], "width": wl["width"], "height": wl["height"],
                "pixelsRay": args.ray, "pyramids": args.levels,
                "parallelism": (f"dp{world}: 4,096-query blocks of one frame pair dealt round-robin, frame B replicated, "
                                f"RCCL all-gather of counts + 64-B survivor records each step") if sharded else
                               (f"dp{world}: one frame pair per rank (weak)" if world > 1 else "1 GPU"),
                "timed": ("match -> NNDR -> DLT -> LM -> survivor records on HBM-resident inputs (descriptors, "
                          "keypoints, image pyramids uploaded/built before the timed region: upload_ms; record "
                          "D2H after it: download_ms)"),
            },
            "upload_ms": upload_ms,
            "download_ms": download_ms,
            "pcie_inclusive_value": all_kept / args.steps / (frame_s + (upload_ms + download_ms) * 1e-3),
            # the input rate beside the kept rate (queries of the frame pair per second)
            "input_keypoints_per_s": wl["keypoints"] * (world if args.weak else 1) / frame_s,
            "roofline": roofline(stats, lm_ms, pix, evals, args, pair, s),
            "cpu_baseline": cpu,
            "stages_ms": {k: last_st[k] for k in ("match_ms", "nndr_ms", "triangulate_ms", "lm_ms", "total_ms")},
            "counts": {k: last_st[k] for k in ("queries", "matches", "inliers", "kept")},
            "lm_profile": lm_profile(last_st["lm"]),
            "setup_s": {"synthetic_generation": round(t_gen, 2)},
        }
        if check is not None:
            out["sharding_check"] = check
        if dist is None:  # bit-identity across builds / boxes (A/B runs compare it)
            out["records_sha256"] = records_digest(mine.tobytes())
            out.update(verify_against_fixture(args, wl, workload, pair, mine))
        elif sharded:  # the merged records of the N-GPU run against the committed oracle run
            out.update(verify_against_fixture(args, wl, workload, pair, merged))
        line = json.dumps(out)
        print(line, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(line + "\n")
    ctx.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def run_c2(args):
    """BASELINE.json configs[1] (C2): 10k SIFT-128 keypoints per 640x480 frame, brute-force L2 match
    (exact u8 path) + NNDR + DLT triangulation, no normals; one GPU.  A step is fm3d_pipeline_run_dlt on
    HBM-resident inputs; the value is the triangulated inliers (matched + triangulated keypoints) per
    second.  The roofline is the match stage's (int8 MFMA), timed by HIP events around it.  Every
    step's matches and points are checked against the CPU oracle (knn2 + NNDR + triangulate)."""
    fm3d = importlib.import_module("3dfeaturematcher_amd")
    synth = importlib.import_module("3dfeaturematcher_amd.synth")
    wl = dict(WORKLOADS["c2"])
    for k in ("keypoints", "width", "height"):
        if getattr(args, k):
            wl[k] = getattr(args, k)
    pair = synth.make_frame_pair(wl["keypoints"], wl["width"], wl["height"], seed=args.seed, desc="sift")
    s = fm3d.Settings.default()
    s.set_camera(pair.cam)
    s.nndrEpsilon = args.nndr
    # the rows as the caller hands them: u8, or the float rows of the reference's cv::Mat
    d1, d2 = ((pair.desc1, pair.desc2) if args.desc_dtype == "u8"
              else (pair.desc1.astype(np.float32), pair.desc2.astype(np.float32)))
    host_io = args.io == "host"
    # a serving loop: `inflight` contexts (one HIP stream each) with the pair resident, a frame pair
    # submitted on one while the previous ones run (fm3d_pipeline_submit_dlt / wait_dlt); the
    # synchronous step (run_dlt, one host wait per pair) is timed beside it.  --io host: every step
    # also stages the pair from host memory (fm3d_pipeline_submit_dlt_pair: staging and the front half
    # queued without a host wait; C2 needs no images) and downloads its matches and inlier points
    nf = max(1, args.inflight)
    ctxs = [fm3d.Context(s) for _ in range(nf)]
    pipes = []
    for ctx in ctxs:
        fm3d.SingleCameraTriangulator(ctx).set_g12(pair.g12)
        pipe = fm3d.Pipeline(ctx)
        pipe.upload(d1, d2, pair.kp1, pair.kp2, None, None)
        pipes.append(pipe)
    for _ in range(args.warmup):
        for pipe in pipes:
            pipe.run_dlt()
    # the stage times (HIP events at the stage boundaries) from their own synchronous steps; the
    # timed loops run without those events (FM3D_STAGE_EVENTS=0: each costs the step a few us)
    os.environ["FM3D_STAGE_EVENTS"] = "1"
    stage_stats = [pipes[0].run_dlt()[1] for _ in range(5)]
    os.environ["FM3D_STAGE_EVENTS"] = "0"
    sync_stats, ts = [], time.perf_counter()
    for _ in range(max(args.steps, 5)):
        sync_stats.append(pipes[0].run_dlt()[1])
    sync_ms = (time.perf_counter() - ts) / len(sync_stats) * 1e3
    stats, lat = [], []
    t_sub = [0.0] * nf
    busy = [False] * nf
    total = 0

    def finish(k):
        n, st = pipes[k].wait_dlt()
        if host_io:  # the pair's matches and inlier points to host memory
            pipes[k].dlt_results(st["matches"], st["inliers"])
        lat.append(time.perf_counter() - t_sub[k])
        stats.append(st)
        return n

    t0 = time.perf_counter()
    for i in range(args.steps):
        k = i % nf
        if busy[k]:
            total += finish(k)
        t_sub[k] = time.perf_counter()
        if host_io:  # staged and queued with no host wait (fm3d_pipeline_submit_dlt_pair)
            pipes[k].submit_dlt_pair(d1, d2, pair.kp1, pair.kp2)
        else:
            pipes[k].submit_dlt()
        busy[k] = True
    for j in range(args.steps, args.steps + nf):
        k = j % nf
        if busy[k]:
            total += finish(k)
            busy[k] = False
    elapsed = time.perf_counter() - t0
    last = sync_stats[-1]
    m, pts, src = pipes[0].dlt_results(last["matches"], last["inliers"])
    same_across = all(np.array_equal(np.asarray(pp.dlt_results(last["matches"], last["inliers"])[1]), np.asarray(pts))
                      for pp in pipes[1:])
    for ctx in ctxs:
        ctx.close()
    # the cpu_baseline leg: the oracle's C2 path on the host cores, whose outputs also check the GPU's
    cpu, (q, t, dist, opts) = (None, (None,) * 4) if args.no_cpu else c2_cpu_baseline(pair, s, args)
    verified = None if q is None else bool(
        np.array_equal(m["queryIdx"], q) and np.array_equal(m["trainIdx"], t) and np.array_equal(m["distance"], dist)
        and np.array_equal(pts, opts))
    n_q, n_t, d = len(pair.desc1), len(pair.desc2), pair.desc1.shape[1]
    os.environ.pop("FM3D_STAGE_EVENTS", None)
    match_ms = float(np.mean([x["match_ms"] for x in stage_stats]))  # isolated launches
    achieved = 2.0 * n_q * n_t * d / (match_ms * 1e-3) / 1e12
    out = {
        "metric": "matched+triangulated keypoints/sec (BASELINE C2: match + DLT triangulate only)",
        "value": total / elapsed,
        "unit": "keypoints/s",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "latency_ms": float(np.mean(lat)) * 1e3,
        "synchronous_ms_per_step": sync_ms,
        "inflight": nf,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8 (exact int32 distances), f64 triangulation",
        "data": "synthetic (ray-cast facet scene, seeded; 3dfeaturematcher_amd/synth.py)",
        "config": {"workload": f"C2: {wl['keypoints'] // 1000}k SIFT-128 ({'float' if args.desc_dtype == 'f32' else 'u8'}) "
                               f"keypoints per {wl['width']}x{wl['height']} "
                               f"frame pair, knnMatch k=2 + NNDR {args.nndr} + DLT triangulation",
                   "keypoints_per_frame": wl["keypoints"], "parallelism": "1 GPU",
                   "descriptor_rows": ("float32 (the reference's cv::Mat of SIFT rows; integer-valued, checked "
                                       "and packed to u8 on the device)" if args.desc_dtype == "f32" else "u8"),
                   "io": args.io,
                   "timed": (f"K frame pairs, each from host memory to host memory: descriptors + keypoints "
                             f"staged (pinned, H2D{', device integer check + u8 pack' if args.desc_dtype == 'f32' else ''}; "
                             f"fm3d_pipeline_submit_dlt_pair, no host wait), "
                             f"match -> NNDR -> compaction -> DLT -> compaction, matches + inlier points D2H; "
                             f"{nf} contexts (HIP streams) in flight" if host_io else
                             f"K frame pairs through match -> NNDR -> compaction -> DLT -> compaction on "
                             f"HBM-resident inputs, {nf} contexts (HIP streams) in flight, every pair's counts read "
                             f"back (page-locked) before its context takes the next") +
                            "; synchronous_ms_per_step: one resident pair at a time"},
        "roofline": {"kernel": "match stage (row constants + knn2_i8_kernel + part merge + NNDR), HIP events",
                     "bound": "mfma", "compute": "int8 MFMA (v_mfma_i32_32x32x32_i8) + VALU top-2 epilogue",
                     "achieved": achieved, "peak": INT8_PEAK_TOPS, "unit": "TOP/s", "frac": achieved / INT8_PEAK_TOPS,
                     "traffic": None, "algorithmic": f"2 x {n_q} x {n_t} x {d} int8 ops per launch",
                     "avg_launch_ms": match_ms},
        "cpu_baseline": cpu,
        "stages_ms": {k: stage_stats[-1][k] for k in ("match_ms", "triangulate_ms", "total_ms")},
        "stages_note": "stages_ms: one synchronous step with HIP events at the stage boundaries (match_ms: row "
                       "constants + knn + NNDR with its compaction, one stage since NNDR is fused into the match's "
                       "last launch); the timed loops run without those events (FM3D_STAGE_EVENTS=0)",
        "counts_identical_across_contexts": bool(same_across),
        "counts": {"queries": n_q, "matches": int(last["matches"]), "inliers": int(last["inliers"])},
        "verified": verified,
        "verification": "matches (query, train, distance) and inlier points byte-equal to the cpu_baseline "
                        "leg's oracle outputs",
    }
    line = json.dumps(out)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


def run_c3(args):
    """BASELINE.json configs[2] (C3) as worded: 10k ORB-256 keypoints per 640x480 frame, Hamming match
    + NNDR 0.8 + DLT, then the NCC scoring of 16 candidate normals (4 x 4, half width 0.4 rad) over the
    pixelsRay-32 neighbourhood (64 x 64) of every inlier -- fm3d_pipeline_run_ncc on HBM-resident
    inputs.  The value is the NCC-scored inliers per second; the roofline is ncc_kernel's (fp64 VALU,
    counted with the LM's 91 flops per pixel evaluation of the same geometry and sampling).  The
    cpu_baseline leg runs the oracle's whole C3 path and its outputs check every score."""
    fm3d = importlib.import_module("3dfeaturematcher_amd")
    synth = importlib.import_module("3dfeaturematcher_amd.synth")
    wl = dict(WORKLOADS["c3"])
    for k in ("keypoints", "width", "height"):
        if getattr(args, k):
            wl[k] = getattr(args, k)
    nndr, ray = args.nndr, args.ray  # C3's own defaults (WORKLOAD_DEFAULTS) unless given
    pair = synth.make_frame_pair(wl["keypoints"], wl["width"], wl["height"], seed=args.seed, desc="orb")
    s = fm3d.Settings.default()
    s.set_camera(pair.cam)
    s.nndrEpsilon = nndr
    s.pixelsRay = ray
    # a serving loop as C2's: `inflight` contexts (one HIP stream each) with the pair resident, a frame
    # pair submitted on one while the previous ones run (fm3d_pipeline_submit_ncc / wait_ncc); the
    # synchronous step (run_ncc, one host wait per pair) is timed beside it
    nf = max(1, args.inflight)
    ctxs = [fm3d.Context(s) for _ in range(nf)]
    pipes = []
    for ctx in ctxs:
        fm3d.SingleCameraTriangulator(ctx).set_g12(pair.g12)
        pipe = fm3d.Pipeline(ctx)
        pipe.upload(pair.desc1, pair.desc2, pair.kp1, pair.kp2, pair.img1, pair.img2, binary=True)
        pipes.append(pipe)
    for _ in range(args.warmup):
        for pipe in pipes:
            pipe.run_ncc(4, 4, 0.4)
    stats, ts = [], time.perf_counter()
    for _ in range(args.steps):
        stats.append(pipes[0].run_ncc(4, 4, 0.4)[1])
    sync_ms = (time.perf_counter() - ts) / len(stats) * 1e3
    lat, t_sub, busy, total = [], [0.0] * nf, [False] * nf, 0
    t0 = time.perf_counter()
    for i in range(args.steps + nf):
        k = i % nf
        if busy[k]:
            n, _ = pipes[k].wait_ncc()
            lat.append(time.perf_counter() - t_sub[k])
            total += n
            busy[k] = False
        if i < args.steps:
            t_sub[k] = time.perf_counter()
            pipes[k].submit_ncc(4, 4, 0.4)
            busy[k] = True
    elapsed = time.perf_counter() - t0
    last = stats[-1]
    P = int(last["inliers"])
    sc, nb, best = pipes[0].ncc_results(P, 16)
    _, pts, _ = pipes[0].dlt_results(int(last["matches"]), P)
    same_across = all(np.array_equal(pp.ncc_results(P, 16)[0], sc) for pp in pipes[1:])
    for ctx in ctxs:
        ctx.close()
    cpu, verified = None, None
    if not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as orc
        quota = cpu_quota()
        cores = len(os.sched_getaffinity(0))
        if quota:
            cores = max(1, min(cores, int(quota)))
        t1 = time.perf_counter()
        q, t, _ = orc.match_nndr(pair.desc1, pair.desc2, orc.BITS, nndr, cores)
        opts, _ = orc.triangulate(pair.cam, pair.g12, s.zThresholdMin, s.zThresholdMax, pair.kp1, pair.kp2, q, t)
        R2, t2 = orc.camera2_from_g12(pair.g12)
        rs, rn, rb = orc.ncc_hypotheses(pair.cam, R2, t2, pair.img1, pair.img2, opts, ray, 4, 4, 0.4,
                                        bound=(s.boundWidth, s.boundHeight), zmax=s.zThresholdMax)
        el = time.perf_counter() - t1
        cpu = {"value": len(opts) / el, "unit": "keypoints/s", "cores": cores, "kind": "port", "cpu_model": cpu_model(),
               "sample": f"the whole C3 frame pair: oracle Hamming knn2 + NNDR + DLT + NCC of {len(opts)} points "
                         f"x 16 hypotheses, {el:.2f} s"}
        verified = bool(np.array_equal(pts, opts) and np.array_equal(sc, rs) and np.array_equal(best, rb) and
                        np.array_equal(nb, rn, equal_nan=True))
    ncc_ms = float(np.mean([x["lm_ms"] for x in stats]))
    # HBM bytes and VALU busy of ncc_kernel from the committed rocprofv3 PMC passes of this command
    # (tools/r05_final_session.sh -> profiles/r05_pmc_c3.json; round 4's file before it), when they
    # are for the same workload
    pmc, pmc_file = None, None
    for name in ("r05_pmc_c3.json", "r04_pmc_c3.json"):
        try:
            with open(os.path.join(ROOT, "profiles", name)) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        w = d.get("workload", {})
        if (w.get("keypoints"), w.get("ray")) == (wl["keypoints"], ray):
            pmc, pmc_file = d, name
            break
    m_dat = sum(1 for i in range(-ray, ray + 1) for j in range(-ray, ray + 1) if i * i + j * j <= ray * ray)
    pix = P * 16 * m_dat
    achieved = FLOPS_PER_PIXEL_EVAL * pix / (ncc_ms * 1e-3) / 1e12 if ncc_ms > 0 else 0.0
    out = {
        "metric": "matched+triangulated+NCC-scored keypoints/sec (BASELINE C3: Hamming match + 64x64 patch NCC "
                  "over 16 normal hypotheses)",
        "value": total / elapsed, "unit": "keypoints/s",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "latency_ms": float(np.mean(lat)) * 1e3, "synchronous_ms_per_step": sync_ms, "inflight": nf,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (ray-cast facet scene, seeded; 3dfeaturematcher_amd/synth.py)",
        "config": {"workload": f"C3: {wl['keypoints'] // 1000}k ORB-256 keypoints per {wl['width']}x{wl['height']} frame "
                               f"pair, Hamming knnMatch k=2 + NNDR {nndr} + DLT + NCC of 4 x 4 normals (span 0.4 rad) "
                               f"over the pixelsRay-{ray} neighbourhood",
                   "keypoints_per_frame": wl["keypoints"], "parallelism": "1 GPU",
                   "timed": f"K frame pairs through match -> NNDR -> DLT -> NCC scoring on HBM-resident inputs "
                            f"(scores stay on the device), {nf} contexts (HIP streams) in flight, every pair's counts "
                            f"read back (page-locked) before its context takes the next; synchronous_ms_per_step: "
                            f"one pair at a time"},
        "roofline": {"kernel": "fm3d::ncc_kernel (NCC over candidate normals)", "bound": "fp64-valu",
                     "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / FP64_PEAK_TFLOPS,
                     "traffic": pmc["hbm_bytes_per_launch"] if pmc else None,
                     "traffic_source": f"profiles/{pmc_file} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes)"
                                       if pmc else None,
                     "valu_busy_per_simd": pmc.get("valu_busy_per_simd") if pmc else None,
                     "l2_hit": pmc.get("l2_hit") if pmc else None,
                     "algorithmic": f"{FLOPS_PER_PIXEL_EVAL} flop per pixel evaluation (the LM's count for the "
                                    f"same geometry + bilinear sample) x {P} points x 16 hypotheses x {m_dat} "
                                    f"neighbourhood pixels (image-bounded pixels count too)",
                     "avg_launch_ms": ncc_ms},
        "cpu_baseline": cpu,
        "stages_ms": {"match_ms": last["match_ms"], "nndr_ms": last["nndr_ms"], "triangulate_ms": last["triangulate_ms"],
                      "ncc_ms": last["lm_ms"], "total_ms": last["total_ms"]},
        "counts": {"queries": int(last["queries"]), "matches": int(last["matches"]), "inliers": P,
                   "scored": int((best >= 0).sum())},
        "scores_identical_across_contexts": bool(same_across),
        "verified": verified,
        "verification": "inlier points, all 16 scores per point, best index and best normal byte-equal to the "
                        "cpu_baseline leg's oracle outputs",
    }
    line = json.dumps(out)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


def c2_cpu_baseline(pair, s, args):
    """The oracle's C2 path (knn2 + NNDR + DLT, C with OpenMP on the granted cores) on the whole 10k
    frame pair: (baseline dict, its outputs)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    quota = cpu_quota()
    cores = len(os.sched_getaffinity(0))
    if quota:
        cores = max(1, min(cores, int(quota)))
    t0 = time.perf_counter()
    q, t, dist = orc.match_nndr(pair.desc1, pair.desc2, orc.U8, args.nndr, cores)
    opts, _ = orc.triangulate(pair.cam, pair.g12, s.zThresholdMin, s.zThresholdMax, pair.kp1, pair.kp2, q, t)
    el = time.perf_counter() - t0
    base = {"value": len(opts) / el, "unit": "keypoints/s", "cores": cores, "kind": "port",
            "cpu_model": cpu_model(),
            "sample": f"the whole C2 frame pair: oracle knn2 of {len(pair.desc1)} x {len(pair.desc2)} u8 rows + "
                      f"NNDR + DLT of {len(q)} matches, {el:.2f} s"}
    return base, (q, t, dist, opts)


def verify_against_fixture(args, wl, workload, pair, rec):
    """The headline run's own correctness proof: the generated inputs' digests and the survivor
    records against the committed oracle run of the same frame pair (the CPU oracle in DETMATH mode,
    made in the container by tests/golden/make_full_fixtures.py): for the default C4 workload and the
    C3 lines (10k ORB, --seed 102 --nndr 0.8, pixelsRay 32 or 64) ALL records (full_c4.npz,
    full_c3r32.npz, full_c3r64.npz); for the default C5 workload -- whole on one GPU or merged from
    N -- the records of every 10th 4,096-query block (full_c5sub.npz, 102,400 queries against all 1M
    train rows).  Other workloads: "verified": null."""
    import importlib.util
    path = os.path.join(ROOT, "tests", "golden", "make_full_fixtures.py")
    spec = importlib.util.spec_from_file_location("make_full_fixtures", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mine = dict(n=wl["keypoints"], w=wl["width"], h=wl["height"], seed=args.seed, desc=args.desc, ray=args.ray,
                levels=args.levels, eps=args.nndr)
    name = next((k for k, v in mod.WORKLOADS.items() if {x: v[x] for x in mine} == mine), None)
    if name is None:
        return {"verified": None, "verified_note": "no committed oracle fixture for this workload"}
    fx = mod.load_fixture(name)
    got = mod.input_digests(pair)
    inputs_ok = all(got[k] == v for k, v in fx["digests"].items())
    checked = rec
    qsel = mod.subset_queries(mod.WORKLOADS[name], len(pair.desc1))
    if qsel is not None:
        checked = rec[np.isin(rec["queryIdx"], qsel)]
    records_ok = checked.tobytes() == fx["records"].tobytes()
    return {"verified": bool(inputs_ok and records_ok),
            "verification": {"fixture": f"tests/golden/full_{name}.npz", "inputs_digest_equal": bool(inputs_ok),
                             "records_equal": bool(records_ok), "records_checked": int(len(checked)),
                             "records": int(len(rec)), "fixture_records": int(len(fx["records"])),
                             "fixture_records_sha256": str(fx["records_sha256"])}}


def check_against_one_gpu(args, fm3d, pair, s, merged, local, rank, dist, torch):
    """Rank 0: the unsharded frame pair on its own GPU (one run, untimed by the metric), byte
    for byte against the merge of the last step's gathered records (query order)."""
    res = None
    if rank == 0 and not args.no_check:
        ctx = fm3d.Context(s, device=local)
        try:
            sct = fm3d.SingleCameraTriangulator(ctx)
            sct.set_g12(pair.g12)
            pipe = fm3d.Pipeline(ctx)
            pipe.upload(pair.desc1, pair.desc2, pair.kp1, pair.kp2, pair.img1, pair.img2)
            t = time.perf_counter()
            k, st = pipe.run()
            one_s = time.perf_counter() - t
            full = pipe.records(k)
        finally:
            ctx.close()
        same = full.tobytes() == merged.tobytes()
        res = {"identical_to_1gpu": bool(same), "records": int(len(merged)),
               "digest_sharded": records_digest(merged.tobytes()), "digest_1gpu": records_digest(full.tobytes()),
               "one_gpu_run": {"ms": one_s * 1e3, "kept_per_s": k / one_s,
                               "note": "the same frame pair unsharded on rank 0's GPU, one run after the timed "
                                       "steps (no warmup of its own)"}}
    ok = torch.tensor([0 if (res is not None and not res["identical_to_1gpu"]) else 1], dtype=torch.int32,
                      device=f"cuda:{local}")
    dist.broadcast(ok, 0)
    if not int(ok.item()):
        raise SystemExit("sharded records differ from the single-GPU run")
    return res


def pmc_traffic(args):
    """HBM bytes per LM launch from the committed rocprofv3 PMC summary of this workload
    (separate --pmc passes; rocprofv3 cannot run inside the timed process)."""
    try:
        with open(args.pmc_json) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    w = d.get("workload", {})
    if (w.get("keypoints"), w.get("ray"), w.get("levels")) != (args.keypoints or 100_000, args.ray, args.levels):
        return None
    return {"bytes": d["hbm_bytes_per_launch"], "source": os.path.relpath(args.pmc_json, ROOT),
            "calibration": d.get("calibration")}


def roofline(stats, lm_ms, pix, evals, args, pair, s):
    """The dominant kernel (lm2_kernel) against its fp64 issue ceiling; HBM traffic beside it."""
    traffic = pmc_traffic(args)
    achieved = FLOPS_PER_PIXEL_EVAL * pix / (lm_ms * 1e-3) / 1e12 if lm_ms > 0 else 0.0
    inliers = float(np.mean([st["inliers"] for st in stats]))
    pyr = 0
    w, h = pair.img1.shape[1], pair.img1.shape[0]
    for _ in range(args.levels + 1):
        pyr += w * h
        w, h = (w + 1) // 2, (h + 1) // 2
    alg_bytes = inliers * (24 + 24 + 4) + 2 * pyr  # point in, normal out, status; both pyramids once
    r = {
        "kernel": "fm3d::lm2_kernel (LM normal refinement)",
        "bound": "fp64-valu",
        "compute": "fp64 VALU (no MFMA); -ffp-contract=off, so every flop is its own instruction",
        "achieved": achieved,
        "peak": FP64_PEAK_TFLOPS,
        "unit": "TFLOP/s",
        "frac": achieved / FP64_PEAK_TFLOPS,
        "peak_no_fma": FP64_PEAK_NO_FMA,
        "frac_no_fma": achieved / FP64_PEAK_NO_FMA,
        "traffic": traffic["bytes"] if traffic else None,
        "traffic_unit": "HBM bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, separate --pmc passes)",
        "traffic_source": traffic["source"] if traffic else None,
        "traffic_calibration": traffic["calibration"] if traffic else None,
        "traffic_per_pixel_eval": traffic["bytes"] / pix if traffic and pix else None,
        "algorithmic_bytes": alg_bytes,
        "traffic_over_algorithmic": traffic["bytes"] / alg_bytes if traffic else None,
        "traffic_GBps": traffic["bytes"] / (lm_ms * 1e6) if traffic and lm_ms > 0 else None,
        "algorithmic": f"{FLOPS_PER_PIXEL_EVAL} flop per pixel evaluation x {pix:.4g} pixel evaluations "
                       f"({evals:.4g} residual evaluations) per launch; bytes: {inliers:.0f} points x 52 B + "
                       f"2 pyramids of {pyr} B",
        "avg_launch_ms": lm_ms,
    }
    return r


def lm_profile(lm):
    """Where the LM kernel's time goes (in-kernel clock counters, fm3d_lm_stats).  Per-group
    lifetimes are the chain wave's (it leaves last)."""
    tot = lm["cycles_total"]
    return {
        "groups": lm["groups"], "passes": lm["passes"],
        "chain_busy": lm["cycles_chain"] / tot if tot else None,    # chain wave adding / group lifetime
        "control_over_terms": lm["cycles_control"] / max(lm["cycles_terms"], 1),  # lmdif bookkeeping
        "wait_over_terms": lm["cycles_wait"] / max(lm["cycles_terms"], 1),        # term waves waiting on the chain
        # mean number of term waves inside a pass over the group lifetime
        "busy_slots_per_group": lm["cycles_terms"] / tot if tot else None,
        "group_life_mean_over_max": lm["wall_ticks_sum"] / max(lm["groups"], 1) / max(lm["wall_ticks_max"], 1),
        "clock_ghz": lm["cycles_total"] / max(lm["wall_ticks_sum"], 1) * lm["wall_clock_khz"] * 1e-6,
        "kcycles_per_pass_by_class": {n: round(cy / max(c, 1) / 1e3, 1) for n, c, cy in
                                      zip(("jac", "eval", "qr", "once"), lm["class_passes"], lm["class_cycles"])},
        "passes_by_class": dict(zip(("jac", "eval", "qr", "once"), lm["class_passes"])),
        "last_group_end_ms": lm["last_group_end_ticks"] / max(lm["wall_clock_khz"], 1),
        "queue_empty_ms": lm.get("queue_empty_ticks", 0) / max(lm["wall_clock_khz"], 1),
        # chain wave: cycles per busy round (up to two chunks of 64 dependent adds per lane) and
        # chunks added per round over the group's lanes
        "chain_cycles_per_round": lm["cycles_chain"] / max(lm.get("chain_rounds", 0), 1),
        "chain_chunks_per_round": lm.get("chain_chunks", 0) / max(lm.get("chain_rounds", 0), 1),
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


def cpu_quota():
    """CPUs the cgroup grants this process (cpu.max), None if unlimited / unknown."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(pair, s, gpu_stats, args):
    """Time the CPU oracle (reference algorithm, C + OpenMP) on a bounded sample of the
    same workload, on every CPU this process may run on, and extrapolate to the frame pair."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    # every CPU the process may run on: its affinity set, capped by the cgroup quota (on the GPU
    # box 256 CPUs are visible and 16 granted; 256 threads on a 16-CPU quota run slower)
    quota = cpu_quota()
    threads = len(os.sched_getaffinity(0))
    if quota:
        threads = max(1, min(threads, int(quota)))
    threads = int(os.environ.get("FM3D_CPU_THREADS", "0") or 0) or threads
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
    # triangulation on the oracle's matches of a query sample
    q, tr, _ = orc.match_nndr(pair.desc1[:2000], pair.desc2, orc.U8, s.nndrEpsilon, threads)
    t = time.perf_counter()
    pts, _ = orc.triangulate(pair.cam, pair.g12, s.zThresholdMin, s.zThresholdMax, pair.kp1, pair.kp2, q, tr)
    t_tri = (time.perf_counter() - t) / max(len(q), 1) * gpu_stats["matches"]
    # LM normals: a seeded random subset (per-point LM cost varies by orders of magnitude), 16
    # points per thread so the dynamic schedule balances
    fm3d = importlib.import_module("3dfeaturematcher_amd")
    R2, t2 = fm3d.camera2_from_g12(pair.g12)
    sub = np.random.default_rng(7).permutation(len(pts))
    npts = min(len(pts), 16 * threads)
    t = time.perf_counter()
    orc.optimize_normals(pair.cam, R2, t2, pair.img1, pair.img2, s.pyramids, pts[sub[:npts]], s.pixelsRay,
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
        "nproc": os.cpu_count(),
        "cpu_quota_cores": cpu_quota(),
        "kind": "port",
        "cpu_model": cpu_model(),
        "single_thread": {"value": gpu_stats["kept"] / total1, "unit": "keypoints/s", "cores": 1,
                          "sample": f"knn2 of 256 queries, LM normals of {n1} points, 1 thread (est. {total1:.0f} s "
                                    f"per frame pair: match {t1_match:.1f}, LM {t1_lm:.1f})"},
        "affinity_cpus": len(os.sched_getaffinity(0)),
        "sample": f"oracle (C, OpenMP {threads} threads = the CPUs granted to the process): knn2 of {qs} queries x "
                  f"{len(pair.desc2)} train, DLT of {len(q)} matches, LM normals of {npts} random points "
                  f"(pixelsRay {s.pixelsRay}); extrapolated to {nA} queries / {gpu_stats['matches']} matches / "
                  f"{gpu_stats['inliers']} points (est. {total:.1f} s per frame pair: match {t_match:.1f}, "
                  f"DLT {t_tri:.3f}, LM {t_lm:.1f})",
    }


if __name__ == "__main__":
    main()
