"""Drive the kernels outside the C4 bench for rocprofv3 --kernel-trace --stats:
SURF detect + describe on the VGA frames (Upright 1 = the reference's settings, and Upright 0),
extractDescriptorsFromPatches, ORB detect + describe and compute (2,000 / 10,000 features), SIFT detect + describe and compute, STAR detection (static and ADAPTIVE), BRISK description, the C3 NCC leg (16 hypotheses at pixelsRay 32 over every DLT inlier
of the 10k-ORB pair) and the circular neighbourhoods of the C4 inliers.  Product path only (no
oracle); each leg timed with host wall clock after a warm-up call, printed as one JSON line.

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_aux -o aux --output-format csv -- python3 tools/prof_aux.py
"""
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
fm3d = importlib.import_module("3dfeaturematcher_amd")
synth = importlib.import_module("3dfeaturematcher_amd.synth")


def timed(f, reps):
    f()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = f()
    return out, (time.perf_counter() - t0) / reps * 1e3


def main():
    res = {}
    pair = synth.make_frame_pair(2000, seed=3)
    for upright in (1, 0):
        s = fm3d.Settings.default()
        s.surfUpright = upright
        ctx = fm3d.Context(s)
        try:
            (k, d), ms = timed(lambda: fm3d.SURF(ctx).detect(pair.img1, with_descriptors=True), 5)
            res[f"surf_detect_describe_vga_upright{upright}"] = {"keypoints": int(len(k)), "ms": round(ms, 3)}
            patches = np.random.default_rng(9).integers(0, 256, (1000, 128, 128), dtype=np.uint8)
            _, ms = timed(lambda: fm3d.SURF(ctx).extractDescriptorsFromPatches(patches), 3)
            res[f"surf_patches_1000x128_upright{upright}"] = {"ms": round(ms, 3)}
        finally:
            ctx.close()
    # ORB (DetectorType / ExtractorType ORB) on the VGA frame: 2,000 and 10,000 features
    for nf in (2000, 10_000):
        s = fm3d.Settings.default()
        s.detectorType = s.extractorType = fm3d.FEAT_ORB
        s.orbNumFeatures = nf
        ctx = fm3d.Context(s)
        try:
            orb = fm3d.ORB(ctx)
            (k, d), ms = timed(lambda: orb.detect(pair.img1, with_descriptors=True), 5)
            res[f"orb_detect_describe_vga_{nf}"] = {"keypoints": int(len(k)), "ms": round(ms, 3)}
            (kc, _, _), ms = timed(lambda: orb.compute(pair.img1, k), 5)
            res[f"orb_compute_vga_{nf}"] = {"keypoints": int(len(kc)), "ms": round(ms, 3)}
        finally:
            ctx.close()
    # SIFT (DetectorType / ExtractorType SIFT, OpenCV's defaults) on the VGA frame: detect + describe,
    # and compute on the detected keypoints (the reference's second call)
    s = fm3d.Settings.default()
    s.detectorType = s.extractorType = fm3d.FEAT_SIFT
    ctx = fm3d.Context(s)
    try:
        sift = fm3d.SIFT(ctx)
        (k, d), ms = timed(lambda: sift.detect(pair.img1, with_descriptors=True), 5)
        res["sift_detect_describe_vga"] = {"keypoints": int(len(k)), "ms": round(ms, 3)}
        _, ms = timed(lambda: sift.detect(pair.img1), 5)
        res["sift_detect_vga"] = {"keypoints": int(len(k)), "ms": round(ms, 3)}
        (kc, _, _), ms = timed(lambda: sift.compute(pair.img1, k), 5)
        res["sift_compute_vga"] = {"keypoints": int(len(kc)), "ms": round(ms, 3)}
    finally:
        ctx.close()
    # STAR (DetectorType STAR, cv::StarDetector's defaults) on the VGA frame, and the StarAdjuster walk
    s = fm3d.Settings.default()
    s.detectorType = fm3d.FEAT_STAR
    ctx = fm3d.Context(s)
    try:
        feats = fm3d.Features(ctx)
        k, ms = timed(lambda: feats.detect(pair.img1), 5)
        res["star_detect_vga"] = {"keypoints": int(len(k)), "ms": round(ms, 3)}
    finally:
        ctx.close()
    s.detectorMode, s.adaptiveMinFeatures, s.adaptiveMaxFeatures, s.adaptiveMaxIters = 1, 400, 500, 30
    ctx = fm3d.Context(s)
    try:
        feats = fm3d.Features(ctx)
        k, ms = timed(lambda: feats.detect(pair.img1), 3)
        res["star_adaptive_vga_400_500"] = {"keypoints": int(len(k)), "ms": round(ms, 3)}
    finally:
        ctx.close()
    # BRISK (ExtractorType BRISK) on the VGA frame's SURF keypoints
    s = fm3d.Settings.default()
    s.extractorType = fm3d.FEAT_BRISK
    ctx = fm3d.Context(s)
    try:
        feats = fm3d.Features(ctx)
        ks = feats.detect(pair.img1)
        (kb, _, _), ms = timed(lambda: feats.compute(pair.img1, ks), 5)
        res["brisk_compute_vga_surf_kpts"] = {"keypoints": int(len(kb)), "ms": round(ms, 3)}
    finally:
        ctx.close()
    # C3 NCC leg: the 10k-ORB pair's DLT inliers, 16 hypotheses, pixelsRay 32
    fp = synth.make_frame_pair(10_000, seed=102, desc="orb")
    s = fm3d.Settings.default()
    s.set_camera(fp.cam)
    s.pixelsRay, s.nndrEpsilon, s.boundWidth, s.boundHeight = 32, 0.8, 640, 480
    ctx = fm3d.Context(s)
    try:
        m = fm3d.DescriptorsMatcher(ctx, binary=True).compareWithNNDR(0.8, fp.desc1, fp.desc2)
        sct = fm3d.SingleCameraTriangulator(ctx)
        sct.set_g12(fp.g12)
        sct.setKeypoints(fp.kp1, fp.kp2, m)
        pts, _ = sct.triangulate()
        no = fm3d.NormalOptimizer(ctx, sct)
        no.setImages(fp.img1, fp.img2)
        (sc, _, b), ms = timed(lambda: no.nccHypotheses(pts, 4, 4, 0.4), 5)
        res["ncc_c3_r32_16hyp"] = {"points": int(len(pts)), "ms": round(ms, 3), "scored": int((b >= 0).sum())}
    finally:
        ctx.close()
    # circular neighbourhoods (Neighborhoods.method 1, 15 thetas x 5 rays) of 36k points
    s.neighMethod, s.neighThetas, s.neighRays = 1, 15, 5
    ctx = fm3d.Context(s)
    try:
        ng = fm3d.NeighborhoodsGenerator(s)
        X = np.tile(pts, (36_000 // len(pts) + 1, 1))[:36_000]
        out, ms = timed(lambda: ng.computeCircularNeighborhoodsByNormals(ctx, X), 5)
        res["circular_36k_points"] = {"points": int(len(X)), "samples": int(out.shape[1]), "ms": round(ms, 3)}
    finally:
        ctx.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
