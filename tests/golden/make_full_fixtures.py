"""Full-size expected records of the BASELINE configurations, from the CPU oracle.

TEST INFRASTRUCTURE (run here, in the container, never on the GPU box):

    python tests/golden/make_full_fixtures.py c4 c3 c5sub [--threads 8]

For each workload it generates the seeded synthetic frame pair exactly as the GPU tests and
bench.py do (3dfeaturematcher_amd/synth.py), records a SHA-256 digest of every input array
(descriptors, keypoints, both images, g12), and runs the whole path through the oracle
(oracle/fm3d_oracle.c): exact brute-force knn + NNDR (descriptorsmatcher.cpp:107-131),
setKeypoints + triangulate (singlecameratriangulator.cpp:145-230) and computeOptimizedNormals
(normaloptimizer.cpp:321-452) in DETMATH mode -- the GPU contract -- over EVERY inlier.  The
survivors become fm3d_record rows (include/fm3d.h), in query order, and are committed as
tests/golden/full_<name>.npz (records + input digests + counts + the records' SHA-256).

The GPU tests first assert the input digests (a box whose numpy generated a different frame
pair fails loudly instead of comparing another workload), then compare every record byte for
byte; bench.py checks its records' digest against the C4 file and reports "verified".
"""
from __future__ import annotations

import argparse
import hashlib
import importlib
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

# fm3d_record (include/fm3d.h)
RECORD = np.dtype([("queryIdx", "<i4"), ("trainIdx", "<i4"), ("distance", "<f4"), ("status", "<i4"),
                   ("point", "<f8", 3), ("normal", "<f8", 3)])

# name -> frame pair + settings, as the GPU tests / bench.py use them
WORKLOADS = {
    # BASELINE configs[3]: the bench workload (bench.py defaults, test_c4_sift100k_full_pipeline)
    "c4": dict(n=100_000, w=640, h=480, seed=7, desc="sift", ray=64, levels=3, eps=0.55),
    # BASELINE configs[2]: 10k ORB-256 in SURVEY.md §8(d)'s two variants (test_c3_orb10k_pipeline)
    "c3r32": dict(n=10_000, w=640, h=480, seed=102, desc="orb", ray=32, levels=3, eps=0.8),
    "c3r64": dict(n=10_000, w=640, h=480, seed=102, desc="orb", ray=64, levels=3, eps=0.8),
    # BASELINE configs[4]: the 1M-keypoint pair; a fixed 10 % of its queries (every tenth
    # 4,096-query block, the unit bench.py deals to the ranks)
    "c5sub": dict(n=1_000_000, w=640, h=480, seed=7, desc="sift", ray=64, levels=3, eps=0.55, blocks=(4096, 10)),
}


def sha(a) -> str:
    a = np.ascontiguousarray(a)
    h = hashlib.sha256()
    h.update(str(a.dtype).encode() + str(a.shape).encode())
    h.update(a.tobytes())
    return h.hexdigest()


def input_digests(fp) -> dict:
    return {k: sha(getattr(fp, k)) for k in ("desc1", "desc2", "kp1", "kp2", "img1", "img2", "g12")}


def subset_queries(wl: dict, n: int) -> np.ndarray | None:
    if "blocks" not in wl:
        return None
    b, every = wl["blocks"]
    q = np.arange(n)
    return q[(q // b) % every == 0]


def make_pair(wl: dict):
    synth = importlib.import_module("3dfeaturematcher_amd.synth")
    return synth.make_frame_pair(wl["n"], wl["w"], wl["h"], seed=wl["seed"], desc=wl["desc"])


def oracle_records(fp, wl: dict, threads: int, log=print) -> tuple[np.ndarray, dict]:
    import oracle as orc
    qsel = subset_queries(wl, len(fp.desc1))
    d1 = fp.desc1 if qsel is None else fp.desc1[qsel]
    k1 = fp.kp1 if qsel is None else fp.kp1[qsel]
    kind = orc.BITS if wl["desc"] == "orb" else orc.U8
    t = time.time()
    q, tr, d = orc.match_nndr(d1, fp.desc2, kind, wl["eps"], threads)
    log(f"  match+nndr: {len(q)} matches ({time.time() - t:.1f} s)")
    pts, mask = orc.triangulate(fp.cam, fp.g12, 1.5, 2.4, k1, fp.kp2, q, tr)
    log(f"  triangulate: {len(pts)} inliers")
    R2, t2 = orc.camera2_from_g12(fp.g12)
    t = time.time()
    ref = orc.optimize_normals(fp.cam, R2, t2, fp.img1, fp.img2, wl["levels"], pts, wl["ray"], mode=orc.DETMATH,
                               nthreads=threads)
    ok = ref["status"] == 0
    log(f"  LM (DETMATH): {int(ok.sum())} kept of {len(pts)} ({time.time() - t:.1f} s)")
    rec = np.zeros(int(ok.sum()), dtype=RECORD)
    qi = q[mask][ok]
    rec["queryIdx"] = qi if qsel is None else qsel[qi]
    rec["trainIdx"] = tr[mask][ok]
    rec["distance"] = d[mask][ok]
    rec["status"] = 0
    rec["point"] = pts[ok]
    rec["normal"] = ref["normals"][ok]
    counts = dict(queries=len(d1), matches=len(q), inliers=len(pts), kept=int(ok.sum()),
                  drops=np.bincount(ref["status"], minlength=8).tolist())
    return rec, counts


def records_digest(rec: np.ndarray) -> str:
    """bench.py's records_sha256 (first 16 hex digits of the SHA-256 of the record bytes)"""
    return hashlib.sha256(np.ascontiguousarray(rec).tobytes()).hexdigest()[:16]


def fixture_path(name: str) -> str:
    return os.path.join(HERE, f"full_{name}.npz")


def load_fixture(name: str) -> dict:
    with np.load(fixture_path(name), allow_pickle=False) as z:
        d = {k: z[k] for k in z.files}
    d["digests"] = dict(zip(d["digest_keys"].tolist(), d["digest_vals"].tolist()))
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("names", nargs="+", choices=sorted(WORKLOADS))
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    args = ap.parse_args()
    for name in args.names:
        wl = WORKLOADS[name]
        print(f"{name}: {wl}", flush=True)
        t = time.time()
        fp = make_pair(wl)
        dig = input_digests(fp)
        print(f"  frame pair generated ({time.time() - t:.1f} s)", flush=True)
        rec, counts = oracle_records(fp, wl, args.threads, log=lambda s: print(s, flush=True))
        keys = sorted(dig)
        np.savez_compressed(fixture_path(name), records=rec, digest_keys=np.array(keys),
                            digest_vals=np.array([dig[k] for k in keys]),
                            counts=np.array([counts["queries"], counts["matches"], counts["inliers"], counts["kept"]]),
                            drops=np.array(counts["drops"]), records_sha256=np.array(records_digest(rec)),
                            workload=np.array(repr(wl)))
        print(f"  {name}: {counts} records_sha256 {records_digest(rec)} -> {fixture_path(name)}", flush=True)


if __name__ == "__main__":
    main()
