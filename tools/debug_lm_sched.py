"""LM schedule check on one GPU: 6,000 points (more than the 3,840 slots) through
computeOptimizedNormals with and without the tail help (FM3D_LM_COOP), several times each, compared with the
oracle (DETMATH); prints the mismatching points.

    python tools/debug_lm_sched.py
"""
import importlib
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def run_one():
    import oracle as orc
    fm3d = importlib.import_module("3dfeaturematcher_amd")
    synth = importlib.import_module("3dfeaturematcher_amd.synth")
    pair = synth.make_frame_pair(3000, seed=11)
    q, t, _ = orc.match_nndr(pair.desc1, pair.desc2, orc.U8, 0.55, 16)
    pts, _ = orc.triangulate(pair.cam, pair.g12, 1.5, 2.4, pair.kp1, pair.kp2, q, t)
    reps = -(-6000 // len(pts))
    P = np.concatenate([pts * (1.0 + 2e-3 * r) for r in range(reps)])[:6000]
    s = fm3d.Settings.default()
    s.set_camera(pair.cam)
    s.pixelsRay = 6
    ctx = fm3d.Context(s)
    sct = fm3d.SingleCameraTriangulator(ctx)
    sct.set_g12(pair.g12)
    R2, t2 = sct.camera2()
    no = fm3d.NormalOptimizer(ctx, sct)
    no.setImages(pair.img1, pair.img2)
    ref = orc.optimize_normals(pair.cam, R2, t2, pair.img1, pair.img2, 3, P, 6, mode=orc.DETMATH, nthreads=16)
    for rep in range(int(os.environ.get("REPS", "4"))):
        _, normals = no.computeOptimizedNormals(P)
        st, info, nfev = no.last_status, no.last_info, no.last_nfev
        bad = np.nonzero((st != ref["status"]) | (nfev[:, :4] != ref["nfev"][:, :4]).any(1))[0]
        ok = ref["status"] == 0
        nbad = int((normals != ref["normals"][ok]).any(1).sum()) if len(normals) == ok.sum() else -1
        print("coop", os.environ.get("FM3D_LM_COOP"), "rep", rep, "mismatches", len(bad),
              "normals", nbad, flush=True)
        for i in bad[:12]:
            print(i, "gpu", st[i], info[i, :4], nfev[i, :4], "ref", ref["status"][i], ref["info"][i, :4], ref["nfev"][i, :4])


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run_one()
    else:
        for coop in ("0", "1"):
            env = dict(os.environ, FM3D_LM_COOP=coop, FM3D_LM_MAX_SECONDS="30")
            subprocess.run([sys.executable, "-u", __file__, "one"], env=env, timeout=240, check=True)
