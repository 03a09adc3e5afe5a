"""BASELINE's C2 through the HBM-resident pipeline (fm3d_pipeline_run_dlt: match -> NNDR -> DLT only),
bit for bit against the oracle (knn2 + NNDR + triangulate), and the same front half inside the full
fm3d_pipeline_run (its matches and inlier points after the LM)."""
import numpy as np
import pytest

from conftest import oracle_threads

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,seed", [(10_000, 7), (2_500, 3)])
def test_pipeline_dlt_bitwise(fm3d, orc, synth, n, seed):
    pair = synth.make_frame_pair(n, seed=seed)
    s = fm3d.Settings.default()
    s.set_camera(pair.cam)
    s.nndrEpsilon = 0.55
    s.pixelsRay, s.pyramids = 8, 1
    ctx = fm3d.Context(s)
    try:
        sct = fm3d.SingleCameraTriangulator(ctx)
        sct.set_g12(pair.g12)
        pipe = fm3d.Pipeline(ctx)
        pipe.upload(pair.desc1, pair.desc2, pair.kp1, pair.kp2, pair.img1, pair.img2)
        P, st = pipe.run_dlt()
        m, pts, src = pipe.dlt_results(st["matches"], st["inliers"])
        P2, st2 = pipe.run_dlt()  # repeatable on the same staged inputs
        _, pts2, _ = pipe.dlt_results(st2["matches"], st2["inliers"])
        kept, _ = pipe.run()  # the full path's front half leaves the same matches / points
        m3, pts3, src3 = pipe.dlt_results(st["matches"], st["inliers"])
    finally:
        ctx.close()
    q, t, dist = orc.match_nndr(pair.desc1, pair.desc2, orc.U8, 0.55, oracle_threads())
    opts, mask = orc.triangulate(pair.cam, pair.g12, s.zThresholdMin, s.zThresholdMax, pair.kp1, pair.kp2, q, t)
    assert len(m) == len(q) > 100 and P == len(opts) > 50
    assert np.array_equal(m["queryIdx"], q) and np.array_equal(m["trainIdx"], t) and np.array_equal(m["distance"], dist)
    assert np.array_equal(pts, opts) and np.array_equal(src, np.flatnonzero(mask))
    assert P2 == P and np.array_equal(pts2, pts)
    assert np.array_equal(m3, m) and np.array_equal(pts3, pts) and np.array_equal(src3, src) and kept <= P
