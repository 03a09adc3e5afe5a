"""BASELINE's C2 through the HBM-resident pipeline (fm3d_pipeline_run_dlt: match -> NNDR -> DLT only),
bit for bit against the oracle (knn2 + NNDR + triangulate), and the same front half inside the full
fm3d_pipeline_run (its matches and inlier points after the LM)."""
import numpy as np
import pytest

from conftest import oracle_threads

pytestmark = pytest.mark.gpu


# 2,500 and 10,000 queries: the one-workgroup compaction; 20,000: the three-kernel one
@pytest.mark.parametrize("n,seed", [(10_000, 7), (2_500, 3), (20_000, 5)])
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


def test_pipeline_dlt_counts_without_copies_and_stage_events(fm3d, orc, synth, monkeypatch):
    """Round 5: the DLT kernel stores (matches, inliers) straight into the page-locked buffer, and
    FM3D_STAGE_EVENTS=0 drops the stage-boundary events.  Alternating pairs with many, few and no
    matches (an NNDR ratio no pair passes) on one context: every step's counts are that pair's
    (never a stale value of the step before: one context alternates the two pairs), its matches and
    points equal the oracle's, and without
    stage events match_ms / triangulate_ms are 0 while total_ms and the results are unchanged."""
    pairs = [synth.make_frame_pair(3000, seed=21), synth.make_frame_pair(700, seed=22)]
    s = fm3d.Settings.default()
    s.set_camera(pairs[0].cam)
    s.pixelsRay, s.pyramids = 8, 1
    ref = {}
    for i, fp in enumerate(pairs):
        for eps in (0.55, 1e-6):
            q, t, _ = orc.match_nndr(fp.desc1, fp.desc2, orc.U8, eps, oracle_threads())
            pts, _ = orc.triangulate(fp.cam, fp.g12, s.zThresholdMin, s.zThresholdMax, fp.kp1, fp.kp2, q, t)
            ref[i, eps] = (q, pts)
    assert len(ref[1, 1e-6][0]) == 0 < len(ref[1, 0.55][0])
    ctxs, pipes = {}, {}
    for eps in (0.55, 1e-6):
        s.nndrEpsilon = eps
        ctxs[eps] = fm3d.Context(s)
        fm3d.SingleCameraTriangulator(ctxs[eps]).set_g12(pairs[0].g12)
        pipes[eps] = fm3d.Pipeline(ctxs[eps])
    try:
        for events in ("1", "0"):
            monkeypatch.setenv("FM3D_STAGE_EVENTS", events)
            for i, eps in [(0, 0.55), (1, 1e-6), (1, 0.55), (0, 1e-6), (0, 0.55), (1, 0.55)]:
                fp = pairs[i]
                pipes[eps].upload(fp.desc1, fp.desc2, fp.kp1, fp.kp2, fp.img1, fp.img2)
                P, st = pipes[eps].run_dlt()
                m, pts, _ = pipes[eps].dlt_results(st["matches"], st["inliers"])
                q, opts = ref[i, eps]
                assert st["matches"] == len(q) and P == st["inliers"] == len(opts)
                assert np.array_equal(m["queryIdx"], q) and np.array_equal(pts, opts)
                assert st["total_ms"] > 0
                if events == "0":
                    assert st["match_ms"] == 0 and st["triangulate_ms"] == 0
                elif len(q):
                    assert st["match_ms"] > 0 and st["triangulate_ms"] > 0
    finally:
        for c in ctxs.values():
            c.close()


def test_pipeline_submit_wait_dlt_two_in_flight(fm3d, orc, synth):
    """fm3d_pipeline_submit_dlt / wait_dlt on two contexts in flight (the C2 serving loop) equal
    fm3d_pipeline_run_dlt; a pending front half blocks the other pipeline calls"""
    pair = synth.make_frame_pair(6000, seed=11)
    s = fm3d.Settings.default()
    s.set_camera(pair.cam)
    s.nndrEpsilon = 0.55
    ctxs = [fm3d.Context(s) for _ in range(2)]
    try:
        pipes = []
        for c in ctxs:
            fm3d.SingleCameraTriangulator(c).set_g12(pair.g12)
            p = fm3d.Pipeline(c)
            p.upload(pair.desc1, pair.desc2, pair.kp1, pair.kp2, pair.img1, pair.img2)
            pipes.append(p)
        P0, st0 = pipes[0].run_dlt()
        ref = pipes[0].dlt_results(st0["matches"], st0["inliers"])
        for _ in range(3):
            pipes[0].submit_dlt()
            pipes[1].submit_dlt()
            with pytest.raises(fm3d.Fm3dError):
                pipes[0].run_dlt()
            with pytest.raises(fm3d.Fm3dError):
                pipes[1].submit_dlt()
            for p in pipes:
                P, st = p.wait_dlt()
                got = p.dlt_results(st["matches"], st["inliers"])
                assert P == P0 and st["matches"] == st0["matches"]
                for a, b in zip(got, ref):
                    assert np.array_equal(a, b)
        with pytest.raises(fm3d.Fm3dError):
            pipes[0].wait_dlt()  # nothing pending
    finally:
        for c in ctxs:
            c.close()


def test_pipeline_submit_wait_ncc_two_in_flight(fm3d, synth):
    """fm3d_pipeline_submit_ncc / wait_ncc on two contexts in flight (the C3 serving loop) equal
    fm3d_pipeline_run_ncc bit for bit; a pending scoring blocks the other pipeline calls and the
    DLT / full waits"""
    pair = synth.make_frame_pair(4000, seed=102, desc="orb")
    s = fm3d.Settings.default()
    s.set_camera(pair.cam)
    s.nndrEpsilon = 0.8
    s.pixelsRay = 16
    ctxs = [fm3d.Context(s) for _ in range(2)]
    try:
        pipes = []
        for c in ctxs:
            fm3d.SingleCameraTriangulator(c).set_g12(pair.g12)
            p = fm3d.Pipeline(c)
            p.upload(pair.desc1, pair.desc2, pair.kp1, pair.kp2, pair.img1, pair.img2, binary=True)
            pipes.append(p)
        P0, st0 = pipes[0].run_ncc(4, 4, 0.4)
        ref = pipes[0].ncc_results(P0, 16)
        assert P0 > 100
        for _ in range(3):
            pipes[0].submit_ncc(4, 4, 0.4)
            pipes[1].submit_ncc(4, 4, 0.4)
            with pytest.raises(fm3d.Fm3dError):
                pipes[0].run_ncc(4, 4, 0.4)
            with pytest.raises(fm3d.Fm3dError):
                pipes[1].wait_dlt()
            for p in pipes:
                P, st = p.wait_ncc()
                assert P == P0 and st["matches"] == st0["matches"]
                for a, b in zip(p.ncc_results(P, 16), ref):
                    assert np.array_equal(a, b, equal_nan=True)
        with pytest.raises(fm3d.Fm3dError):
            pipes[0].wait_ncc()  # nothing pending
    finally:
        for c in ctxs:
            c.close()


def test_pipeline_ncc_bitwise(fm3d, orc, synth):
    """BASELINE's C3 as worded through the pipeline (fm3d_pipeline_run_ncc): Hamming match -> NNDR ->
    DLT -> NCC of 4 x 4 normals at pixelsRay 32, every inlier's scores against the oracle on a sample"""
    fp = synth.make_frame_pair(10_000, seed=102, desc="orb")
    s = fm3d.Settings.default()
    s.set_camera(fp.cam)
    s.nndrEpsilon, s.pixelsRay = 0.8, 32
    ctx = fm3d.Context(s)
    try:
        sct = fm3d.SingleCameraTriangulator(ctx)
        sct.set_g12(fp.g12)
        R2, t2 = sct.camera2()
        pipe = fm3d.Pipeline(ctx)
        pipe.upload(fp.desc1, fp.desc2, fp.kp1, fp.kp2, fp.img1, fp.img2, binary=True)
        P, st = pipe.run_ncc(4, 4, 0.4)
        sc, nb, b = pipe.ncc_results(P, 16)
        _, pts, _ = pipe.dlt_results(st["matches"], P)
    finally:
        ctx.close()
    q, t, _ = orc.match_nndr(fp.desc1, fp.desc2, orc.BITS, 0.8, oracle_threads())
    opts, _ = orc.triangulate(fp.cam, fp.g12, s.zThresholdMin, s.zThresholdMax, fp.kp1, fp.kp2, q, t)
    assert P == len(opts) > 5000 and np.array_equal(pts, opts)
    sel = np.sort(np.random.default_rng(34).choice(P, 800, replace=False))
    rs, rn, rb = orc.ncc_hypotheses(fp.cam, R2, t2, fp.img1, fp.img2, opts[sel], 32, 4, 4, 0.4,
                                    bound=(s.boundWidth, s.boundHeight), zmax=s.zThresholdMax)
    assert np.array_equal(sc[sel], rs) and np.array_equal(b[sel], rb) and np.array_equal(nb[sel], rn, equal_nan=True)
    assert (b >= 0).mean() > 0.3


def test_pipeline_float_sift_rows_packed_on_device(fm3d, orc, synth):
    """SIFT rows as the reference hands them to knnMatch (float cv::Mat,
    descriptorsmatcher.cpp:114-117).  fm3d_pipeline_submit with float32 rows: the device checks them
    (integers in [0, 255]) and packs them to u8, so the survivor records equal the u8 rows' byte for
    byte and the oracle's matches; rows with one non-integer element take the float kernels and
    equal the oracle's float (FLANN-order) matching; upload without images runs C2's path."""
    pair = synth.make_frame_pair(4000, seed=31)
    s = fm3d.Settings.default()
    s.set_camera(pair.cam)
    s.nndrEpsilon = 0.55
    s.pixelsRay, s.pyramids = 12, 2
    ctx = fm3d.Context(s)
    try:
        fm3d.SingleCameraTriangulator(ctx).set_g12(pair.g12)
        pipe = fm3d.Pipeline(ctx)
        out = {}
        for kind in ("u8", "f32"):
            d1 = pair.desc1 if kind == "u8" else pair.desc1.astype(np.float32)
            d2 = pair.desc2 if kind == "u8" else pair.desc2.astype(np.float32)
            pipe.submit(d1, d2, pair.kp1, pair.kp2, pair.img1, pair.img2)
            rec, st = pipe.wait()
            out[kind] = (rec.copy(), st)
        assert len(out["u8"][0]) > 100 and out["u8"][0].tobytes() == out["f32"][0].tobytes()
        q, t, dist = orc.match_nndr(pair.desc1, pair.desc2, orc.U8, 0.55, oracle_threads())
        assert out["f32"][1]["matches"] == len(q)
        # C2's front half from float rows, staged without images
        pipe.upload(pair.desc1.astype(np.float32), pair.desc2.astype(np.float32), pair.kp1, pair.kp2, None, None)
        P, st = pipe.run_dlt()
        m, pts, _ = pipe.dlt_results(st["matches"], st["inliers"])
        opts, _ = orc.triangulate(pair.cam, pair.g12, s.zThresholdMin, s.zThresholdMax, pair.kp1, pair.kp2, q, t)
        assert np.array_equal(m["queryIdx"], q) and np.array_equal(m["trainIdx"], t)
        assert np.array_equal(m["distance"], dist) and np.array_equal(pts, opts)
        # one element off the integers: the float path (FLANN's L2 order), against the oracle's F32 scan
        f1 = pair.desc1.astype(np.float32)
        f2 = pair.desc2.astype(np.float32)
        f2[17, 5] += 0.25
        pipe.upload(f1, f2, pair.kp1, pair.kp2, None, None)
        P, st = pipe.run_dlt()
        m, pts, _ = pipe.dlt_results(st["matches"], st["inliers"])
        qf, tf, df = orc.match_nndr(f1, f2, orc.F32, 0.55, oracle_threads())
        assert np.array_equal(m["queryIdx"], qf) and np.array_equal(m["trainIdx"], tf)
        assert np.array_equal(m["distance"], df)
    finally:
        ctx.close()


def test_submit_dlt_pair_equals_upload_and_run_dlt(fm3d, orc, synth):
    """fm3d_pipeline_submit_dlt_pair (C2 from host memory without a host wait; bench.py --workload
    c2 --io host): u8 rows, integer float rows (packed on the device and matched as u8 before their
    flag is read) and float rows with one non-integer element (wait_dlt reads the flag and runs
    the front half again on the float rows), on two contexts in flight, interleaved.  Each pair's
    matches and points equal fm3d_pipeline_upload + run_dlt of the same rows, and the oracle's."""
    pair = synth.make_frame_pair(4000, seed=35)
    s = fm3d.Settings.default()
    s.set_camera(pair.cam)
    s.nndrEpsilon = 0.55
    f1 = pair.desc1.astype(np.float32)
    f2 = pair.desc2.astype(np.float32)
    g2 = f2.copy()
    g2[23, 7] += 0.5
    cases = {"u8": (pair.desc1, pair.desc2), "f32": (f1, f2), "f32_frac": (f1, g2)}
    ctxs = [fm3d.Context(s) for _ in range(2)]
    try:
        pipes = []
        for ctx in ctxs:
            fm3d.SingleCameraTriangulator(ctx).set_g12(pair.g12)
            pipes.append(fm3d.Pipeline(ctx))
        ref = {}
        for name, (a, b) in cases.items():
            pipes[0].upload(a, b, pair.kp1, pair.kp2, None, None)
            P, st = pipes[0].run_dlt()
            m, pts, src = pipes[0].dlt_results(st["matches"], st["inliers"])
            ref[name] = (m.copy(), pts.copy(), src.copy())
        order = ["f32", "f32_frac", "u8", "f32_frac", "f32", "u8", "f32", "f32_frac"]
        pend = [None, None]
        got = []
        for i, name in enumerate(order + [None, None]):
            k = i % 2
            if pend[k] is not None:
                P, st = pipes[k].wait_dlt()
                m, pts, src = pipes[k].dlt_results(st["matches"], st["inliers"])
                got.append((pend[k], m.copy(), pts.copy(), src.copy()))
                pend[k] = None
            if name is not None:
                a, b = cases[name]
                pipes[k].submit_dlt_pair(a, b, pair.kp1, pair.kp2)
                pend[k] = name
        assert len(got) == len(order)
        for name, m, pts, src in got:
            rm, rp, rs = ref[name]
            assert m.tobytes() == rm.tobytes() and pts.tobytes() == rp.tobytes() and src.tobytes() == rs.tobytes(), name
    finally:
        for ctx in ctxs:
            ctx.close()
    q, t, dist = orc.match_nndr(pair.desc1, pair.desc2, orc.U8, 0.55, oracle_threads())
    assert np.array_equal(ref["f32"][0]["queryIdx"], q) and np.array_equal(ref["f32"][0]["distance"], dist)
    qf, tf, df = orc.match_nndr(f1, g2, orc.F32, 0.55, oracle_threads())
    assert np.array_equal(ref["f32_frac"][0]["queryIdx"], qf) and np.array_equal(ref["f32_frac"][0]["trainIdx"], tf)
    assert np.array_equal(ref["f32_frac"][0]["distance"], df)
    assert len(ref["u8"][1]) > 1000


def test_pipeline_no_images_full_path_fails_cleanly(fm3d, synth):
    """a context staged without images runs C2's front half; the full path refuses (no pyramids)"""
    pair = synth.make_frame_pair(1500, seed=32)
    s = fm3d.Settings.default()
    s.set_camera(pair.cam)
    ctx = fm3d.Context(s)
    try:
        fm3d.SingleCameraTriangulator(ctx).set_g12(pair.g12)
        pipe = fm3d.Pipeline(ctx)
        pipe.upload(pair.desc1, pair.desc2, pair.kp1, pair.kp2, None, None)
        P, _ = pipe.run_dlt()
        assert P > 0
        with pytest.raises(fm3d.Fm3dError):
            pipe.run()
    finally:
        ctx.close()


def test_lookback_epoch_wrap_and_counter_reset(fm3d, orc, synth, monkeypatch):
    """the fused compactions' look-back.  Each launch takes block indices
    0 .. n-1 from a counter its last block resets (no host-side base), and the 32-bit launch tag
    skips 0 (the zeroed status words' "not yet") when it wraps.  A context started 3 tags before the
    wrap runs C2's front half eight times across it, alternating two pairs: every result equals the
    oracle's."""
    pairs = [synth.make_frame_pair(3000, seed=41), synth.make_frame_pair(9000, seed=42)]
    s = fm3d.Settings.default()
    s.set_camera(pairs[0].cam)
    s.nndrEpsilon = 0.55
    ref = []
    for fp in pairs:
        q, t, _ = orc.match_nndr(fp.desc1, fp.desc2, orc.U8, 0.55, oracle_threads())
        pts, _ = orc.triangulate(fp.cam, fp.g12, s.zThresholdMin, s.zThresholdMax, fp.kp1, fp.kp2, q, t)
        ref.append((q, pts))
    monkeypatch.setenv("FM3D_DEBUG_LB_EPOCH", str(2 ** 32 - 3))
    ctx = fm3d.Context(s)
    monkeypatch.delenv("FM3D_DEBUG_LB_EPOCH")
    try:
        fm3d.SingleCameraTriangulator(ctx).set_g12(pairs[0].g12)
        pipe = fm3d.Pipeline(ctx)
        for i in range(8):  # two look-back launches per step: the tag wraps in the second step
            fp = pairs[i % 2]
            pipe.upload(fp.desc1, fp.desc2, fp.kp1, fp.kp2, None, None)
            P, st = pipe.run_dlt()
            m, pts, _ = pipe.dlt_results(st["matches"], st["inliers"])
            q, opts = ref[i % 2]
            assert np.array_equal(m["queryIdx"], q) and np.array_equal(pts, opts), i
    finally:
        ctx.close()
