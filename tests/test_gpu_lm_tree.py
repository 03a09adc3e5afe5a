"""The LM kernel's tree-reduction mode (fm3d_settings.lmReduction = 1, lm2_kernel<.., TREE>;
DESIGN.md §3.4b) bit for bit against the oracle's ORC_LM_TREE | ORC_LM_GRAM mode: statuses, lmdif
info and evaluation counts per level, normals.  The mode is opt-in: it does not replay the
reference's pixel-order sums (tools/full_parity.py measures how far its normals move), but it is
exactly as reproducible as the default mode."""
import numpy as np
import pytest

from conftest import oracle_threads

pytestmark = pytest.mark.gpu


def _settings(fm3d, cam, **kw):
    s = fm3d.Settings.default()
    s.set_camera(cam)
    for k, v in kw.items():
        setattr(s, k, v)
    return s


@pytest.fixture(scope="module")
def pair(synth):
    return synth.make_frame_pair(3000, seed=11)


@pytest.fixture(scope="module")
def points(orc, pair):
    q, t, _ = orc.match_nndr(pair.desc1, pair.desc2, orc.U8, 0.55, oracle_threads())
    pts, _ = orc.triangulate(pair.cam, pair.g12, 1.5, 2.4, pair.kp1, pair.kp2, q, t)
    extra = np.array([[-1.3, -0.95, 2.0], [5.0, 5.0, 2.0], [0.0, 0.0, 2.0]])
    return np.concatenate([pts[:150], extra])


def _run(fm3d, orc, pair, P, ray, levels=3, bound=(1024, 768)):
    s = _settings(fm3d, pair.cam, pixelsRay=ray, boundWidth=bound[0], boundHeight=bound[1], pyramids=levels,
                  lmReduction=1)
    ctx = fm3d.Context(s)
    try:
        sct = fm3d.SingleCameraTriangulator(ctx)
        sct.set_g12(pair.g12)
        R2, t2 = sct.camera2()
        no = fm3d.NormalOptimizer(ctx, sct)
        no.setImages(pair.img1, pair.img2)
        kept, normals = no.computeOptimizedNormals(P)
        st, info, nfev = no.last_status, no.last_info, no.last_nfev
    finally:
        ctx.close()
    orc.tree_stats(reset=True)
    ref = orc.optimize_normals(pair.cam, R2, t2, pair.img1, pair.img2, levels, P, ray, bound[0], bound[1],
                               mode=orc.DETMATH | orc.TREE | orc.GRAM, nthreads=oracle_threads())
    return kept, normals, st, info, nfev, ref, orc.tree_stats()


def _check(kept, normals, st, info, nfev, ref, P, L=4):
    assert np.array_equal(st, ref["status"])
    assert np.array_equal(info[:, :L], ref["info"][:, :L])
    assert np.array_equal(nfev[:, :L], ref["nfev"][:, :L])
    ok = ref["status"] == 0
    assert np.array_equal(normals, ref["normals"][ok])
    assert np.array_equal(kept, P[ok])
    return ok


@pytest.mark.parametrize("ray,safe", [(8, 0), (16, 0), (16, 1)])
def test_tree_normals_bitwise_vs_tree_oracle(fm3d, orc, pair, points, ray, safe, monkeypatch):
    monkeypatch.setenv("FM3D_LM_SAFE", str(safe))
    kept, normals, st, info, nfev, ref, stats = _run(fm3d, orc, pair, points, ray)
    ok = _check(kept, normals, st, info, nfev, ref, points)
    assert ok.sum() > 10
    assert stats[0] > 100  # the Gram form ran
    print("tree paths (gram, householder, sequential enorm):", stats)


def test_tree_normals_reference_config_ray64(fm3d, orc, pair, points):
    kept, normals, st, info, nfev, ref, _ = _run(fm3d, orc, pair, points[:40], 64)
    assert _check(kept, normals, st, info, nfev, ref, points[:40]).sum() > 5


def test_tree_normals_vga_bounds_pyramids(fm3d, orc, pair, points):
    for levels in (0, 1):
        kept, normals, st, info, nfev, ref, _ = _run(fm3d, orc, pair, points[:60], 12, levels=levels,
                                                     bound=(640, 480))
        _check(kept, normals, st, info, nfev, ref, points[:60], L=levels + 1)


def test_tree_mode_moves_normals_not_statuses(fm3d, orc, pair, points):
    """The tree mode is not the reference's summation order: against the default (pixel-order)
    mode the statuses agree on these points and most normals agree to well below 1e-4, but they
    are not the same bits."""
    P = points[:100]
    kept, normals, st, *_ = _run(fm3d, orc, pair, P, 16)
    seq = orc.optimize_normals(pair.cam, *fm3d.camera2_from_g12(pair.g12), pair.img1, pair.img2, 3, P, 16,
                               mode=orc.DETMATH, nthreads=oracle_threads())
    assert np.array_equal(st, seq["status"])
    d = np.abs(normals - seq["normals"][seq["status"] == 0]).max(axis=1)
    assert np.median(d) < 1e-9 and (d > 0).any()


def test_tree_pipeline_linked_equals_run(fm3d, synth):
    """lmReduction = 1 through the pipeline, two linked frame pairs in one launch: each pair's
    records equal its own run; linking a tree context to a pixel-order one fails loudly."""
    pairs = [synth.make_frame_pair(3000, seed=11), synth.make_frame_pair(2500, seed=12)]
    s = _settings(fm3d, pairs[0].cam, pixelsRay=12, pyramids=2, lmReduction=1)

    def mk(settings):
        c = fm3d.Context(settings)
        fm3d.SingleCameraTriangulator(c).set_g12(pairs[0].g12)
        return c, fm3d.Pipeline(c)

    ref = []
    c, p = mk(s)
    try:
        for fp in pairs:
            p.upload(fp.desc1, fp.desc2, fp.kp1, fp.kp2, fp.img1, fp.img2)
            k, _ = p.run()
            ref.append(p.records(k))
    finally:
        c.close()
    (cm, m), (cl, l) = mk(s), mk(s)
    try:
        m.link(l)
        a, b = pairs
        m.submit(a.desc1, a.desc2, a.kp1, a.kp2, a.img1, a.img2)
        l.submit(b.desc1, b.desc2, b.kp1, b.kp2, b.img1, b.img2)
        assert m.wait()[0].tobytes() == ref[0].tobytes()
        assert l.wait()[0].tobytes() == ref[1].tobytes()
    finally:
        cm.close()
        cl.close()
    s0 = _settings(fm3d, pairs[0].cam, pixelsRay=12, pyramids=2, lmReduction=0)
    (cm, m), (cl, l) = mk(s0), mk(s)
    try:
        m.link(l)
        a, b = pairs
        m.submit(a.desc1, a.desc2, a.kp1, a.kp2, a.img1, a.img2)
        with pytest.raises(fm3d.Fm3dError):
            l.submit(b.desc1, b.desc2, b.kp1, b.kp2, b.img1, b.img2)
        m.wait()  # the member's LM alone
    finally:
        cm.close()
        cl.close()
