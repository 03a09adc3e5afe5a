"""The C++ compat shim (include/fm3d_compat.hpp) and the drop-in consumer
examples/fm3d_main.cpp that mirrors main.cpp:91-155: settings.yml + PGM images +
keypoint/descriptor side files in, matches / points / normals out."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, oracle_threads

EXE = os.path.join(ROOT, "examples", "fm3d_main")


def test_compat_header_compiles():
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "examples", "fm3d_main.cpp")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_example_binary_built_and_usage():
    assert os.path.exists(EXE), "run __graft_entry__.build() (make -C examples)"
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "usage" in r.stderr


def write_pgm(path, img):
    h, w = img.shape
    with open(path, "wb") as f:
        f.write(b"P5\n# fm3d test\n%d %d\n255\n" % (w, h))
        f.write(np.ascontiguousarray(img, dtype=np.uint8).tobytes())


def settings_yml(cam, pos1, pos2, ray, levels, eps):
    k0, k1, p1, p2, k2 = cam.k
    f = lambda v: repr(float(v))
    return f"""%YAML:1.0
IMAGES:
   img1: img1.pgm
   img2: img2.pgm
   pos1: [{', '.join(f(v) for v in pos1)}]
   pos2: [{', '.join(f(v) for v in pos2)}]
NNDR:
   epsilon: {f(eps)}
Neighborhoods:
   epsilonLMMIN: 1e-10
   pixelsRay: {ray}
   pyramids: {levels}
CameraSettings:
   rodriguesIC: [-1.2005, 1.1981, -1.2041]
   translationIC: [0.0, 0.015, -0.051]
   Fx: {f(cam.fx)}
   Fy: {f(cam.fy)}
   Cx: {f(cam.cx)}
   Cy: {f(cam.cy)}
   p1: {f(p1)}
   p2: {f(p2)}
   k0: {f(k0)}
   k1: {f(k1)}
   k2: {f(k2)}
   zThresholdMin: 1.5
   zThresholdMax: 2.4
"""


@pytest.mark.gpu
def test_example_main_matches_python_api(fm3d, synth, orc, tmp_path):
    pair = synth.make_frame_pair(1500, seed=21)
    d = tmp_path
    write_pgm(d / "img1.pgm", pair.img1)
    write_pgm(d / "img2.pgm", pair.img2)
    pair.kp1.astype(np.float32).tofile(d / "kp1.f32")
    pair.kp2.astype(np.float32).tofile(d / "kp2.f32")
    pair.desc1.tofile(d / "desc1.u8")
    pair.desc2.tofile(d / "desc2.u8")
    (d / "settings.yml").write_text(settings_yml(pair.cam, synth.REF_POS1, synth.REF_POS2, 10, 2, 0.55))
    r = subprocess.run([EXE, "-s", str(d / "settings.yml"), "-d", str(d)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    matches = np.fromfile(d / "out_matches.bin", dtype=fm3d.DMATCH)
    pts = np.fromfile(d / "out_points.f64").reshape(-1, 3)
    nrm = np.fromfile(d / "out_normals.f64").reshape(-1, 3)
    # the same calls through the Python mirror of the reference classes
    s = fm3d.Settings.load(str(d / "settings.yml"))
    ctx = fm3d.Context(s)
    try:
        m = fm3d.DescriptorsMatcher(ctx).compareWithNNDR(s.nndrEpsilon, pair.desc1, pair.desc2)
        sct = fm3d.SingleCameraTriangulator(ctx)
        sct.setg12(s.pos1[:3], s.pos2[:3], s.pos1[3:], s.pos2[3:])
        sct.setKeypoints(pair.kp1, pair.kp2, m)
        P, _ = sct.triangulate()
        no = fm3d.NormalOptimizer(ctx, sct)
        no.setImages(pair.img1, pair.img2)
        kept, normals = no.computeOptimizedNormals(P)
    finally:
        ctx.close()
    assert matches.tobytes() == m.tobytes()
    q, t, _ = orc.match_nndr(pair.desc1, pair.desc2, orc.U8, s.nndrEpsilon, oracle_threads())
    assert np.array_equal(matches["queryIdx"], q) and np.array_equal(matches["trainIdx"], t)
    assert len(kept) > 10
    assert np.array_equal(pts, kept) and np.array_equal(nrm, normals)
    # main.cpp:157-180: patch_<i>.pgm of the normal-rectified patches (P5 128 128, like results/)
    s2 = fm3d.Settings.load(str(d / "settings.yml"))
    ctx = fm3d.Context(s2)
    try:
        no = fm3d.NormalOptimizer(ctx)
        no.setImages(pair.img1, pair.img2)
        frames = no.computeFeaturesFrames(kept, normals)
        patches = fm3d.SingleCameraTriangulator(ctx).projectReferencePointsToImageWithFrames(None, frames)
    finally:
        ctx.close()
    for i in range(min(16, len(kept))):
        raw = (d / f"patch_{i}.pgm").read_bytes()
        assert raw.startswith(b"P5\n128 128\n255\n")
        assert raw[len(b"P5\n128 128\n255\n"):] == patches[i].tobytes()


DROPIN = os.path.join(ROOT, "examples", "main_dropin")


def test_dropin_main_compiles_against_cv_standins():
    """examples/main_dropin.cpp (main.cpp's call sequence with only the includes replaced by
    include/fm3d_cv.hpp) compiles warning-free."""
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-I",
                        os.path.join(ROOT, "include"), os.path.join(ROOT, "examples", "main_dropin.cpp")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([DROPIN], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "Usage" in r.stdout


REF_MAIN = "/root/reference/main.cpp"


@pytest.mark.skipif(not os.access(REF_MAIN, os.R_OK), reason="the reference tree is not on this machine")
def test_reference_main_compiles_with_includes_swapped(tmp_path):
    """north_star's "main.cpp drops in unchanged": the reference's own main.cpp, copied at test time
    (no reference text is stored in this repository) with only its include block (main.cpp:8-20:
    lmmin.h, the OpenCV headers, the four class headers, pclvisualizerthread.h, tools.h) replaced by
    include/fm3d_cv.hpp, compiles with -Wall and links against libfm3d.so; run without arguments it
    prints the reference's usage line and exits -1 (main.cpp:45-49)."""
    lines = open(REF_MAIN).read().split("\n")
    assert lines[7].startswith("#include <lmmin.h>") and lines[19].startswith('#include "tools.h"')
    src = tmp_path / "main.cpp"
    src.write_text("\n".join(lines[:7] + ['#include "fm3d_cv.hpp"'] + lines[20:]))
    exe = tmp_path / "main_ref"
    libdir = os.path.join(ROOT, "3dfeaturematcher_amd")
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe),
                        "-L" + libdir, "-lfm3d", "-Wl,-rpath," + libdir, "-L/opt/rocm/lib", "-Wl,-rpath-link,/opt/rocm/lib"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert "warning" not in r.stderr, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 255 and "Usage: 3dfeaturematcher -s <settings.yml>" in r.stdout


def test_reference_rng_colours():
    """drawMatches' colours (tools.cpp:116-120, 159-167): cv::RNG(0xFFF0FF0F) + CV_RGB.  The first
    15 are the colours of the 15 frames painted in the reference's build/projectedPatches.pgm (RGB
    order in the file); tests/golden/ref_pins.npz holds them as read from that file."""
    src = r'''
#include "fm3d_cv.hpp"
#include <cstdio>
int main() { cv::RNG rng(0xFFF0FF0F); for (int i = 0; i < 23; i++) { cv::Scalar c = cv::random_color(rng);
  std::printf("%d %d %d\n", (int)c[2], (int)c[1], (int)c[0]); } return 0; }
'''
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        open(os.path.join(d, "c.cpp"), "w").write(src)
        r = subprocess.run(["g++", "-std=c++17", "-I", os.path.join(ROOT, "include"), os.path.join(d, "c.cpp"), "-o",
                            os.path.join(d, "c")], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
        out = subprocess.run([os.path.join(d, "c")], capture_output=True, text=True).stdout.split("\n")
    rgb = [tuple(int(v) for v in line.split()) for line in out if line]
    assert rgb[0] == (150, 195, 189) and rgb[14] == (62, 232, 43) and rgb[22] == (172, 160, 148)


def test_settings_lookup_filestorage_nodes(fm3d, tmp_path):
    """fm3d_settings_lookup (cv::FileNode of the stand-ins) on the reference's settings layout."""
    import ctypes
    p = tmp_path / "s.yml"
    p.write_text("%YAML:1.0\nIMAGES:\n#TIME : 1 POS : 1 2 3\n\n   img1: /data/img_7809.pgm\n"
                 "   pos1: [5.301099, 8.031408, 1.977258, 0.153433, 0.149941, -2.658648]\n"
                 "NNDR:\n   epsilon: 0.55\nFeatureOptions:\n   SurfDetector:\n      Extended: 1\n"
                 "   ExtractorType: SURF\n")
    lib = fm3d.lib()

    def look(key):
        n = ctypes.c_int(0)
        buf = ctypes.create_string_buffer(256)
        rc = lib.fm3d_settings_lookup(str(p).encode(), key.encode(), buf, 256, ctypes.byref(n))
        return rc, buf.value.decode(), n.value

    assert look("IMAGES.img1") == (0, "/data/img_7809.pgm", len("/data/img_7809.pgm"))
    assert look("NNDR.epsilon")[1] == "0.55"
    assert look("IMAGES.pos1")[1].startswith("[5.301099,")
    assert look("FeatureOptions.SurfDetector.Extended")[1] == "1"
    assert look("FeatureOptions.ExtractorType")[1] == "SURF"
    assert look("FeatureOptions.Missing")[0] == fm3d.ERR_INVALID
    n = ctypes.c_int(0)
    assert lib.fm3d_settings_lookup(str(tmp_path / "nope.yml").encode(), b"A", None, 0, ctypes.byref(n)) == fm3d.ERR_PARSE


@pytest.mark.gpu
def test_dropin_main_matches_python_api(fm3d, synth, orc, tmp_path):
    """main_dropin -s settings.yml (the reference command line): matches, triangulated points and
    normals equal the Python mirror's on the same inputs; patch_<i>.pgm of every kept point equal
    the patch export; the square neighbourhood of frame 0 equals the oracle's."""
    pair = synth.make_frame_pair(1500, seed=23)
    d = tmp_path
    write_pgm(d / "img1.pgm", pair.img1)
    write_pgm(d / "img2.pgm", pair.img2)
    # the upstream detector's output, as the images' feature side files
    pair.kp1.astype(np.float32).tofile(d / "img1.pgm.kpts.f32")
    pair.kp2.astype(np.float32).tofile(d / "img2.pgm.kpts.f32")
    pair.desc1.tofile(d / "img1.pgm.desc.u8")
    pair.desc2.tofile(d / "img2.pgm.desc.u8")
    yml = settings_yml(pair.cam, synth.REF_POS1, synth.REF_POS2, 10, 2, 0.55)
    yml = yml.replace("img1: img1.pgm", f"img1: {d / 'img1.pgm'}").replace("img2: img2.pgm", f"img2: {d / 'img2.pgm'}")
    # a detector type the reference does not build (GFTT): the side files are read
    yml += "FeatureOptions:\n   DetectorType: GFTT\n   ExtractorType: SIFT\n"
    (d / "settings.yml").write_text(yml)
    r = subprocess.run([DROPIN, "-s", str(d / "settings.yml")], capture_output=True, text=True, timeout=120, cwd=d)
    assert r.returncode == 0, r.stderr + r.stdout
    matches = np.fromfile(d / "out_matches.bin", dtype=fm3d.DMATCH)
    pts = np.fromfile(d / "out_points.f64").reshape(-1, 3)
    nrm = np.fromfile(d / "out_normals.f64").reshape(-1, 3)
    s = fm3d.Settings.load(str(d / "settings.yml"))
    ctx = fm3d.Context(s)
    try:
        m = fm3d.DescriptorsMatcher(ctx).compareWithNNDR(s.nndrEpsilon, pair.desc1, pair.desc2)
        sct = fm3d.SingleCameraTriangulator(ctx)
        sct.setg12(s.pos1[:3], s.pos2[:3], s.pos1[3:], s.pos2[3:])
        sct.setKeypoints(pair.kp1, pair.kp2, m)
        P, _ = sct.triangulate()
        no = fm3d.NormalOptimizer(ctx, sct)
        no.setImages(pair.img1, pair.img2)
        kept, normals = no.computeOptimizedNormals(P)
        frames = no.computeFeaturesFrames(kept, normals)
        patches = sct.projectReferencePointsToImageWithFrames(None, frames)
    finally:
        ctx.close()
    assert matches.tobytes() == m.tobytes()
    q, t, _ = orc.match_nndr(pair.desc1, pair.desc2, orc.U8, s.nndrEpsilon, oracle_threads())
    assert np.array_equal(matches["queryIdx"], q) and np.array_equal(matches["trainIdx"], t)
    assert len(kept) > 10
    assert np.array_equal(pts, kept) and np.array_equal(nrm, normals)
    for i in range(len(kept)):
        raw = (d / f"patch_{i}.pgm").read_bytes()
        assert raw == b"P5\n128 128\n255\n" + patches[i].tobytes()
    nb0 = np.fromfile(d / "out_neighborhoods.f64").reshape(-1, 3)
    assert np.array_equal(nb0, orc.square_neighborhoods(frames[:1])[0])
    for f in ("matches.pgm", "projectedPatches.pgm"):
        assert (d / f).read_bytes().startswith(b"P6\n")


SURF_OPTIONS = """FeatureOptions:
   DetectorType: SURF
   DetectorMode: STATIC
   SurfDetector:
      HessianThreshold: 400
      NumOctaves: 4
      NumOctaveLayers: 2
      Extended: 1
      Upright: 1
   ExtractorType: SURF
"""


def _python_chain(fm3d, s, img1, img2):
    """main.cpp:91-183 through the Python mirror: SURF compareWithNNDR from the images, triangulation,
    normals, frames, patches, patch descriptors."""
    ctx = fm3d.Context(s)
    try:
        m, ka, kb, _, _ = fm3d.DescriptorsMatcher(ctx).compareWithNNDRImages(s.nndrEpsilon, img1, img2)
        sct = fm3d.SingleCameraTriangulator(ctx)
        sct.setg12(s.pos1[:3], s.pos2[:3], s.pos1[3:], s.pos2[3:])
        xy = lambda k: np.stack([k["x"], k["y"]], axis=1).astype(np.float32)
        sct.setKeypoints(xy(ka), xy(kb), m)
        P, _ = sct.triangulate()
        no = fm3d.NormalOptimizer(ctx, sct)
        no.setImages(img1, img2)
        kept, normals = no.computeOptimizedNormals(P)
        frames = no.computeFeaturesFrames(kept, normals)
        patches = sct.projectReferencePointsToImageWithFrames(None, frames)
        feats = fm3d.Features(ctx)
        cols, dt = feats.descriptor_info()
        desc = feats.extractDescriptorsFromPatches(patches) if len(patches) else np.zeros((0, cols), dt)
    finally:
        ctx.close()
    return m, kept, normals, patches, desc


@pytest.mark.gpu
def test_dropin_main_surf_detection(fm3d, synth, orc, tmp_path):
    """main_dropin -s settings.yml with the reference's FeatureOptions (STATIC SURF, upright,
    extended): features detected and described on the GPU from the images alone, and the patch
    descriptors of main.cpp:182-183 -- all equal to the Python mirror; the patch descriptors equal
    the SURF oracle's."""
    pair = synth.make_frame_pair(1500, seed=24)
    d = tmp_path
    write_pgm(d / "img1.pgm", pair.img1)
    write_pgm(d / "img2.pgm", pair.img2)
    yml = settings_yml(pair.cam, synth.REF_POS1, synth.REF_POS2, 10, 2, 0.6)
    yml = yml.replace("img1: img1.pgm", f"img1: {d / 'img1.pgm'}").replace("img2: img2.pgm", f"img2: {d / 'img2.pgm'}")
    (d / "settings.yml").write_text(yml + SURF_OPTIONS)
    r = subprocess.run([DROPIN, "-s", str(d / "settings.yml")], capture_output=True, text=True, timeout=120, cwd=d)
    assert r.returncode == 0, r.stderr + r.stdout
    s = fm3d.Settings.load(str(d / "settings.yml"))
    assert s.detectorType == 0 and s.extractorType == 0 and s.surfExtended == 1 and s.surfUpright == 1
    m, kept, normals, patches, desc = _python_chain(fm3d, s, pair.img1, pair.img2)
    assert np.fromfile(d / "out_matches.bin", dtype=fm3d.DMATCH).tobytes() == m.tobytes()
    assert np.array_equal(np.fromfile(d / "out_points.f64").reshape(-1, 3), kept)
    assert np.array_equal(np.fromfile(d / "out_normals.f64").reshape(-1, 3), normals)
    assert len(m) > 50 and len(kept) > 5
    pd = np.fromfile(d / "out_patch_desc.f32", dtype=np.float32).reshape(-1, 128)
    assert np.array_equal(pd, desc)
    kp = np.zeros(1, dtype=fm3d.KEYPOINT)
    kp["x"] = kp["y"] = 64
    kp["size"] = 128
    kp["angle"] = -1
    ref = np.stack([orc.surf_describe(p, kp)[2][0] for p in patches[:8]])
    assert np.array_equal(pd[:8], ref)


SIFT_OPTIONS = """FeatureOptions:
   DetectorType: SIFT
   DetectorMode: STATIC
   SiftDetector:
      NumFeatures: 0
      NumOctaveLayers: 3
      ContrastThreshold: 0.04
      EdgeThreshold: 10
      Sigma: 1.6
   ExtractorType: SIFT
"""


@pytest.mark.gpu
def test_dropin_main_sift_detection(fm3d, synth, orc, tmp_path):
    """main_dropin -s settings.yml with FeatureOptions SIFT: SIFT detection + description of both
    images on the GPU (the reference's detect, then compute), and the patch descriptors of
    main.cpp:182-183 by the SIFT extractor -- equal to the Python mirror; the patch descriptors equal
    the SIFT oracle's (SIFT::operator() on each patch with its centred keypoint)."""
    pair = synth.make_frame_pair(1500, seed=26)
    d = tmp_path
    write_pgm(d / "img1.pgm", pair.img1)
    write_pgm(d / "img2.pgm", pair.img2)
    yml = settings_yml(pair.cam, synth.REF_POS1, synth.REF_POS2, 10, 2, 0.6)
    yml = yml.replace("img1: img1.pgm", f"img1: {d / 'img1.pgm'}").replace("img2: img2.pgm", f"img2: {d / 'img2.pgm'}")
    (d / "settings.yml").write_text(yml + SIFT_OPTIONS)
    r = subprocess.run([DROPIN, "-s", str(d / "settings.yml")], capture_output=True, text=True, timeout=120, cwd=d)
    assert r.returncode == 0, r.stderr + r.stdout
    s = fm3d.Settings.load(str(d / "settings.yml"))
    assert s.detectorType == fm3d.FEAT_SIFT and s.extractorType == fm3d.FEAT_SIFT and s.siftOctaveLayers == 3
    m, kept, normals, patches, desc = _python_chain(fm3d, s, pair.img1, pair.img2)
    assert np.fromfile(d / "out_matches.bin", dtype=fm3d.DMATCH).tobytes() == m.tobytes()
    assert np.array_equal(np.fromfile(d / "out_points.f64").reshape(-1, 3), kept)
    assert np.array_equal(np.fromfile(d / "out_normals.f64").reshape(-1, 3), normals)
    assert len(m) > 50 and len(kept) > 5
    pd = np.fromfile(d / "out_patch_desc.f32", dtype=np.float32).reshape(-1, 128)
    assert np.array_equal(pd, desc)
    kp = np.zeros(1, dtype=fm3d.KEYPOINT)
    kp["x"] = kp["y"] = 64
    kp["size"] = 128
    kp["angle"] = -1
    kp["response"] = 1
    ref = np.stack([orc.sift_compute(p, kp)[2][0] for p in patches[:8]])
    assert np.array_equal(pd[:8], ref)


STAR_OPTIONS = """FeatureOptions:
   DetectorType: STAR
   DetectorMode: STATIC
   StarDetector:
      MaxSize: 45
      Response: 20
      LineThreshold: 10
      LineBinarized: 8
      Suppression: 5
   ExtractorType: SIFT
"""


@pytest.mark.gpu
def test_dropin_main_star_detection(fm3d, synth, orc, tmp_path):
    """main_dropin -s settings.yml with DetectorType STAR and ExtractorType SIFT (a pair the reference
    builds from two FeatureOptions entries): STAR detection and SIFT description of both images on the
    GPU through fm3d_detect / fm3d_compute; matches, points and normals equal the Python mirror's, the
    keypoints of image 1 equal the oracle chain's."""
    pair = synth.make_frame_pair(1500, seed=27)
    d = tmp_path
    write_pgm(d / "img1.pgm", pair.img1)
    write_pgm(d / "img2.pgm", pair.img2)
    yml = settings_yml(pair.cam, synth.REF_POS1, synth.REF_POS2, 10, 2, 0.6)
    yml = yml.replace("img1: img1.pgm", f"img1: {d / 'img1.pgm'}").replace("img2: img2.pgm", f"img2: {d / 'img2.pgm'}")
    (d / "settings.yml").write_text(yml + STAR_OPTIONS)
    r = subprocess.run([DROPIN, "-s", str(d / "settings.yml")], capture_output=True, text=True, timeout=120, cwd=d)
    assert r.returncode == 0, r.stderr + r.stdout
    s = fm3d.Settings.load(str(d / "settings.yml"))
    assert (s.detectorType, s.extractorType, s.starResponse) == (fm3d.FEAT_STAR, fm3d.FEAT_SIFT, 20)
    m, kept, normals, patches, desc = _python_chain(fm3d, s, pair.img1, pair.img2)
    assert np.fromfile(d / "out_matches.bin", dtype=fm3d.DMATCH).tobytes() == m.tobytes()
    assert np.array_equal(np.fromfile(d / "out_points.f64").reshape(-1, 3), kept)
    assert np.array_equal(np.fromfile(d / "out_normals.f64").reshape(-1, 3), normals)
    assert len(m) > 20 and len(kept) > 3
    pd = np.fromfile(d / "out_patch_desc.f32", dtype=np.float32).reshape(-1, 128)
    assert np.array_equal(pd, desc)
    ko, _, dk = orc.sift_compute(pair.img1, orc.star_detect(pair.img1, 45, 20, 10, 8, 5))
    q, t, _ = orc.match_nndr(dk.astype(np.uint8), orc.sift_compute(
        pair.img2, orc.star_detect(pair.img2, 45, 20, 10, 8, 5))[2].astype(np.uint8), orc.U8, s.nndrEpsilon)
    assert np.array_equal(m["queryIdx"], q) and np.array_equal(m["trainIdx"], t)


@pytest.mark.gpu
@pytest.mark.parametrize("det,ex", [("ORB", "ORB"), ("FAST", "BRISK")])
def test_dropin_main_binary_extractors(fm3d, synth, orc, tmp_path, det, ex):
    """main_dropin -s settings.yml with a binary extractor (ORB; BRISK, whose BriskDetector block the
    reference's settings.yml carries): Hamming matching, the pipeline and the patch descriptors of
    main.cpp:182-183 equal the Python mirror's; ORB's patch rows equal the ORB oracle on each patch,
    BRISK's are zero (its pattern reaches past every centred patch keypoint, so OpenCV's rows stay
    Mat::zeros)."""
    pair = synth.make_frame_pair(1500, seed=28)
    d = tmp_path
    write_pgm(d / "img1.pgm", pair.img1)
    write_pgm(d / "img2.pgm", pair.img2)
    yml = settings_yml(pair.cam, synth.REF_POS1, synth.REF_POS2, 10, 2, 0.8)
    yml = yml.replace("img1: img1.pgm", f"img1: {d / 'img1.pgm'}").replace("img2: img2.pgm", f"img2: {d / 'img2.pgm'}")
    yml += (f"FeatureOptions:\n   DetectorType: {det}\n   DetectorMode: STATIC\n   BriskDetector:\n"
            f"      Threshold: 25\n      Octaves: 0\n   ExtractorType: {ex}\n")
    (d / "settings.yml").write_text(yml)
    r = subprocess.run([DROPIN, "-s", str(d / "settings.yml")], capture_output=True, text=True, timeout=120, cwd=d)
    assert r.returncode == 0, r.stderr + r.stdout
    s = fm3d.Settings.load(str(d / "settings.yml"))
    m, kept, normals, patches, desc = _python_chain(fm3d, s, pair.img1, pair.img2)
    assert np.fromfile(d / "out_matches.bin", dtype=fm3d.DMATCH).tobytes() == m.tobytes()
    assert np.array_equal(np.fromfile(d / "out_points.f64").reshape(-1, 3), kept)
    assert np.array_equal(np.fromfile(d / "out_normals.f64").reshape(-1, 3), normals)
    assert len(m) > 10 and len(kept) > 3
    cols = 32 if ex == "ORB" else 64
    pd = np.fromfile(d / "out_patch_desc.u8", dtype=np.uint8).reshape(-1, cols)
    assert pd.shape == (len(patches), cols) and np.array_equal(pd, desc)
    if ex == "BRISK":
        assert not pd.any()
    else:
        kp = np.zeros(1, dtype=fm3d.KEYPOINT)
        kp["x"] = kp["y"] = 64
        kp["size"] = 128
        kp["angle"] = -1
        kp["response"] = 1
        ref = np.stack([orc.orb_compute(p, kp)[2][0] for p in patches[:6]])
        assert np.array_equal(pd[:6], ref)


@pytest.mark.gpu
def test_dropin_main_orb_pattern_from_env(fm3d, synth, orc, tmp_path):
    """the drop-in takes OpenCV's tables from FM3D_ORB_PATTERN / FM3D_FREAK_PAIRS; without
    them ORB at patchSize 31 warns once that it runs on makeRandomPattern(31).  With a table given the
    patch descriptors are the ORB oracle's on that table, and nothing is printed."""
    pair = synth.make_frame_pair(1500, seed=28)
    d = tmp_path
    write_pgm(d / "img1.pgm", pair.img1)
    write_pgm(d / "img2.pgm", pair.img2)
    yml = settings_yml(pair.cam, synth.REF_POS1, synth.REF_POS2, 10, 2, 0.8)
    yml = yml.replace("img1: img1.pgm", f"img1: {d / 'img1.pgm'}").replace("img2: img2.pgm", f"img2: {d / 'img2.pgm'}")
    yml += "FeatureOptions:\n   DetectorType: ORB\n   DetectorMode: STATIC\n   ExtractorType: ORB\n"
    (d / "settings.yml").write_text(yml)
    env = {k: v for k, v in os.environ.items() if k not in ("FM3D_ORB_PATTERN", "FM3D_FREAK_PAIRS")}
    r = subprocess.run([DROPIN, "-s", str(d / "settings.yml")], capture_output=True, text=True, timeout=120, cwd=d,
                       env=env)
    assert r.returncode == 0, r.stderr + r.stdout
    assert r.stderr.count("makeRandomPattern(31)") == 1
    # another valid 512-point table: the default one with its tests reversed
    pat = np.ascontiguousarray(orc.orb_random_pattern(31).reshape(256, 2, 2)[::-1].reshape(512, 2), dtype=np.int32)
    pat.tofile(d / "pattern.i32")
    r = subprocess.run([DROPIN, "-s", str(d / "settings.yml")], capture_output=True, text=True, timeout=120, cwd=d,
                       env=dict(env, FM3D_ORB_PATTERN=str(d / "pattern.i32")))
    assert r.returncode == 0, r.stderr + r.stdout
    assert "makeRandomPattern" not in r.stderr and "ignored" not in r.stderr
    pd = np.fromfile(d / "out_patch_desc.u8", dtype=np.uint8).reshape(-1, 32)
    kp = np.zeros(1, dtype=fm3d.KEYPOINT)
    kp["x"] = kp["y"] = 64
    kp["size"] = 128
    kp["angle"] = -1
    kp["response"] = 1
    s = fm3d.Settings.load(str(d / "settings.yml"))
    _, _, _, patches, _ = _python_chain(fm3d, s, pair.img1, pair.img2)
    assert len(pd) == len(patches) > 3
    ref = np.stack([orc.orb_compute(p, kp, pattern=pat)[2][0] for p in patches[:6]])
    assert np.array_equal(pd[:6], ref)
    assert not np.array_equal(ref, np.stack([orc.orb_compute(p, kp)[2][0] for p in patches[:6]]))


@pytest.mark.gpu
def test_mosaic_python_and_cpp(fm3d, synth, tmp_path):
    """MOSAIC (mosaic.h:47-70, mosaic.cpp:32-73): the Python class and the C++ one (mosaic_demo,
    include/fm3d_cv.hpp) run the same pipeline; their patch descriptors and points equal the
    step-by-step chain."""
    pair = synth.make_frame_pair(1500, seed=25)
    d = tmp_path
    write_pgm(d / "img1.pgm", pair.img1)
    write_pgm(d / "img2.pgm", pair.img2)
    yml = settings_yml(pair.cam, synth.REF_POS1, synth.REF_POS2, 10, 2, 0.6)
    yml = yml.replace("img1: img1.pgm", f"img1: {d / 'img1.pgm'}").replace("img2: img2.pgm", f"img2: {d / 'img2.pgm'}")
    (d / "settings.yml").write_text(yml + SURF_OPTIONS)
    s = fm3d.Settings.load(str(d / "settings.yml"))
    m, kept, normals, patches, desc = _python_chain(fm3d, s, pair.img1, pair.img2)
    ctx = fm3d.Context(s)
    try:
        mo = fm3d.MOSAIC(ctx, pair.img1, pair.img2, s.pos1[:3], s.pos2[:3], s.pos1[3:], s.pos2[3:])
        md = mo.compute()
    finally:
        ctx.close()
    assert mo.matches.tobytes() == m.tobytes()
    assert np.array_equal(mo.triangulated_points, kept) and np.array_equal(mo.normals, normals)
    assert np.array_equal(mo.patches, patches) and np.array_equal(md, desc) and md.shape[1] == 128
    exe = os.path.join(ROOT, "examples", "mosaic_demo")
    r = subprocess.run([exe, "-s", str(d / "settings.yml")], capture_output=True, text=True, timeout=120, cwd=d)
    assert r.returncode == 0, r.stderr + r.stdout
    assert np.array_equal(np.fromfile(d / "mosaic_desc.f32", dtype=np.float32).reshape(-1, 128), desc)
    assert np.array_equal(np.fromfile(d / "mosaic_points.f64").reshape(-1, 3), kept)
