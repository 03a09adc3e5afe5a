"""The C ABI library: loads, exports every symbol include/fm3d.h declares, host-only
entry points (settings, g12 algebra) -- no GPU compute here."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SETTINGS_YML = """%YAML:1.0
IMAGES:
   img1: /nonexistent/img_0000007809.pgm
   img2: /nonexistent/img_0000007825.pgm
   pos1: [5.301099, 8.031408, 1.977258, 0.153433, 0.149941, -2.658648]
   pos2: [4.735536, 7.691893, 1.913166, 0.252828, 0.048977, -2.676886]
NNDR:
   epsilon: 0.6
Neighborhoods:
   #Part for normal optimization: take pixels in the image
   epsilonLMMIN: 1e-10
   pixelsRay: 32
   pyramids: 2
   method: square
   cmPerPixel: 0.25
   epsilon: 0.16
FeatureOptions:
   DetectorType: SURF
   SurfDetector:
      HessianThreshold: 400
      Extended: 1
CameraSettings:
   rodriguesIC: [-1.2005, 1.1981, -1.2041]
   translationIC: [0.0, 0.015, -0.051]
   Fx: 572.4765
   Fy: 572.69354
   Cx: 549.75189
   Cy: 411.68039
   p1: -6.6e-05
   p2: 0.000567
   k0: -0.299957
   k1: 0.124129
   k2: -0.028357
   zThresholdMin: 1.5
   zThresholdMax: 2.4
"""


def header_symbols():
    with open(os.path.join(ROOT, "include", "fm3d.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(fm3d_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_header_symbol(fm3d):
    lib = fm3d.lib()
    syms = header_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(syms) == set(fm3d.EXPORTS)


def test_struct_layouts(fm3d):
    assert fm3d.DMATCH.itemsize == 16          # cv::DMatch
    assert fm3d.RECORD.itemsize == 64
    # every fm3d_settings / fm3d_keypoint field at the C compiler's offset (the Python mirror and the header agree)
    import subprocess
    import tempfile
    fields = [f for f, _ in fm3d.Settings._fields_]
    src = "#include <stdio.h>\n#include <stddef.h>\n#include \"fm3d.h\"\nint main(void){printf(\"%zu %zu\\n\", sizeof(fm3d_settings), sizeof(fm3d_keypoint));"
    src += "".join(f'printf("%zu\\n", offsetof(fm3d_settings, {f}));' for f in fields) + "return 0;}"
    with tempfile.TemporaryDirectory() as d:
        c, exe = os.path.join(d, "s.c"), os.path.join(d, "s")
        open(c, "w").write(src)
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()
    assert int(out[0]) == ctypes.sizeof(fm3d.Settings) and int(out[1]) == fm3d.KEYPOINT.itemsize == 28
    assert [int(v) for v in out[2:]] == [getattr(fm3d.Settings, f).offset for f in fields]


def test_settings_default_is_reference_file(fm3d):
    s = fm3d.Settings.default()
    assert (s.Fx, s.Fy, s.Cx, s.Cy) == (572.4765, 572.69354, 549.75189, 411.68039)
    assert (s.pixelsRay, s.pyramids, s.nndrEpsilon, s.epsilonLMMIN) == (64, 3, 0.55, 1e-10)
    assert (s.boundWidth, s.boundHeight) == (1024, 768)


def test_settings_yaml_subset(fm3d, tmp_path):
    p = tmp_path / "settings.yml"
    p.write_text(SETTINGS_YML)
    s = fm3d.Settings.load(str(p))
    assert s.pixelsRay == 32 and s.pyramids == 2 and s.nndrEpsilon == 0.6
    assert list(s.pos2) == [4.735536, 7.691893, 1.913166, 0.252828, 0.048977, -2.676886]
    assert list(s.translationIC) == [0.0, 0.015, -0.051]
    assert s.k0 == -0.299957 and s.zThresholdMax == 2.4
    assert (s.neighMethod, s.neighThetas, s.neighRays) == (0, 15, 5)
    with pytest.raises(fm3d.Fm3dError):
        fm3d.Settings.load(str(tmp_path / "missing.yml"))


def test_settings_neighborhood_method(fm3d, tmp_path):
    """Neighborhoods.method / thetas / rays (neighborhoodsgenerator.cpp:38-73): circular reads its two
    counts; any other method is the reference's exit(-10), here a ValueError of the generator."""
    p = tmp_path / "settings.yml"
    p.write_text(SETTINGS_YML.replace("method: square", "method: circular\n   thetas: 12\n   rays: 4"))
    s = fm3d.Settings.load(str(p))
    assert (s.neighMethod, s.neighThetas, s.neighRays) == (1, 12, 4)
    fm3d.NeighborhoodsGenerator(s)
    p.write_text(SETTINGS_YML.replace("method: square", "method: hexagonal"))
    s = fm3d.Settings.load(str(p))
    assert s.neighMethod == -1
    with pytest.raises(ValueError):
        fm3d.NeighborhoodsGenerator(s)


def test_g12_host_algebra_bitwise_vs_oracle(fm3d, orc):
    s = fm3d.Settings.default()
    g = fm3d.g12_from_poses(s, s.pos1[:3], s.pos2[:3], s.pos1[3:], s.pos2[3:])
    go = orc.setg12(list(s.rodriguesIC), list(s.translationIC), s.pos1[:3], s.pos2[:3], s.pos1[3:], s.pos2[3:])
    assert np.array_equal(g, go)
    R2, t2 = fm3d.camera2_from_g12(g)
    R2o, t2o = orc.camera2_from_g12(go)
    assert np.array_equal(R2, R2o) and np.array_equal(t2, t2o)
    # R2 = Rodrigues(Rodrigues^-1(R12)) stays within ulps of the rotation block of g12
    assert np.abs(R2 - g[:3, :3]).max() < 1e-14


def test_compute_without_gpu_fails_loudly(fm3d):
    """No CPU fallback: without a HIP device the context cannot be created."""
    import subprocess
    import sys
    code = ("import importlib,sys; sys.path.insert(0, %r); f = importlib.import_module('3dfeaturematcher_amd');\n"
            "try:\n    f.Context()\nexcept f.Fm3dError as e:\n    print('ERR', e.code)\nelse:\n    print('OK')") % ROOT
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120).stdout
    has_gpu = os.path.exists("/dev/kfd") and os.environ.get("HIP_VISIBLE_DEVICES", "x") != ""
    if not has_gpu:
        assert "ERR" in out


def test_new_entry_points_reject_bad_arguments(fm3d):
    """The batch MSER and the NCC submit / wait entry points validate their arguments on the host
    (FM3D_ERR_INVALID for a null context or sizes) before any device work -- no GPU needed"""
    import ctypes
    L = ctypes.CDLL(fm3d.LIB_PATH)
    invalid = fm3d.ERR_INVALID
    img = (ctypes.c_uint8 * 16)()
    cnt = (ctypes.c_int32 * 2)()
    tot = ctypes.c_int(0)
    kp = (ctypes.c_uint8 * 64)()
    r = L.fm3d_mser_detect_batch(None, img, 2, 4, 2, 5, 60, 14400, ctypes.c_double(0.25), ctypes.c_double(0.2),
                                 kp, 0, cnt, ctypes.byref(tot))
    assert r == invalid
    n = ctypes.c_int(0)
    assert L.fm3d_pipeline_submit_ncc(None, 4, 4, ctypes.c_double(0.4)) == invalid
    assert L.fm3d_pipeline_wait_ncc(None, ctypes.byref(n), None) == invalid


def test_gravity_and_patch_size_host(fm3d, orc):
    s = fm3d.Settings.default()
    g = np.zeros(3)
    assert fm3d.lib().fm3d_gravity(ctypes.byref(s), g.ctypes.data_as(ctypes.POINTER(ctypes.c_double))) == 0
    assert np.array_equal(g, orc.gravity(list(s.rodriguesIC)))  # same operations, bit for bit
    assert fm3d.lib().fm3d_patch_size(ctypes.byref(s)) == 128
    assert fm3d.NeighborhoodsGenerator(s).getReferenceSquaredNeighborhood().shape == (128 * 128, 3)


def test_settings_feature_options(fm3d, tmp_path):
    """FeatureOptions (descriptorsmatcher.cpp:176-359): SIFT's five constructor values, FAST's
    threshold / suppression, the ADAPTIVE mode and its bounds; OpenCV's defaults where the file names
    none; detector types with no GPU implementation map to FEAT_OTHER."""
    def load(text):
        p = tmp_path / "s.yml"
        p.write_text("%YAML:1.0\n" + text)
        return fm3d.Settings.load(str(p))

    s = load("FeatureOptions:\n   DetectorMode: STATIC\n   DetectorType: SIFT\n   ExtractorType: SIFT\n"
             "   SiftDetector:\n      NumFeatures: 300\n      NumOctaveLayers: 4\n      ContrastThreshold: 0.03\n"
             "      EdgeThreshold: 12\n      Sigma: 1.5\n")
    assert (s.detectorType, s.extractorType, s.detectorMode) == (fm3d.FEAT_SIFT, fm3d.FEAT_SIFT, 0)
    assert (s.siftNumFeatures, s.siftOctaveLayers) == (300, 4)
    assert (s.siftContrastThreshold, s.siftEdgeThreshold, s.siftSigma) == (0.03, 12.0, 1.5)
    s = load("FeatureOptions:\n   DetectorType: SIFT\n   ExtractorType: ORB\n")
    assert (s.siftNumFeatures, s.siftOctaveLayers, s.siftContrastThreshold, s.siftEdgeThreshold, s.siftSigma) == \
        (0, 3, 0.04, 10.0, 1.6)
    assert s.extractorType == fm3d.FEAT_ORB
    s = load("FeatureOptions:\n   DetectorMode: STATIC\n   DetectorType: FAST\n   ExtractorType: SIFT\n"
             "   FastDetector:\n      Threshold: 33\n      NonMaxSuppression: 0\n")
    assert (s.detectorType, s.fastThreshold, s.fastNonmax) == (fm3d.FEAT_FAST, 33, 0)
    s = load("FeatureOptions:\n   DetectorMode: ADAPTIVE\n   DetectorType: SURF\n   ExtractorType: SURF\n"
             "   Adaptive:\n      MinFeatures: 100\n      MaxFeatures: 200\n      MaxIters: 7\n")
    assert (s.detectorType, s.detectorMode) == (fm3d.FEAT_SURF, 1)
    assert (s.adaptiveMinFeatures, s.adaptiveMaxFeatures, s.adaptiveMaxIters) == (100, 200, 7)
    s = load("FeatureOptions:\n   DetectorMode: STATIC\n   DetectorType: STAR\n   ExtractorType: SIFT\n"
             "   StarDetector:\n      MaxSize: 32\n      Response: 25\n      LineThreshold: 9\n"
             "      LineBinarized: 7\n      Suppression: 4\n")
    assert (s.detectorType, s.starMaxSize, s.starResponse, s.starLineThreshold, s.starLineBinarized,
            s.starSuppression) == (fm3d.FEAT_STAR, 32, 25, 9, 7, 4)
    s = load("FeatureOptions:\n   DetectorMode: ADAPTIVE\n   DetectorType: STAR\n")
    assert (s.detectorType, s.detectorMode) == (fm3d.FEAT_STAR, 1)
    assert (s.starMaxSize, s.starResponse, s.starLineThreshold, s.starLineBinarized, s.starSuppression) == \
        (45, 30, 10, 8, 5)
    s = load("FeatureOptions:\n   DetectorType: SURF\n   DetectorMode: STATIC\n   BriskDetector:\n"
             "      Threshold: 25\n      Octaves: 0\n   ExtractorType: BRISK\n")  # build/settings.yml:46-48
    assert (s.extractorType, s.briskThreshold, s.briskOctaves) == (fm3d.FEAT_BRISK, 25, 0)
    assert (fm3d.Settings.default().briskThreshold, fm3d.Settings.default().briskOctaves) == (30, 3)
    assert load("FeatureOptions:\n   DetectorType: BRISK\n").detectorType == fm3d.FEAT_OTHER  # no BRISK detector
    assert load("FeatureOptions:\n   ExtractorType: FREAK\n").extractorType == fm3d.FEAT_FREAK
    assert load("FeatureOptions:\n   DetectorMode: STATIC\n   DetectorType: MSER\n").detectorType == fm3d.FEAT_MSER
    s = load("FeatureOptions:\n   DetectorType: MSER\n   MSERDetector:\n      Delta: 3\n      MinArea: 30\n"
             "      MaxArea: 5000\n      MaxVariation: 0.4\n      MinDiversity: 0.1\n      MaxEvolution: 100\n"
             "      AreaThreshold: 1.2\n      MinMargin: 0.01\n      EdgeBlurSize: 3\n")
    assert (s.mserDelta, s.mserMinArea, s.mserMaxArea, s.mserMaxVariation, s.mserMinDiversity, s.mserMaxEvolution,
            s.mserAreaThreshold, s.mserMinMargin, s.mserEdgeBlurSize) == (3, 30, 5000, 0.4, 0.1, 100, 1.2, 0.01, 3)
    d = fm3d.Settings.default()  # cv::MSER's defaults
    assert (d.mserDelta, d.mserMinArea, d.mserMaxArea, d.mserMaxVariation, d.mserMinDiversity, d.mserMaxEvolution,
            d.mserAreaThreshold, d.mserMinMargin, d.mserEdgeBlurSize) == (5, 60, 14400, 0.25, 0.2, 200, 1.01, 0.003, 5)
    for mode, det in (("ADAPTIVE", "ORB"), ("ADAPTIVE", "MSER"), ("STATIC", "GFTT"), ("OTHER", "SURF")):
        s = load(f"FeatureOptions:\n   DetectorMode: {mode}\n   DetectorType: {det}\n")
        assert s.detectorType == fm3d.FEAT_OTHER, (mode, det)
    d = fm3d.Settings.default()
    assert (d.fastThreshold, d.fastNonmax, d.adaptiveMinFeatures, d.adaptiveMaxFeatures, d.adaptiveMaxIters) == \
        (10, 1, 400, 500, 5)
