"""3dfeaturematcher_amd -- MI355X-native hot path of caomw/3DFeatureMatcher.

Python mirror of the reference's operator interface for the path
(``DescriptorsMatcher`` / ``SingleCameraTriangulator`` / ``NormalOptimizer``,
``main.cpp:91-155``), bound with ctypes to the C ABI of ``libfm3d.so``
(``include/fm3d.h``).  All compute runs in the HIP kernels of the library; there
is no CPU fallback -- constructing a context without the library or without a
GPU raises ``Fm3dError``.

The package directory name starts with a digit, so import it with
``importlib.import_module("3dfeaturematcher_amd")``.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# FM3D_LIB selects another in-tree build of the same library (A/B performance experiments)
LIB_PATH = os.environ.get("FM3D_LIB") or os.path.join(_HERE, "libfm3d.so")

FM3D_OK = 0
ERR_INVALID, ERR_HIP, ERR_UNSUPPORTED, ERR_NOMEM, ERR_PARSE, ERR_NAN_PLANE = -1, -2, -3, -4, -5, -6
FEAT_SURF, FEAT_ORB, FEAT_SIFT, FEAT_FAST, FEAT_STAR, FEAT_BRISK, FEAT_FREAK, FEAT_MSER, FEAT_OTHER = 0, 1, 2, 3, 4, 5, 6, 7, -1  # fm3d_settings.detectorType / extractorType
DESC_F32, DESC_U8, DESC_BITS = 0, 1, 2
ST_OK, ST_NO_PIXELS, ST_ABORT_BBOX, ST_ABORT_PIX1, ST_ABORT_PIX2, ST_NAN_PLANE, ST_NAN_NORMAL = range(7)

# every symbol include/fm3d.h declares (tests check the library exports all of them)
EXPORTS = (
    "fm3d_settings_default", "fm3d_settings_load", "fm3d_settings_lookup", "fm3d_ctx_create", "fm3d_ctx_destroy", "fm3d_last_error",
    "fm3d_ctx_set_stream", "fm3d_knn2", "fm3d_match_nndr", "fm3d_setg12", "fm3d_g12_from_poses",
    "fm3d_camera2_from_g12", "fm3d_set_g12", "fm3d_get_camera2", "fm3d_triangulate", "fm3d_set_images",
    "fm3d_get_pyramid_level", "fm3d_optimize_normals", "fm3d_pipeline_upload", "fm3d_pipeline_run",
    "fm3d_records_download", "fm3d_pyrdown", "fm3d_neighborhood", "fm3d_undistort", "fm3d_version",
    "fm3d_gravity", "fm3d_features_frames", "fm3d_patch_size", "fm3d_export_patches", "fm3d_square_neighborhoods",
    "fm3d_circular_neighborhoods", "fm3d_surf_detect", "fm3d_surf_compute", "fm3d_extract_descriptors_from_patches", "fm3d_extract_descriptors_from_patches_any", "fm3d_pipeline_run_dlt", "fm3d_pipeline_dlt_download", "fm3d_pipeline_run_ncc",
    "fm3d_pipeline_ncc_download",
    "fm3d_orb_detect", "fm3d_orb_compute", "fm3d_orb_set_pattern", "fm3d_sift_detect", "fm3d_sift_compute",
    "fm3d_sift_pyramid", "fm3d_fast_detect", "fm3d_star_detect", "fm3d_brisk_compute", "fm3d_star_responses", "fm3d_detect", "fm3d_descriptor_info", "fm3d_compute",
    "fm3d_ncc_hypotheses", "fm3d_mgpu_create", "fm3d_mgpu_destroy", "fm3d_mgpu_last_error", "fm3d_mgpu_set_g12",
    "fm3d_mgpu_pipeline_upload", "fm3d_mgpu_pipeline_run", "fm3d_share_queries", "fm3d_merge_shares",
    "fm3d_plane_to_image2", "fm3d_pipeline_submit", "fm3d_pipeline_wait",
    "fm3d_mgpu_submit", "fm3d_mgpu_wait", "fm3d_pipeline_link", "fm3d_freak_compute", "fm3d_freak_set_pairs",
    "fm3d_mser_detect", "fm3d_mser_detect_batch", "fm3d_mser_regions", "fm3d_pipeline_submit_dlt", "fm3d_pipeline_submit_dlt_pair",
    "fm3d_pipeline_submit_ncc", "fm3d_pipeline_wait_ncc", "fm3d_pipeline_wait_dlt", "fm3d_device_count",
)


class Fm3dError(RuntimeError):
    def __init__(self, code, msg=""):
        super().__init__(f"fm3d error {code}: {msg}")
        self.code = code


class Settings(ctypes.Structure):
    """fm3d_settings (the build/settings.yml keys of the path)."""
    _fields_ = [
        ("Fx", ctypes.c_double), ("Fy", ctypes.c_double), ("Cx", ctypes.c_double), ("Cy", ctypes.c_double),
        ("p1", ctypes.c_double), ("p2", ctypes.c_double), ("k0", ctypes.c_double), ("k1", ctypes.c_double),
        ("k2", ctypes.c_double), ("rodriguesIC", ctypes.c_double * 3), ("translationIC", ctypes.c_double * 3),
        ("zThresholdMin", ctypes.c_double), ("zThresholdMax", ctypes.c_double), ("epsilonLMMIN", ctypes.c_double),
        ("pixelsRay", ctypes.c_int), ("pyramids", ctypes.c_int), ("nndrEpsilon", ctypes.c_double),
        ("pos1", ctypes.c_double * 6), ("pos2", ctypes.c_double * 6), ("boundWidth", ctypes.c_int),
        ("boundHeight", ctypes.c_int), ("strictNanExit", ctypes.c_int), ("lmWaves", ctypes.c_int),
        ("neighEpsilon", ctypes.c_double), ("cmPerPixel", ctypes.c_double),
        ("neighMethod", ctypes.c_int), ("neighThetas", ctypes.c_int), ("neighRays", ctypes.c_int),
        ("detectorType", ctypes.c_int), ("extractorType", ctypes.c_int), ("surfHessianThreshold", ctypes.c_double),
        ("surfOctaves", ctypes.c_int), ("surfOctaveLayers", ctypes.c_int), ("surfExtended", ctypes.c_int),
        ("surfUpright", ctypes.c_int),
        ("orbNumFeatures", ctypes.c_int), ("orbScaleFactor", ctypes.c_double), ("orbNumLevels", ctypes.c_int),
        ("orbEdgeThreshold", ctypes.c_int), ("orbPatchSize", ctypes.c_int), ("orbFastThreshold", ctypes.c_int),
        ("siftNumFeatures", ctypes.c_int), ("siftOctaveLayers", ctypes.c_int),
        ("siftContrastThreshold", ctypes.c_double), ("siftEdgeThreshold", ctypes.c_double),
        ("siftSigma", ctypes.c_double),
        ("detectorMode", ctypes.c_int), ("fastThreshold", ctypes.c_int), ("fastNonmax", ctypes.c_int),
        ("adaptiveMinFeatures", ctypes.c_int), ("adaptiveMaxFeatures", ctypes.c_int), ("adaptiveMaxIters", ctypes.c_int),
        ("starMaxSize", ctypes.c_int), ("starResponse", ctypes.c_int), ("starLineThreshold", ctypes.c_int),
        ("starLineBinarized", ctypes.c_int), ("starSuppression", ctypes.c_int),
        ("briskThreshold", ctypes.c_int), ("briskOctaves", ctypes.c_int),
        ("mserDelta", ctypes.c_int), ("mserMinArea", ctypes.c_int), ("mserMaxArea", ctypes.c_int),
        ("mserMaxVariation", ctypes.c_double), ("mserMinDiversity", ctypes.c_double),
        ("mserMaxEvolution", ctypes.c_int), ("mserAreaThreshold", ctypes.c_double),
        ("mserMinMargin", ctypes.c_double), ("mserEdgeBlurSize", ctypes.c_int),
        ("lmReduction", ctypes.c_int),
        ("dltSolver", ctypes.c_int),
    ]

    @staticmethod
    def default() -> "Settings":
        s = Settings()
        _check(lib().fm3d_settings_default(ctypes.byref(s)))
        return s

    @staticmethod
    def load(path: str) -> "Settings":
        s = Settings()
        _check(lib().fm3d_settings_load(path.encode(), ctypes.byref(s)))
        return s

    def camera(self):
        """(fx, fy, cx, cy, (k1, k2, p1, p2, k3)) in OpenCV order."""
        return self.Fx, self.Fy, self.Cx, self.Cy, (self.k0, self.k1, self.p1, self.p2, self.k2)

    def set_camera(self, cam) -> None:
        self.Fx, self.Fy, self.Cx, self.Cy = cam.fx, cam.fy, cam.cx, cam.cy
        self.k0, self.k1, self.p1, self.p2, self.k2 = cam.k


DMATCH = np.dtype([("queryIdx", "<i4"), ("trainIdx", "<i4"), ("imgIdx", "<i4"), ("distance", "<f4")])
KEYPOINT = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                     ("octave", "<i4"), ("class_id", "<i4")])  # cv::KeyPoint (fm3d_keypoint)
RECORD = np.dtype([("queryIdx", "<i4"), ("trainIdx", "<i4"), ("distance", "<f4"), ("status", "<i4"),
                   ("point", "<f8", (3,)), ("normal", "<f8", (3,))])


class LMStats(ctypes.Structure):
    _fields_ = [("points_in", ctypes.c_int64), ("points_kept", ctypes.c_int64), ("evaluations", ctypes.c_int64),
                ("pixel_evaluations", ctypes.c_int64), ("drops", ctypes.c_int64 * 8), ("kernel_ms", ctypes.c_double),
                ("groups", ctypes.c_int64), ("passes", ctypes.c_int64), ("cycles_terms", ctypes.c_int64),
                ("cycles_chain", ctypes.c_int64), ("cycles_control", ctypes.c_int64), ("cycles_total", ctypes.c_int64),
                ("wall_ticks_sum", ctypes.c_int64), ("wall_ticks_max", ctypes.c_int64),
                ("wall_clock_khz", ctypes.c_int64), ("class_passes", ctypes.c_int64 * 4),
                ("class_cycles", ctypes.c_int64 * 4), ("last_group_start_ticks", ctypes.c_int64),
                ("last_group_end_ticks", ctypes.c_int64), ("cycles_wait", ctypes.c_int64),
                ("chain_rounds", ctypes.c_int64), ("chain_chunks", ctypes.c_int64),
                ("queue_empty_ticks", ctypes.c_int64)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_}
        for k in ("drops", "class_passes", "class_cycles"):
            d[k] = list(d[k])
        return d


class PipelineStats(ctypes.Structure):
    _fields_ = [("queries", ctypes.c_int64), ("trains", ctypes.c_int64), ("matches", ctypes.c_int64),
                ("inliers", ctypes.c_int64), ("kept", ctypes.c_int64), ("match_ms", ctypes.c_double),
                ("nndr_ms", ctypes.c_double), ("triangulate_ms", ctypes.c_double), ("pyramid_ms", ctypes.c_double),
                ("lm_ms", ctypes.c_double), ("total_ms", ctypes.c_double), ("lm", LMStats)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_ if k != "lm"}
        d["lm"] = self.lm.as_dict()
        return d


_LIB = None


def lib():
    """Load libfm3d.so (built by __graft_entry__.build()); raises if absent."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise Fm3dError(ERR_HIP, f"{LIB_PATH} missing: build it with __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        L.fm3d_last_error.restype = ctypes.c_char_p
        L.fm3d_version.restype = ctypes.c_char_p
        L.fm3d_mgpu_last_error.restype = ctypes.c_char_p
        _LIB = L
    return _LIB


def _check(code, ctx=None):
    if code != FM3D_OK:
        msg = ""
        if ctx is not None:
            msg = (lib().fm3d_last_error(ctx) or b"").decode(errors="replace")
        raise Fm3dError(code, msg)


def _ptr(a, t=ctypes.c_double):
    return a.ctypes.data_as(ctypes.POINTER(t))


def _vp(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


class Context:
    """One fm3d_ctx: device buffers + a HIP stream on one GPU."""

    def __init__(self, settings: Settings | None = None, device: int = 0):
        self.settings = settings if settings is not None else Settings.default()
        self._h = ctypes.c_void_p()
        rc = lib().fm3d_ctx_create(ctypes.byref(self.settings), ctypes.c_int(device), ctypes.byref(self._h))
        if rc != FM3D_OK:
            raise Fm3dError(rc, "fm3d_ctx_create failed (no HIP device / runtime?)")

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            lib().fm3d_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, code):
        _check(code, self._h)

    def set_stream(self, hip_stream: int | None):
        self.check(lib().fm3d_ctx_set_stream(self._h, ctypes.c_void_p(hip_stream or 0)))


def _desc_type(desc: np.ndarray, binary: bool) -> int:
    if binary:
        return DESC_BITS
    if desc.dtype == np.uint8:
        return DESC_U8
    if desc.dtype == np.float32:
        return DESC_F32
    raise TypeError("descriptors must be uint8 (SIFT-like), float32 or binary uint8 (binary=True)")


class DescriptorsMatcher:
    """DescriptorsMatcher (DescriptorsMatcher/descriptorsmatcher.h:39-111), matcher + NNDR part.

    Feature detection/description (descriptorsmatcher.cpp:110-115) is upstream of
    the hot path: this class takes the descriptor matrices directly.
    """

    def __init__(self, ctx: Context, binary: bool = False):
        self.ctx = ctx
        self.binary = binary

    def knn_match(self, desc_a: np.ndarray, desc_b: np.ndarray) -> np.ndarray:
        """knnMatch(A, B, k=2) (descriptorsmatcher.cpp:89-105) -> (nA, 2) DMATCH array."""
        a = np.ascontiguousarray(desc_a)
        b = np.ascontiguousarray(desc_b)
        out = np.zeros((a.shape[0], 2), dtype=DMATCH)
        self.ctx.check(lib().fm3d_knn2(self.ctx.handle, _vp(a), a.shape[0], _vp(b), b.shape[0], a.shape[1],
                                       _desc_type(a, self.binary), _vp(out)))
        return out

    def compareWithNNDRImages(self, epsilon: float, image_a: np.ndarray, image_b: np.ndarray,
                              matches: np.ndarray | None = None):
        """compareWithNNDR (descriptorsmatcher.cpp:107-131) with the detection it starts with: the
        settings' detector + extractor on both images on the GPU (SURF; SIFT; or ORB: detect, then
        compute on the detected keypoints as the reference's two calls, Hamming matching as its binary
        extractor types select, :64), knnMatch, NNDR.  Returns (matches appended as the reference
        does, kpts_a, kpts_b, desc_a, desc_b)."""
        S = self.ctx.settings
        if S.detectorMode == 1 or S.detectorType in (FEAT_SIFT, FEAT_FAST, FEAT_STAR) or S.extractorType != S.detectorType:
            # the reference's two calls with any detector / extractor pair built here (fm3d_detect,
            # fm3d_compute): detect, then compute on the detected keypoints
            feats = Features(self.ctx)
            ka, _, da = feats.compute(image_a, feats.detect(image_a))
            kb, _, db = feats.compute(image_b, feats.detect(image_b))
            binary = S.extractorType in (FEAT_ORB, FEAT_BRISK, FEAT_FREAK)
            m = DescriptorsMatcher(self.ctx, binary=binary).compareWithNNDR(epsilon, da, db, matches)
            return m, ka, kb, da, db
        if S.detectorType == FEAT_ORB and S.extractorType == FEAT_ORB:
            orb = ORB(self.ctx)
            ka, _, da = orb.compute(image_a, orb.detect(image_a))
            kb, _, db = orb.compute(image_b, orb.detect(image_b))
            m = DescriptorsMatcher(self.ctx, binary=True).compareWithNNDR(epsilon, da, db, matches)
            return m, ka, kb, da, db
        surf = SURF(self.ctx)
        ka, da = surf.detect(image_a, with_descriptors=True)
        kb, db = surf.detect(image_b, with_descriptors=True)
        m = self.compareWithNNDR(epsilon, da, db, matches)
        return m, ka, kb, da, db

    def compareWithNNDR(self, epsilon: float, desc_a: np.ndarray, desc_b: np.ndarray,
                        matches: np.ndarray | None = None) -> np.ndarray:
        """compareWithNNDR (descriptorsmatcher.cpp:107-131).  Like the reference, new
        matches are APPENDED to `matches` (the reference pushes back without clearing)."""
        a = np.ascontiguousarray(desc_a)
        b = np.ascontiguousarray(desc_b)
        out = np.zeros(max(a.shape[0], 1), dtype=DMATCH)
        n = ctypes.c_int(0)
        self.ctx.check(lib().fm3d_match_nndr(self.ctx.handle, _vp(a), a.shape[0], _vp(b), b.shape[0], a.shape[1],
                                             _desc_type(a, self.binary), ctypes.c_double(epsilon), _vp(out),
                                             ctypes.byref(n)))
        new = out[:n.value].copy()
        return new if matches is None else np.concatenate([matches, new])


class SURF:
    """The settings' SURF detector / extractor (DescriptorsMatcher::generateDetector /
    generateExtractor, descriptorsmatcher.cpp:176-359; OpenCV 2.4 nonfree SURF, upright) on the GPU."""

    def __init__(self, ctx: Context):
        self.ctx = ctx

    @property
    def descriptorSize(self) -> int:
        return 128 if self.ctx.settings.surfExtended else 64

    def detect(self, image: np.ndarray, with_descriptors: bool = False):
        """FeatureDetector::detect (descriptorsmatcher.cpp:110-111): KEYPOINT records in
        KeypointGreater order; with_descriptors: (keypoints, descriptors) of the same call."""
        img = np.ascontiguousarray(image, dtype=np.uint8)
        h, w = img.shape
        # one detection with room for one keypoint per 64 pixels; again only if more were found
        cap = max(4096, w * h // 64)
        while True:
            k = np.zeros(cap, dtype=KEYPOINT)
            d = np.zeros((cap, self.descriptorSize), dtype=np.float32) if with_descriptors else None
            n = ctypes.c_int(0)
            self.ctx.check(lib().fm3d_surf_detect(self.ctx.handle, _ptr(img, ctypes.c_uint8), w, h, _vp(k), cap,
                                                  ctypes.byref(n), _ptr(d, ctypes.c_float) if d is not None else None))
            if n.value <= cap:
                break
            cap = n.value
        k = k[:n.value]
        return (k, d[:n.value]) if with_descriptors else k

    def compute(self, image: np.ndarray, keypoints: np.ndarray):
        """DescriptorExtractor::compute (descriptorsmatcher.cpp:113-114): (kept keypoints, input index
        of each, descriptors float32 n x 128|64)."""
        img = np.ascontiguousarray(image, dtype=np.uint8)
        h, w = img.shape
        kin = np.ascontiguousarray(keypoints, dtype=KEYPOINT)
        n = len(kin)
        kout = np.zeros(max(n, 1), dtype=KEYPOINT)
        kept = np.zeros(max(n, 1), dtype=np.int32)
        desc = np.zeros((max(n, 1), self.descriptorSize), dtype=np.float32)
        m = ctypes.c_int(0)
        self.ctx.check(lib().fm3d_surf_compute(self.ctx.handle, _ptr(img, ctypes.c_uint8), w, h, _vp(kin), n,
                                               _vp(kout), _ptr(kept, ctypes.c_int32), ctypes.byref(m),
                                               _ptr(desc, ctypes.c_float)))
        return kout[:m.value], kept[:m.value], desc[:m.value]

    def extractDescriptorsFromPatches(self, patches: np.ndarray) -> np.ndarray:
        """DescriptorsMatcher::extractDescriptorsFromPatches (descriptorsmatcher.cpp:133-174): one
        keypoint per square patch at (floor(size/2), floor(size/2)), size = the patch edge, angle -1,
        then the extractor: (P, 128|64) float32."""
        P = np.ascontiguousarray(patches, dtype=np.uint8)
        if P.ndim != 3 or P.shape[1] != P.shape[2]:
            raise ValueError("patches: (P, size, size) uint8")
        out = np.zeros((max(P.shape[0], 1), self.descriptorSize), dtype=np.float32)
        self.ctx.check(lib().fm3d_extract_descriptors_from_patches(self.ctx.handle, _ptr(P, ctypes.c_uint8),
                                                                   P.shape[0], P.shape[1], _ptr(out, ctypes.c_float)))
        return out[:P.shape[0]]


class ORB:
    """The settings' ORB detector / extractor (FeatureOptions DetectorType / ExtractorType ORB,
    descriptorsmatcher.cpp:273-279, 336-341: cv::ORB(NumFeatures, ScaleFactor, NumLevels) of OpenCV
    2.4) on the GPU.  Descriptors are 32 bytes (Hamming)."""

    descriptorSize = 32

    def __init__(self, ctx: Context):
        self.ctx = ctx

    def set_pattern(self, xy) -> None:
        """the 512 rBRIEF test points (OpenCV's bit_pattern_31_ for patchSize 31); None: the default
        makeRandomPattern(orbPatchSize)"""
        if xy is None:
            self.ctx.check(lib().fm3d_orb_set_pattern(self.ctx.handle, None, 0))
            return
        p = np.ascontiguousarray(xy, dtype=np.int32).reshape(-1)
        if p.size != 1024:
            raise ValueError("pattern: 512 (x, y) points")
        self.ctx.check(lib().fm3d_orb_set_pattern(self.ctx.handle, _ptr(p, ctypes.c_int32), 512))

    def detect(self, image: np.ndarray, with_descriptors: bool = False):
        """FeatureDetector::detect (descriptorsmatcher.cpp:110-111): KEYPOINT records, level-major;
        with_descriptors: (keypoints, (n, 32) uint8) of ORB::operator()'s one call"""
        img = np.ascontiguousarray(image, dtype=np.uint8)
        h, w = img.shape
        cap = max(1024, self.ctx.settings.orbNumFeatures * 2)
        while True:
            k = np.zeros(cap, dtype=KEYPOINT)
            d = np.zeros((cap, 32), dtype=np.uint8) if with_descriptors else None
            n = ctypes.c_int(0)
            self.ctx.check(lib().fm3d_orb_detect(self.ctx.handle, _ptr(img, ctypes.c_uint8), w, h, _vp(k), cap,
                                                 ctypes.byref(n), _ptr(d, ctypes.c_uint8) if d is not None else None))
            if n.value <= cap:
                break
            cap = n.value
        k = k[:n.value]
        return (k, d[:n.value]) if with_descriptors else k

    def compute(self, image: np.ndarray, keypoints: np.ndarray):
        """DescriptorExtractor::compute (descriptorsmatcher.cpp:113-114): (kept keypoints level-major,
        input index of each, (m, 32) uint8)"""
        img = np.ascontiguousarray(image, dtype=np.uint8)
        h, w = img.shape
        kin = np.ascontiguousarray(keypoints, dtype=KEYPOINT)
        n = len(kin)
        kout = np.zeros(max(n, 1), dtype=KEYPOINT)
        kept = np.zeros(max(n, 1), dtype=np.int32)
        desc = np.zeros((max(n, 1), 32), dtype=np.uint8)
        m = ctypes.c_int(0)
        self.ctx.check(lib().fm3d_orb_compute(self.ctx.handle, _ptr(img, ctypes.c_uint8), w, h, _vp(kin), n, _vp(kout),
                                              _ptr(kept, ctypes.c_int32), ctypes.byref(m), _ptr(desc, ctypes.c_uint8)))
        return kout[:m.value], kept[:m.value], desc[:m.value]


class SIFT:
    """The settings' SIFT detector / extractor (FeatureOptions DetectorType / ExtractorType SIFT,
    descriptorsmatcher.cpp:243-257, 302-315: cv::SIFT(NumFeatures, NumOctaveLayers, ContrastThreshold,
    EdgeThreshold, Sigma) of OpenCV 2.4 nonfree) on the GPU.  Descriptors are 128 floats holding the
    integers 0..255 (the matcher takes them on its exact integer path)."""

    descriptorSize = 128

    def __init__(self, ctx: Context):
        self.ctx = ctx

    def detect(self, image: np.ndarray, with_descriptors: bool = False):
        """FeatureDetector::detect (descriptorsmatcher.cpp:110-111): KEYPOINT records in the
        reference's order; with_descriptors: (keypoints, (n, 128) float32) -- the extractor's compute
        on the same image"""
        img = np.ascontiguousarray(image, dtype=np.uint8)
        h, w = img.shape
        cap = max(4096, self.ctx.settings.siftNumFeatures * 2)
        while True:
            k = np.zeros(cap, dtype=KEYPOINT)
            d = np.zeros((cap, 128), dtype=np.float32) if with_descriptors else None
            n = ctypes.c_int(0)
            self.ctx.check(lib().fm3d_sift_detect(self.ctx.handle, _ptr(img, ctypes.c_uint8), w, h, _vp(k), cap,
                                                  ctypes.byref(n), _ptr(d, ctypes.c_float) if d is not None else None))
            if n.value <= cap:
                break
            cap = n.value
        k = k[:n.value]
        return (k, d[:n.value]) if with_descriptors else k

    def pyramid(self, image: np.ndarray, first_octave: int = -1, octaves: int | None = None, dog: bool = False):
        """buildGaussianPyramid (dog False) / buildDoGPyramid levels, octave-major: float32 images"""
        img = np.ascontiguousarray(image, dtype=np.uint8)
        h, w = img.shape
        if octaves is None:
            bw, bh = (2 * w, 2 * h) if first_octave < 0 else (w, h)
            octaves = int(np.rint(np.log(min(bw, bh)) / np.log(2.0) - 2)) - first_octave
        nl = octaves * (self.ctx.settings.siftOctaveLayers + (2 if dog else 3))
        sizes = np.zeros(2 * nl, dtype=np.int32)
        tot = ctypes.c_int64(0)
        args = (self.ctx.handle, _ptr(img, ctypes.c_uint8), w, h, first_octave, octaves, 1 if dog else 0)
        self.ctx.check(lib().fm3d_sift_pyramid(*args, None, _ptr(sizes, ctypes.c_int32), ctypes.byref(tot)))
        out = np.zeros(max(tot.value, 1), dtype=np.float32)
        self.ctx.check(lib().fm3d_sift_pyramid(*args, _ptr(out, ctypes.c_float), None, ctypes.byref(tot)))
        levels, o = [], 0
        for i in range(nl):
            lw, lh = int(sizes[2 * i]), int(sizes[2 * i + 1])
            levels.append(out[o:o + lw * lh].reshape(lh, lw))
            o += lw * lh
        return levels

    def compute(self, image: np.ndarray, keypoints: np.ndarray):
        """DescriptorExtractor::compute (descriptorsmatcher.cpp:113-114): (kept keypoints, input index
        of each, (m, 128) float32)"""
        img = np.ascontiguousarray(image, dtype=np.uint8)
        h, w = img.shape
        kin = np.ascontiguousarray(keypoints, dtype=KEYPOINT)
        n = len(kin)
        kout = np.zeros(max(n, 1), dtype=KEYPOINT)
        kept = np.zeros(max(n, 1), dtype=np.int32)
        desc = np.zeros((max(n, 1), 128), dtype=np.float32)
        m = ctypes.c_int(0)
        self.ctx.check(lib().fm3d_sift_compute(self.ctx.handle, _ptr(img, ctypes.c_uint8), w, h, _vp(kin), n,
                                               _vp(kout), _ptr(kept, ctypes.c_int32), ctypes.byref(m),
                                               _ptr(desc, ctypes.c_float)))
        return kout[:m.value], kept[:m.value], desc[:m.value]

    extractDescriptorsFromPatches = SURF.extractDescriptorsFromPatches  # the C ABI picks the settings' extractor


class Features:
    """The settings' detector and extractor, whatever their types (descriptorsmatcher.cpp:176-359):
    STATIC SURF / ORB / SIFT / FAST / STAR or ADAPTIVE FAST / SURF / STAR detection (fm3d_detect), SURF / SIFT / ORB / BRISK /
    FREAK description (fm3d_compute) on any keypoints."""

    def __init__(self, ctx: Context):
        self.ctx = ctx

    def descriptor_info(self):
        """(columns, numpy dtype) of the extractor's rows"""
        cols, typ = ctypes.c_int(0), ctypes.c_int(0)
        self.ctx.check(lib().fm3d_descriptor_info(self.ctx.handle, ctypes.byref(cols), ctypes.byref(typ)))
        return cols.value, (np.uint8 if typ.value == DESC_BITS else np.float32)

    def detect(self, image: np.ndarray) -> np.ndarray:
        """feature_detector_->detect (descriptorsmatcher.cpp:110-111): KEYPOINT records"""
        img = np.ascontiguousarray(image, dtype=np.uint8)
        h, w = img.shape
        cap = 4096
        while True:
            k = np.zeros(cap, dtype=KEYPOINT)
            n = ctypes.c_int(0)
            self.ctx.check(lib().fm3d_detect(self.ctx.handle, _ptr(img, ctypes.c_uint8), w, h, _vp(k), cap,
                                             ctypes.byref(n)))
            if n.value <= cap:
                return k[:n.value]
            cap = n.value

    def compute(self, image: np.ndarray, keypoints: np.ndarray):
        """descriptor_extractor_->compute (descriptorsmatcher.cpp:113-114): (kept keypoints, input index
        of each, descriptor rows)"""
        img = np.ascontiguousarray(image, dtype=np.uint8)
        h, w = img.shape
        cols, dt = self.descriptor_info()
        kin = np.ascontiguousarray(keypoints, dtype=KEYPOINT)
        n = len(kin)
        kout = np.zeros(max(n, 1), dtype=KEYPOINT)
        kept = np.zeros(max(n, 1), dtype=np.int32)
        desc = np.zeros((max(n, 1), cols), dtype=dt)
        m = ctypes.c_int(0)
        self.ctx.check(lib().fm3d_compute(self.ctx.handle, _ptr(img, ctypes.c_uint8), w, h, _vp(kin), n, _vp(kout),
                                          _ptr(kept, ctypes.c_int32), ctypes.byref(m), _vp(desc)))
        return kout[:m.value], kept[:m.value], desc[:m.value]

    def set_freak_pairs(self, pairs=None):
        """fm3d_freak_set_pairs: FREAK's 512 selected pairs (indices into the 903 point pairs); None restores
        the default table (include/fm3d_freak.h)"""
        if pairs is None:
            self.ctx.check(lib().fm3d_freak_set_pairs(self.ctx.handle, None, 0))
        else:
            a = np.ascontiguousarray(pairs, dtype=np.int32)
            self.ctx.check(lib().fm3d_freak_set_pairs(self.ctx.handle, _ptr(a, ctypes.c_int32), len(a)))

    def fast(self, image: np.ndarray, threshold: int = 10, nonmax: bool = True) -> np.ndarray:
        """cv::FastFeatureDetector(threshold, nonmax).detect: KEYPOINT records in raster order"""
        img = np.ascontiguousarray(image, dtype=np.uint8)
        h, w = img.shape
        cap = 4096
        while True:
            k = np.zeros(cap, dtype=KEYPOINT)
            n = ctypes.c_int(0)
            self.ctx.check(lib().fm3d_fast_detect(self.ctx.handle, _ptr(img, ctypes.c_uint8), w, h, threshold,
                                                  1 if nonmax else 0, _vp(k), cap, ctypes.byref(n)))
            if n.value <= cap:
                return k[:n.value]
            cap = n.value


    def extractDescriptorsFromPatches(self, patches: np.ndarray) -> np.ndarray:
        """DescriptorsMatcher::extractDescriptorsFromPatches (descriptorsmatcher.cpp:133-174) with any of
        the settings' extractors: (P, cols) rows of the extractor's type (zero rows where the extractor
        drops the centred keypoint)"""
        P = np.ascontiguousarray(patches, dtype=np.uint8)
        if P.ndim != 3 or P.shape[1] != P.shape[2]:
            raise ValueError("patches must be (P, size, size)")
        cols, dt = self.descriptor_info()
        out = np.zeros((P.shape[0], cols), dtype=dt)
        self.ctx.check(lib().fm3d_extract_descriptors_from_patches_any(self.ctx.handle, _ptr(P, ctypes.c_uint8),
                                                                       P.shape[0], P.shape[1], _vp(out)))
        return out

    def star(self, image: np.ndarray, max_size: int = 45, response: int = 30, line_threshold: int = 10,
             line_binarized: int = 8, suppression: int = 5) -> np.ndarray:
        """cv::StarFeatureDetector(maxSize, response, lineThreshold, lineBinarized, suppression).detect:
        KEYPOINT records in tile order"""
        img = np.ascontiguousarray(image, dtype=np.uint8)
        h, w = img.shape
        cap = 4096
        while True:
            k = np.zeros(cap, dtype=KEYPOINT)
            n = ctypes.c_int(0)
            self.ctx.check(lib().fm3d_star_detect(self.ctx.handle, _ptr(img, ctypes.c_uint8), w, h, max_size, response,
                                                  line_threshold, line_binarized, suppression, _vp(k), cap,
                                                  ctypes.byref(n)))
            if n.value <= cap:
                return k[:n.value]
            cap = n.value


    def star_responses(self, image: np.ndarray, max_size: int = 45):
        """StarDetectorComputeResponses: (border, float32 responses, int16 signed sizes)"""
        img = np.ascontiguousarray(image, dtype=np.uint8)
        h, w = img.shape
        R = np.zeros((h, w), np.float32)
        Z = np.zeros((h, w), np.int16)
        b = ctypes.c_int(0)
        self.ctx.check(lib().fm3d_star_responses(self.ctx.handle, _ptr(img, ctypes.c_uint8), w, h, max_size,
                                                 _ptr(R, ctypes.c_float), _ptr(Z, ctypes.c_int16), ctypes.byref(b)))
        return b.value, R, Z

    def mser(self, image: np.ndarray, delta: int = 5, min_area: int = 60, max_area: int = 14400,
             max_variation: float = 0.25, min_diversity: float = 0.2) -> np.ndarray:
        """cv::MserFeatureDetector(delta, minArea, maxArea, maxVariation, minDiversity, ...).detect:
        KEYPOINT records in region order"""
        img = np.ascontiguousarray(image, dtype=np.uint8)
        h, w = img.shape
        cap = 4096
        while True:
            k = np.zeros(cap, dtype=KEYPOINT)
            n = ctypes.c_int(0)
            self.ctx.check(lib().fm3d_mser_detect(self.ctx.handle, _ptr(img, ctypes.c_uint8), w, h, delta, min_area,
                                                  max_area, ctypes.c_double(max_variation),
                                                  ctypes.c_double(min_diversity), _vp(k), cap, ctypes.byref(n)))
            if n.value <= cap:
                return k[:n.value]
            cap = n.value

    def mser_batch(self, images, delta: int = 5, min_area: int = 60, max_area: int = 14400,
                   max_variation: float = 0.25, min_diversity: float = 0.2):
        """mser() on several images of one size in one call (fm3d_mser_detect_batch: every image's floods
        side by side): a list of KEYPOINT arrays, each equal to mser(image)"""
        imgs = np.ascontiguousarray(np.stack([np.asarray(i, dtype=np.uint8) for i in images]))
        count, h, w = imgs.shape
        cap = 4096 * count
        counts = np.zeros(count, np.int32)
        while True:
            k = np.zeros(cap, dtype=KEYPOINT)
            tot = ctypes.c_int(0)
            self.ctx.check(lib().fm3d_mser_detect_batch(
                self.ctx.handle, _ptr(imgs, ctypes.c_uint8), count, w, h, delta, min_area, max_area,
                ctypes.c_double(max_variation), ctypes.c_double(min_diversity), _vp(k), cap,
                _ptr(counts, ctypes.c_int32), ctypes.byref(tot)))
            if tot.value <= cap:
                break
            cap = tot.value
        out, off = [], 0
        for c in counts:
            out.append(k[off:off + int(c)].copy())
            off += int(c)
        return out

    def mser_regions(self, image: np.ndarray, delta: int = 5, min_area: int = 60, max_area: int = 14400,
                     max_variation: float = 0.25, min_diversity: float = 0.2):
        """MSER::operator()(img, msers): [(colour -1 | +1, (k, 2) int32 points (x, y) in region-list order)]"""
        img = np.ascontiguousarray(image, dtype=np.uint8)
        h, w = img.shape
        cap, pcap = 1024, 1 << 18
        while True:
            color = np.zeros(cap, np.int32)
            count = np.zeros(cap, np.int32)
            pts = np.zeros((pcap, 2), np.int32)
            nr, npt = ctypes.c_int(0), ctypes.c_int64(0)
            self.ctx.check(lib().fm3d_mser_regions(
                self.ctx.handle, _ptr(img, ctypes.c_uint8), w, h, delta, min_area, max_area,
                ctypes.c_double(max_variation), ctypes.c_double(min_diversity), _ptr(color, ctypes.c_int32),
                _ptr(count, ctypes.c_int32), cap, _ptr(pts, ctypes.c_int32), ctypes.c_int64(pcap), ctypes.byref(nr),
                ctypes.byref(npt)))
            if nr.value <= cap and npt.value <= pcap:
                break
            cap, pcap = max(cap, nr.value), max(pcap, npt.value)
        out, off = [], 0
        for i in range(nr.value):
            out.append((int(color[i]), pts[off:off + count[i]].copy()))
            off += int(count[i])
        return out


class SingleCameraTriangulator:
    """SingleCameraTriangulator (Triangulator/singlecameratriangulator.h:52-93), hot-path methods."""

    def __init__(self, ctx: Context):
        self.ctx = ctx
        self._kp1 = self._kp2 = self._matches = None

    def setg12(self, T1, T2, r1, r2) -> np.ndarray:
        g = np.zeros(16)
        f64 = lambda v: np.ascontiguousarray(v, dtype=np.float64)
        self.ctx.check(lib().fm3d_setg12(self.ctx.handle, _ptr(f64(T1)), _ptr(f64(T2)), _ptr(f64(r1)),
                                         _ptr(f64(r2)), _ptr(g)))
        return g.reshape(4, 4)

    def set_g12(self, g12) -> None:
        self.ctx.check(lib().fm3d_set_g12(self.ctx.handle, _ptr(np.ascontiguousarray(g12, dtype=np.float64))))

    def camera2(self):
        R2 = np.zeros(9)
        t2 = np.zeros(3)
        self.ctx.check(lib().fm3d_get_camera2(self.ctx.handle, _ptr(R2), _ptr(t2)))
        return R2.reshape(3, 3), t2

    def plane_to_image2(self, X, n):
        """fm3d_plane_to_image2 (device kernel): extractPixelsContour(X) and the level-0 projection of
        those pixels through the plane (X, n) into image 2 -- (image-1 pixels (m, 2), image-2 uv
        (m, 2), status (m,))."""
        X = np.ascontiguousarray(X, dtype=np.float64)
        n = np.ascontiguousarray(n, dtype=np.float64)
        R = self.ctx.settings.pixelsRay
        cap = (2 * R + 1) ** 2
        xy = np.zeros((cap, 2))
        uv = np.zeros((cap, 2))
        st = np.zeros(cap, dtype=np.int32)
        m = ctypes.c_int(0)
        self.ctx.check(lib().fm3d_plane_to_image2(self.ctx.handle, _ptr(X), _ptr(n), _ptr(xy), _ptr(uv),
                                                  _ptr(st, ctypes.c_int32), cap, ctypes.byref(m)))
        k = m.value
        return xy[:k], uv[:k], st[:k]

    def setKeypoints(self, kpts1: np.ndarray, kpts2: np.ndarray, matches: np.ndarray) -> None:
        """setKeypoints (:145-171): keypoint positions (N, 2) float32 + DMATCH array."""
        self._kp1 = np.ascontiguousarray(kpts1, dtype=np.float32)
        self._kp2 = np.ascontiguousarray(kpts2, dtype=np.float32)
        self._matches = np.ascontiguousarray(matches, dtype=DMATCH)

    def triangulate(self):
        """triangulate (:173-230) -> (points (P, 3) float64, outliersMask (K,) bool)."""
        K = self._matches.shape[0]
        pts = np.zeros((max(K, 1), 3))
        mask = np.zeros(max(K, 1), dtype=np.uint8)
        n = ctypes.c_int(0)
        self.ctx.check(lib().fm3d_triangulate(self.ctx.handle, _vp(self._kp1), self._kp1.shape[0], _vp(self._kp2),
                                              self._kp2.shape[0], _vp(self._matches), K, _ptr(pts),
                                              _ptr(mask, ctypes.c_uint8), ctypes.byref(n)))
        return pts[:n.value].copy(), mask[:K].astype(bool)

    def projectReferencePointsToImageWithFrames(self, referenceNeighborhood, featuresFrames, image_points=False):
        """singlecameratriangulator.cpp:769-849 on image 1 of setImages: (P, size, size) uint8 patches,
        patch[j, i] = sample of reference point (i, j); optionally the (P, size*size, 2) projections.
        The reference neighbourhood must be the square one of the settings (it is rebuilt on the GPU)."""
        F = np.ascontiguousarray(featuresFrames, dtype=np.float64).reshape(-1, 16)
        size = lib().fm3d_patch_size(ctypes.byref(self.ctx.settings))
        if referenceNeighborhood is not None and len(referenceNeighborhood) != size * size:
            raise ValueError(f"reference neighbourhood has {len(referenceNeighborhood)} points, settings give {size}^2")
        n = F.shape[0]
        patches = np.zeros((max(n, 1), size, size), dtype=np.uint8)
        pts = np.zeros((max(n, 1), size * size, 2)) if image_points else None
        self.ctx.check(lib().fm3d_export_patches(self.ctx.handle, _ptr(F), n, _ptr(patches, ctypes.c_uint8),
                                                 _ptr(pts) if pts is not None else None))
        return (patches[:n], pts[:n]) if image_points else patches[:n]


class NeighborhoodsGenerator:
    """NeighborhoodsGenerator (Triangulator/neighborhoodsgenerator.h:78-97): the square method and the
    circular one (Neighborhoods.method; the reference constructor exits with -10 on anything else,
    here ValueError)."""

    def __init__(self, settings: Settings):
        if settings.neighMethod not in (0, 1):
            raise ValueError("Unsupported method for plane neighborhood extraction")  # :69-73 exit(-10)
        self.settings = settings

    def computeCircularNeighborhoodsByNormals(self, ctx: "Context", points, normals=None) -> np.ndarray:
        """neighborhoodsgenerator.cpp:160-224: (P, thetas*rays, 3) samples on concentric circles in the
        tangent plane of every point, ray outer / angle inner; normals None -> the initial guess X/|X|
        (the reference fills its empty normals Mat the same way).  points / normals: (P, 3) (the
        reference's 3 x N Mats, transposed).  Computed on the GPU of ctx."""
        X = np.ascontiguousarray(points, dtype=np.float64).reshape(-1, 3)
        N = None if normals is None or len(normals) == 0 else np.ascontiguousarray(normals, dtype=np.float64).reshape(-1, 3)
        if N is not None and N.shape != X.shape:
            raise ValueError("normals and points differ in shape")
        n, S = X.shape[0], self.settings.neighThetas * self.settings.neighRays
        out = np.zeros((max(n, 1), max(S, 1), 3))
        ctx.check(lib().fm3d_circular_neighborhoods(ctx.handle, _ptr(X), _ptr(N) if N is not None else None, n,
                                                    _ptr(out)))
        return out[:n, :S]

    def computeCircularNeighborhoodByNormal(self, ctx: "Context", point, normal=(0.0, 0.0, 0.0)) -> np.ndarray:
        """neighborhoodsgenerator.cpp:226-277 (one point; a zero normal -> X/|X|): (thetas*rays, 3)."""
        nz = not any(float(v) != 0.0 for v in normal)
        return self.computeCircularNeighborhoodsByNormals(ctx, [point], None if nz else [normal])[0]

    def size(self) -> int:
        return lib().fm3d_patch_size(ctypes.byref(self.settings))

    def computeSquareNeighborhoodsByNormals(self, ctx: "Context", featuresFrames) -> np.ndarray:
        """neighborhoodsgenerator.cpp:76-132 (main.cpp:187): (P, size*size, 3) points of the square
        grid transformed by each feature frame, point order i*size + j; computed on the GPU of ctx."""
        F = np.ascontiguousarray(featuresFrames, dtype=np.float64).reshape(-1, 16)
        n, size = F.shape[0], self.size()
        out = np.zeros((max(n, 1), size * size, 3))
        ctx.check(lib().fm3d_square_neighborhoods(ctx.handle, _ptr(F), n, _ptr(out)))
        return out[:n]

    def getReferenceSquaredNeighborhood(self) -> np.ndarray:
        """neighborhoodsgenerator.cpp:134-158: (size*size, 3) points (-eps + inc*i, -eps + inc*j, 0),
        i outer."""
        eps, inc, n = self.settings.neighEpsilon, self.settings.cmPerPixel * 0.01, self.size()
        out = np.zeros((n * n, 3))
        for i in range(n):
            for j in range(n):
                out[i * n + j, 0] = -eps + inc * i
                out[i * n + j, 1] = -eps + inc * j
        return out


class NormalOptimizer:
    """NormalOptimizer (Triangulator/normaloptimizer.h:43-59), hot-path methods."""

    def __init__(self, ctx: Context, sct: SingleCameraTriangulator | None = None):
        self.ctx = ctx
        self.sct = sct
        self.last_status = self.last_info = self.last_nfev = None
        self.last_stats = None

    def setImages(self, img1: np.ndarray, img2: np.ndarray) -> None:
        a = np.ascontiguousarray(img1, dtype=np.uint8)
        b = np.ascontiguousarray(img2, dtype=np.uint8)
        if a.shape != b.shape or a.ndim != 2:
            raise ValueError("two gray images of the same size expected")
        h, w = a.shape
        self.ctx.check(lib().fm3d_set_images(self.ctx.handle, _ptr(a, ctypes.c_uint8), _ptr(b, ctypes.c_uint8), w, h, w))

    def pyramid(self, which: int, level: int) -> np.ndarray:
        w = ctypes.c_int(0)
        h = ctypes.c_int(0)
        self.ctx.check(lib().fm3d_get_pyramid_level(self.ctx.handle, which, level, None, ctypes.byref(w),
                                                    ctypes.byref(h)))
        out = np.zeros((h.value, w.value), dtype=np.uint8)
        self.ctx.check(lib().fm3d_get_pyramid_level(self.ctx.handle, which, level, _ptr(out, ctypes.c_uint8),
                                                    ctypes.byref(w), ctypes.byref(h)))
        return out

    def getGravity(self) -> np.ndarray:
        """getGravity (normaloptimizer.cpp:185-188): Rodrigues(rodriguesIC)^-1 (0, 0, -1)."""
        g = np.zeros(3)
        _check(lib().fm3d_gravity(ctypes.byref(self.ctx.settings), _ptr(g)))
        return g

    def nccHypotheses(self, points3D: np.ndarray, hphi: int = 4, htheta: int = 4, span: float = 0.4):
        """NCC scoring of hphi x htheta candidate normals per point (fm3d_ncc_hypotheses; BASELINE's
        "patch NCC over 16 / 32 normal hypotheses" -- an extension, the reference has no NCC search):
        (scores (P, H) float64, -2 = invalid; best normals (P, 3); best index (P,), -1 = none).
        Needs setImages and the camera-2 pose of the triangulator."""
        X = np.ascontiguousarray(points3D, dtype=np.float64).reshape(-1, 3)
        n, H = X.shape[0], hphi * htheta
        scores = np.zeros((max(n, 1), H))
        normals = np.zeros((max(n, 1), 3))
        best = np.zeros(max(n, 1), dtype=np.int32)
        self.ctx.check(lib().fm3d_ncc_hypotheses(self.ctx.handle, _ptr(X), n, hphi, htheta, ctypes.c_double(span),
                                                 _ptr(scores), _ptr(normals), _ptr(best, ctypes.c_int32)))
        return scores[:n], normals[:n], best[:n]

    def computeFeaturesFrames(self, points3D: np.ndarray, normals: np.ndarray) -> np.ndarray:
        """computeFeaturesFrames (normaloptimizer.cpp:454-504): (P, 4, 4) frames, on the GPU."""
        P = np.ascontiguousarray(points3D, dtype=np.float64).reshape(-1, 3)
        N = np.ascontiguousarray(normals, dtype=np.float64).reshape(-1, 3)
        n = min(P.shape[0], N.shape[0])  # the reference walks both vectors together
        frames = np.zeros((max(n, 1), 4, 4))
        self.ctx.check(lib().fm3d_features_frames(self.ctx.handle, _ptr(P), _ptr(N), n, _ptr(frames)))
        return frames[:n]

    def startVisualizerThread(self):  # PCL viewer: out of scope, no-op
        pass

    def stopVisualizerThread(self):
        pass

    def computeOptimizedNormals(self, points3D: np.ndarray):
        """computeOptimizedNormals (normaloptimizer.cpp:321-452).

        Returns (kept points, normals): failed points are erased (stable order),
        exactly like the reference mutates its std::vector.  Per-input-point status,
        lmdif info and evaluation counts are left in last_status / last_info / last_nfev.
        """
        P = np.ascontiguousarray(points3D, dtype=np.float64).reshape(-1, 3).copy()
        n = P.shape[0]
        normals = np.zeros((max(n, 1), 3))
        status = np.zeros(max(n, 1), dtype=np.int32)
        info = np.zeros((max(n, 1), 8), dtype=np.int32)
        nfev = np.zeros((max(n, 1), 8), dtype=np.int32)
        kept = ctypes.c_int(0)
        st = LMStats()
        self.ctx.check(lib().fm3d_optimize_normals(self.ctx.handle, _ptr(P), n, _ptr(normals),
                                                   _ptr(status, ctypes.c_int32), _ptr(info, ctypes.c_int32),
                                                   _ptr(nfev, ctypes.c_int32), ctypes.byref(kept), ctypes.byref(st)))
        self.last_status, self.last_info, self.last_nfev = status[:n], info[:n], nfev[:n]
        self.last_stats = st.as_dict()
        k = kept.value
        return P[:k].copy(), normals[:k].copy()


class Pipeline:
    """Whole hot path with inputs resident in HBM (bench / multi-GPU shards)."""

    def __init__(self, ctx: Context):
        self.ctx = ctx
        self.n_queries = 0

    def upload(self, desc_a, desc_b, kp1, kp2, img1, img2, binary=False, query_offset=0):
        """fm3d_pipeline_upload; img1 = img2 = None stages no images (C2's match + DLT)"""
        a = np.ascontiguousarray(desc_a)
        b = np.ascontiguousarray(desc_b)
        k1 = np.ascontiguousarray(kp1, dtype=np.float32)
        k2 = np.ascontiguousarray(kp2, dtype=np.float32)
        if img1 is None and img2 is None:
            i1 = i2 = None
            h = w = 0
        else:
            i1 = np.ascontiguousarray(img1, dtype=np.uint8)
            i2 = np.ascontiguousarray(img2, dtype=np.uint8)
            h, w = i1.shape
        self.n_queries = a.shape[0]
        self.ctx.check(lib().fm3d_pipeline_upload(self.ctx.handle, _vp(a), a.shape[0], _vp(b), b.shape[0],
                                                  a.shape[1], _desc_type(a, binary), _vp(k1), _vp(k2),
                                                  None if i1 is None else _ptr(i1, ctypes.c_uint8),
                                                  None if i2 is None else _ptr(i2, ctypes.c_uint8), w, h,
                                                  query_offset))

    def run(self, records_dev_ptr: int | None = None):
        """One pass; returns (n_kept, stats dict).  records_dev_ptr: device buffer
        (e.g. a torch tensor's data_ptr()) with room for n_queries records."""
        n = ctypes.c_int(0)
        st = PipelineStats()
        self.ctx.check(lib().fm3d_pipeline_run(self.ctx.handle, ctypes.c_void_p(records_dev_ptr or 0),
                                               ctypes.byref(n), ctypes.byref(st)))
        return n.value, st.as_dict()

    def submit(self, desc_a, desc_b, kp1, kp2, img1, img2, binary=False, query_offset=0):
        """fm3d_pipeline_submit: stage one frame pair (H2D through pinned buffers, pyramids) and queue the
        whole path on the context stream without waiting.  The arrays are copied before it returns."""
        a = np.ascontiguousarray(desc_a)
        b = np.ascontiguousarray(desc_b)
        k1 = np.ascontiguousarray(kp1, dtype=np.float32)
        k2 = np.ascontiguousarray(kp2, dtype=np.float32)
        i1 = np.ascontiguousarray(img1, dtype=np.uint8)
        i2 = np.ascontiguousarray(img2, dtype=np.uint8)
        h, w = i1.shape
        self.n_queries = a.shape[0]
        self.ctx.check(lib().fm3d_pipeline_submit(self.ctx.handle, _vp(a), a.shape[0], _vp(b), b.shape[0],
                                                  a.shape[1], _desc_type(a, binary), _vp(k1), _vp(k2),
                                                  _ptr(i1, ctypes.c_uint8), _ptr(i2, ctypes.c_uint8), w, h,
                                                  query_offset))

    def link(self, leader: "Pipeline"):
        """fm3d_pipeline_link(self, leader): this context's pairs join the leader's LM launches."""
        self.ctx.check(lib().fm3d_pipeline_link(self.ctx.handle, leader.ctx.handle))

    def wait(self, out: np.ndarray | None = None):
        """fm3d_pipeline_wait: (survivor records (host), stats dict) of the submitted frame pair.  out: a
        RECORD array with room for n_queries records (reused across calls), or None to allocate."""
        if out is None:
            out = np.zeros(max(self.n_queries, 1), dtype=RECORD)
        n = ctypes.c_int(0)
        st = PipelineStats()
        self.ctx.check(lib().fm3d_pipeline_wait(self.ctx.handle, _vp(out), len(out), ctypes.byref(n),
                                                ctypes.byref(st)))
        return out[:n.value], st.as_dict()

    def run_dlt(self):
        """C2's path: match -> NNDR -> triangulate only; returns (n_inliers, stats dict)"""
        n = ctypes.c_int(0)
        st = PipelineStats()
        self.ctx.check(lib().fm3d_pipeline_run_dlt(self.ctx.handle, ctypes.byref(n), ctypes.byref(st)))
        return n.value, st.as_dict()

    def submit_dlt(self) -> None:
        """fm3d_pipeline_submit_dlt: C2's path queued on the context stream (returns at once)"""
        self.ctx.check(lib().fm3d_pipeline_submit_dlt(self.ctx.handle))

    def submit_dlt_pair(self, desc_a, desc_b, kp1, kp2, binary=False, query_offset=0) -> None:
        """fm3d_pipeline_submit_dlt_pair: stage a pair from host memory (no images) and queue C2's path,
        with no host wait (float rows are checked on the device; wait_dlt redoes non-integer ones)"""
        a = np.ascontiguousarray(desc_a)
        b = np.ascontiguousarray(desc_b)
        k1 = np.ascontiguousarray(kp1, dtype=np.float32)
        k2 = np.ascontiguousarray(kp2, dtype=np.float32)
        self.n_queries = a.shape[0]
        self.ctx.check(lib().fm3d_pipeline_submit_dlt_pair(self.ctx.handle, _vp(a), a.shape[0], _vp(b), b.shape[0],
                                                           a.shape[1], _desc_type(a, binary), _vp(k1), _vp(k2),
                                                           query_offset))

    def wait_dlt(self):
        """fm3d_pipeline_wait_dlt: (n_inliers, stats dict) of the submitted front half"""
        n = ctypes.c_int(0)
        st = PipelineStats()
        self.ctx.check(lib().fm3d_pipeline_wait_dlt(self.ctx.handle, ctypes.byref(n), ctypes.byref(st)))
        return n.value, st.as_dict()

    def run_ncc(self, hphi: int = 4, htheta: int = 4, span: float = 0.4):
        """C3's path: match -> NNDR -> triangulate -> NCC scoring of hphi x htheta normals per inlier;
        returns (n_points, stats dict)"""
        n = ctypes.c_int(0)
        st = PipelineStats()
        self.ctx.check(lib().fm3d_pipeline_run_ncc(self.ctx.handle, hphi, htheta, ctypes.c_double(span), ctypes.byref(n),
                                                   ctypes.byref(st)))
        return n.value, st.as_dict()

    def submit_ncc(self, hphi: int = 4, htheta: int = 4, span: float = 0.4) -> None:
        """fm3d_pipeline_submit_ncc: C3's path queued on the context stream (returns at once)"""
        self.ctx.check(lib().fm3d_pipeline_submit_ncc(self.ctx.handle, hphi, htheta, ctypes.c_double(span)))

    def wait_ncc(self):
        """fm3d_pipeline_wait_ncc: (n_points, stats dict) of the submitted C3 path"""
        n = ctypes.c_int(0)
        st = PipelineStats()
        self.ctx.check(lib().fm3d_pipeline_wait_ncc(self.ctx.handle, ctypes.byref(n), ctypes.byref(st)))
        return n.value, st.as_dict()

    def ncc_results(self, n_points: int, H: int):
        """(scores (P, H), best normals (P, 3), best index (P,)) of the last run_ncc"""
        sc = np.zeros((max(n_points, 1), H))
        nr = np.zeros((max(n_points, 1), 3))
        b = np.zeros(max(n_points, 1), dtype=np.int32)
        self.ctx.check(lib().fm3d_pipeline_ncc_download(self.ctx.handle, _vp(sc), _vp(nr), _ptr(b, ctypes.c_int32)))
        return sc[:n_points], nr[:n_points], b[:n_points]

    def dlt_results(self, n_matches: int, n_inliers: int):
        """(matches (K,) DMATCH, inlier points (P, 3), match index of each point) of the last run"""
        m = np.zeros(max(n_matches, 1), dtype=DMATCH)
        pts = np.zeros((max(n_inliers, 1), 3))
        src = np.zeros(max(n_inliers, 1), dtype=np.int32)
        self.ctx.check(lib().fm3d_pipeline_dlt_download(self.ctx.handle, _vp(m), _vp(pts), _ptr(src, ctypes.c_int32)))
        return m[:n_matches], pts[:n_inliers], src[:n_inliers]

    def records(self, n: int, records_dev_ptr: int | None = None) -> np.ndarray:
        out = np.zeros(max(n, 1), dtype=RECORD)
        self.ctx.check(lib().fm3d_records_download(self.ctx.handle, ctypes.c_void_p(records_dev_ptr or 0), n,
                                                   _vp(out)))
        return out[:n]


SHARE_BLOCK = 4096  # queries per block of the block-cyclic partition (fm3d_mgpu, shard.py)


def device_count() -> int:
    """fm3d_device_count: the GPUs HIP sees (hipGetDeviceCount), without importing torch."""
    n = ctypes.c_int(0)
    _check(lib().fm3d_device_count(ctypes.byref(n)))
    return n.value


def share_queries(n: int, shares: int, s: int, block: int = SHARE_BLOCK) -> np.ndarray:
    """fm3d_share_queries: global query indices of share s (blocks dealt round-robin)."""
    cnt = ctypes.c_int(0)
    _check(lib().fm3d_share_queries(n, shares, s, block, None, 0, ctypes.byref(cnt)))
    idx = np.zeros(max(cnt.value, 1), dtype=np.int32)
    _check(lib().fm3d_share_queries(n, shares, s, block, _ptr(idx, ctypes.c_int32), len(idx), ctypes.byref(cnt)))
    return idx[:cnt.value].astype(np.int64)


def merge_shares(parts, n: int, block: int = SHARE_BLOCK) -> np.ndarray:
    """fm3d_merge_shares (the C++ merge of fm3d_mgpu_pipeline_run, host only): parts[s] = share s's
    survivor records with local query indices -> all records with global indices, query order."""
    parts = [np.ascontiguousarray(p, dtype=RECORD) for p in parts]
    shares = len(parts)
    ptrs = (ctypes.c_void_p * max(shares, 1))(*[p.ctypes.data for p in parts])
    counts = np.array([len(p) for p in parts], dtype=np.int32)
    out = np.zeros(max(int(counts.sum()), 1), dtype=RECORD)
    k = ctypes.c_int(0)
    _check(lib().fm3d_merge_shares(n, shares, block, ptrs, _ptr(counts, ctypes.c_int32), _vp(out), ctypes.byref(k)))
    return out[:k.value]


class MultiGPU:
    """fm3d_mgpu: the whole path over several GPUs in one process -- query
    blocks dealt round-robin over `shares` logical shares (share s on devices[s % ndev]), frame B
    and the images replicated, RCCL all-gather of the survivor records, merged in query order."""

    def __init__(self, settings: Settings, devices=(0,), shares: int | None = None, block: int = SHARE_BLOCK):
        self.settings = settings
        devs = np.ascontiguousarray(devices, dtype=np.int32)
        self.ndev = len(devs)
        self.shares = shares or self.ndev
        self._h = ctypes.c_void_p()
        rc = lib().fm3d_mgpu_create(ctypes.byref(settings), self.ndev, _ptr(devs, ctypes.c_int32), self.shares, block,
                                    ctypes.byref(self._h))
        if rc != FM3D_OK:
            why = (lib().fm3d_mgpu_last_error(None) or b"").decode(errors="replace")
            raise Fm3dError(rc, "fm3d_mgpu_create failed" + (f": {why}" if why else " (no HIP devices / RCCL?)"))
        self.n_queries = 0

    def check(self, rc):
        if rc != FM3D_OK:
            raise Fm3dError(rc, lib().fm3d_mgpu_last_error(self._h).decode(errors="replace"))

    def set_g12(self, g12):
        self.check(lib().fm3d_mgpu_set_g12(self._h, _ptr(np.ascontiguousarray(g12, dtype=np.float64).ravel())))

    def upload(self, desc_a, desc_b, kp1, kp2, img1, img2, binary=False):
        a = np.ascontiguousarray(desc_a)
        b = np.ascontiguousarray(desc_b)
        k1 = np.ascontiguousarray(kp1, dtype=np.float32)
        k2 = np.ascontiguousarray(kp2, dtype=np.float32)
        i1 = np.ascontiguousarray(img1, dtype=np.uint8)
        i2 = np.ascontiguousarray(img2, dtype=np.uint8)
        h, w = i1.shape
        self.n_queries = a.shape[0]
        self.check(lib().fm3d_mgpu_pipeline_upload(self._h, _vp(a), a.shape[0], _vp(b), b.shape[0], a.shape[1],
                                                   _desc_type(a, binary), _vp(k1), _vp(k2), _ptr(i1, ctypes.c_uint8),
                                                   _ptr(i2, ctypes.c_uint8), w, h))

    def submit(self, desc_a, desc_b, kp1, kp2, img1, img2, binary=False):
        """fm3d_mgpu_submit: one frame pair staged on every device and queued (two may be in flight)."""
        a = np.ascontiguousarray(desc_a)
        b = np.ascontiguousarray(desc_b)
        k1 = np.ascontiguousarray(kp1, dtype=np.float32)
        k2 = np.ascontiguousarray(kp2, dtype=np.float32)
        i1 = np.ascontiguousarray(img1, dtype=np.uint8)
        i2 = np.ascontiguousarray(img2, dtype=np.uint8)
        h, w = i1.shape
        self.n_queries = a.shape[0]
        self.check(lib().fm3d_mgpu_submit(self._h, _vp(a), a.shape[0], _vp(b), b.shape[0], a.shape[1],
                                          _desc_type(a, binary), _vp(k1), _vp(k2), _ptr(i1, ctypes.c_uint8),
                                          _ptr(i2, ctypes.c_uint8), w, h))

    def wait(self, out: np.ndarray | None = None):
        """fm3d_mgpu_wait: (merged records of the oldest submitted pair, stats dict)."""
        if out is None:
            out = np.zeros(max(self.n_queries, 1), dtype=RECORD)
        n = ctypes.c_int(0)
        st = PipelineStats()
        self.check(lib().fm3d_mgpu_wait(self._h, _vp(out), len(out), ctypes.byref(n), ctypes.byref(st)))
        return out[:n.value], st.as_dict()

    def run(self):
        """One pass over all devices: (records in query order, stats dict)."""
        out = np.zeros(max(self.n_queries, 1), dtype=RECORD)
        n = ctypes.c_int(0)
        st = PipelineStats()
        self.check(lib().fm3d_mgpu_pipeline_run(self._h, _vp(out), ctypes.byref(n), ctypes.byref(st)))
        return out[:n.value], st.as_dict()

    def close(self):
        if self._h:
            lib().fm3d_mgpu_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def g12_from_poses(settings: Settings, T1, T2, r1, r2) -> np.ndarray:
    """Context-free setg12 algebra (host only)."""
    g = np.zeros(16)
    f64 = lambda v: np.ascontiguousarray(v, dtype=np.float64)
    _check(lib().fm3d_g12_from_poses(ctypes.byref(settings), _ptr(f64(T1)), _ptr(f64(T2)), _ptr(f64(r1)),
                                     _ptr(f64(r2)), _ptr(g)))
    return g.reshape(4, 4)


def camera2_from_g12(g12):
    R2 = np.zeros(9)
    t2 = np.zeros(3)
    _check(lib().fm3d_camera2_from_g12(_ptr(np.ascontiguousarray(g12, dtype=np.float64).ravel()), _ptr(R2), _ptr(t2)))
    return R2.reshape(3, 3), t2


class MOSAIC:
    """MOSAIC (mosaic.h:47-70, mosaic.cpp:32-73): the reference's descriptor extractor built on the
    whole pipeline.  The constructor runs the reference's seven steps on the GPU -- SURF
    compareWithNNDR on the two images, setg12, setKeypoints + triangulate, setImages +
    computeOptimizedNormals + computeFeaturesFrames, the reference square neighbourhood, and the
    normal-rectified patches of image A (projectReferencePointsToImageWithFrames).  The reference's
    computeImpl is empty (mosaic.cpp:75-79); compute() finishes it the way the reference's main()
    does (main.cpp:182-183): extractDescriptorsFromPatches of the patches, one SURF row per kept
    feature (descriptorType CV_32F, descriptorSize 128)."""

    descriptorSize = 128

    def __init__(self, ctx: Context, imgA: np.ndarray, imgB: np.ndarray, tA, tB, rA, rB):
        self.ctx = ctx
        s = ctx.settings
        self.imgA = np.ascontiguousarray(imgA, dtype=np.uint8)
        self.imgB = np.ascontiguousarray(imgB, dtype=np.uint8)
        # 2 - matches (descriptorsmatcher.cpp:107-131 from the images)
        self.dm = DescriptorsMatcher(ctx)
        self.matches, self.kptsA, self.kptsB, _, _ = self.dm.compareWithNNDRImages(s.nndrEpsilon, self.imgA, self.imgB)
        # 3 - g12 (singlecameratriangulator.cpp:123-143)
        self.sct = SingleCameraTriangulator(ctx)
        self.gAB = self.sct.setg12(tA, tB, rA, rB)
        # 4 - triangulation of the matches (:145-230)
        xy = lambda k: np.stack([k["x"], k["y"]], axis=1).astype(np.float32)
        self.sct.setKeypoints(xy(self.kptsA), xy(self.kptsB), self.matches)
        pts, self.outliersMask = self.sct.triangulate()
        # 5 - normals and feature frames (normaloptimizer.cpp:191-504)
        self.no = NormalOptimizer(ctx, self.sct)
        self.no.setImages(self.imgA, self.imgB)
        self.triangulated_points, self.normals = self.no.computeOptimizedNormals(pts)
        self.features_frames = self.no.computeFeaturesFrames(self.triangulated_points, self.normals)
        # 6 - the reference neighbourhood (neighborhoodsgenerator.cpp:134-158)
        self.ng = NeighborhoodsGenerator(s)
        self.reference_neighborhood = self.ng.getReferenceSquaredNeighborhood()
        # 7 - patches of image A (singlecameratriangulator.cpp:769-849)
        self.patches, self.image_points = self.sct.projectReferencePointsToImageWithFrames(
            self.reference_neighborhood, self.features_frames, image_points=True)

    def descriptorType(self):
        return np.float32

    def compute(self) -> np.ndarray:
        """The patch descriptors: (kept features, cols) rows of the settings' extractor (float32 for
        SURF / SIFT, uint8 for ORB / BRISK)."""
        feats = Features(self.ctx)
        if len(self.patches) == 0:
            cols, dt = feats.descriptor_info()
            return np.zeros((0, cols), dtype=dt)
        return feats.extractDescriptorsFromPatches(self.patches)
