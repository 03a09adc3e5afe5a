/*
 * fm3d.h -- C ABI of the MI355X-native 3DFeatureMatcher hot path.
 *
 * The reference (caomw/3DFeatureMatcher) exposes this path as three C++ classes
 * called from main.cpp:91-155.  Every entry point below replaces one of their
 * methods; the citation names the reference interface it stands in for.  Plain
 * C types only (no OpenCV / torch types): the C++ shim in
 * include/fm3d_compat.hpp re-exposes the reference class signatures on top of
 * this ABI, and INTEGRATION.md shows the bindings.
 *
 * Conventions
 *   - every function returns FM3D_OK (0) or a negative FM3D_ERR_* code; the
 *     reference's exit() paths become error returns (fm3d_last_error() has the text);
 *   - host pointers unless the name ends in _dev; the caller owns all buffers;
 *   - a context owns its device buffers (grown on demand, reused across calls),
 *     one HIP stream, and is not thread-safe (one host thread per context);
 *   - the per-point "erase" of the reference (normaloptimizer.cpp:366,378) is a
 *     stable compaction: survivors keep their input order.
 */
#ifndef FM3D_H
#define FM3D_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FM3D_OK 0
#define FM3D_ERR_INVALID (-1)     /* bad argument / state (the reference would exit(-1)) */
#define FM3D_ERR_HIP (-2)         /* HIP runtime error */
#define FM3D_ERR_UNSUPPORTED (-3) /* e.g. pixelsRay larger than the kernel supports */
#define FM3D_ERR_NOMEM (-4)
#define FM3D_ERR_PARSE (-5)       /* settings file could not be read */
#define FM3D_ERR_NAN_PLANE (-6)   /* strictNanExit: projectPointToPlane exit(-6),
                                     singlecameratriangulator.cpp:465-469 */

/* per-point outcome of the normal optimisation */
#define FM3D_ST_OK 0
#define FM3D_ST_NO_PIXELS 1   /* "Not enough pixels!"  normaloptimizer.cpp:364-369 */
#define FM3D_ST_ABORT_BBOX 2  /* isInBoundingBox failed, singlecameratriangulator.cpp:557-560 */
#define FM3D_ST_ABORT_PIX1 3  /* image-1 pixel outside isPixelGood, :580-584 */
#define FM3D_ST_ABORT_PIX2 4  /* image-2 projection outside isPixelGood, :623-626 */
#define FM3D_ST_NAN_PLANE 5   /* ray parallel to the plane (reference: exit(-6)) */
#define FM3D_ST_NAN_NORMAL 6  /* sph2car produced NaN, normaloptimizer.cpp:81-85 */

typedef struct fm3d_ctx fm3d_ctx;

/* Settings: the keys of build/settings.yml the hot path reads. */
typedef struct fm3d_settings {
    /* CameraSettings (singlecameratriangulator.cpp:45-109) */
    double Fx, Fy, Cx, Cy;
    double p1, p2, k0, k1, k2; /* OpenCV order (k1,k2,p1,p2,k3) = (k0,k1,p1,p2,k2) */
    double rodriguesIC[3];
    double translationIC[3];
    double zThresholdMin, zThresholdMax;
    /* Neighborhoods (normaloptimizer.cpp:154-156, singlecameratriangulator.cpp:112) */
    double epsilonLMMIN;
    int pixelsRay;
    int pyramids;
    /* NNDR (main.cpp:94) */
    double nndrEpsilon;
    /* IMAGES.pos1 / pos2: T(3) then Rodrigues(3) (main.cpp:96-114) */
    double pos1[6], pos2[6];
    /* --- extensions (not in the reference file) --- */
    int boundWidth, boundHeight; /* literal 1024 x 768 of extractPixelsContour (:359) */
    int strictNanExit;           /* 1: NaN plane makes fm3d_optimize_normals fail with FM3D_ERR_NAN_PLANE */
    int lmWaves;                 /* LM workgroups to launch (0 = fill the GPU) */
    /* Neighborhoods.epsilon / cmPerPixel (neighborhoodsgenerator.cpp:43-44): patch export */
    double neighEpsilon, cmPerPixel;
    /* Neighborhoods.method (neighborhoodsgenerator.cpp:38-73): 0 square, 1 circular, -1 anything
       else (the reference's exit(-10)); thetas / rays of the circular method (:47-48) */
    int neighMethod, neighThetas, neighRays;
    /* FeatureOptions (descriptorsmatcher.cpp:176-359): DetectorMode STATIC + DetectorType /
       ExtractorType SURF are FM3D_FEAT_SURF, ORB FM3D_FEAT_ORB; anything else FM3D_FEAT_OTHER (no GPU
       implementation).
       SurfDetector.HessianThreshold / NumOctaves / NumOctaveLayers / Extended / Upright */
    int detectorType, extractorType;
    double surfHessianThreshold;
    int surfOctaves, surfOctaveLayers, surfExtended, surfUpright;
    /* FeatureOptions.OrbDetector.NumFeatures / ScaleFactor / NumLevels (cv::ORB's first three
       arguments, descriptorsmatcher.cpp:276-279, 338-341); defaults OpenCV's 500 / 1.2 / 8.  The
       extensions after them are cv::ORB's defaulted arguments: edgeThreshold 31, patchSize 31, and
       computeKeyPoints' hard-coded FAST threshold 20 */
    int orbNumFeatures;
    double orbScaleFactor;
    int orbNumLevels, orbEdgeThreshold, orbPatchSize, orbFastThreshold;
    /* FeatureOptions.SiftDetector.NumFeatures / NumOctaveLayers / ContrastThreshold / EdgeThreshold /
       Sigma (cv::SIFT's five arguments, descriptorsmatcher.cpp:246-251, 305-310); OpenCV's defaults
       0 / 3 / 0.04 / 10 / 1.6 when the file names none (the reference would read 0 from a missing
       node) */
    int siftNumFeatures, siftOctaveLayers;
    double siftContrastThreshold, siftEdgeThreshold, siftSigma;
    /* FeatureOptions.DetectorMode: 0 STATIC, 1 ADAPTIVE (DynamicAdaptedFeatureDetector over
       AdjusterAdapter::create(DetectorType), :185-201; FAST, SURF and STAR run on the GPU);
       FeatureOptions.FastDetector.Threshold / NonMaxSuppression (:215-222, cv::FastFeatureDetector's
       defaults 10 / 1); FeatureOptions.Adaptive.MinFeatures / MaxFeatures / MaxIters (the
       DynamicAdaptedFeatureDetector defaults 400 / 500 / 5) */
    int detectorMode;
    int fastThreshold, fastNonmax;
    int adaptiveMinFeatures, adaptiveMaxFeatures, adaptiveMaxIters;
    /* FeatureOptions.StarDetector.MaxSize / Response / LineThreshold / LineBinarized / Suppression
       (:207-212, cv::StarDetector's defaults 45 / 30 / 10 / 8 / 5) */
    int starMaxSize, starResponse, starLineThreshold, starLineBinarized, starSuppression;
    /* FeatureOptions.BriskDetector.Threshold / Octaves (:345-347, build/settings.yml:46-48): cv::BRISK's
       detection parameters, which its descriptor does not use (OpenCV defaults 30 / 3) */
    int briskThreshold, briskOctaves;
    /* FeatureOptions.MSERDetector.Delta / MinArea / MaxArea / MaxVariation / MinDiversity / MaxEvolution /
       AreaThreshold / MinMargin / EdgeBlurSize (:258-272, cv::MSER's nine arguments; OpenCV's defaults
       5 / 60 / 14400 / 0.25 / 0.2 / 200 / 1.01 / 0.003 / 5).  On grey images only the first five
       steer the result (the last four drive OpenCV's colour-image MSCR). */
    int mserDelta, mserMinArea, mserMaxArea;
    double mserMaxVariation, mserMinDiversity;
    int mserMaxEvolution;
    double mserAreaThreshold, mserMinMargin;
    int mserEdgeBlurSize;
    /* The LM's reduction order (not a reference key; Fm3d.lmReduction in the settings file):
       0 = every m_dat-long sum (enorm of the residual, the Jacobian column norms, the Householder
       products) in pixel order, MINPACK's and so the reference's -- the default, the parity
       contract; 1 = the fixed blocked tree of DESIGN.md §3.4b (faster; bit-exact to the oracle's
       ORC_LM_TREE | ORC_LM_GRAM mode, but the normals leave the reference's by more than 1e-4 on a
       share of the points, profiles/r05_full_parity.json) */
    int lmReduction;
    /* The DLT's null-vector solver (not a reference key; Fm3d.dltSolver in the settings file):
       0 = OpenCV 2.4's cvTriangulatePoints -- the 6 x 4 system and JacobiSVD, include/fm3d_cvsvd.h --
       the default, the parity contract; 1 = the 4-row system and a round-robin Jacobi of rounds 1-5
       (opt-in; its points leave OpenCV's in the last bits) */
    int dltSolver;
} fm3d_settings;

#define FM3D_FEAT_SURF 0
#define FM3D_FEAT_ORB 1
#define FM3D_FEAT_SIFT 2
#define FM3D_FEAT_FAST 3
#define FM3D_FEAT_STAR 4
#define FM3D_FEAT_BRISK 5 /* extractor only: the reference's generateDetector has no BRISK branch */
#define FM3D_FEAT_FREAK 6 /* extractor only (cv::FREAK(), descriptorsmatcher.cpp:350-353) */
#define FM3D_FEAT_MSER 7  /* detector only (cv::MserFeatureDetector, descriptorsmatcher.cpp:258-272) */
#define FM3D_FEAT_OTHER (-1)

/* cv::DMatch layout */
typedef struct fm3d_dmatch {
    int32_t queryIdx, trainIdx, imgIdx;
    float distance;
} fm3d_dmatch;

/* cv::KeyPoint::pt */
typedef struct fm3d_point2f {
    float x, y;
} fm3d_point2f;

/* cv::KeyPoint (28 bytes) */
typedef struct fm3d_keypoint {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} fm3d_keypoint;

typedef enum fm3d_desc_type {
    FM3D_DESC_F32 = 0,  /* float rows (SURF/SIFT): FLANN L2 order, distance = sqrt */
    FM3D_DESC_U8 = 1,   /* uint8 rows (SIFT saturated to uchar): exact integer L2 */
    FM3D_DESC_BITS = 2  /* binary strings, dim = bytes (ORB/BRISK/FREAK): Hamming */
} fm3d_desc_type;

/* one surviving keypoint of the whole hot path (64 bytes) */
typedef struct fm3d_record {
    int32_t queryIdx, trainIdx;
    float distance;
    int32_t status;
    double point[3];
    double normal[3];
} fm3d_record;

typedef struct fm3d_lm_stats {
    int64_t points_in;
    int64_t points_kept;
    int64_t evaluations;       /* residual evaluations, all points and levels */
    int64_t pixel_evaluations; /* sum over evaluations of m_dat */
    int64_t drops[8];          /* points per FM3D_ST_* code */
    double kernel_ms;          /* LM kernel time (HIP events on the context stream) */
    int64_t groups;            /* LM workgroups launched (15 points in flight each, one per term wave) */
    int64_t passes;            /* summed neighbourhood passes (residual, Jacobian, Householder), all points */
    /* core clock cycles, summed over workgroups or waves: term waves inside passes
       (including waits), the chain wave busy adding, term waves in the lmdif bookkeeping,
       workgroup 0-th wave lifetime */
    int64_t cycles_terms, cycles_chain, cycles_control, cycles_total;
    /* workgroup lifetimes in constant-rate wall-clock ticks: sum and max over workgroups */
    int64_t wall_ticks_sum, wall_ticks_max, wall_clock_khz;
    /* passes and term-wave cycles by class: [0] Jacobian (two residual evaluations),
       [1] one residual evaluation, [2] Householder products, [3] once per point / level */
    int64_t class_passes[4], class_cycles[4];
    /* wall-clock ticks from the first workgroup start to the last start / the last end */
    int64_t last_group_start_ticks, last_group_end_ticks;
    /* term-wave cycles spent waiting on the chain lanes (ring full, pass results) */
    int64_t cycles_wait;
    /* chain wave: busy rounds (each adds up to two chunks per lane) and chunks added, summed
       over workgroups and lanes */
    int64_t chain_rounds, chain_chunks;
    /* wall-clock ticks from the first workgroup start to the last point handed out (the queue
       runs dry there: the rest of the launch is the tail) */
    int64_t queue_empty_ticks;
} fm3d_lm_stats;

/* match_ms: row constants + knn + NNDR with its compaction (NNDR is fused into the match's last
   launch, so nndr_ms is always 0); triangulate_ms: DLT + inlier compaction.  Both are 0 when the step
   recorded no stage events (FM3D_STAGE_EVENTS=0).  In a stream of frame pairs the stage events of a
   pair also span the time its launches wait behind other pairs' work on the GPU: stage costs come from
   a pair run alone. */
typedef struct fm3d_pipeline_stats {
    int64_t queries, trains, matches, inliers, kept;
    double match_ms, nndr_ms, triangulate_ms, pyramid_ms, lm_ms, total_ms; /* HIP events */
    fm3d_lm_stats lm;
} fm3d_pipeline_stats;

/* ---------------- settings / context ---------------- */
/* build/settings.yml values (the reference's defaults) */
int fm3d_settings_default(fm3d_settings *s);
/* read a %YAML:1.0 cv::FileStorage file (the subset settings.yml uses) */
int fm3d_settings_load(const char *path, fm3d_settings *s);
/* cv::FileStorage node lookup (fs["IMAGES"]["img1"] >> ..., main.cpp:74-98): the raw text of the
   dotted key "IMAGES.img1" in a %YAML:1.0 file -- a scalar or a flow sequence "[a, b]", quotes
   removed.  out: cap bytes, NUL-terminated (may be NULL to ask for *len); *len = text length.
   FM3D_ERR_PARSE: the file cannot be read; FM3D_ERR_INVALID: no such key (or a map node). */
int fm3d_settings_lookup(const char *path, const char *key, char *out, int cap, int *len);
int fm3d_ctx_create(const fm3d_settings *s, int device, fm3d_ctx **out);
void fm3d_ctx_destroy(fm3d_ctx *ctx);
const char *fm3d_last_error(const fm3d_ctx *ctx);
/* use an external hipStream_t (e.g. torch.cuda.current_stream().cuda_stream); NULL = own stream */
int fm3d_ctx_set_stream(fm3d_ctx *ctx, void *hip_stream);

/* ---------------- DescriptorsMatcher ---------------- */
/* knnMatch(A, B, k=2) of DescriptorsMatcher::compare (descriptorsmatcher.cpp:89-105), exact
   brute force in (distance, trainIdx) order.  out: nA*2 entries, trainIdx -1 when nB < 2. */
int fm3d_knn2(fm3d_ctx *ctx, const void *descA, int nA, const void *descB, int nB, int dim, int type,
              fm3d_dmatch *out);
/* matcher + NNDR of DescriptorsMatcher::compareWithNNDR (descriptorsmatcher.cpp:117-129):
   keep m[0] iff two neighbours exist and m[0].distance <= epsilon * m[1].distance.
   matches: capacity nA, written in query order; *nMatches = count. */
int fm3d_match_nndr(fm3d_ctx *ctx, const void *descA, int nA, const void *descB, int nB, int dim, int type,
                    double epsilon, fm3d_dmatch *matches, int *nMatches);

/* ---------------- SingleCameraTriangulator ---------------- */
/* setg12 (singlecameratriangulator.cpp:123-143): g12 = gIC^-1 g2^-1 g1 gIC, row-major 4x4 */
int fm3d_setg12(fm3d_ctx *ctx, const double T1[3], const double T2[3], const double r1[3], const double r2[3],
                double g12[16]);
/* context-free versions of the two above (pure host algebra, usable without a GPU) */
int fm3d_g12_from_poses(const fm3d_settings *s, const double T1[3], const double T2[3], const double r1[3],
                        const double r2[3], double g12[16]);
int fm3d_camera2_from_g12(const double g12[16], double R2[9], double t2[3]);
/* install a g12 computed elsewhere */
int fm3d_set_g12(fm3d_ctx *ctx, const double g12[16]);
/* R2, t2 that projectPointsToImage2 projects with: Rodrigues(Rodrigues^-1(R12)), t12 (:591-602) */
int fm3d_get_camera2(const fm3d_ctx *ctx, double R2[9], double t2[3]);
/* setKeypoints (:145-171) + triangulate (:173-230).  points: capacity 3*nMatches (compacted,
   match order); inlierMask: nMatches bytes (the outliersMask). */
int fm3d_triangulate(fm3d_ctx *ctx, const fm3d_point2f *kpts1, int n1, const fm3d_point2f *kpts2, int n2,
                     const fm3d_dmatch *matches, int nMatches, double *points, uint8_t *inlierMask, int *nPoints);

/* ---------------- NormalOptimizer ---------------- */
/* setImages (normaloptimizer.cpp:191-221): 8-bit gray images, builds both pyramids */
int fm3d_set_images(fm3d_ctx *ctx, const uint8_t *img1, const uint8_t *img2, int width, int height, int stride);
/* copy pyramid level `level` of image `which` (1 or 2) to host; *w,*h receive its size */
int fm3d_get_pyramid_level(const fm3d_ctx *ctx, int which, int level, uint8_t *out, int *w, int *h);
/* computeOptimizedNormals (normaloptimizer.cpp:321-452).  points: in/out, 3*P doubles, compacted
   in place to the kept points (reference erase semantics); normals: capacity 3*P; status: P
   codes per INPUT point (may be NULL); info/nfev: 8 ints per input point (lmdif info and
   evaluation count per pyramid level, may be NULL). */
int fm3d_optimize_normals(fm3d_ctx *ctx, double *points, int P, double *normals, int32_t *status,
                          int32_t *info, int32_t *nfev, int *nKept, fm3d_lm_stats *stats);

/* NCC scoring of Hphi x Htheta candidate normals per point (BASELINE.json's "patch NCC over 16 / 32
   normal hypotheses"; the reference has no such search -- SURVEY.md D2 -- so this is an extension on
   the reference's evaluateNormal geometry, normaloptimizer.cpp:65-149): normals sph2car(phi0 + dphi,
   theta0 + dtheta) on a grid of half width span (radians) around car2sph(X/|X|), scored by the NCC of
   the pyramid-level-0 image-1 samples of the extractPixelsContour neighbourhood and the image-2
   samples through each normal's plane (-2: a pixel fails the bounding box / isPixelGood, or a flat
   patch).  Needs fm3d_set_images and the camera-2 pose (fm3d_set_g12).  scores: P x H doubles
   (hypothesis h = iphi*Htheta + itheta); normals: P x 3, the best scoring normal (lowest h on ties;
   the initial guess if none scores); best: P (-1 if none).  H <= 32. */
int fm3d_ncc_hypotheses(fm3d_ctx *ctx, const double *points, int P, int Hphi, int Htheta, double span, double *scores,
                        double *normals, int32_t *best);

/* ---------------- feature frames + patch export (after the hot path) ---------------- */
/* gravity_ of the NormalOptimizer ctor (normaloptimizer.cpp:160-178):
   Rodrigues(rodriguesIC).inv() * (0, 0, -1) */
int fm3d_gravity(const fm3d_settings *s, double g[3]);
/* computeFeaturesFrames (normaloptimizer.cpp:454-504): one row-major 4x4 frame per (point, normal),
   frames: 16*P doubles */
int fm3d_features_frames(fm3d_ctx *ctx, const double *points, const double *normals, int P, double *frames);
/* numberOfPointsPerEdge of getReferenceSquaredNeighborhood (neighborhoodsgenerator.cpp:134-158):
   2*floor(epsilon / (0.01*cmPerPixel)) -- 128 with build/settings.yml */
int fm3d_patch_size(const fm3d_settings *s);
/* getReferenceSquaredNeighborhood + projectReferencePointsToImageWithFrames
   (singlecameratriangulator.cpp:769-849) on image 1 of fm3d_set_images: per frame a size x size
   8-bit patch, patches[f][j][i] = sample of reference point (i, j) (the reference's transposed
   patch.at<uchar>(col, row)); imagePoints (may be NULL): 2*size*size doubles per frame, point order
   i*size + j.  patches: P*size*size bytes. */
int fm3d_export_patches(fm3d_ctx *ctx, const double *frames, int P, uint8_t *patches, double *imagePoints);
/* NeighborhoodsGenerator::computeSquareNeighborhoodsByNormals (neighborhoodsgenerator.cpp:76-132,
   called at main.cpp:187): per frame the size x size square grid (-eps + inc*i, -eps + inc*j, 0),
   inc = 0.01*cmPerPixel, transformed by the frame (Matx44d * Vec4d; scaled by 1/w when w != 1).
   out: P*size*size*3 doubles, point order i*size + j (host buffer; computed in HBM in chunks). */
int fm3d_square_neighborhoods(fm3d_ctx *ctx, const double *frames, int P, double *out);
/* NeighborhoodsGenerator::computeCircularNeighborhoodsByNormals (neighborhoodsgenerator.cpp:160-224;
   the single-point computeCircularNeighborhoodByNormal :226-277 is P = 1): per point thetas*rays
   samples X + r_i*(s + (W s) sin t_j + 2 sin^2(t_j/2) (W W s)) with the constructor's lookup table
   (:50-64), s = epsilon*(0, 1, -n1/n2)/|(0, 1, -n1/n2)|, W = skew(n), in Matx / Vec operation order.
   points: P*3 doubles (the reference's 3 x N Mat, transposed); normals: P*3 doubles, or NULL for the
   initial guess X/|X| (the reference's empty-normals branch, :167-183).  out: P*thetas*rays*3
   doubles, sample order (ray outer, angle inner).  FM3D_ERR_INVALID unless neighMethod is circular
   (the reference constructor reads thetas / rays only then). */
int fm3d_circular_neighborhoods(fm3d_ctx *ctx, const double *points, const double *normals, int P, double *out);

/* ---------------- feature detection + description (SURF, OpenCV 2.4 nonfree) ---------------- */
/* FeatureDetector::detect of the settings' SURF detector (descriptorsmatcher.cpp:110-111 via
   generateDetector :176-293): fastHessianDetector + the SURFInvoker pass (Upright 1: angle 270;
   Upright 0: the dominant orientation, keypoints without one removed), keypoints in KeypointGreater
   order (response, size, octave, y, x descending).  *n = all keypoints found; the first min(*n, cap)
   are written to kpts.  desc (may be NULL): their descriptors too (the extractor's compute on the
   same image, :113-114), min(*n, cap) x (surfExtended ? 128 : 64) floats.
   FM3D_ERR_UNSUPPORTED unless detector (and, with desc, extractor) is SURF. */
int fm3d_surf_detect(fm3d_ctx *ctx, const uint8_t *img, int width, int height, fm3d_keypoint *kpts, int cap, int *n,
                     float *desc);
/* DescriptorExtractor::compute of the settings' SURF extractor for given keypoints (:113-114,
   extractDescriptorsFromPatches :133-174): keypoints whose 2*round(2s) wavelet does not fit the
   image are removed, the others get angle 270 (upright).  kout / kept (input index of each kept
   keypoint, may be NULL): capacity n; desc: n x (128 | 64) floats; *nOut = kept count. */
int fm3d_surf_compute(fm3d_ctx *ctx, const uint8_t *img, int width, int height, const fm3d_keypoint *kpts, int n,
                      fm3d_keypoint *kout, int32_t *kept, int *nOut, float *desc);

/* DescriptorsMatcher::extractDescriptorsFromPatches (descriptorsmatcher.cpp:133-174): per square
   patch (P x size x size bytes, e.g. the fm3d_export_patches output) one keypoint at
   (floor(size/2), floor(size/2)) of size `size`, angle -1, octave 0, described by the settings' SURF
   extractor (P x (128 | 64) floats) or SIFT extractor (P x 128 floats: the patch's own firstOctave-0
   level 0, as SIFT::operator() with that keypoint builds it); the reference's descriptors Mat, one
   row per patch. */
int fm3d_extract_descriptors_from_patches(fm3d_ctx *ctx, const uint8_t *patches, int P, int size, float *desc);
/* The same for any extractor of the settings, rows laid out as fm3d_descriptor_info says: SURF / SIFT
   as above (floats), ORB (32 bytes) and BRISK (64 bytes) per patch through their compute on the patch
   (fm3d_orb_compute / fm3d_brisk_compute).  A patch whose keypoint the extractor drops keeps a zero
   row, as the reference's Mat::zeros + copyTo of an empty row leaves it (BRISK drops every centred
   patch keypoint: its pattern reaches ~1.5 x size); FM3D_ERR_INVALID when the first patch's row is
   dropped by ORB (the reference's matrix would have 0 columns). */
int fm3d_extract_descriptors_from_patches_any(fm3d_ctx *ctx, const uint8_t *patches, int P, int size, void *desc);

/* ---------------- feature detection + description (ORB, OpenCV 2.4) ---------------- */
/* FeatureDetector::detect of the settings' ORB detector (descriptorsmatcher.cpp:273-279:
   cv::ORB(orbNumFeatures, orbScaleFactor, orbNumLevels), edgeThreshold / patchSize orbEdgeThreshold /
   orbPatchSize, FAST threshold orbFastThreshold): level-major keypoints (FAST + Harris retainBest
   per level, IC_Angle orientation), positions scaled to the image.  *n = all; min(*n, cap) written.
   desc (may be NULL): ORB::operator()'s descriptors of the same call, min(*n, cap) x 32 bytes (the
   reference computes them with a separate compute, fm3d_orb_compute, whose float round trip of the
   positions can move them by an ulp).  FM3D_ERR_UNSUPPORTED unless the detector is ORB. */
int fm3d_orb_detect(fm3d_ctx *ctx, const uint8_t *img, int width, int height, fm3d_keypoint *kpts, int cap, int *n,
                    uint8_t *desc);
/* DescriptorExtractor::compute of the settings' ORB extractor (descriptorsmatcher.cpp:113-114,
   336-341): size < FLT_EPSILON and the orbEdgeThreshold border (rounded positions) removed, the rest
   grouped by octave (level-major, input order within a level) and described on the blurred level
   of their octave.  kout / kept (input index, may be NULL): capacity n; desc: n x 32 bytes; *nOut =
   kept count.  FM3D_ERR_INVALID for a kept keypoint with a negative octave. */
int fm3d_orb_compute(fm3d_ctx *ctx, const uint8_t *img, int width, int height, const fm3d_keypoint *kpts, int n,
                     fm3d_keypoint *kout, int32_t *kept, int *nOut, uint8_t *desc);
/* the 512 rBRIEF test points (x, y interleaved): OpenCV's bit_pattern_31_ for patchSize 31 is not
   part of this library -- pass it here for descriptor parity with OpenCV; NULL restores the default,
   makeRandomPattern(orbPatchSize) (cv::RNG(0x34985739), OpenCV's pattern for every other patchSize). */
int fm3d_orb_set_pattern(fm3d_ctx *ctx, const int32_t *xy, int npoints);

/* ---------------- feature detection + description (SIFT, OpenCV 2.4 nonfree) ---------------- */
/* FeatureDetector::detect of the settings' SIFT detector (descriptorsmatcher.cpp:243-251:
   cv::SIFT(siftNumFeatures, siftOctaveLayers, siftContrastThreshold, siftEdgeThreshold, siftSigma)):
   the doubled-image scale space, DoG extrema in scan order (octave, layer, row, column), one keypoint
   per orientation peak, removeDuplicated, retainBest(NumFeatures) when > 0; octave codes and
   positions as OpenCV returns them (octave -1 = the doubled image).  *n = all; min(*n, cap) written.
   desc (may be NULL): the extractor's compute on the same image (:113-114, 302-310), min(*n, cap) x
   128 floats holding integers 0..255.  FM3D_ERR_UNSUPPORTED unless the detector (and, with desc, the
   extractor) is SIFT, or when a blur needs more than 65 taps (sigma above ~8). */
int fm3d_sift_detect(fm3d_ctx *ctx, const uint8_t *img, int width, int height, fm3d_keypoint *kpts, int cap, int *n,
                     float *desc);
/* DescriptorExtractor::compute of the settings' SIFT extractor (:113-114, 302-310): keypoints with
   size < FLT_EPSILON removed (input order kept), the rest described on the pyramid of firstOctave =
   min(0, their octaves).  kout / kept (input index, may be NULL): capacity n; desc: n x 128 floats;
   *nOut = kept count.  FM3D_ERR_INVALID for an octave below -1, a layer above NumOctaveLayers + 2 or an
   octave the image cannot hold (OpenCV asserts there). */
int fm3d_sift_compute(fm3d_ctx *ctx, const uint8_t *img, int width, int height, const fm3d_keypoint *kpts, int n,
                      fm3d_keypoint *kout, int32_t *kept, int *nOut, float *desc);
/* the scale space SIFT builds (cv::SIFT::buildGaussianPyramid / buildDoGPyramid, public in OpenCV 2.4):
   firstOctave -1 (doubled) or 0, nOctaves octaves of NumOctaveLayers + 3 Gaussian levels (dog 0) or
   NumOctaveLayers + 2 DoG levels (dog 1), concatenated octave-major.  *total = floats; sizes (may be
   NULL): (w, h) per level; out (may be NULL to ask for the sizes): *total floats. */
int fm3d_sift_pyramid(fm3d_ctx *ctx, const uint8_t *img, int width, int height, int firstOctave, int nOctaves, int dog,
                      float *out, int32_t *sizes, int64_t *total);

/* ---------------- any detector / extractor of the settings ---------------- */
/* cv::FastFeatureDetector(threshold, nonmax).detect (descriptorsmatcher.cpp:215-222): FAST-9 on the
   image, KeyPoint(x, y, 7, -1, score) in raster order (score 0 without non-max suppression). */
int fm3d_fast_detect(fm3d_ctx *ctx, const uint8_t *img, int width, int height, int threshold, int nonmax,
                     fm3d_keypoint *kpts, int cap, int *n);
/* descriptor_extractor_->compute(img, kpts, desc) of the settings' BRISK extractor
   (descriptorsmatcher.cpp:343-348: cv::BRISK(Threshold, Octaves); OpenCV 2.4.9 brisk.cpp, the default
   pattern, no orientation step for given keypoints): keypoints of size < FLT_EPSILON and those within
   the pattern's reach of the border dropped (order kept; kept[] = input index, may be NULL), then 64
   bytes (512 bits) per kept keypoint. */
int fm3d_brisk_compute(fm3d_ctx *ctx, const uint8_t *img, int width, int height, const fm3d_keypoint *kpts, int n,
                       fm3d_keypoint *kout, int32_t *kept, int *nOut, uint8_t *desc);
/* descriptor_extractor_->compute(img, kpts, desc) of the settings' FREAK extractor
   (descriptorsmatcher.cpp:350-353: cv::FREAK() -- orientation and scale normalised, patternScale 22,
   4 octaves; OpenCV 2.4.9 freak.cpp): keypoints of size < FLT_EPSILON and those within their scale's
   pattern size of the border dropped (order kept; kept[] = input index, may be NULL), kout's angle set
   to FREAK's orientation, then 64 bytes (512 bits, the SSE2 build's bit order) per kept keypoint. */
int fm3d_freak_compute(fm3d_ctx *ctx, const uint8_t *img, int width, int height, const fm3d_keypoint *kpts, int n,
                       fm3d_keypoint *kout, int32_t *kept, int *nOut, uint8_t *desc);
/* the 512 selected pairs, as indices into the 903 pairs (i, j < i) of the 43 pattern points in
   generation order: OpenCV's FREAK::DEF_PAIRS is restated in include/fm3d_freak.h (unverified: OpenCV
   is not in this image) -- pass OpenCV's own table here for parity with it; NULL restores the default. */
int fm3d_freak_set_pairs(fm3d_ctx *ctx, const int32_t *pairs, int n);
/* cv::StarFeatureDetector(maxSize, response, lineThreshold, lineBinarized, suppression).detect
   (descriptorsmatcher.cpp:204-213; OpenCV 2.4.9 StarDetector, CenSurE): KeyPoint(x, y, size, -1,
   response) in tile order.  FM3D_ERR_INVALID where OpenCV's result is undefined (min(w, h) <= 6,
   maxSize > 128, suppression / 2 beyond the pattern border). */
int fm3d_star_detect(fm3d_ctx *ctx, const uint8_t *img, int width, int height, int maxSize, int response,
                     int lineThreshold, int lineBinarized, int suppression, fm3d_keypoint *kpts, int cap, int *n);
/* StarDetectorComputeResponses (the step fm3d_star_detect starts with): per pixel the float response and
   the signed pattern size (0 in the border), w*h each; *border the pattern border. */
int fm3d_star_responses(fm3d_ctx *ctx, const uint8_t *img, int width, int height, int maxSize, float *resp,
                        int16_t *sizes, int *border);
/* cv::MserFeatureDetector(delta, minArea, maxArea, maxVariation, minDiversity, ...).detect
   (descriptorsmatcher.cpp:258-272; OpenCV 2.4.9 mser.cpp on a grey image): per maximally stable region
   (pass 1 on 255 - I, then pass 2 on I, each in the flood's order) KeyPoint(centre, sqrt(w * h)) of its
   fitEllipse, kept when the diameter exceeds FLT_EPSILON and the rounded centre is inside the image
   (angle -1, response 0).  FM3D_ERR_INVALID where OpenCV throws (a region under 5 points, MinArea < 4).
   Each flood pass is sequential by construction (its order is part of the output) and runs as one GPU
   lane; fitEllipse runs one wave per region (fm3d_mser_detect_batch: many images at once). */
int fm3d_mser_detect(fm3d_ctx *ctx, const uint8_t *img, int width, int height, int delta, int minArea, int maxArea,
                     double maxVariation, double minDiversity, fm3d_keypoint *kpts, int cap, int *n);
/* fm3d_mser_detect on `count` images of width x height stored one after the other (the reference's
   detect(image_a), detect(image_b) of descriptorsmatcher.cpp:77-78 in one call): every image's two
   floods run side by side (one workgroup each), so a batch takes about the time of one image.  The
   keypoints of image 0, then image 1, ... (each exactly fm3d_mser_detect's); counts[i] = image i's,
   *total = all; min(*total, cap) written.  FM3D_ERR_INVALID as fm3d_mser_detect for any image. */
int fm3d_mser_detect_batch(fm3d_ctx *ctx, const uint8_t *imgs, int count, int width, int height, int delta,
                           int minArea, int maxArea, double maxVariation, double minDiversity, fm3d_keypoint *kpts,
                           int cap, int32_t *counts, int *total);
/* MSER::operator()(img, msers): *nRegions regions, color[i] -1 (pass 1) or +1, count[i] points, the
   points (x, y) concatenated in pts in each region's list order (MSERToContour); *nPoints = all points.
   min(regions, cap) and min(points, ptsCap) written. */
int fm3d_mser_regions(fm3d_ctx *ctx, const uint8_t *img, int width, int height, int delta, int minArea, int maxArea,
                      double maxVariation, double minDiversity, int32_t *color, int32_t *count, int cap, int32_t *pts,
                      int64_t ptsCap, int *nRegions, int64_t *nPoints);
/* feature_detector_->detect(img, kpts) of generateDetector (descriptorsmatcher.cpp:110-111, 176-293):
   STATIC SURF / ORB / SIFT / FAST / STAR / MSER, or ADAPTIVE with the FAST, SURF or STAR adjuster (the
   threshold walk of DynamicAdaptedFeatureDetector).  *n = all; min(*n, cap) written.
   FM3D_ERR_UNSUPPORTED for a type the reference does not build (FM3D_FEAT_OTHER). */
int fm3d_detect(fm3d_ctx *ctx, const uint8_t *img, int width, int height, fm3d_keypoint *kpts, int cap, int *n);
/* the row layout of the settings' extractor: SURF 64 | 128 and SIFT 128 (FM3D_DESC_F32), ORB 32 bytes,
   BRISK and FREAK 64 bytes (FM3D_DESC_BITS). */
int fm3d_descriptor_info(const fm3d_ctx *ctx, int *cols, int *type);
/* descriptor_extractor_->compute(img, kpts, desc) of generateExtractor (:113-114, 295-359): the
   settings' SURF / SIFT / ORB extractor on any keypoints (fm3d_surf_compute / fm3d_sift_compute /
   fm3d_orb_compute); desc: n rows of fm3d_descriptor_info's layout. */
int fm3d_compute(fm3d_ctx *ctx, const uint8_t *img, int width, int height, const fm3d_keypoint *kpts, int n,
                 fm3d_keypoint *kout, int32_t *kept, int *nOut, void *desc);

/* ---------------- the whole hot path, device resident ---------------- */
/* Stage inputs in HBM (H2D once).  queryOffset is added to queryIdx (sharding).
   type FM3D_DESC_F32 (the float cv::Mat rows knnMatch receives, descriptorsmatcher.cpp:114-117): the
   rows go to the device as they are and a kernel checks them; rows that hold integers in [0, 255]
   (SIFT) are packed to u8 on the device and take the exact u8 matcher (same ranking and distances),
   others the float matchers.  This choice costs the call one wait for its own copies.
   img1 = img2 = NULL: no images (C2's match + DLT needs none; the context keeps earlier ones, and
   the full path fails without any). */
int fm3d_pipeline_upload(fm3d_ctx *ctx, const void *descA, int nA, const void *descB, int nB, int dim, int type,
                         const fm3d_point2f *kpts1, const fm3d_point2f *kpts2, const uint8_t *img1,
                         const uint8_t *img2, int width, int height, int queryOffset);
/* Run match -> NNDR -> triangulate -> pyramids -> LM normals on the staged inputs.
   recordsDev: device buffer with capacity nA records (NULL: internal); *nKept: survivors.
   Synchronises the context stream before returning. */
int fm3d_pipeline_run(fm3d_ctx *ctx, fm3d_record *recordsDev, int *nKept, fm3d_pipeline_stats *stats);
/* The same path for a stream of frame pairs (a serving loop keeps two contexts, i.e. two pairs, in
   flight): fm3d_pipeline_submit stages one frame pair's inputs through page-locked buffers (H2D of
   descriptors, keypoints and images, the pyramids) and queues match -> NNDR -> triangulate -> LM
   normals -> survivor records on the context stream, then returns without waiting: every count
   stays on the device and sizes nothing the host launches.  fm3d_pipeline_wait waits for it and
   copies the survivor records to out (host, capacity cap; may be NULL); stats.pyramid_ms = the
   inputs' H2D + pyramids, total_ms = submit to results.  One submit per context may be pending; the
   other pipeline calls on that context fail with FM3D_ERR_INVALID until it is waited for. */
int fm3d_pipeline_submit(fm3d_ctx *ctx, const void *descA, int nA, const void *descB, int nB, int dim, int type,
                         const fm3d_point2f *kpts1, const fm3d_point2f *kpts2, const uint8_t *img1,
                         const uint8_t *img2, int width, int height, int queryOffset);
int fm3d_pipeline_wait(fm3d_ctx *ctx, fm3d_record *out, int cap, int *nKept, fm3d_pipeline_stats *stats);
/* Join contexts' LM launches (same device, camera and LM settings; up to 3 members per leader):
   after the link a submit on `member` queues its pair's front half only, and the next submit on
   `leader` queues ONE LM launch over its pair's and every queued member pair's points -- the
   workgroups whose slots run out of one pair's points take the next's, so the pairs fill each
   other's end-of-queue tail -- followed by each pair's records on its own stream.  A member waited
   for before its leader's next submit runs its LM alone.  Each pair's results are those of its own
   fm3d_pipeline_run, bit for bit.  fm3d_pipeline_run and the other calls of a linked context run
   unlinked. */
int fm3d_pipeline_link(fm3d_ctx *member, fm3d_ctx *leader);
/* BASELINE.json's C2 ("brute-force L2 match + DLT triangulate only"): match -> NNDR -> triangulate on
   the staged inputs, no normals; *nInliers = the triangulated points kept by the z filter (stats:
   match / NNDR-compaction / triangulate / total HIP-event times). */
int fm3d_pipeline_run_dlt(fm3d_ctx *ctx, int *nInliers, fm3d_pipeline_stats *stats);
/* fm3d_pipeline_run_dlt as submit / wait (a serving loop keeps two contexts in flight): submit queues the
   staged pair's front half (match -> NNDR -> compaction -> DLT -> compaction) on the context stream with
   its counts copied to page-locked memory and returns; wait blocks on that copy and reports as
   fm3d_pipeline_run_dlt.  Until the wait the other pipeline calls on the context fail. */
int fm3d_pipeline_submit_dlt(fm3d_ctx *ctx);
int fm3d_pipeline_wait_dlt(fm3d_ctx *ctx, int *nInliers, fm3d_pipeline_stats *stats);
/* fm3d_pipeline_upload (no images) + fm3d_pipeline_submit_dlt in one call that never waits for the
   device: a serving loop of C2 from host memory overlaps one context's staging copy with another's
   DMA.  Float rows (FM3D_DESC_F32) are packed on the device and matched as u8 rows before their
   "integer-valued" flag is read; fm3d_pipeline_wait_dlt reads it and, for rows that are not, runs the
   front half again on the float rows, so the results are always those of fm3d_pipeline_upload +
   fm3d_pipeline_run_dlt.  The arrays are copied before it returns.  (Round 6.) */
int fm3d_pipeline_submit_dlt_pair(fm3d_ctx *ctx, const void *descA, int nA, const void *descB, int nB, int dim,
                                  int type, const fm3d_point2f *kpts1, const fm3d_point2f *kpts2, int queryOffset);
/* after fm3d_pipeline_run(_dlt): the compacted matches (K), the inlier points (P x 3 doubles, the
   z-filtered triangulation in match order) and each point's match index (P); any may be NULL */
int fm3d_pipeline_dlt_download(fm3d_ctx *ctx, fm3d_dmatch *matches, double *points, int32_t *matchIdx);
/* BASELINE.json's C3 as worded ("Hamming popcount match + 64x64 patch NCC over 16 normal hypotheses"):
   match -> NNDR -> triangulate, then fm3d_ncc_hypotheses' scoring of every inlier on the device
   (pixelsRay 32 gives the 64 x 64 neighbourhood); *nPoints = inliers scored; stats.lm_ms is the NCC
   kernel's time.  Needs the camera-2 pose (fm3d_set_g12).  Results via fm3d_pipeline_ncc_download
   (scores P x H, best normals P x 3, best index P; any may be NULL). */
int fm3d_pipeline_run_ncc(fm3d_ctx *ctx, int Hphi, int Htheta, double span, int *nPoints, fm3d_pipeline_stats *stats);
/* fm3d_pipeline_run_ncc split for serving (as fm3d_pipeline_submit_dlt / wait_dlt): submit queues the
   front half and the NCC scoring on the context stream and returns; wait blocks on the counts' copy
   and reports as run_ncc.  Until the wait the other pipeline calls on the context fail. */
int fm3d_pipeline_submit_ncc(fm3d_ctx *ctx, int Hphi, int Htheta, double span);
int fm3d_pipeline_wait_ncc(fm3d_ctx *ctx, int *nPoints, fm3d_pipeline_stats *stats);
int fm3d_pipeline_ncc_download(fm3d_ctx *ctx, double *scores, double *normals, int32_t *best);
/* copy n records from a device record buffer (NULL = internal) to host */
int fm3d_records_download(fm3d_ctx *ctx, const fm3d_record *recordsDev, int n, fm3d_record *out);

/* ---------------- several GPUs of one node, one process ---------------- */
/* The reference runs main.cpp:91-155 in one process on one device; these calls are the same
   pipeline over ndev devices.  The queries split into `shares` logical shares (blocks of `block`
   queries, 0 = 4096, dealt round-robin; share s belongs to devices[s % ndev], shares >= ndev).  Each
   device holds ONE replica -- its shares' queries gathered in increasing order, frame B, its
   keypoints and both images, staged once -- and runs the whole path over them in one pass (one LM
   launch); the survivor counts and 64-byte records are all-gathered with RCCL over xGMI
   (ncclCommInitAll, ncclAllGather, queued behind each device's records); the host merge returns the
   records in query order, byte-identical to fm3d_pipeline_run of the whole frame pair.  devices may
   be NULL (0..ndev-1); FM3D_ERR_INVALID when a device index is not visible (fewer GPUs than asked
   for) or repeats; FM3D_ERR_UNSUPPORTED when RCCL (librccl.so.1) cannot be loaded.
   Memory pre-flight: fm3d_mgpu_create checks every device's free memory (hipMemGetInfo) for the LM
   slabs of its four context sets, and the first upload / submit of a larger frame pair for the
   per-pair buffers and exchange slots, before anything grows: too little is FM3D_ERR_NOMEM with the
   shortfall in the error text (fm3d_mgpu_last_error(NULL) after a failed create), never an
   allocation failure in the middle of a run.  The merge is linear (blocks in order, no sort). */
typedef struct fm3d_mgpu fm3d_mgpu;
/* the GPUs visible to this process (hipGetDeviceCount; 0 when HIP finds none): what a multi-GPU
   host checks before fm3d_mgpu_create, without loading another runtime (bench.py --gpus N) */
int fm3d_device_count(int *n);
int fm3d_mgpu_create(const fm3d_settings *s, int ndev, const int *devices, int shares, int block, fm3d_mgpu **out);
void fm3d_mgpu_destroy(fm3d_mgpu *m);
const char *fm3d_mgpu_last_error(const fm3d_mgpu *m);
/* setg12 result for every device (else each device uses the settings' pos1 / pos2) */
int fm3d_mgpu_set_g12(fm3d_mgpu *m, const double g12[16]);
int fm3d_mgpu_pipeline_upload(fm3d_mgpu *m, const void *descA, int nA, const void *descB, int nB, int dim, int type,
                              const fm3d_point2f *kpts1, const fm3d_point2f *kpts2, const uint8_t *img1,
                              const uint8_t *img2, int width, int height);
/* out: host buffer, capacity nA records; stats: counts summed over the devices, total_ms / lm_ms =
   the slowest device's */
int fm3d_mgpu_pipeline_run(fm3d_mgpu *m, fm3d_record *out, int *nKept, fm3d_pipeline_stats *stats);
/* A stream of frame pairs over the devices (up to four in flight, as fm3d_pipeline_submit / _wait
   on one GPU, two pairs per LM launch through fm3d_pipeline_link): submit stages one frame pair on
   every device (host-asynchronous, one host thread per device) and queues its path and all-gather;
   wait returns the oldest submitted pair's merged records (out: capacity cap).  Pairs in flight
   together must have the same query count. */
int fm3d_mgpu_submit(fm3d_mgpu *m, const void *descA, int nA, const void *descB, int nB, int dim, int type,
                     const fm3d_point2f *kpts1, const fm3d_point2f *kpts2, const uint8_t *img1, const uint8_t *img2,
                     int width, int height);
int fm3d_mgpu_wait(fm3d_mgpu *m, fm3d_record *out, int cap, int *nKept, fm3d_pipeline_stats *stats);
/* the block-cyclic partition: global query indices of share s (increasing); idx NULL asks for *n */
int fm3d_share_queries(int nA, int shares, int s, int block, int32_t *idx, int cap, int *n);
/* the merge (host only, no GPU): recs[s] holds counts[s] records of share s with LOCAL query
   indices (positions in share s's query list, increasing); out (capacity nA) receives them with
   global indices in query order.  FM3D_ERR_INVALID on a local index outside the share or out of
   order. */
int fm3d_merge_shares(int nA, int shares, int block, const fm3d_record *const *recs, const int *counts,
                      fm3d_record *out, int *nOut);

/* ---------------- building blocks exposed for tests ---------------- */
/* cv::pyrDown of one 8-bit image (normaloptimizer.cpp:216-217) */
int fm3d_pyrdown(fm3d_ctx *ctx, const uint8_t *src, int width, int height, uint8_t *dst);
/* extractPixelsContour(Vec3d) (:376-397): kept pixel coordinates (2*cap doubles), returns m via *m */
int fm3d_neighborhood(fm3d_ctx *ctx, const double X[3], double *xy, int cap, int *m);
/* extractPixelsContour(X) (singlecameratriangulator.cpp:341-397) and the level-0 geometry of one
   evaluateNormal call through the plane (X, n) -- get3dPointsFromImage1Pixels (:530-574) +
   projectPointsToImage2 (:591-626) at scale 1 -- on the device: what the reference's image2pixels
   drawing code paints (normaloptimizer.cpp:421-445).  Uses the context's camera, pixelsRay,
   bounds, zThresholdMax and camera-2 pose.  xy / uv: 2*cap doubles (image-1 pixel, image-2
   projection), status: cap codes (0, FM3D_ST_NAN_PLANE, FM3D_ST_ABORT_BBOX, FM3D_ST_ABORT_PIX2
   against the fm3d_set_images size); any may be NULL.  *m = kept pixels (m_dat). */
int fm3d_plane_to_image2(fm3d_ctx *ctx, const double X[3], const double n[3], double *xy, double *uv, int32_t *status,
                         int cap, int *m);
/* cv::undistortPoints of n pixel coordinates (device kernel) */
int fm3d_undistort(fm3d_ctx *ctx, const double *xy, int n, double *out);

/* library version string */
const char *fm3d_version(void);

#ifdef __cplusplus
}
#endif
#endif /* FM3D_H */
