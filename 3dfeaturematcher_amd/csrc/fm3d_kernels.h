// fm3d_kernels.h -- kernel parameter blocks and host-side launchers.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fm3d.h"
#include "fm3d_device.h"

// LM ray slab layout: 1 = one (ux, uy) record of 16 bytes per entry (one 16-byte load per
// entry), 0 = separate ux and uy arrays (two 8-byte loads; round 2's first layout).  Same-box
// A/B at C4 (profiles/r02_lm_ray_aos_ab.json): with the single-evaluation passes' slab bases
// in scalar registers (FM3D_EVAL_HOIST), 3.6 % fewer cycles per single-evaluation pass (launch
// within box noise, 0.5-1.2 % fewer cycles), bit-identical records.
#ifndef FM3D_RAY_AOS
#define FM3D_RAY_AOS 1
#endif

namespace fm3d {

struct LevelDesc {
    const uint8_t* img1;  // pyramid level of image 1 (+ zero guard)
    const uint8_t* img2;
    int w, h;
};

// camera-2 projection constants (projectPointsToImage2, singlecameratriangulator.cpp:591-644)
struct ProjConst {
    double R[9], t[3];
    Camera cam;
    // LM slab array bases (grid-uniform): the summed passes re-read them per chunk
    // with scalar loads and address entries by one 32-bit byte offset
    const char *slabRX, *slabRY, *slabI1;
    char *slabDF, *slabDJ0, *slabDJ1;
    // 2 k[2], 2 k[3] (exact): the tangential 2xy terms as (2k) RN(xy), the same bits as k RN(2xy)
    double k2d, k3d;
};

// one frame pair's points in an LM launch (a launch may take the points of several: the slots
// of a workgroup whose first pair runs dry take the next pair's points)
struct LMProblem {
    const double* points;     // P x 3
    const int* Pdev;          // the point count on the device (may be null: P)
    const LevelDesc* lvl;     // its pyramids, levels+1 entries
    double* normals;          // P x 3
    int* status;              // P
    int* info;                // P x 8
    int* nfev;                // P x 8
    int* mdat;                // P
    unsigned long long* stat; // [residual evaluations, pixel evaluations] of its points
    int P;                    // points, or their bound when Pdev is set
    unsigned projOff;         // byte offset of its ProjConst (camera-2 pose) in LMParams::proj
};

struct LMParams {
    // (the field order of the single-problem layout is kept: the kernel's register allocation
    // follows the kernarg layout; points .. mdat are unused, the problem table holds them)
    const double* points_;
    int P_;
    const int* Pdev_;
    Camera cam;                 // shared by the problems (one camera)
    double R2_[9], t2_[3];
    const ProjConst* proj;      // per problem: R2, t2, cam (+ the slab bases, the same in each)
    const LevelDesc* lvl_;
    int levels;
    const int2* offsets;  // circle offsets (i, j) in reference order, padded to nOffPad
    int nOff, nOffPad;
    int boundW, boundH;
    double epsfcn;
    int cmax;
    int* queue;
    double* slab;    // rays: 2 arrays x (groups*kLM2Slots) slots x nOffPad entries
    float* slabI1;   // I1, fvec dI, 2 Jacobian dI, compact index: 5 arrays, same shape
    long nWaves;     // number of workgroups
    double* normals_;
    int* status_;
    int* info_;
    int* nfev_;
    int* mdat_;
    unsigned long long* statEval;
    unsigned long long* statPix;
    long long maxIter;       // safety bound on passes per slot
    long long maxTicks;      // safety bound on wall-clock ticks per workgroup
    int* overflow;           // set to 1 if a workgroup hit a guard
    int coop;                // 1: waves without points help busy slots (tail of the launch)
    int safe;                // 1: every pass takes the guarded (per-lane) form (tests of that form)
    // [passes, cycles terms, cycles chain, cycles control, cycles total, wall ticks sum, wall ticks
    //  max, class passes x4, class cycles x4, max start, max end, min start, ..., producer waits]
    unsigned long long* statPass;
    int nProb;                  // frame pairs of the launch (problems, <= kLMMaxProblems)
    const LMProblem* prob;      // device table
};
constexpr int kLMMaxProblems = 4;

constexpr int kLMRunning = 0x100;  // status of a point still in flight

// wave-per-point LM kernel (fm3d_lm2.hip): kLM2Slots term waves + 1 chain wave, one
// 1024-thread workgroup per CU (4 waves per SIMD; 141 KB of LDS)
constexpr int kLM2Slots = 15;
constexpr int kLM2Ring = 8;  // chunks of 64 entries in flight per slot
constexpr int kLM2Threads = 64 * (kLM2Slots + 1);
// MULTI: the problems' ProjConst entries differ (per-pass pose offset); false: entry 0 for all.
// TREE: the tree-summed reduction mode (kLM2Slots + 1 term waves, no chain wave)
template <bool MULTI, bool TREE>
__global__ void lm2_kernel(LMParams p);

// ---------------- matching ----------------
struct KnnOut {
    int* idx;       // nA x 2 train indices (-1 = none)
    int* key;       // nA x 2 ranking keys (u8: d2, bits: hamming)
    float* fkey;    // nA x 2 (f32: FLANN squared distance)
};

// u8 rows (dim padded to a multiple of 128 with value 128 on both sides -> no effect)
// u8 rows: `parts` train-tile ranges (knn2_u8_parts), merged through partIdx/partKey
int knn2_u8_parts(int nA, int nB, int nCU, int qPerBlock, int tileRows);
int knn2_i8_queries_per_block(int dimPad, int bits);
int knn2_i8_tile_rows(int dimPad, int bits);
// int8-MFMA matcher for u8 rows (bits = 0) and for 32-byte binary rows unpacked by
// launch_unpack_bits (bits = 1, dimPad 256); ctB = packed train row constants
// deferMerge: with parts > 1 the parts' lists stay in partIdx / partKey (launch_nndr_compact merges them)
void launch_knn2_i8(const uint8_t* A, int nA, const uint8_t* B, int nB, int dimPad, int bits, const int* cqA,
                    const int* ctB, int parts, int* partIdx, int* partKey, int* idx, int* key, hipStream_t s,
                    bool deferMerge = false);
// row constants of both sides: cq = |a'|^2 per query row, ctp = packed train constants
void launch_rowconst_u8(const uint8_t* A, int nA, const uint8_t* B, int nB, int dimPad, int* cq, int* ctp,
                        hipStream_t s);
// float rows (nA x dim, nB x dim) -> u8 rows padded to dimPad with 128, and *notU8 |= 1 when any element
// is not an integer in [0, 255] (the caller zeroes it; (nA + nB) * dimPad / 4 < 2^32)
void launch_f32_pack_u8(const float* A, int nA, const float* B, int nB, int dim, int dimPad, uint8_t* Au,
                        uint8_t* Bu, int* notU8, hipStream_t s);
// 32-byte binary rows -> 256 int8 (query 0/1, train -1/+1) + packed train constants popc(b)
void launch_unpack_bits(const uint8_t* A, int nA, const uint8_t* B, int nB, uint8_t* outA, uint8_t* outB, int* ctp,
                        hipStream_t s);
// f32 rows (dim 64 / 128): `parts` train ranges (knn2_parts), merged through partIdx/partKey (parts*nA*2 each)
int knn2_parts(int nA, int nB, int dim, int nCU);
size_t knn2_f32_pairs_bytes(int nB, int dim);  // the row-pair copy of B (dim 64 / 128)
void launch_knn2_f32(const float* A, int nA, const float* B, int nB, int dim, int parts, int* partIdx,
                     float* partKey, float* pairs, int* idx, float* key, hipStream_t s);
// f32 rows (dim 64 / 128) through the bf16 MFMA prefilter (fm3d_match.hip): the same top-2 and keys
// as launch_knn2_f32; work: knn2_f32_mfma_bytes(nA, nB, dim, parts) bytes of device scratch
size_t knn2_f32_mfma_bytes(int nA, int nB, int dim, int parts);
int knn2_f32_mfma_parts(int nA, int nB, int nCU);
// fused: one MFMA pass listing the rows under each lane's running bound (default); else two passes
// (the bound first, then the lists: fewer candidates per query)
void launch_knn2_f32_mfma(const float* A, int nA, const float* B, int nB, int dim, int parts, bool fused, void* work,
                          int* idx, float* key, hipStream_t s);
// the number of queries the prefilter could not settle (device int in work), and their exact rescan
int* knn2_f32_mfma_rescan_count(void* work, int nA, int nB, int dim, int parts);
void launch_knn2_f32_mfma_rescan(const float* A, const float* B, int nB, int dim, void* work, int nA, int parts,
                                 int nResc, int* idx, float* key, hipStream_t s);
// binary rows: `parts` train ranges (knn2_parts), merged through partIdx/partKey
void launch_knn2_bits(const uint8_t* A, int nA, const uint8_t* B, int nB, int dimBytes, int parts, int* partIdx,
                      int* partKey, int* idx, int* key, hipStream_t s);
// distances + NNDR flag per query; type 0 f32 keys in fkey, 1 u8, 2 bits
void launch_nndr(int type, const int* idx, const int* key, const float* fkey, int nA, int nB, double eps,
                 int queryOffset, fm3d_dmatch* knnOut, fm3d_dmatch* cand, int* flag, hipStream_t s);

// ---------------- NCC normal hypotheses (fm3d_ncc.hip) ----------------
struct NccParams {
    const double* points;  // P x 3
    int P;                 // points, or their bound when Pdev is set (one workgroup each)
    const int* Pdev;       // the point count on the device (may be null)
    Camera cam;
    double R2[9], t2[3];
    const uint8_t *img1, *img2;  // pyramid level 0 (+ zero guard)
    int w, h;
    const int2* offsets;  // circle offsets in reference order, padded
    int nOff, nOffPad, boundW, boundH, cmax;
    int Hphi, Htheta;  // hypotheses: Hphi x Htheta grid (H <= 32)
    double span;       // grid half width in radians
    double* scores;    // P x H (-2: a failing pixel or a flat patch)
    double* normals;   // P x 3 best normal (the initial guess if none scores)
    int* best;         // P (-1: none)
};
void launch_ncc_hypotheses(const NccParams& p, hipStream_t s);

// ---------------- SURF (fm3d_surf.hip) ----------------
struct SurfHF {  // a box of a resized Haar pattern: sum[p0] + sum[p3] - sum[p1] - sum[p2], weight w
    int p0, p1, p2, p3;
    float w;
};
struct SurfLayer {     // one scale-space layer (calcLayerDetAndTrace)
    long long first;   // first thread of this layer in the Hessian launch
    size_t off;        // det / trace offset of the layer (rows x cols floats)
    int size, step, margin, si, sj, rows, cols;
    SurfHF hf[10];     // Dx (3), Dy (3), Dxy (4)
};
struct SurfMid {  // a middle layer searched for maxima (findMaximaInLayer)
    long long first;
    int layer, octave, rows, cols, margin;
};
struct SurfCand {
    float x, y, size, response;
    int octave, class_id;
    long long seq;  // discovery order: (layer << 42) | (row << 21) | column
};
// SURFInvoker's orientation samples: the disc of radius 6 (x outer, y inner), Gaussian weights
constexpr int kOriMax = 128;
struct SurfOri {
    int n;
    int ax[kOriMax], ay[kOriMax];
    float w[kOriMax];
};
void launch_integral(const uint8_t* img, int w, int h, int* sum, hipStream_t s);
// nb images of w x h back to back, their (w+1) x (h+1) sums back to back
// the row pass alone: rows[(y + 1) * (w + 1) + k] = sum of image row y's first k pixels (row 0 untouched)
void launch_integral_rows(const uint8_t* img, int w, int h, int* rows, hipStream_t s);
void launch_integral_batch(const uint8_t* img, int w, int h, int nb, int* sum, hipStream_t s);
// Upright 0: flag[q] / angle[q] of keypoint q = (x, y, size) at kp + q*kstride, on the integral
// image sum + q*sumStride
void launch_surf_orient(const void* kp, size_t kstride, int n, const int* sum, size_t sumStride, int w, int h,
                        const SurfOri& ori, int* flag, float* angle, hipStream_t s);
void launch_surf_hessian(const int* sum, int w, const SurfLayer* layers, int nL, long long total, float* det,
                         float* tr, hipStream_t s);
void launch_surf_maxima(const float* det, const float* tr, const SurfLayer* layers, const SurfMid* mids, int nM,
                        long long total, float thr, SurfCand* cand, int* count, int cap, hipStream_t s);
size_t surf_sort_tmp_bytes(int n);
void launch_surf_sort(SurfCand* cand, int n, void* tmp, size_t tmpBytes, hipStream_t s);
// angle == nullptr: the upright pass (flags computed here, angle 270); else flag / angle from
// launch_surf_orient
void launch_surf_upright(const SurfCand* cand, const int* count, int n, int w, int h, int* flag, int* pos, int* total,
                         void* scanTmp, fm3d_keypoint* out, int* src, const float* angle, hipStream_t s);
void launch_surf_keep(const fm3d_keypoint* in, int n, int w, int h, int* flag, int* pos, int* total, void* scanTmp,
                      fm3d_keypoint* out, int* src, const float* angle, hipStream_t s);
void launch_surf_describe(const uint8_t* img, size_t imgStride, int w, int h, const fm3d_keypoint* kp, int n,
                          const float* DW, int extended, int upright, float* desc, hipStream_t s);

// ---------------- ORB (fm3d_orb.hip) ----------------
struct OrbLevel {     // one pyramid level, levels concatenated pixel after pixel
    int w, h;
    long long first;  // first pixel of the level in the concatenation (== its byte offset)
};
struct OrbUmax {  // computeKeyPoints' umax (halfPatchSize <= 62)
    int u[64];
};
struct OrbBlurK {  // GaussianBlur(7x7, 2): the x256 fixed-point kernel; the SSE2 column weights
    int ik[7];
    float fk[4];
};
void launch_orb_resize(const uint8_t* src, int sw, int sh, uint8_t* dst, int dw, int dh, const int* xofs,
                       const short* alpha, const int* yofs, const short* beta, int xmax, int xs, hipStream_t s);
// map: corner | score per pixel; flag: the keypoints FAST (+ non-max when nonmax) + the edge border keep
void launch_orb_fast(const uint8_t* pyr, const OrbLevel* L, int nL, long long total, int thr, int border, int nonmax,
                     uint16_t* map, int* flag, hipStream_t s);
void launch_orb_fast_scatter(const uint16_t* map, const OrbLevel* L, int nL, long long total, const int* flag,
                             const int* pos, fm3d_keypoint* out, hipStream_t s);
void launch_orb_harris(const uint8_t* pyr, const OrbLevel* L, fm3d_keypoint* kp, int n, hipStream_t s);
void launch_orb_angle(const uint8_t* pyr, const OrbLevel* L, fm3d_keypoint* kp, int n, int half, const OrbUmax& um,
                      hipStream_t s);
void launch_orb_blur(const uint8_t* pyr, const OrbLevel* L, int nL, long long total, const OrbBlurK& bk, int* R,
                     uint8_t* out, hipStream_t s);
void launch_orb_desc(const uint8_t* blur, const OrbLevel* L, const fm3d_keypoint* kp, int n, const int* pattern,
                     uint8_t* desc, hipStream_t s);

// ---------------- SIFT (fm3d_sift.hip) ----------------
struct SiftLevel {    // one pyramid level, levels concatenated float after float
    int w, h;
    long long first;  // first float of the level
};
struct SiftResize {   // createInitialImage: gray (sw x sh) -> float (dw x dh), doubled with INTER_LINEAR
    int sw, sh, dw, dh, xmax, doubled;
    double scx, scy;  // 1 / inv_scale
};
struct SiftScan {     // one DoG layer scanned by findScaleSpaceExtrema, flags concatenated
    long long first;  // first flag of the layer
    int dog, octave, layer, pad;
};
struct SiftCand {     // a scale-space extremum, then adjustLocalExtrema's keypoint
    float x, y, size, response;
    int koct;              // KeyPoint::octave: octv + (layer << 8) + (round((xi + 0.5) * 255) << 16)
    int octave, layer, r, c, ok;
};
// batch: that many equal-size images back to back (patches)
void launch_sift_init(const uint8_t* img, float* dst, const SiftResize& p, int batch, hipStream_t s);
size_t sift_blur_lds(int n);
// dst = GaussianBlur(src, taps[0..n)), dog = dst - src (dog may be null); batch images back to back
void launch_sift_blur(const float* src, float* dst, float* dog, int w, int h, const float* taps, int n, int batch,
                      hipStream_t s);
void launch_sift_down(const float* src, int sw, int sh, float* dst, int dw, int dh, double ifx, double ify,
                      hipStream_t s);
void launch_sift_extrema(const float* dog, const SiftLevel* DL, const SiftScan* S, int nS, long long total,
                         int threshold, int* flag, hipStream_t s);
void launch_sift_cand_scatter(const SiftLevel* DL, const SiftScan* S, int nS, long long total, const int* flag,
                              const int* pos, SiftCand* cand, hipStream_t s);
void launch_sift_adjust(const float* dog, const SiftLevel* DL, int L, float contrastThreshold, float edgeThreshold,
                        float sigma, SiftCand* cand, int n, hipStream_t s);
// angles: 36 per candidate (the first npk[q] are its peaks, in bin order)
void launch_sift_orient(const float* gp, const SiftLevel* GL, int L, const SiftCand* cand, int n, float* angles,
                        int* npk, hipStream_t s);
// lvl (may be null): the level of keypoint q, else its octave code's (octave - firstOctave) * (L + 3) + layer
void launch_sift_desc(const float* gp, const SiftLevel* GL, int L, int firstOctave, const fm3d_keypoint* kp,
                      const int* lvl, int n, float* desc, hipStream_t s);

// ---------------- compaction ----------------
// out[k] = in[i] for flag[i] != 0, stable; *count (device) = number kept.  tmp >= scan_tmp_bytes(n).
size_t scan_tmp_bytes(int n);
void launch_compact_dmatch(const fm3d_dmatch* in, const int* flag, int n, fm3d_dmatch* out, int* count, void* tmp,
                           hipStream_t s);
// nDev (may be null): the item count on the device, n its bound (device-sized launches: no host sync)
void launch_compact_points(const double* in, const int* flag, int n, const int* nDev, double* out, int* count,
                           int* srcIndex, void* tmp, hipStream_t s);
void launch_exclusive_scan(const int* flag, int n, int* offsets, int* total, void* tmp, hipStream_t s);

// ---------------- triangulation ----------------
struct TriParams {
    Camera cam;
    double g12[16];
    double zmin, zmax;
    const fm3d_point2f* kp1;
    const fm3d_point2f* kp2;
    const fm3d_dmatch* matches;
    int K;            // matches, or their bound when Kdev is set
    const int* Kdev;  // the match count on the device (may be null)
    int queryOffset;  // matches[].queryIdx - queryOffset indexes kp1
    double* pts;      // K x 3 (match order, not compacted)
    int* mask;        // K
    uint8_t* mask8;   // K (optional)
    int dltSolver;    // fm3d_settings.dltSolver: 0 OpenCV 2.4's cvSVD (6 x 4), 1 the round-robin 4 x 4 Jacobi
};
void launch_triangulate(const TriParams& p, hipStream_t s);

// The LM launch's resets in one kernel (it replaced eleven fill launches per launch: each a blit
// kernel that, in a stream of frame pairs, waits for CUs behind the other pairs' LM launches):
// the launch counters (stat: 32 words, word 20 = ~0, the minimum start), the work queue, and per
// problem its pair counters (pcnt + 16 bytes), its statuses (kLMRunning) and lmdif info / nfev.
struct LMReset {
    unsigned long long* stat;
    int* queue;  // 64 ints, or null (no points)
    int nProb;
    int* pcnt16[kLMMaxProblems];  // 4 ints each
    int* status[kLMMaxProblems];
    int* info[kLMMaxProblems];
    int* nfev[kLMMaxProblems];
    int P[kLMMaxProblems];  // the problems' point bounds (0: only the counters)
};
void launch_lm_reset(const LMReset& r, hipStream_t s);

// ---------------- stable compaction fused into its producer (decoupled look-back) ----------------
// One launch produces the items and compacts them in order: each block counts its kept items,
// publishes the count, and adds up its predecessors' (their inclusive prefix as soon as one is
// published) to place its items.  Blocks take their index from a counter in launch order, so a block
// only ever waits for blocks that started before it.
struct LookBack {
    unsigned long long* st;  // per block of the launch: (epoch << 32) | (flag << 30) | value
    unsigned* ctr;           // block counter: 0 at every launch's start (lookback_block_id)
    unsigned epoch;  // the launch's tag (never 0): status words of earlier launches read as "not yet"
};
// A block's index in launch order.  The block that takes the last index resets the counter for the
// next launch on the stream: every other block of this launch took its index before it (one
// modification order per address), so each launch's indices are 0 .. gridDim.x - 1 whatever the
// earlier launches did -- a launch that never ran leaves the counter at 0 (no host-side
// base to fall out of step with the device).
__device__ inline int lookback_block_id(const LookBack& lb) {
    const unsigned id = atomicAdd(lb.ctr, 1u);
    if (id == gridDim.x - 1) __hip_atomic_store(lb.ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (int)id;
}
// NNDR (descriptorsmatcher.cpp:119-129) with the parts' top-2 merge (int keys; parts = 1: idx / key
// as merged lists) and the stable compaction of the kept matches: out[0 .. *count)
void launch_nndr_compact(int type, const int* idx, const int* key, const float* fkey, const int* partIdx,
                         const int* partKey, int parts, int nA, double eps, int queryOffset, fm3d_dmatch* out,
                         int* count, const LookBack& lb, hipStream_t s);
int nndr_compact_blocks(int nA);
// setKeypoints + triangulate with the compaction of the inliers: out (P x 3), srcIdx (P), *count = P;
// mask (K) as launch_triangulate
void launch_triangulate_compact(const TriParams& p, double* out, int* srcIdx, int* count, const LookBack& lb,
                                hipStream_t s, int* hostCnt = nullptr);
int triangulate_compact_blocks(int K);

// ---------------- images ----------------
void launch_pyrdown(const uint8_t* src, int w, int h, uint8_t* dst, hipStream_t s);
void launch_undistort(const Camera& cam, const double* xy, int n, double* out, hipStream_t s);

// extractPixelsContour + the level-0 geometry of evaluateNormal through a given plane (fm3d_misc.hip)
struct PlaneProjParams {
    Camera cam;
    double R2[9], t2[3], X[3], n[3];
    double cmax;  // int(2 * zThresholdMax), isInBoundingBox :648
    const int2* offsets;
    int nOff, boundW, boundH, w, h;
    double *xy, *uv;
    int *keep, *status;
};
void launch_plane_project(const PlaneProjParams& p, hipStream_t s);

// ---------------- feature frames + patch export (fm3d_patch.hip) ----------------
void launch_features_frames(const double* pts, const double* nrm, int P, const double g[3], double* frames,
                            hipStream_t s);
// computeSquareNeighborhoodsByNormals: out P*size*size*3 doubles (device)
// computeCircularNeighborhoodsByNormals: P points (P*3), normals (P*3 or NULL: X/|X|), S samples per
// point from lut (S*3: r, sin t, 2 sin^2(t/2)) -> out P*S*3
void launch_circular_neighborhoods(const double* pts, const double* nrm, int P, int S, const double* lut, double eps,
                                   double* out, hipStream_t s);
void launch_square_neighborhoods(const double* frames, int P, int size, double eps, double inc, double* out,
                                 hipStream_t s);
// RT: 12 doubles of scratch per frame
void launch_export_patches(const double* frames, int P, int size, double eps, double inc, const Camera& cam,
                           const uint8_t* img, int w, int h, double* RT, uint8_t* patches, double* imagePoints,
                           hipStream_t s);

// ---------------- records ----------------
// nDev (may be null): the count on the device, nInl / n its bound
void launch_make_records(const fm3d_dmatch* matches, const int* inlierSrc, int nInl, const int* nDev, const double* pts,
                         const double* normals, const int* status, fm3d_record* rec, int* flag, hipStream_t s);
void launch_compact_records(const fm3d_record* in, const int* flag, int n, const int* nDev, fm3d_record* out,
                            int* count, void* tmp, hipStream_t s);

// ---------------------------------------------------------------- STAR (fm3d_star.hip)
struct StarPat {   // StarDetectorComputeResponses' pattern set (oracle/orc_star.c orc_star_patterns)
    int np, maxIdx, border, nsimd;  // pairs, largest pattern, border, columns of the SSE2 block
    int sizes1[17];                 // pattern sizes, the range's ends negated
    int ofs[17 * 8];                // integral offsets per pattern: 0-3 into S, 4 and 7 into T, 5 and 6 into F
    float inv[24];                  // per pair 1/outerArea, 1/innerArea
};
struct StarNms {   // StarDetectorSuppressNonmax's tiling and thresholds
    int border, delta, nx, ny, respThr, lineProj, lineBin;
};
size_t star_tilted_lds_bytes(int w);
int star_tilted_max_width();
void launch_star_tilted(const uint8_t* img, int w, int h, int* T, int* F, hipStream_t s);
size_t star_diag_bytes(int w, int h);
void launch_star_tilted_diag(const uint8_t* img, int w, int h, void* work, int* T, int* F, hipStream_t s);
void launch_star_resp(const int* S, const int* T, const int* F, int w, int h, const StarPat& P, float* resp,
                      short* sizes, hipStream_t s);
void launch_star_nms(const float* resp, const short* sizes, int w, int h, const StarNms& N, fm3d_keypoint* kp, int* flag,
                     hipStream_t s);
void launch_star_scatter(const fm3d_keypoint* kp, const int* flag, const int* pos, int n, fm3d_keypoint* out,
                         hipStream_t s);

// ---------------------------------------------------------------- FREAK (fm3d_freak.hip)
constexpr int kFreakScales = 64, kFreakOrient = 256, kFreakPoints = 43, kFreakOrientPairs = 45;
// lut: (x, y, sigma, 0) per (scale, orientation, point); opairs: (i, j, weight_dx, weight_dy); pairs: the
// 512 (i, j); scale: each keypoint's pattern scale; angle / desc: n floats / n x 64 bytes
void launch_freak_desc(const uint8_t* img, const int* sum, int w, const fm3d_keypoint* kp, const int* scale, int n,
                       const float4* lut, const int4* opairs, const int2* pairs, float* angle, uint8_t* desc,
                       hipStream_t s);

// ---------------------------------------------------------------- MSER (fm3d_mser.hip)
struct MserParams {
    int delta, minArea, maxArea;
    double maxVariation, minDiversity;
};
struct MserHist {  // MSERGrowHistory by index
    int shortcut, child, stable, val, size;
};
// the workspace of one pass over a w x h image (both passes: twice, pass-major)
struct MserLayout {
    int w, h;
    int pw;              // the padded width w + 2 (the flood works on the (w + 2) x (h + 2) grid)
    int visInLds;        // the visited bitmap in LDS ((w + 2)(h + 2) <= kMserLdsBits), else in HBM
    long long visWords;  // ceil((w + 2)(h + 2) / 32)
    long long padBytes;  // one pass's padded grey image, rounded up to whole dwords
    long long heapEntries;  // w * h + 256: {padded pixel + 1 | direction << 28, x | y << 16}
    long long nodes;     // w * h: {next node, x | y << 16}
    long long hists;     // 2 w h + 2 (a bound: one per raise and per merge)
    long long regCap;    // region records per pass
};
constexpr long long kMserLdsBits = 120 * 1024 * 8;
MserLayout mser_layout(int w, int h);
// both flood passes of `count` images of w x h (stored one after the other), one workgroup per slot
// (slot = 2 * image + pass; pass 0 on 255 - I, colour -1; pass 1 on I, colour +1):
// reg[slot * regCap + r] = {colour, head node, point count, 0}; nreg[slot] = regions (all, even past
// regCap); pad: 2 * count * padBytes of scratch (each slot's grey values on the padded grid)
void launch_mser_flood(const uint8_t* img, int count, const MserLayout& L, const MserParams& P, uint8_t* pad,
                       unsigned* vis, int2* heap, int2* node, MserHist* hist, int4* reg, int* nreg, hipStream_t s);
// the point lists of all slots ranked (list ranking): node g = slot * nodes + i sits at
// pts[base[last[g]] + rank[g]] (its list's points stored backwards from the end); work: mser_rank_bytes
struct MserRank {
    const int *rank, *last, *base, *pts;
};
size_t mser_rank_bytes(long long nodes, int slots);
MserRank launch_mser_rank(const int2* node, long long nodes, int slots, int* work, hipStream_t s);
// fitEllipse per region (one wave each): reg[r] = {colour, head node, count, slot} (all slots' regions
// in slot order), its points at off[r] in xy (gathered from the ranked lists) and 5 * count doubles
// of scratch at 5 * off[r]; kp[r] = KeyPoint(centre, sqrt(w h)), flag[r] = kept (diameter >
// FLT_EPSILON, rounded centre inside)
void launch_mser_fit(const int4* reg, int n, const MserRank& K, long long nodes, const long long* off,
                     const MserLayout& L, int2* xy, double* scratch, fm3d_keypoint* kp, int* flag, float* box,
                     hipStream_t s);

// ---------------------------------------------------------------- BRISK (fm3d_brisk.hip)
// pat: 60 (x, y, sigma, 0) pattern points per (scale, rotation) in use; pidx: each keypoint's row of pat;
// pairs: the short pairs (i, j); desc: n x 64 bytes
void launch_brisk_desc(const uint8_t* img, const int* II, int w, const fm3d_keypoint* kp, const int* pidx, int n,
                       const float4* pat, const int2* pairs, int npairs, uint8_t* desc, hipStream_t s);

}  // namespace fm3d
