// fm3d_host.cpp -- C ABI (include/fm3d.h): context, host algebra, orchestration.
//
// Host-side algebra restates the reference's scalar code (setg12, Rodrigues,
// Matx44d::inv) with the same operation order as oracle/fm3d_oracle.c; the heavy
// per-keypoint work runs in the HIP kernels of fm3d_match.hip, fm3d_misc.hip and
// fm3d_lm.hip.  There is no CPU fallback: without a GPU every compute entry point
// fails with FM3D_ERR_HIP.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "fm3d.h"
#include "fm3d_freak.h"
#include "fm3d_kernels.h"

using fm3d::Camera;
using fm3d::LevelDesc;

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    hipError_t ensure(size_t n) {
        if (n <= bytes) return hipSuccess;
        if (p) hipFree(p);
        p = nullptr;
        bytes = 0;
        size_t alloc = n < 256 ? 256 : n;
        hipError_t e = hipMalloc(&p, alloc);
        if (e == hipSuccess) bytes = alloc;
        return e;
    }
    void release() {
        if (p) hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <typename T>
    T* as() const {
        return (T*)p;
    }
};

constexpr size_t kGuard(int w) { return (size_t)4 * w + 64; }

// page-locked host staging (hipHostMalloc): the H2D copies of the inputs run asynchronously from
// it, at full PCIe rate, and the host may return before they execute (fm3d_pipeline_submit)
struct HostBuf {
    void* p = nullptr;
    size_t bytes = 0;
    hipError_t ensure(size_t n) {
        if (n <= bytes) return hipSuccess;
        if (p) hipHostFree(p);
        p = nullptr;
        bytes = 0;
        size_t alloc = n < 4096 ? 4096 : n;
        hipError_t e = hipHostMalloc(&p, alloc, hipHostMallocDefault);
        if (e == hipSuccess) bytes = alloc;
        return e;
    }
    void release() {
        if (p) hipHostFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <typename T>
    T* as() const {
        return (T*)p;
    }
};

// the pipeline's small device -> host results of one frame pair (one D2H, pinned)
struct PipeSmall {
    int32_t cnt[4];                 // matches K, inliers P, kept, pad (c->pcnt bytes 0..15)
    unsigned long long prob[2];     // this pair's residual / pixel evaluations (c->pcnt bytes 16..31)
    unsigned long long lm[26];      // the LM launch's counters (fm3d_lm2.hip statPass layout)
};

}  // namespace

struct fm3d_ctx {
    fm3d_settings s;
    int device = 0;
    hipStream_t stream = nullptr;
    bool ownStream = false;
    Camera cam{};
    double g12[16];
    double R2[9], t2[3];
    bool haveG12 = false;
    // pyramids
    int w = 0, h = 0;
    std::vector<int> lw, lh;
    std::vector<DevBuf> pyr1, pyr2;
    int pyrGuardW = -1, pyrGuardH = -1, pyrGuardLevels = -1;  // the geometry whose guards are zero
    DevBuf lvlDesc;
    // circle offsets of pixelsRay
    DevBuf offsets;
    int nOff = 0, nOffPad = 0;
    // work buffers
    DevBuf A, B, cqA, ctB, idx, key, fkey, knnOut, cand, flag, matches, count, scanTmp;
    DevBuf partIdx, partKey;  // per-part top-2 lists of the split matchers
    DevBuf A8, B8;            // binary rows unpacked to int8 for the MFMA matcher; u8 rows packed from floats
    DevBuf u8Flag;            // launch_f32_pack_u8's "not integer-valued" flag
    bool specU8 = false;      // the staged float rows went to the u8 matcher before their flag was read
    // SURF detection / description
    DevBuf sfImg, sfSum, sfDet, sfTr, sfLayers, sfMids, sfCand, sfCount, sfSortTmp, sfFlag, sfPos, sfKp, sfKin, sfSrc,
        sfDesc, sfDW, sfAng;
    // ORB detection / description
    DevBuf orbPyr, orbTab, orbLev, orbMap, orbFlag, orbPos, orbKp, orbR, orbBlur, orbDesc, orbPat;
    std::vector<int> orbUserPattern;  // fm3d_orb_set_pattern (empty: makeRandomPattern(orbPatchSize))
    // SIFT detection / description
    DevBuf siftImg, siftBase, siftG, siftD, siftGL, siftDL, siftTaps, siftScan, siftFlag, siftPos, siftCand, siftAng,
        siftNpk, siftKp, siftDesc;
    // BRISK description
    DevBuf brImg, brSum, brKp, brIdx, brPat, brPairs, brDesc;
    // FREAK description (frLut: the whole default pattern, uploaded once)
    DevBuf frImg, frSum, frKp, frScale, frLut, frOp, frPairs, frAng, frDesc;
    DevBuf msImg, msWork, msHeap, msNode, msHist, msReg, msCnt, msOff, msXY, msScr, msKp, msFlag, msPos, msOut, msRank,
        msPad, msRegC;
    std::vector<int> freakUserPairs;  // fm3d_freak_set_pairs (empty: FM3D_FREAK_DEF_PAIRS)
    // STAR detection
    DevBuf starImg, starS, starT, starF, starR, starZ, starKp, starFlag, starPos, starOut, starWork;
    // NCC hypotheses over the pipeline's inliers (fm3d_pipeline_run_ncc)
    DevBuf nccS, nccN, nccB;
    int nccH = 0;
    DevBuf bPairs;            // the f32 train rows in interleaved pairs
    DevBuf f32Work;           // the bf16 MFMA prefilter's scratch (rows, norms, bounds, candidates)
    int nCU = 0;
    DevBuf kp1, kp2, triPts, triMask, triMask8, pts, srcIdx;
    long lmGroups = 0;
    int wallKhz = 0;
    DevBuf lmNormals, lmStatus, lmInfo, lmNfev, lmMdat, lmQueue, lmStat, slab, slabI1;
    // the fused compactions' look-back state (fm3d_kernels.h LookBack): status words, block counter
    DevBuf lbSt, lbCtr;
    unsigned lbEpoch = 0;  // the last look-back launch's tag (fm3d_kernels.h LookBack)
    DevBuf records, recTmp, recFlag;
    DevBuf lmProj;  // camera-2 projection constants for the LM kernel (fm3d::ProjConst)
    DevBuf pcnt;    // the pipeline's device counts: [0] matches K, [1] inliers P, [2] kept
    // pinned staging: descriptors A / B (padded rows), keypoints, images, small tables, results
    HostBuf hA, hB, hK1, hK2, hImg, hTab, hProj, hSmall, hFlag;
    hipEvent_t evStage = nullptr;  // after the last H2D copy from the staging buffers
    hipEvent_t evProj = nullptr;   // after the last H2D copy of the LM constants (hProj)
    bool pending = false;          // a fm3d_pipeline_submit awaiting fm3d_pipeline_wait
    // fm3d_pipeline_link: a member's submit queues its front half only; the leader's next submit
    // queues ONE LM launch over both pairs' points and the member's records behind it
    fm3d_ctx* linkLeader = nullptr;        // (member) the context that launches its LM
    std::vector<fm3d_ctx*> linkMembers;    // (leader) the contexts whose pairs join its launches
    bool frontOnly = false;          // (member) submitted, its LM not queued yet
    fm3d_record* subOut = nullptr;   // the submitted pair's record destination (device; null: internal)
    hipEvent_t evFront = nullptr;    // (member) after its front half
    hipEvent_t evLm = nullptr;       // (leader) after a joint LM launch
    fm3d_lm_stats subLm{};         // the pending submit's LM launch data
    bool pendingDlt = false;       // the pending submit is fm3d_pipeline_submit_dlt's front half
    bool pendingNcc = false;       // the pending submit is fm3d_pipeline_submit_ncc's front half + NCC
    int nccHPending = 0;           // its hypotheses per point
    fm3d_record* pendOut = nullptr;  // the device records of the pending / last run
    // staged pipeline inputs
    int stNA = 0, stNB = 0, stDim = 0, stType = 0, stDimPad = 0, stQueryOffset = 0;
    int stK = 0, stP = 0;  // matches and inliers of the last fm3d_pipeline_run_dlt
    bool stageEv = true;   // the last pipeline_front recorded ev[3] / ev[5] (FM3D_STAGE_EVENTS)
    int* frontHostCnt = nullptr;  // pipeline_front: the DLT kernel also stores (K, P) here (device pointer)
    int nccP = 0;          // points of the last successful fm3d_pipeline_run_ncc (its score rows)
    bool staged = false;
    hipEvent_t ev[10];     // [0..1] standalone LM, [2..7] pipeline stages, [8] submit start, [1] end
    std::string err;
};

namespace {

int fail(fm3d_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

#define HIPCHK(ctx, expr)                                                                         \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess) return fail((ctx), FM3D_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

// ---------------- host algebra (same operation order as the oracle) ----------------
void rodrigues_v2m(const double r[3], double R[9]) {
    double rx = r[0], ry = r[1], rz = r[2];
    double theta = std::sqrt(rx * rx + ry * ry + rz * rz);
    if (theta < DBL_EPSILON) {
        for (int k = 0; k < 9; k++) R[k] = (k % 4 == 0) ? 1. : 0.;
        return;
    }
    const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    double c = std::cos(theta), s = std::sin(theta), c1 = 1. - c;
    double itheta = theta ? 1. / theta : 0.;
    rx *= itheta;
    ry *= itheta;
    rz *= itheta;
    const double rrt[9] = {rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz};
    const double rxm[9] = {0, -rz, ry, rz, 0, -rx, -ry, rx, 0};
    for (int k = 0; k < 9; k++) R[k] = c * I[k] + c1 * rrt[k] + s * rxm[k];
}

// cvRodrigues2 matrix -> vector: R replaced by its polar factor U V^T from OpenCV 2.4's SVD
// (include/fm3d_cvsvd.h, the same JacobiSVD the oracle restates), then the skew part and trace
void rodrigues_m2v(const double Rin[9], double r[3]) {
    double R[9];
    fm3d_cv::polar3(Rin, R);
    double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
    double s = std::sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    double c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    double theta = std::acos(c);
    if (s < 1e-5) {
        double t;
        if (c > 0)
            rx = ry = rz = 0;
        else {
            t = (R[0] + 1) * 0.5;
            rx = std::sqrt(t > 0. ? t : 0.);
            t = (R[4] + 1) * 0.5;
            ry = std::sqrt(t > 0. ? t : 0.) * (R[1] < 0 ? -1. : 1.);
            t = (R[8] + 1) * 0.5;
            rz = std::sqrt(t > 0. ? t : 0.) * (R[2] < 0 ? -1. : 1.);
            if (std::fabs(rx) < std::fabs(ry) && std::fabs(rx) < std::fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
            theta /= std::sqrt(rx * rx + ry * ry + rz * rz);
            rx *= theta;
            ry *= theta;
            rz *= theta;
        }
    } else {
        double vth = 1 / (2 * s);
        vth *= theta;
        rx *= vth;
        ry *= vth;
        rz *= vth;
    }
    r[0] = rx;
    r[1] = ry;
    r[2] = rz;
}

void compose(const double R[9], const double T[3], double G[16]) {  // tools.cpp:87-99
    G[0] = R[0]; G[1] = R[1]; G[2] = R[2]; G[3] = T[0];
    G[4] = R[3]; G[5] = R[4]; G[6] = R[5]; G[7] = T[1];
    G[8] = R[6]; G[9] = R[7]; G[10] = R[8]; G[11] = T[2];
    G[12] = 0; G[13] = 0; G[14] = 0; G[15] = 1;
}

void inv4(const double Ain[16], double B[16]) {  // Matx44d::inv(DECOMP_LU)
    double A[16];
    std::memcpy(A, Ain, sizeof(A));
    for (int i = 0; i < 16; i++) B[i] = (i % 5 == 0) ? 1. : 0.;
    for (int i = 0; i < 4; i++) {
        int k = i;
        for (int j = i + 1; j < 4; j++)
            if (std::fabs(A[j * 4 + i]) > std::fabs(A[k * 4 + i])) k = j;
        if (k != i) {
            for (int j = i; j < 4; j++) std::swap(A[i * 4 + j], A[k * 4 + j]);
            for (int j = 0; j < 4; j++) std::swap(B[i * 4 + j], B[k * 4 + j]);
        }
        double d = -1 / A[i * 4 + i];
        for (int j = i + 1; j < 4; j++) {
            double alpha = A[j * 4 + i] * d;
            for (int kk = i + 1; kk < 4; kk++) A[j * 4 + kk] += alpha * A[i * 4 + kk];
            for (int kk = 0; kk < 4; kk++) B[j * 4 + kk] += alpha * B[i * 4 + kk];
        }
        A[i * 4 + i] = -d;
    }
    for (int i = 3; i >= 0; i--)
        for (int j = 0; j < 4; j++) {
            double s = B[i * 4 + j];
            for (int kk = i + 1; kk < 4; kk++) s -= A[i * 4 + kk] * B[kk * 4 + j];
            B[i * 4 + j] = s * A[i * 4 + i];
        }
}

void mul4(const double a[16], const double b[16], double c[16]) {
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            double s = 0;
            for (int k = 0; k < 4; k++) s += a[i * 4 + k] * b[k * 4 + j];
            c[i * 4 + j] = s;
        }
}

void camera2_from_g12(const double g12[16], double R2[9], double t2[3]) {
    double R[9] = {g12[0], g12[1], g12[2], g12[4], g12[5], g12[6], g12[8], g12[9], g12[10]};
    double r[3];
    rodrigues_m2v(R, r);  // decomposeTransformation (tools.cpp:101-114)
    rodrigues_v2m(r, R2); // cvProjectPoints2 converts r2 back to a matrix
    t2[0] = g12[3];
    t2[1] = g12[7];
    t2[2] = g12[11];
}

void install_g12(fm3d_ctx* c, const double g[16]) {
    std::memcpy(c->g12, g, sizeof(c->g12));
    camera2_from_g12(c->g12, c->R2, c->t2);
    c->haveG12 = true;
}

int ensure_offsets(fm3d_ctx* c) {
    if (c->nOff > 0) return FM3D_OK;
    const int R = c->s.pixelsRay;
    std::vector<int2> off;
    for (int i = -R; i <= R; i++)      // extractPixelsContour (:345-351): i outer (x), j inner (y)
        for (int j = -R; j <= R; j++)
            if (i * i + j * j <= R * R) off.push_back(make_int2(i, j));
    c->nOff = (int)off.size();
    // pad to a multiple of the LM kernel's 64-entry chunk with offsets that are never
    // inside the image
    while (off.size() % 64) off.push_back(make_int2(1 << 20, 1 << 20));
    c->nOffPad = (int)off.size();
    HIPCHK(c, c->offsets.ensure(off.size() * sizeof(int2)));
    HIPCHK(c, hipMemcpy(c->offsets.p, off.data(), off.size() * sizeof(int2), hipMemcpyHostToDevice));
    return FM3D_OK;
}

int upload(fm3d_ctx* c, DevBuf& b, const void* src, size_t bytes) {
    HIPCHK(c, b.ensure(bytes));
    if (bytes) HIPCHK(c, hipMemcpyAsync(b.p, src, bytes, hipMemcpyHostToDevice, c->stream));
    return FM3D_OK;
}

// The staging buffers are refilled only after the H2D copies of the previous call out of them
// have run (c->evStage, recorded after them on the context stream).
int staging_wait(fm3d_ctx* c) {
    HIPCHK(c, hipEventSynchronize(c->evStage));
    return FM3D_OK;
}

// bytes from a host array to a device buffer through the pinned staging buffer h: one memcpy, one
// DMA copy (1 MiB pieces issued as they were copied, and the memcpy split over host threads, were
// both slower on the C2 and C4 lines)
int upload_pinned(fm3d_ctx* c, DevBuf& dst, HostBuf& h, const void* src, size_t bytes) {
    HIPCHK(c, dst.ensure(bytes));
    if (!bytes) return FM3D_OK;
    HIPCHK(c, h.ensure(bytes));
    std::memcpy(h.p, src, bytes);
    HIPCHK(c, hipMemcpyAsync(dst.p, h.p, bytes, hipMemcpyHostToDevice, c->stream));
    return FM3D_OK;
}

// rows of bytes padded to dimPad (multiple of 128) with value 128 (x - 128 == 0: no effect on d2)
void pad_u8(uint8_t* o, const uint8_t* x, int n, int dim, int dimPad) {
    if (dim == dimPad) {
        std::memcpy(o, x, (size_t)n * dim);
        return;
    }
    for (int i = 0; i < n; i++) {
        std::memcpy(o + (size_t)i * dimPad, x + (size_t)i * dim, dim);
        std::memset(o + (size_t)i * dimPad + dim, 128, dimPad - dim);
    }
}
// stage descriptors on the device (asynchronous H2D from the pinned staging buffers; the stream
// orders every later use); returns the effective kernel type
// (waitStaging false: the caller waited for the staging buffers already, stage_pipeline)
int stage_descriptors(fm3d_ctx* c, const void* descA, int nA, const void* descB, int nB, int dim, int type,
                      int* effType, int* dimPad, bool waitStaging = true, bool speculate = false) {
    if (dim <= 0 || nA < 0 || nB < 0) return fail(c, FM3D_ERR_INVALID, "bad descriptor shape");
    int r;
    if (waitStaging && (r = staging_wait(c))) return r;
    c->specU8 = false;
    int t = type;
    if (type == FM3D_DESC_F32 && ((dim + 127) / 128) * 128 <= 256) {
        // float rows as the reference hands them to knnMatch (descriptorsmatcher.cpp:114-117): to the
        // device as they are; one kernel packs them into padded u8 rows and flags any element that is not
        // an integer in [0, 255].  Integer-valued rows (SIFT) take the u8 kernel -- exact, the same
        // ranking and distances as the float scan -- others the float kernels.  The choice of kernels
        // needs the flag: one host wait for this context's copies and the pack (the float path waits
        // on the device once more anyway, run_match)
        const int dp = ((dim + 127) / 128) * 128;
        int r2;
        if ((r2 = upload_pinned(c, c->A, c->hA, descA, (size_t)nA * dim * 4))) return r2;
        if ((r2 = upload_pinned(c, c->B, c->hB, descB, (size_t)nB * dim * 4))) return r2;
        HIPCHK(c, c->A8.ensure((size_t)nA * dp + 16));
        HIPCHK(c, c->B8.ensure((size_t)nB * dp + 16));
        HIPCHK(c, c->u8Flag.ensure(64));
        HIPCHK(c, c->hFlag.ensure(64));
        HIPCHK(c, hipMemsetAsync(c->u8Flag.p, 0, sizeof(int), c->stream));
        fm3d::launch_f32_pack_u8(c->A.as<float>(), nA, c->B.as<float>(), nB, dim, dp, c->A8.as<uint8_t>(),
                                 c->B8.as<uint8_t>(), c->u8Flag.as<int>(), c->stream);
        HIPCHK(c, hipGetLastError());
        *c->hFlag.as<int>() = -1;  // "not arrived" (the previous pair's copies into it have run: staging_wait)
        HIPCHK(c, hipMemcpyAsync(c->hFlag.p, c->u8Flag.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
        if (speculate) {
            // no host wait (fm3d_pipeline_submit_dlt_pair): the u8 matcher runs on the packed rows, and
            // the wait re-runs the front half on the float rows if the flag then says they were not
            // integers (redo_float_front)
            std::swap(c->A, c->A8);
            std::swap(c->B, c->B8);
            *dimPad = dp;
            *effType = FM3D_DESC_U8;
            c->specU8 = true;
            return FM3D_OK;
        }
        HIPCHK(c, hipEventRecord(c->evStage, c->stream));
        HIPCHK(c, hipEventSynchronize(c->evStage));
        if (*c->hFlag.as<int>() == 0) {
            std::swap(c->A, c->A8);  // the packed rows become the matcher's inputs
            std::swap(c->B, c->B8);
            *dimPad = dp;
            *effType = FM3D_DESC_U8;
        } else {
            *dimPad = dim;
            *effType = FM3D_DESC_F32;
        }
        return FM3D_OK;
    }
    if (t == FM3D_DESC_U8) {
        int dp = ((dim + 127) / 128) * 128;
        if (dp > 256) return fail(c, FM3D_ERR_UNSUPPORTED, "u8 descriptors longer than 256 bytes");
        const size_t ba = (size_t)nA * dp, bb = (size_t)nB * dp;
        if (dim == dp) {  // rows already padded (SIFT's 128 bytes): the copy overlapped with the DMA
            if ((r = upload_pinned(c, c->A, c->hA, descA, ba))) return r;
            if ((r = upload_pinned(c, c->B, c->hB, descB, bb))) return r;
        } else {
            HIPCHK(c, c->hA.ensure(ba + 1));
            HIPCHK(c, c->hB.ensure(bb + 1));
            pad_u8(c->hA.as<uint8_t>(), (const uint8_t*)descA, nA, dim, dp);
            pad_u8(c->hB.as<uint8_t>(), (const uint8_t*)descB, nB, dim, dp);
            HIPCHK(c, c->A.ensure(ba));
            HIPCHK(c, c->B.ensure(bb));
            if (ba) HIPCHK(c, hipMemcpyAsync(c->A.p, c->hA.p, ba, hipMemcpyHostToDevice, c->stream));
            if (bb) HIPCHK(c, hipMemcpyAsync(c->B.p, c->hB.p, bb, hipMemcpyHostToDevice, c->stream));
        }
        *dimPad = dp;
    } else if (t == FM3D_DESC_F32) {
        if ((r = upload_pinned(c, c->A, c->hA, descA, (size_t)nA * dim * 4))) return r;
        if ((r = upload_pinned(c, c->B, c->hB, descB, (size_t)nB * dim * 4))) return r;
        *dimPad = dim;
    } else if (t == FM3D_DESC_BITS) {
        int words = (dim + 3) / 4;
        int wp = (words == 4 || words == 8 || words == 16) ? words : 16;
        if (words > 16) return fail(c, FM3D_ERR_UNSUPPORTED, "binary descriptors longer than 64 bytes");
        const size_t ba = (size_t)nA * wp * 4, bb = (size_t)nB * wp * 4;
        HIPCHK(c, c->hA.ensure(ba + 1));
        HIPCHK(c, c->hB.ensure(bb + 1));
        std::memset(c->hA.p, 0, ba);
        std::memset(c->hB.p, 0, bb);
        for (int i = 0; i < nA; i++) std::memcpy(c->hA.as<uint8_t>() + (size_t)i * wp * 4, (const uint8_t*)descA + (size_t)i * dim, dim);
        for (int i = 0; i < nB; i++) std::memcpy(c->hB.as<uint8_t>() + (size_t)i * wp * 4, (const uint8_t*)descB + (size_t)i * dim, dim);
        HIPCHK(c, c->A.ensure(ba));
        HIPCHK(c, c->B.ensure(bb));
        if (ba) HIPCHK(c, hipMemcpyAsync(c->A.p, c->hA.p, ba, hipMemcpyHostToDevice, c->stream));
        if (bb) HIPCHK(c, hipMemcpyAsync(c->B.p, c->hB.p, bb, hipMemcpyHostToDevice, c->stream));
        *dimPad = wp * 4;
    } else {
        return fail(c, FM3D_ERR_INVALID, "unknown descriptor type");
    }
    HIPCHK(c, hipEventRecord(c->evStage, c->stream));
    *effType = t;
    return FM3D_OK;
}

// FM3D_BITS_MFMA=0 keeps 256-bit binary rows on the popcount kernel (A/B comparisons)
bool bits_mfma() {
    const char* e = getenv("FM3D_BITS_MFMA");
    return !(e && e[0] == '0');
}

// FM3D_F32_MFMA=0 keeps float rows on the exact VALU scan (A/B comparisons)
bool f32_mfma() {
    const char* e = getenv("FM3D_F32_MFMA");
    return !(e && e[0] == '0');
}

// knn2 + NNDR flags on staged descriptors (device), results in c->idx/key/fkey/cand/flag
// the look-back state of one fused-compaction launch of nBlocks blocks on c's stream
bool stage_events() {
    const char* e = getenv("FM3D_STAGE_EVENTS");
    return !(e && e[0] == '0');
}

// match_ms (row constants, knn, NNDR and its compaction: one stage since NNDR is fused into the
// match's last launch; nndr_ms stays 0) and triangulate_ms, when the step recorded its stage events
void stage_times(fm3d_ctx* c, fm3d_pipeline_stats* stats) {
    float ms = 0;
    stats->match_ms = stats->nndr_ms = stats->triangulate_ms = 0;  // 0 when the step recorded no stage events
    if (!c->stageEv) return;
    hipEventElapsedTime(&ms, c->ev[2], c->ev[3]);
    stats->match_ms = ms;
    stats->nndr_ms = 0;
    hipEventElapsedTime(&ms, c->ev[3], c->ev[5]);
    stats->triangulate_ms = ms;
}

int make_lookback(fm3d_ctx* c, int nBlocks, fm3d::LookBack* lb) {
    if (!c->lbCtr.p) {
        HIPCHK(c, c->lbCtr.ensure(64));
        HIPCHK(c, hipMemsetAsync(c->lbCtr.p, 0, 64, c->stream));  // each launch leaves it at 0
    }
    bool zero = false;
    if (c->lbSt.bytes < (size_t)nBlocks * 8) {
        HIPCHK(c, c->lbSt.ensure((size_t)nBlocks * 8 * 2));
        zero = true;
    }
    if (++c->lbEpoch == 0) {  // the 32-bit tag wrapped: 0 is the zeroed words' "not yet"
        c->lbEpoch = 1;
        zero = true;
    }
    if (zero) HIPCHK(c, hipMemsetAsync(c->lbSt.p, 0, c->lbSt.bytes, c->stream));  // epoch 0: "not yet"
    lb->st = c->lbSt.as<unsigned long long>();
    lb->ctr = c->lbCtr.as<unsigned>();
    lb->epoch = c->lbEpoch;
    return FM3D_OK;
}

// compactOut / compactCount (the pipeline): NNDR, the parts' merge (int keys) and the stable
// compaction of the kept matches in one launch (launch_nndr_compact); else the NNDR flags and
// candidates in c->flag / c->cand
int run_match(fm3d_ctx* c, int nA, int nB, int type, int dimPad, double eps, int queryOffset, bool wantKnn,
              fm3d_dmatch* compactOut = nullptr, int* compactCount = nullptr) {
    const bool fuse = compactOut != nullptr && !wantKnn;
    int mergeParts = 1;  // > 1: the parts' lists are merged by launch_nndr_compact
    HIPCHK(c, c->idx.ensure((size_t)nA * 2 * sizeof(int) + 16));
    HIPCHK(c, c->key.ensure((size_t)nA * 2 * sizeof(int) + 16));
    HIPCHK(c, c->fkey.ensure((size_t)nA * 2 * sizeof(float) + 16));
    HIPCHK(c, c->cand.ensure((size_t)nA * sizeof(fm3d_dmatch) + 16));
    HIPCHK(c, c->flag.ensure((size_t)nA * sizeof(int) + 16));
    if (wantKnn) HIPCHK(c, c->knnOut.ensure((size_t)nA * 2 * sizeof(fm3d_dmatch) + 16));
    if (c->nCU <= 0) {
        int n = 0;
        HIPCHK(c, hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, c->device));
        c->nCU = n > 0 ? n : 1;
    }
    if (type == FM3D_DESC_U8) {
        const int nAPad = nA, nBPad = nB;
        HIPCHK(c, c->cqA.ensure((size_t)(nAPad + 1) * sizeof(int)));
        HIPCHK(c, c->ctB.ensure((size_t)(nBPad + 1) * sizeof(int)));
        fm3d::launch_rowconst_u8(c->A.as<uint8_t>(), nA, c->B.as<uint8_t>(), nB, dimPad, c->cqA.as<int>(),
                                 c->ctB.as<int>(), c->stream);
        const int parts = fm3d::knn2_u8_parts(nA, nB, c->nCU, fm3d::knn2_i8_queries_per_block(dimPad, 0),
                                              fm3d::knn2_i8_tile_rows(dimPad, 0));
        if (parts > 1) {
            HIPCHK(c, c->partIdx.ensure((size_t)parts * nA * 2 * sizeof(int) + 16));
            HIPCHK(c, c->partKey.ensure((size_t)parts * nA * 2 * sizeof(int) + 16));
        }
        if (fuse && parts > 1) mergeParts = parts;
        fm3d::launch_knn2_i8(c->A.as<uint8_t>(), nA, c->B.as<uint8_t>(), nB, dimPad, 0, c->cqA.as<int>(),
                             c->ctB.as<int>(), parts, c->partIdx.as<int>(), c->partKey.as<int>(), c->idx.as<int>(),
                             c->key.as<int>(), c->stream, mergeParts > 1);
    } else if (type == FM3D_DESC_F32 && (dimPad == 64 || dimPad == 128) && nB >= 64 &&
               (long long)nA * nB >= (1LL << 22) && f32_mfma()) {
        // float rows (SURF): the bf16 MFMA prefilter lists each query's possible top-2 rows, whose exact
        // FLANN-order distances decide (fm3d_match.hip); the same result as the full exact scan
        const int parts = fm3d::knn2_f32_mfma_parts(nA, nB, c->nCU);
        HIPCHK(c, c->f32Work.ensure(fm3d::knn2_f32_mfma_bytes(nA, nB, dimPad, parts)));
        // one fused pass; when more than 1/8 of the queries overflow its lists, the two-pass form (whose
        // lists hold only the rows under the final bound); FM3D_F32_FUSED=0 starts with the two-pass form
        const char* fe = getenv("FM3D_F32_FUSED");
        bool fused = !(fe && fe[0] == '0');
        int nResc = 0;
        for (;;) {
            fm3d::launch_knn2_f32_mfma(c->A.as<float>(), nA, c->B.as<float>(), nB, dimPad, parts, fused, c->f32Work.p,
                                       c->idx.as<int>(), c->fkey.as<float>(), c->stream);
            HIPCHK(c, hipMemcpyAsync(&nResc, fm3d::knn2_f32_mfma_rescan_count(c->f32Work.p, nA, nB, dimPad, parts),
                                     sizeof(int), hipMemcpyDeviceToHost, c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
            if (!fused || nResc <= nA / 8) break;
            fused = false;
        }
        if (nResc > 0 && nResc <= nA / 8) {
            // the queries whose bound held more rows than the candidate list: an exact wave-per-query scan
            fm3d::launch_knn2_f32_mfma_rescan(c->A.as<float>(), c->B.as<float>(), nB, dimPad, c->f32Work.p, nA, parts,
                                              nResc, c->idx.as<int>(), c->fkey.as<float>(), c->stream);
        } else if (nResc > 0) {
            // descriptors with no margin between neighbours (e.g. uniform noise in high dimension):
            // the full exact scan for every query
            const int p2 = fm3d::knn2_parts(nA, nB, dimPad, c->nCU);
            if (p2 > 1) {
                HIPCHK(c, c->partIdx.ensure((size_t)p2 * nA * 2 * sizeof(int) + 16));
                HIPCHK(c, c->partKey.ensure((size_t)p2 * nA * 2 * sizeof(float) + 16));
            }
            HIPCHK(c, c->bPairs.ensure(fm3d::knn2_f32_pairs_bytes(nB, dimPad) + 16));
            fm3d::launch_knn2_f32(c->A.as<float>(), nA, c->B.as<float>(), nB, dimPad, p2, c->partIdx.as<int>(),
                                  c->partKey.as<float>(), c->bPairs.as<float>(), c->idx.as<int>(), c->fkey.as<float>(),
                                  c->stream);
        }
    } else if (type == FM3D_DESC_F32) {
        const int parts = (dimPad == 64 || dimPad == 128) ? fm3d::knn2_parts(nA, nB, dimPad, c->nCU) : 1;
        if (parts > 1) {
            HIPCHK(c, c->partIdx.ensure((size_t)parts * nA * 2 * sizeof(int) + 16));
            HIPCHK(c, c->partKey.ensure((size_t)parts * nA * 2 * sizeof(float) + 16));
        }
        HIPCHK(c, c->bPairs.ensure(fm3d::knn2_f32_pairs_bytes(nB, dimPad) + 16));
        fm3d::launch_knn2_f32(c->A.as<float>(), nA, c->B.as<float>(), nB, dimPad, parts, c->partIdx.as<int>(),
                              c->partKey.as<float>(), c->bPairs.as<float>(), c->idx.as<int>(), c->fkey.as<float>(),
                              c->stream);
    } else if (dimPad == 32 && bits_mfma()) {
        // 256-bit rows (ORB): unpacked to int8 and matched on the int8 MFMA kernel (exact integer
        // Hamming distances popc(b) - a.b', same ranking rule)
        HIPCHK(c, c->A8.ensure((size_t)nA * 256 + 16));
        HIPCHK(c, c->B8.ensure((size_t)nB * 256 + 16));
        HIPCHK(c, c->ctB.ensure((size_t)(nB + 1) * sizeof(int)));
        fm3d::launch_unpack_bits(c->A.as<uint8_t>(), nA, c->B.as<uint8_t>(), nB, c->A8.as<uint8_t>(),
                                 c->B8.as<uint8_t>(), c->ctB.as<int>(), c->stream);
        const int parts = fm3d::knn2_u8_parts(nA, nB, c->nCU, fm3d::knn2_i8_queries_per_block(256, 1),
                                              fm3d::knn2_i8_tile_rows(256, 1));
        if (parts > 1) {
            HIPCHK(c, c->partIdx.ensure((size_t)parts * nA * 2 * sizeof(int) + 16));
            HIPCHK(c, c->partKey.ensure((size_t)parts * nA * 2 * sizeof(int) + 16));
        }
        if (fuse && parts > 1) mergeParts = parts;
        fm3d::launch_knn2_i8(c->A8.as<uint8_t>(), nA, c->B8.as<uint8_t>(), nB, 256, 1, nullptr, c->ctB.as<int>(),
                             parts, c->partIdx.as<int>(), c->partKey.as<int>(), c->idx.as<int>(), c->key.as<int>(),
                             c->stream, mergeParts > 1);
    } else {
        const int parts = fm3d::knn2_parts(nA, nB, dimPad, c->nCU);
        if (parts > 1) {
            HIPCHK(c, c->partIdx.ensure((size_t)parts * nA * 2 * sizeof(int) + 16));
            HIPCHK(c, c->partKey.ensure((size_t)parts * nA * 2 * sizeof(int) + 16));
        }
        fm3d::launch_knn2_bits(c->A.as<uint8_t>(), nA, c->B.as<uint8_t>(), nB, dimPad, parts, c->partIdx.as<int>(),
                               c->partKey.as<int>(), c->idx.as<int>(), c->key.as<int>(), c->stream);
    }
    HIPCHK(c, hipGetLastError());
    if (fuse) {
        fm3d::LookBack lb;
        int r;
        if ((r = make_lookback(c, fm3d::nndr_compact_blocks(nA), &lb))) return r;
        fm3d::launch_nndr_compact(type, c->idx.as<int>(), c->key.as<int>(), c->fkey.as<float>(), c->partIdx.as<int>(),
                                  c->partKey.as<int>(), mergeParts, nA, eps, queryOffset, compactOut, compactCount, lb,
                                  c->stream);
    } else {
        fm3d::launch_nndr(type, c->idx.as<int>(), c->key.as<int>(), c->fkey.as<float>(), nA, nB, eps, queryOffset,
                          wantKnn ? c->knnOut.as<fm3d_dmatch>() : nullptr, c->cand.as<fm3d_dmatch>(), c->flag.as<int>(),
                          c->stream);
    }
    HIPCHK(c, hipGetLastError());
    return FM3D_OK;
}

int ensure_scan_tmp(fm3d_ctx* c, int n) {
    HIPCHK(c, c->scanTmp.ensure(fm3d::scan_tmp_bytes(n < 1 ? 1 : n)));
    HIPCHK(c, c->count.ensure(64));
    return FM3D_OK;
}

void fill_lm_cycles(const fm3d_ctx* c, const unsigned long long* cnt, fm3d_lm_stats* st) {
    st->groups = c->lmGroups;
    st->passes = (int64_t)cnt[3];
    st->cycles_terms = (int64_t)cnt[4];
    st->cycles_chain = (int64_t)cnt[5];
    st->cycles_control = (int64_t)cnt[6];
    st->cycles_total = (int64_t)cnt[7];
    st->wall_ticks_sum = (int64_t)cnt[8];
    st->wall_ticks_max = (int64_t)cnt[9];
    st->wall_clock_khz = c->wallKhz;
    for (int k = 0; k < 4; k++) {
        st->class_passes[k] = (int64_t)cnt[10 + k];
        st->class_cycles[k] = (int64_t)cnt[14 + k];
    }
    st->last_group_start_ticks = (int64_t)(cnt[18] - cnt[20]);
    st->last_group_end_ticks = (int64_t)(cnt[19] - cnt[20]);
    st->cycles_wait = (int64_t)cnt[24];
    st->chain_rounds = (int64_t)cnt[21];
    st->chain_chunks = (int64_t)cnt[22];
    st->queue_empty_ticks = cnt[25] ? (int64_t)(cnt[25] - cnt[20]) : 0;
}

// The LM kernel's camera: the settings' camera with a principal point of -0.0 replaced by +0.0.
// The kernel's isPixelGood compares bit patterns (0 <= u <= xmax as bits(u) <= bits(xmax)), which
// differs from the reference's comparison only for u == -0.0; u = xd*fx + cx (and the image-1
// centre, the same sum) is -0.0 only when cx is -0.0 and xd*fx is -0.0.  With +0.0 that sum is
// +0.0: the reference's test is true for both zeros, and the bilinear sample at a +-0 coordinate is
// the same.  Every other principal point (zero, negative, outside the image) gives the reference's
// bits: a negative u or NaN lies above bits(xmax) as the reference's comparison is false, and the
// fused a2 = r2 + 2x^2 differs only where x*x is subnormal, where u's float sample coordinate
// rounds to the same value (tests/test_gpu_parity.py::test_principal_point_zero_and_negative).
fm3d::Camera lm_camera(const fm3d::Camera& cam) {
    fm3d::Camera k = cam;
    if (k.cx == 0.) k.cx = 0.;  // -0.0 -> +0.0
    if (k.cy == 0.) k.cy = 0.;
    return k;
}

// One frame pair's points for an LM launch: its context (pyramids c->lvlDesc, pose c->R2/t2,
// outputs c->lm*, per-pair counters c->pcnt + 16 bytes) and the points (c->pts): P of them, or
// P their bound when Pdev holds the count on the device (the pipeline: no host sync)
struct LMSrc {
    fm3d_ctx* c;
    int P;
    const int* Pdev;
};

// LM normals over the points of nProb frame pairs in ONE launch on c's stream (c's slabs, queue
// and launch counters): the slots that find one pair's points used up take the next pair's, so
// a second pair fills the launch's end-of-queue tail (fm3d_pipeline_link).  Every problem's
// context must be ordered before this stream by the caller (its points, pyramids).
// the LM launch's workgroups for Ptot points (Ptot < 0: as many as the GPU holds): the settings'
// lmWaves, or every CU at the kernel's occupancy, bounded by the points, the slabs' HBM budget and
// their 32-bit offsets
int lm_groups(fm3d_ctx* c, const void* kptr, int slots, long Ptot, long* out) {
    long groups = c->s.lmWaves;
    if (groups <= 0) {
        int cus = 0, perCU = 0;
        HIPCHK(c, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
        HIPCHK(c, hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCU, kptr, fm3d::kLM2Threads, 0));
        if (perCU < 1) perCU = 1;
        groups = (long)cus * perCU;
    }
    if (Ptot >= 0) {
        const long needed = (Ptot + slots - 1) / slots;
        if (groups > needed) groups = needed;
    }
    const size_t ents = (size_t)c->nOffPad * slots;
    // per slot and entry: rays (2 doubles) + I1, fvec dI, two Jacobian dI (float) + compact index
    const size_t perGroup = ents * (2 * sizeof(double) + 5 * 4);
    const size_t budget = (size_t)48 << 30;  // HBM budget for the per-slot pixel slabs
    long cap = (long)(budget / perGroup);
    if (cap < 1) cap = 1;
    if (groups > cap) groups = cap;
    // the summed passes address a slab array with a 32-bit byte offset
    const long cap32 = (long)((((size_t)1 << 32) - ((size_t)1 << 20)) / (ents * sizeof(double) * (FM3D_RAY_AOS ? 2 : 1)));
    if (groups > cap32) groups = cap32;
    if (groups < 1) groups = 1;
    *out = groups;
    return FM3D_OK;
}

int run_lm_multi(fm3d_ctx* c, const LMSrc* src, int nProb, fm3d_lm_stats* stats, hipEvent_t e0, hipEvent_t e1) {
    int r;
    if (nProb < 1 || nProb > fm3d::kLMMaxProblems) return fail(c, FM3D_ERR_INVALID, "bad LM problem count");
    if ((r = ensure_offsets(c))) return r;
    const fm3d::Camera cam = lm_camera(c->cam);
    const int levels = c->s.pyramids;
    long Ptot = 0;
    for (int j = 0; j < nProb; j++) {
        fm3d_ctx* q = src[j].c;
        if (q->pyr1.empty()) return fail(c, FM3D_ERR_INVALID, "fm3d_set_images (NormalOptimizer::setImages) not called");
        if (!q->haveG12) return fail(c, FM3D_ERR_INVALID, "g12 not set (SingleCameraTriangulator::setg12)");
        if (q != c && (q->device != c->device || q->s.pyramids != levels || q->s.pixelsRay != c->s.pixelsRay ||
                       std::memcmp(&q->cam, &c->cam, sizeof(c->cam)) != 0 || q->s.boundWidth != c->s.boundWidth ||
                       q->s.boundHeight != c->s.boundHeight || q->s.zThresholdMax != c->s.zThresholdMax ||
                       q->s.epsilonLMMIN != c->s.epsilonLMMIN || q->s.lmReduction != c->s.lmReduction))
            return fail(c, FM3D_ERR_INVALID, "linked contexts need one device, camera and LM settings");
        const int P = src[j].P;
        HIPCHK(c, q->lmNormals.ensure((size_t)(P + 1) * 3 * sizeof(double)));
        HIPCHK(c, q->lmStatus.ensure((size_t)(P + 1) * sizeof(int)));
        HIPCHK(c, q->lmInfo.ensure((size_t)(P + 1) * 8 * sizeof(int)));
        HIPCHK(c, q->lmNfev.ensure((size_t)(P + 1) * 8 * sizeof(int)));
        HIPCHK(c, q->lmMdat.ensure((size_t)(P + 1) * sizeof(int)));
        HIPCHK(c, q->pcnt.ensure(64));
        Ptot += P;
    }
    HIPCHK(c, c->lmQueue.ensure(64 * sizeof(int)));
    HIPCHK(c, c->lmStat.ensure(256));
    // persistent workgroups of fm3d::kLM2Slots term waves (one point each) + a chain wave, or in the
    // tree-reduction mode kLM2Slots + 1 term waves; slots refill from the queue (fm3d_lm2.hip)
    // the settings field alone picks the mode (no environment override: ADVICE r05; the tree mode
    // fails the parity gate, profiles/r05_full_parity.json)
    if (c->s.lmReduction != 0 && c->s.lmReduction != 1)
        return fail(c, FM3D_ERR_INVALID, "lmReduction must be 0 (pixel order) or 1 (tree)");
    const bool tree = c->s.lmReduction != 0;
    const int slots = fm3d::kLM2Slots + (tree ? 1 : 0);
    // one pose for all problems: the single-pose kernel (entry 0 of the table serves them all)
    bool multiPose = false;
    for (int j = 1; j < nProb; j++)
        multiPose |= std::memcmp(src[j].c->R2, src[0].c->R2, sizeof(c->R2)) != 0 ||
                     std::memcmp(src[j].c->t2, src[0].c->t2, sizeof(c->t2)) != 0;
    const void* kptr = tree ? (multiPose ? reinterpret_cast<const void*>(fm3d::lm2_kernel<true, true>)
                                         : reinterpret_cast<const void*>(fm3d::lm2_kernel<false, true>))
                            : (multiPose ? reinterpret_cast<const void*>(fm3d::lm2_kernel<true, false>)
                                         : reinterpret_cast<const void*>(fm3d::lm2_kernel<false, false>));
    long groups = 0;
    int r0;
    if ((r0 = lm_groups(c, kptr, slots, Ptot, &groups))) return r0;
    const size_t ents = (size_t)c->nOffPad * slots;
    // +8 KiB: the passes prefetch up to eight 64-entry chunks past a slot's last entry
    HIPCHK(c, c->slab.ensure(ents * 2 * sizeof(double) * groups + 16384));
    HIPCHK(c, c->slabI1.ensure(ents * 5 * 4 * groups + 16384));
    fm3d::LMParams p{};
    p.nProb = nProb;
    p.cam = cam;
    {   // per problem: its pose as a small global table (re-read per chunk by the LM kernel), and
        // the problem table; both from pinned memory (the copies may run after this returns)
        HIPCHK(c, hipEventSynchronize(c->evProj));  // the previous launch's copies out of hProj ran
        const size_t pcBytes = (sizeof(fm3d::ProjConst) + 255) / 256 * 256;
        HIPCHK(c, c->hProj.ensure(pcBytes * nProb + sizeof(fm3d::LMProblem) * nProb));
        char* hp = c->hProj.as<char>();
        fm3d::LMProblem* hpr = (fm3d::LMProblem*)(hp + pcBytes * nProb);
        HIPCHK(c, c->lmProj.ensure(pcBytes * nProb + sizeof(fm3d::LMProblem) * nProb));
        const size_t Gn = (size_t)groups * slots * c->nOffPad;  // entries per slab array
        for (int j = 0; j < nProb; j++) {
            fm3d_ctx* q = src[j].c;
            fm3d::ProjConst& pc = *(fm3d::ProjConst*)(hp + pcBytes * j);
            std::memcpy(pc.R, q->R2, sizeof(pc.R));
            std::memcpy(pc.t, q->t2, sizeof(pc.t));
            pc.cam = cam;
            pc.k2d = 2. * cam.k[2];
            pc.k3d = 2. * cam.k[3];
            pc.slabRX = (const char*)c->slab.p;
            pc.slabRY = FM3D_RAY_AOS ? pc.slabRX + sizeof(double) : pc.slabRX + Gn * sizeof(double);
            pc.slabI1 = (const char*)c->slabI1.p;
            pc.slabDF = (char*)c->slabI1.p + Gn * 4;
            pc.slabDJ0 = pc.slabDF + Gn * 4;
            pc.slabDJ1 = pc.slabDJ0 + Gn * 4;
            fm3d::LMProblem& pr = hpr[j];
            pr.points = q->pts.as<double>();
            pr.Pdev = src[j].Pdev;
            pr.P = src[j].P;
            pr.lvl = q->lvlDesc.as<LevelDesc>();
            pr.normals = q->lmNormals.as<double>();
            pr.status = q->lmStatus.as<int>();
            pr.info = q->lmInfo.as<int>();
            pr.nfev = q->lmNfev.as<int>();
            pr.mdat = q->lmMdat.as<int>();
            pr.stat = (unsigned long long*)(q->pcnt.as<char>() + 16);
            pr.projOff = (unsigned)(pcBytes * j);
        }
        HIPCHK(c, hipMemcpyAsync(c->lmProj.p, hp, pcBytes * nProb + sizeof(fm3d::LMProblem) * nProb,
                                 hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipEventRecord(c->evProj, c->stream));
        p.proj = c->lmProj.as<fm3d::ProjConst>();
        p.prob = (const fm3d::LMProblem*)(c->lmProj.as<char>() + pcBytes * nProb);
    }
    p.levels = levels;
    p.offsets = c->offsets.as<int2>();
    p.nOff = c->nOff;
    p.nOffPad = c->nOffPad;
    p.boundW = c->s.boundWidth;
    p.boundH = c->s.boundHeight;
    p.epsfcn = c->s.epsilonLMMIN;
    p.cmax = (int)(2 * c->s.zThresholdMax);  // isInBoundingBox: int cMax = 2*z_threshold_max_ (:648)
    p.queue = c->lmQueue.as<int>();
    p.slab = c->slab.as<double>();
    p.slabI1 = c->slabI1.as<float>();
    p.nWaves = groups;
    p.statEval = c->lmStat.as<unsigned long long>();
    p.statPix = c->lmStat.as<unsigned long long>() + 1;
    p.overflow = (int*)(c->lmStat.as<unsigned long long>() + 2);
    p.statPass = c->lmStat.as<unsigned long long>() + 3;
    c->lmGroups = groups;
    {   // guards against a broken state machine (never expected to trigger): passes per slot
        // <= its points x levels x (300 evaluations + QR passes), and a wall-clock limit
        const long long perSlot = (Ptot + groups * slots - 1) / (groups * slots) + 1;
        p.maxIter = perSlot * (long long)(levels + 1) * 1600 + 10000;
        int khz = 0;
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device) != hipSuccess || khz <= 0) khz = 100000;
        const char* ms = getenv("FM3D_LM_MAX_SECONDS");  // watchdog (tests lower it; fractions allowed)
        const double secs = ms && atof(ms) > 0 ? atof(ms) : 300.;
        p.maxTicks = (long long)((double)khz * 1000. * secs);
        c->wallKhz = khz;
        const char* co = getenv("FM3D_LM_COOP");  // A/B switch for the tail help
        p.coop = co ? atoi(co) : 1;
        if (tree) p.coop = 0;  // a helper's chunks would leave the lanes' chunk order of the tree
        const char* sf = getenv("FM3D_LM_SAFE");  // test switch: the guarded pass forms only
        p.safe = sf ? atoi(sf) : 0;
    }
    // the counters (incl. the overflow word) are reset for every call, also for P == 0; with points,
    // the queue, the min-start word and every problem's statuses / info / nfev too -- one kernel
    {
        fm3d::LMReset rz{};
        rz.stat = c->lmStat.as<unsigned long long>();
        rz.queue = Ptot > 0 ? c->lmQueue.as<int>() : nullptr;
        rz.nProb = nProb;
        for (int j = 0; j < nProb; j++) {
            fm3d_ctx* q = src[j].c;
            rz.pcnt16[j] = q->pcnt.as<int>() + 4;
            rz.status[j] = q->lmStatus.as<int>();
            rz.info[j] = q->lmInfo.as<int>();
            rz.nfev[j] = q->lmNfev.as<int>();
            rz.P[j] = Ptot > 0 && src[j].P > 0 ? src[j].P : 0;
        }
        if (Ptot > 0) HIPCHK(c, hipEventRecord(e0, c->stream));
        fm3d::launch_lm_reset(rz, c->stream);
        HIPCHK(c, hipGetLastError());
    }
    if (Ptot > 0) {
        // one launch: every slot runs its point through all levels, coarsest first
        // (optimize_pyramid :225-241)
        // through the runtime's launch by address (not a call through a cast function pointer, which
        // the host sanitizers' function-type check rejects: tests/test_sanitizers.py)
        void* kargs[] = {&p};
        HIPCHK(c, hipLaunchKernel(kptr, dim3((unsigned)groups), dim3(fm3d::kLM2Threads), kargs, 0, c->stream));
        HIPCHK(c, hipEventRecord(e1, c->stream));
    }
    if (stats) {
        std::memset(stats, 0, sizeof(*stats));
        stats->points_in = Ptot;
    }
    return FM3D_OK;
}

// LM normals over c's own points (c->pts: P, or the bound P with the count at Pdev)
int run_lm(fm3d_ctx* c, int P, const int* Pdev, fm3d_lm_stats* stats, hipEvent_t e0, hipEvent_t e1) {
    const LMSrc one{c, P, Pdev};
    return run_lm_multi(c, &one, 1, stats, e0, e1);
}

// the two images into pinned staging and their pyramids (pyrDown chain) on the context stream;
// sync: wait for them before returning (fm3d_set_images: the caller may read them back at once)
int set_images_impl(fm3d_ctx* c, const uint8_t* img1, const uint8_t* img2, int width, int height, int stride,
                    bool sync = true, bool waitStaging = true) {
    if (!img1 || !img2 || width <= 0 || height <= 0 || stride < width)
        return fail(c, FM3D_ERR_INVALID, "bad image arguments");
    const int levels = c->s.pyramids;
    if (levels < 0 || levels > 7) return fail(c, FM3D_ERR_UNSUPPORTED, "pyramids must be in [0, 7]");
    int r;
    if (waitStaging && (r = staging_wait(c))) return r;
    c->w = width;
    c->h = height;
    c->lw.assign(levels + 1, 0);
    c->lh.assign(levels + 1, 0);
    c->pyr1.resize(levels + 1);
    c->pyr2.resize(levels + 1);
    c->lw[0] = width;
    c->lh[0] = height;
    for (int L = 1; L <= levels; L++) {  // cv::pyrDown size ((w+1)/2, (h+1)/2)
        c->lw[L] = (c->lw[L - 1] + 1) / 2;
        c->lh[L] = (c->lh[L - 1] + 1) / 2;
    }
    // the zero guards: cleared when a level's buffer is new or the image size changed, not per frame
    // pair -- nothing but the guard clearing writes past a level's w x h pixels, so they stay zero
    // (each clear is a fill kernel, which in a stream of frame pairs waits for CUs behind the other
    // pairs' LM launches)
    bool fresh = c->pyrGuardW != width || c->pyrGuardH != height || c->pyrGuardLevels != levels;
    for (int L = 0; L <= levels; L++) {
        size_t bytes = (size_t)c->lw[L] * c->lh[L] + kGuard(c->lw[L]);
        void* p1 = c->pyr1[L].p;
        void* p2 = c->pyr2[L].p;
        HIPCHK(c, c->pyr1[L].ensure(bytes));
        HIPCHK(c, c->pyr2[L].ensure(bytes));
        fresh |= c->pyr1[L].p != p1 || c->pyr2[L].p != p2;
    }
    for (int L = 0; fresh && L <= levels; L++) {
        // a level's pixels are overwritten (level 0 by the copy below, the others by pyrDown): the
        // guard past them is what needs clearing
        const size_t img = (size_t)c->lw[L] * c->lh[L];
        HIPCHK(c, hipMemsetAsync((char*)c->pyr1[L].p + img, 0, c->pyr1[L].bytes - img, c->stream));
        HIPCHK(c, hipMemsetAsync((char*)c->pyr2[L].p + img, 0, c->pyr2[L].bytes - img, c->stream));
    }
    c->pyrGuardW = width;
    c->pyrGuardH = height;
    c->pyrGuardLevels = levels;
    const size_t wh = (size_t)width * height;
    HIPCHK(c, c->hImg.ensure(2 * wh));
    for (int y = 0; y < height; y++) {
        std::memcpy(c->hImg.as<uint8_t>() + (size_t)y * width, img1 + (size_t)y * stride, width);
        std::memcpy(c->hImg.as<uint8_t>() + wh + (size_t)y * width, img2 + (size_t)y * stride, width);
    }
    HIPCHK(c, hipMemcpyAsync(c->pyr1[0].p, c->hImg.p, wh, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->pyr2[0].p, c->hImg.as<uint8_t>() + wh, wh, hipMemcpyHostToDevice, c->stream));
    for (int L = 1; L <= levels; L++) {
        fm3d::launch_pyrdown(c->pyr1[L - 1].as<uint8_t>(), c->lw[L - 1], c->lh[L - 1], c->pyr1[L].as<uint8_t>(),
                             c->stream);
        fm3d::launch_pyrdown(c->pyr2[L - 1].as<uint8_t>(), c->lw[L - 1], c->lh[L - 1], c->pyr2[L].as<uint8_t>(),
                             c->stream);
    }
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, c->hTab.ensure((levels + 1) * sizeof(LevelDesc)));
    LevelDesc* d = c->hTab.as<LevelDesc>();
    for (int L = 0; L <= levels; L++) d[L] = LevelDesc{c->pyr1[L].as<uint8_t>(), c->pyr2[L].as<uint8_t>(), c->lw[L], c->lh[L]};
    HIPCHK(c, c->lvlDesc.ensure((levels + 1) * sizeof(LevelDesc)));
    HIPCHK(c, hipMemcpyAsync(c->lvlDesc.p, d, (levels + 1) * sizeof(LevelDesc), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipEventRecord(c->evStage, c->stream));
    if (sync) HIPCHK(c, hipStreamSynchronize(c->stream));
    return FM3D_OK;
}

// ---------------- SURF plan (host side of fm3d_surf.hip; the oracle's orc_surf.c formulas) ----------------
int cv_round_h(double v) { return (int)std::lrint(v); }

// resizeHaarPattern (surf.cpp) in float, cvRound to nearest even
void surf_resize_haar(const int src[][5], fm3d::SurfHF* dst, int n, int oldSize, int newSize, int widthStep) {
    const float ratio = (float)newSize / oldSize;
    for (int k = 0; k < n; k++) {
        const int dx1 = cv_round_h(ratio * src[k][0]), dy1 = cv_round_h(ratio * src[k][1]);
        const int dx2 = cv_round_h(ratio * src[k][2]), dy2 = cv_round_h(ratio * src[k][3]);
        dst[k].p0 = dy1 * widthStep + dx1;
        dst[k].p1 = dy2 * widthStep + dx1;
        dst[k].p2 = dy1 * widthStep + dx2;
        dst[k].p3 = dy2 * widthStep + dx2;
        dst[k].w = src[k][4] / ((float)(dx2 - dx1) * (dy2 - dy1));
    }
}

struct SurfPlan {
    std::vector<fm3d::SurfLayer> L;
    std::vector<fm3d::SurfMid> M;
    size_t detFloats = 0;
    long long hTotal = 0, mTotal = 0, candCap = 0;
};

// fastHessianDetector's layer table: (nOctaveLayers + 2) * nOctaves layers, size (9 + 6*layer) <<
// octave, sample step 1 << octave; calcLayerDetAndTrace skips layers larger than the image
SurfPlan surf_plan(int w, int h, int octaves, int layers) {
    static const int dx_s[3][5] = {{0, 2, 3, 7, 1}, {3, 2, 6, 7, -2}, {6, 2, 9, 7, 1}};
    static const int dy_s[3][5] = {{2, 0, 7, 3, 1}, {2, 3, 7, 6, -2}, {2, 6, 7, 9, 1}};
    static const int dxy_s[4][5] = {{1, 1, 4, 4, 1}, {5, 1, 8, 4, -1}, {1, 5, 4, 8, -1}, {5, 5, 8, 8, 1}};
    SurfPlan P;
    for (int o = 0; o < octaves; o++)
        for (int l = 0; l < layers + 2; l++) {
            fm3d::SurfLayer y{};
            y.size = (9 + 6 * l) << o;
            y.step = 1 << o;
            y.rows = h / y.step;
            y.cols = w / y.step;
            y.off = P.detFloats;
            P.detFloats += (size_t)y.rows * y.cols;
            y.first = P.hTotal;
            if (y.size <= h && y.size <= w) {
                y.si = 1 + (h - y.size) / y.step;
                y.sj = 1 + (w - y.size) / y.step;
                y.margin = (y.size / 2) / y.step;
                surf_resize_haar(dx_s, y.hf, 3, 9, y.size, w + 1);
                surf_resize_haar(dy_s, y.hf + 3, 3, 9, y.size, w + 1);
                surf_resize_haar(dxy_s, y.hf + 6, 4, 9, y.size, w + 1);
            }
            P.hTotal += (long long)y.si * y.sj;
            P.L.push_back(y);
        }
    for (int o = 0; o < octaves; o++)
        for (int l = 1; l <= layers; l++) {
            const int idx = o * (layers + 2) + l;
            fm3d::SurfMid m{};
            m.layer = idx;
            m.octave = o;
            m.rows = P.L[idx].rows;
            m.cols = P.L[idx].cols;
            m.margin = (P.L[idx + 1].size / 2) / P.L[idx].step + 1;
            m.first = P.mTotal;
            P.mTotal += (long long)m.rows * m.cols;
            // strict maxima of a 3x3 neighbourhood: at most one per 2x2 block
            P.candCap += (long long)((m.rows + 1) / 2) * ((m.cols + 1) / 2);
            P.M.push_back(m);
        }
    P.candCap += 16;
    return P;
}

// getGaussianKernel(20, 3.3, CV_32F) outer product: SURFInvoker's descriptor weights DW
std::vector<float> surf_dw() {
    float g[20];
    const double scale2X = -0.5 / (3.3 * 3.3);
    double sum = 0;
    for (int i = 0; i < 20; i++) {
        const double x = i - (20 - 1) * 0.5;
        g[i] = (float)std::exp(scale2X * x * x);
        sum += g[i];
    }
    sum = 1. / sum;
    for (int i = 0; i < 20; i++) g[i] = (float)(g[i] * sum);
    std::vector<float> dw(400);
    for (int i = 0; i < 20; i++)
        for (int j = 0; j < 20; j++) dw[i * 20 + j] = g[i] * g[j];
    return dw;
}

// SURFInvoker's orientation samples (the constructor's apt / aptw): the disc of radius 6, i (x)
// outer, j (y) inner, weights G(i) * G(j), G = getGaussianKernel(13, 2.5, CV_32F)
const fm3d::SurfOri& surf_ori() {
    static const fm3d::SurfOri ori = [] {
        fm3d::SurfOri o{};
        float g[13];
        const double scale2X = -0.5 / (2.5 * 2.5);
        double sum = 0;
        for (int i = 0; i < 13; i++) {
            const double x = i - (13 - 1) * 0.5;
            g[i] = (float)std::exp(scale2X * x * x);
            sum += g[i];
        }
        sum = 1. / sum;
        for (int i = 0; i < 13; i++) g[i] = (float)(g[i] * sum);
        for (int i = -6; i <= 6; i++)
            for (int j = -6; j <= 6; j++)
                if (i * i + j * j <= 36) {
                    o.ax[o.n] = i;
                    o.ay[o.n] = j;
                    o.w[o.n++] = g[i + 6] * g[j + 6];
                }
        return o;
    }();
    return ori;
}

// ---------------- ORB (host side of fm3d_orb.hip; the oracle's orc_orb.c formulas) ----------------
// getScale (orb.cpp): (float)pow(scaleFactor, level)
float orb_scale(double scaleFactor, int level) { return (float)std::pow(scaleFactor, (double)level); }

struct OrbPlan {
    std::vector<fm3d::OrbLevel> L;
    long long total = 0;
};

// the pyramid levels: size cvRound(cols * (1 / getScale)), concatenated pixel after pixel
OrbPlan orb_plan(int w, int h, double scaleFactor, int nl) {
    OrbPlan P;
    for (int l = 0; l < nl; l++) {
        const float scale = 1 / orb_scale(scaleFactor, l);
        fm3d::OrbLevel v;
        v.w = (int)std::lrint((float)(w * scale));
        v.h = (int)std::lrint((float)(h * scale));
        v.first = P.total;
        P.total += (long long)std::max(v.w, 0) * std::max(v.h, 0);
        P.L.push_back(v);
    }
    return P;
}

short sat_short(float v) {
    const long i = std::lrint(v);
    return (short)(i < -32768 ? -32768 : (i > 32767 ? 32767 : i));
}

// resize(INTER_LINEAR)'s fixed-point tables for src (sw x sh) -> dst (dw x dh), packed as
// [xofs dw][yofs dh] ints then [alpha 2dw][beta 2dh] shorts; returns xmax
int orb_resize_tabs(int sw, int sh, int dw, int dh, std::vector<int>& ofs, std::vector<short>& ab) {
    const double scale_x = 1. / ((double)dw / sw), scale_y = 1. / ((double)dh / sh);
    int xmax = dw;
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = (int)std::floor(fx);
        fx -= sx;
        if (sx < 0) {
            fx = 0;
            sx = 0;
        }
        if (sx + 1 >= sw) {
            xmax = std::min(xmax, dx);
            if (sx >= sw - 1) {
                fx = 0;
                sx = sw - 1;
            }
        }
        ofs.push_back(sx);
        ab.push_back(sat_short((1.f - fx) * 2048));
        ab.push_back(sat_short(fx * 2048));
    }
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        const int sy = (int)std::floor(fy);
        fy -= sy;
        ofs.push_back(sy);
        ab.push_back(sat_short((1.f - fy) * 2048));
        ab.push_back(sat_short(fy * 2048));
    }
    return xmax;
}

// VResizeLinearVec_32s8u's columns: the 16-wide loop, then the 4-wide one while x < width - 4
int orb_vresize_sse_end(int width) {
    int x = 0;
    for (; x <= width - 16; x += 16) {}
    for (; x < width - 4; x += 4) {}
    return x;
}

// image -> level 0, then every level from the previous one (orb.cpp's pyramid loop)
int orb_build_pyramid(fm3d_ctx* c, const uint8_t* img, int w, int h, const OrbPlan& P) {
    const int nl = (int)P.L.size();
    HIPCHK(c, c->orbPyr.ensure((size_t)P.total + 64));
    HIPCHK(c, c->orbLev.ensure(P.L.size() * sizeof(fm3d::OrbLevel)));
    HIPCHK(c, hipMemcpyAsync(c->orbPyr.p, img, (size_t)w * h, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->orbLev.p, P.L.data(), P.L.size() * sizeof(fm3d::OrbLevel), hipMemcpyHostToDevice,
                             c->stream));
    std::vector<int> ofs;
    std::vector<short> ab;
    std::vector<int> xmax(nl, 0);
    std::vector<size_t> oOfs(nl, 0), oAb(nl, 0);
    for (int l = 1; l < nl; l++) {
        oOfs[l] = ofs.size();
        oAb[l] = ab.size();
        xmax[l] = orb_resize_tabs(P.L[l - 1].w, P.L[l - 1].h, P.L[l].w, P.L[l].h, ofs, ab);
    }
    const size_t ofsBytes = ofs.size() * sizeof(int);
    HIPCHK(c, c->orbTab.ensure(ofsBytes + ab.size() * sizeof(short) + 64));
    if (!ofs.empty()) {
        HIPCHK(c, hipMemcpyAsync(c->orbTab.p, ofs.data(), ofsBytes, hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipMemcpyAsync(static_cast<char*>(c->orbTab.p) + ofsBytes, ab.data(), ab.size() * sizeof(short),
                                 hipMemcpyHostToDevice, c->stream));
    }
    const int* T = c->orbTab.as<int>();
    const short* A = reinterpret_cast<const short*>(static_cast<const char*>(c->orbTab.p) + ofsBytes);
    uint8_t* pyr = c->orbPyr.as<uint8_t>();
    for (int l = 1; l < nl; l++) {
        const fm3d::OrbLevel &s0 = P.L[l - 1], &d0 = P.L[l];
        if (d0.w <= 0 || d0.h <= 0 || s0.w <= 0 || s0.h <= 0) continue;
        fm3d::launch_orb_resize(pyr + s0.first, s0.w, s0.h, pyr + d0.first, d0.w, d0.h, T + oOfs[l], A + oAb[l],
                                T + oOfs[l] + d0.w, A + oAb[l] + 2 * d0.w, xmax[l], orb_vresize_sse_end(d0.w),
                                c->stream);
    }
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(c->stream));  // ofs / ab leave scope
    return FM3D_OK;
}

// KeyPointsFilter::retainBest with libstdc++'s own nth_element / partition (the order they leave
// decides which tied keypoints survive and the output order)
int orb_retain_best(fm3d_keypoint* k, int n, int npts) {
    if (npts >= 0 && n > npts) {
        if (npts == 0) return 0;
        auto greater = [](const fm3d_keypoint& a, const fm3d_keypoint& b) { return a.response > b.response; };
        std::nth_element(k, k + npts, k + n, greater);
        const float amb = k[npts - 1].response;
        return (int)(std::partition(k + npts, k + n, [amb](const fm3d_keypoint& p) { return p.response >= amb; }) - k);
    }
    return n;
}

// the 512-point pattern: the caller's, else makeRandomPattern(patchSize) (cv::RNG(0x34985739))
int orb_upload_pattern(fm3d_ctx* c, int patchSize) {
    std::vector<int> xy = c->orbUserPattern;
    if (xy.empty()) {
        uint64_t state = 0x34985739;
        const int a = -patchSize / 2, b = patchSize / 2 + 1;
        for (int i = 0; i < 1024; i++) {
            state = (uint64_t)(unsigned)state * 4164903690U + (unsigned)(state >> 32);
            xy.push_back((int)((unsigned)state % (unsigned)(b - a) + (unsigned)a));
        }
    }
    HIPCHK(c, c->orbPat.ensure(1024 * sizeof(int)));
    HIPCHK(c, hipMemcpyAsync(c->orbPat.p, xy.data(), 1024 * sizeof(int), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return FM3D_OK;
}

fm3d::OrbBlurK orb_blur_kernel() {
    fm3d::OrbBlurK k;
    float g[7];
    const double scale2X = -0.5 / (2.0 * 2.0);
    double sum = 0;
    for (int i = 0; i < 7; i++) {
        const double x = i - 3.0;
        g[i] = (float)std::exp(scale2X * x * x);
        sum += g[i];
    }
    sum = 1. / sum;
    for (int i = 0; i < 7; i++) g[i] = (float)(g[i] * sum);
    for (int i = 0; i < 7; i++) k.ik[i] = (int)std::lrint(g[i] * 256.f);
    for (int i = 0; i < 4; i++) k.fk[i] = (float)(k.ik[3 + i] * (1. / 65536));
    return k;
}

// blurred levels + descriptors of the (device) keypoints kp[0..n) in level coordinates
int orb_describe(fm3d_ctx* c, const OrbPlan& P, int n, uint8_t* desc) {
    if (n <= 0) return FM3D_OK;
    int r;
    if ((r = orb_upload_pattern(c, c->s.orbPatchSize))) return r;
    HIPCHK(c, c->orbR.ensure((size_t)P.total * sizeof(int) + 64));
    HIPCHK(c, c->orbBlur.ensure((size_t)P.total + 64));
    HIPCHK(c, c->orbDesc.ensure((size_t)n * 32));
    fm3d::launch_orb_blur(c->orbPyr.as<uint8_t>(), c->orbLev.as<fm3d::OrbLevel>(), (int)P.L.size(), P.total,
                          orb_blur_kernel(), c->orbR.as<int>(), c->orbBlur.as<uint8_t>(), c->stream);
    fm3d::launch_orb_desc(c->orbBlur.as<uint8_t>(), c->orbLev.as<fm3d::OrbLevel>(), c->orbKp.as<fm3d_keypoint>(), n,
                          c->orbPat.as<int>(), c->orbDesc.as<uint8_t>(), c->stream);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(desc, c->orbDesc.p, (size_t)n * 32, hipMemcpyDeviceToHost, c->stream));
    return FM3D_OK;
}

int orb_check_settings(fm3d_ctx* c) {
    const fm3d_settings& S = c->s;
    if (S.orbNumLevels < 1 || S.orbNumLevels > 64 || !(S.orbScaleFactor > 1.0) || S.orbNumFeatures < 0 ||
        S.orbEdgeThreshold < 0 || S.orbPatchSize < 2 || S.orbPatchSize > 124 || S.orbFastThreshold < 0)
        return fail(c, FM3D_ERR_INVALID, "ORB NumLevels / ScaleFactor / NumFeatures / edgeThreshold / patchSize out of range");
    // the descriptor reads pattern points up to patchSize/2 * sqrt(2) + 1 from the centre and the
    // blur 3 more: inside the edge border, as OpenCV's defaults guarantee
    if (S.orbEdgeThreshold < (int)std::ceil(S.orbPatchSize / 2 * 1.4143) + 4)
        return fail(c, FM3D_ERR_INVALID, "ORB edgeThreshold too small for patchSize (reads past the level border)");
    return FM3D_OK;
}

// ---------------- SIFT (host side of fm3d_sift.hip; the oracle's orc_sift.c formulas) ----------------
// the pyramid plan: level sizes and offsets, Gaussian levels nOct * (L + 3), DoG levels nOct * (L + 2)
struct SiftPlan {
    int firstOctave = 0, nOct = 0, L = 0;
    std::vector<fm3d::SiftLevel> G, D;
    long long gTotal = 0, dTotal = 0;
};

// false when an octave would be empty (OpenCV's resize asserts there)
bool sift_plan(int w, int h, int firstOctave, int nOct, int L, SiftPlan& P) {
    P = SiftPlan{};
    P.firstOctave = firstOctave;
    P.nOct = nOct;
    P.L = L;
    int ow = firstOctave < 0 ? 2 * w : w, oh = firstOctave < 0 ? 2 * h : h;
    for (int o = 0; o < nOct; o++) {
        if (o > 0) {
            ow /= 2;
            oh /= 2;
        }
        if (ow < 1 || oh < 1) return false;
        for (int i = 0; i < L + 3; i++) {
            P.G.push_back({ow, oh, P.gTotal});
            P.gTotal += (long long)ow * oh;
        }
        for (int i = 0; i < L + 2; i++) {
            P.D.push_back({ow, oh, P.dTotal});
            P.dTotal += (long long)ow * oh;
        }
    }
    return true;
}

int sift_num_octaves(int w, int h, int firstOctave) {
    const int bw = firstOctave < 0 ? 2 * w : w, bh = firstOctave < 0 ? 2 * h : h;
    return (int)std::lrint(std::log((double)std::min(bw, bh)) / std::log(2.) - 2) - firstOctave;
}

// getGaussianKernel(cvRound(sigma*8+1)|1, sigma, CV_32F)
std::vector<float> sift_gauss_kernel(double sigma) {
    const int n = (int)std::lrint(sigma * 4 * 2 + 1) | 1;
    std::vector<float> cf(n);
    const double scale2X = -0.5 / (sigma * sigma);
    double sum = 0;
    for (int i = 0; i < n; i++) {
        const double x = i - (n - 1) * 0.5;
        cf[i] = (float)std::exp(scale2X * x * x);
        sum += cf[i];
    }
    sum = 1. / sum;
    for (int i = 0; i < n; i++) cf[i] = (float)(cf[i] * sum);
    return cf;
}

constexpr int kSiftMaxTaps = 65;  // the blur tile's LDS (r <= 32: sigma up to ~8)

// createInitialImage + buildGaussianPyramid (+ buildDoGPyramid) into siftG / siftD
int sift_build(fm3d_ctx* c, const uint8_t* img, int w, int h, const SiftPlan& P, bool dog) {
    const fm3d_settings& S = c->s;
    const int L = P.L, nl = L + 3;
    // the blur kernels: [0] sig_diff of the initial image, [i] sig[i] of the octave levels
    std::vector<std::vector<float>> taps(nl);
    {
        const float sigma = (float)S.siftSigma;
        const float sd = P.firstOctave < 0 ? std::sqrt(std::max(sigma * sigma - 0.5f * 0.5f * 4, 0.01f))
                                           : std::sqrt(std::max(sigma * sigma - 0.5f * 0.5f, 0.01f));
        taps[0] = sift_gauss_kernel(sd);
        const double k = std::pow(2., 1. / L);
        for (int i = 1; i < nl; i++) {
            const double sig_prev = std::pow(k, (double)(i - 1)) * S.siftSigma;
            const double sig_total = sig_prev * k;
            taps[i] = sift_gauss_kernel(std::sqrt(sig_total * sig_total - sig_prev * sig_prev));
        }
    }
    for (auto& t : taps)
        if ((int)t.size() > kSiftMaxTaps)
            return fail(c, FM3D_ERR_UNSUPPORTED, "SIFT sigma too large for the GPU blur tile (kernel > 65 taps)");
    std::vector<float> tapBuf((size_t)nl * 128, 0.f);
    for (int i = 0; i < nl; i++) std::copy(taps[i].begin(), taps[i].end(), tapBuf.begin() + (size_t)i * 128);
    HIPCHK(c, c->siftTaps.ensure(tapBuf.size() * sizeof(float)));
    HIPCHK(c, hipMemcpyAsync(c->siftTaps.p, tapBuf.data(), tapBuf.size() * sizeof(float), hipMemcpyHostToDevice,
                             c->stream));
    HIPCHK(c, c->siftImg.ensure((size_t)w * h));
    HIPCHK(c, hipMemcpyAsync(c->siftImg.p, img, (size_t)w * h, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, c->siftG.ensure((size_t)P.gTotal * sizeof(float) + 64));
    if (dog) HIPCHK(c, c->siftD.ensure((size_t)P.dTotal * sizeof(float) + 64));
    const int bw = P.G[0].w, bh = P.G[0].h;
    HIPCHK(c, c->siftBase.ensure((size_t)bw * bh * sizeof(float)));
    float* G = c->siftG.as<float>();
    float* D = dog ? c->siftD.as<float>() : nullptr;
    const float* T = c->siftTaps.as<float>();
    {
        fm3d::SiftResize rp{};
        rp.sw = w;
        rp.sh = h;
        rp.dw = bw;
        rp.dh = bh;
        rp.doubled = P.firstOctave < 0;
        rp.scx = 1. / ((double)bw / w);
        rp.scy = 1. / ((double)bh / h);
        rp.xmax = bw;
        for (int dx = 0; dx < bw; dx++) {  // resize's xmax: the first column whose right tap leaves the row
            const float fx = (float)((dx + 0.5) * rp.scx - 0.5);
            if ((int)std::floor(fx) + 1 >= w) {
                rp.xmax = dx;
                break;
            }
        }
        fm3d::launch_sift_init(c->siftImg.as<uint8_t>(), c->siftBase.as<float>(), rp, 1, c->stream);
        fm3d::launch_sift_blur(c->siftBase.as<float>(), G, nullptr, bw, bh, T, (int)taps[0].size(), 1, c->stream);
    }
    for (int o = 0; o < P.nOct; o++)
        for (int i = 0; i < nl; i++) {
            const fm3d::SiftLevel& d = P.G[o * nl + i];
            if (o == 0 && i == 0) continue;
            if (i == 0) {
                const fm3d::SiftLevel& s = P.G[(o - 1) * nl + L];
                fm3d::launch_sift_down(G + s.first, s.w, s.h, G + d.first, d.w, d.h, 1. / ((double)d.w / s.w),
                                       1. / ((double)d.h / s.h), c->stream);
            } else {
                const fm3d::SiftLevel& s = P.G[o * nl + i - 1];
                fm3d::launch_sift_blur(G + s.first, G + d.first, D ? D + P.D[o * (L + 2) + i - 1].first : nullptr, d.w,
                                       d.h, T + (size_t)i * 128, (int)taps[i].size(), 1, c->stream);
            }
        }
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, c->siftGL.ensure(P.G.size() * sizeof(fm3d::SiftLevel)));
    HIPCHK(c, hipMemcpyAsync(c->siftGL.p, P.G.data(), P.G.size() * sizeof(fm3d::SiftLevel), hipMemcpyHostToDevice,
                             c->stream));
    if (dog) {
        HIPCHK(c, c->siftDL.ensure(P.D.size() * sizeof(fm3d::SiftLevel)));
        HIPCHK(c, hipMemcpyAsync(c->siftDL.p, P.D.data(), P.D.size() * sizeof(fm3d::SiftLevel), hipMemcpyHostToDevice,
                                 c->stream));
    }
    // the host vectors leave scope: finish the copies
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return FM3D_OK;
}

int sift_check_settings(fm3d_ctx* c) {
    const fm3d_settings& S = c->s;
    if (S.siftOctaveLayers < 1 || S.siftOctaveLayers > 16 || S.siftNumFeatures < 0 || !(S.siftSigma > 0) ||
        !(S.siftContrastThreshold >= 0) || !(S.siftEdgeThreshold >= 0))
        return fail(c, FM3D_ERR_INVALID, "SIFT NumOctaveLayers / NumFeatures / Sigma / thresholds out of range");
    return FM3D_OK;
}

// KeyPointsFilter::removeDuplicated: KeyPoint_LessThan order with the index as the last key, the
// first of each group of equal (pt, size, angle) kept, input order preserved
int sift_remove_duplicated(std::vector<fm3d_keypoint>& k) {
    const int n = (int)k.size();
    if (n < 2) return n;
    std::vector<int> idx(n);
    for (int i = 0; i < n; i++) idx[i] = i;
    std::sort(idx.begin(), idx.end(), [&](int i, int j) {
        const fm3d_keypoint &a = k[i], &b = k[j];
        if (a.x != b.x) return a.x < b.x;
        if (a.y != b.y) return a.y < b.y;
        if (a.size != b.size) return a.size > b.size;
        if (a.angle != b.angle) return a.angle < b.angle;
        if (a.response != b.response) return a.response > b.response;
        if (a.octave != b.octave) return a.octave > b.octave;
        if (a.class_id != b.class_id) return a.class_id > b.class_id;
        return i < j;
    });
    std::vector<uint8_t> mask(n, 1);
    for (int i = 1, j = 0; i < n; i++) {
        const fm3d_keypoint &a = k[idx[i]], &b = k[idx[j]];
        if (a.x != b.x || a.y != b.y || a.size != b.size || a.angle != b.angle)
            j = i;
        else
            mask[idx[i]] = 0;
    }
    int j = 0;
    for (int i = 0; i < n; i++)
        if (mask[i]) k[j++] = k[i];
    k.resize(j);
    return j;
}

void sift_unpack_octave(const fm3d_keypoint& k, int& octave, int& layer) {
    octave = k.octave & 255;
    layer = (k.octave >> 8) & 255;
    octave = octave < 128 ? octave : (-128 | octave);
}

// SIFT::operator()(img, Mat(), kpts, desc, true) on keypoints that passed runByKeypointSize:
// the pyramid from firstOctave = min(0, octaves), nOctaves = max - first + 1 (reused when the detect
// call just built the same levels), calcDescriptors.  desc: m x 128 floats (host)
int sift_describe(fm3d_ctx* c, const uint8_t* img, int w, int h, const std::vector<fm3d_keypoint>& k, float* desc,
                  const SiftPlan* built) {
    const int m = (int)k.size(), L = c->s.siftOctaveLayers;
    if (m == 0) return FM3D_OK;
    int firstOctave = 0, maxOctave = INT_MIN, actualNLayers = 0;
    for (const auto& q : k) {
        int o, l;
        sift_unpack_octave(q, o, l);
        firstOctave = std::min(firstOctave, o);
        maxOctave = std::max(maxOctave, o);
        actualNLayers = std::max(actualNLayers, l - 2);
    }
    firstOctave = std::min(firstOctave, 0);
    if (firstOctave < -1 || actualNLayers > L)
        return fail(c, FM3D_ERR_INVALID, "SIFT compute: a keypoint octave < -1 or layer > nOctaveLayers + 2");
    const int nOct = maxOctave - firstOctave + 1;
    int r;
    SiftPlan P;
    if (built && built->firstOctave == firstOctave && built->nOct >= nOct) {
        P = *built;
    } else {
        if (!sift_plan(w, h, firstOctave, nOct, L, P))
            return fail(c, FM3D_ERR_INVALID, "SIFT compute: a keypoint octave the image cannot hold");
        if ((r = sift_build(c, img, w, h, P, false))) return r;
    }
    HIPCHK(c, c->siftKp.ensure((size_t)m * sizeof(fm3d_keypoint)));
    HIPCHK(c, c->siftDesc.ensure((size_t)m * 128 * sizeof(float)));
    HIPCHK(c, hipMemcpyAsync(c->siftKp.p, k.data(), (size_t)m * sizeof(fm3d_keypoint), hipMemcpyHostToDevice,
                             c->stream));
    fm3d::launch_sift_desc(c->siftG.as<float>(), c->siftGL.as<fm3d::SiftLevel>(), L, firstOctave,
                           c->siftKp.as<fm3d_keypoint>(), nullptr, m, c->siftDesc.as<float>(), c->stream);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(desc, c->siftDesc.p, (size_t)m * 128 * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return FM3D_OK;
}

// extractDescriptorsFromPatches with the SIFT extractor (descriptorsmatcher.cpp:133-174, 302-310): per
// patch SIFT::operator()(patch, Mat(), {kp}, desc, true) with kp = (center, size, angle -1, octave 0):
// firstOctave 0, one octave, and the descriptor reads level 0 of it, blur(patch, sig_diff) -- so every
// patch needs only that level (batched: one init and one blur launch for all patches)
int sift_patches(fm3d_ctx* c, const uint8_t* patches, int P, int size, float* desc) {
    int r;
    if ((r = sift_check_settings(c))) return r;
    if (P == 0) return FM3D_OK;
    hipSetDevice(c->device);
    const fm3d_settings& S = c->s;
    const float center = (float)(int)std::floor(size / 2);
    const fm3d_keypoint k{center, center, (float)size, -1.f, 1.f, 0, 0};
    const float sigma = (float)S.siftSigma;
    const std::vector<float> taps = sift_gauss_kernel(std::sqrt(std::max(sigma * sigma - 0.5f * 0.5f, 0.01f)));
    if ((int)taps.size() > kSiftMaxTaps)
        return fail(c, FM3D_ERR_UNSUPPORTED, "SIFT sigma too large for the GPU blur tile (kernel > 65 taps)");
    const size_t per = (size_t)size * size;
    std::vector<fm3d::SiftLevel> GL((size_t)P);
    std::vector<int> lvl((size_t)P);
    for (int p = 0; p < P; p++) {
        GL[p] = {size, size, (long long)(p * per)};
        lvl[p] = p;
    }
    std::vector<fm3d_keypoint> kp((size_t)P, k);
    HIPCHK(c, c->siftTaps.ensure(128 * sizeof(float)));
    HIPCHK(c, c->siftImg.ensure((size_t)P * per));
    HIPCHK(c, c->siftBase.ensure((size_t)P * per * sizeof(float)));
    HIPCHK(c, c->siftG.ensure((size_t)P * per * sizeof(float)));
    HIPCHK(c, c->siftGL.ensure((size_t)P * sizeof(fm3d::SiftLevel)));
    HIPCHK(c, c->siftPos.ensure((size_t)P * sizeof(int)));
    HIPCHK(c, c->siftKp.ensure((size_t)P * sizeof(fm3d_keypoint)));
    HIPCHK(c, c->siftDesc.ensure((size_t)P * 128 * sizeof(float)));
    HIPCHK(c, hipMemcpyAsync(c->siftTaps.p, taps.data(), taps.size() * sizeof(float), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->siftImg.p, patches, (size_t)P * per, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->siftGL.p, GL.data(), GL.size() * sizeof(fm3d::SiftLevel), hipMemcpyHostToDevice,
                             c->stream));
    HIPCHK(c, hipMemcpyAsync(c->siftPos.p, lvl.data(), lvl.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->siftKp.p, kp.data(), kp.size() * sizeof(fm3d_keypoint), hipMemcpyHostToDevice,
                             c->stream));
    fm3d::SiftResize rp{};
    rp.sw = rp.dw = size;
    rp.sh = rp.dh = size;
    rp.doubled = 0;
    fm3d::launch_sift_init(c->siftImg.as<uint8_t>(), c->siftBase.as<float>(), rp, P, c->stream);
    fm3d::launch_sift_blur(c->siftBase.as<float>(), c->siftG.as<float>(), nullptr, size, size, c->siftTaps.as<float>(),
                           (int)taps.size(), P, c->stream);
    fm3d::launch_sift_desc(c->siftG.as<float>(), c->siftGL.as<fm3d::SiftLevel>(), S.siftOctaveLayers, 0,
                           c->siftKp.as<fm3d_keypoint>(), c->siftPos.as<int>(), P, c->siftDesc.as<float>(), c->stream);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(desc, c->siftDesc.p, (size_t)P * 128 * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return FM3D_OK;
}

// FastFeatureDetector(thr, nonmax).detect (features2d/src/fast.cpp): FAST-9 on the image itself, the
// ORB level-0 kernels with no edge border; KeyPoint(x, y, 7, -1, score) in raster order, the score 0
// without non-max suppression (FAST_t computes it only for the suppression)
int fast_detect(fm3d_ctx* c, const uint8_t* img, int w, int h, int thr, bool nonmax, std::vector<fm3d_keypoint>& k) {
    k.clear();
    thr = std::min(std::max(thr, 0), 255);
    const long long total = (long long)w * h;
    if (total > INT32_MAX / 2) return fail(c, FM3D_ERR_INVALID, "image too large for FAST");
    const fm3d::OrbLevel lv{w, h, 0};
    int r;
    if ((r = ensure_scan_tmp(c, (int)total))) return r;
    HIPCHK(c, c->orbPyr.ensure((size_t)total + 64));
    HIPCHK(c, c->orbLev.ensure(sizeof(fm3d::OrbLevel)));
    HIPCHK(c, c->orbMap.ensure((size_t)total * sizeof(uint16_t) + 64));
    HIPCHK(c, c->orbFlag.ensure((size_t)(total + 1) * sizeof(int)));
    HIPCHK(c, c->orbPos.ensure((size_t)(total + 1) * sizeof(int)));
    HIPCHK(c, hipMemcpyAsync(c->orbPyr.p, img, (size_t)total, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->orbLev.p, &lv, sizeof(lv), hipMemcpyHostToDevice, c->stream));
    fm3d::launch_orb_fast(c->orbPyr.as<uint8_t>(), c->orbLev.as<fm3d::OrbLevel>(), 1, total, thr, 0, nonmax ? 1 : 0,
                          c->orbMap.as<uint16_t>(), c->orbFlag.as<int>(), c->stream);
    fm3d::launch_exclusive_scan(c->orbFlag.as<int>(), (int)total, c->orbPos.as<int>(), c->count.as<int>(), c->scanTmp.p,
                                c->stream);
    HIPCHK(c, hipGetLastError());
    int nc = 0;
    HIPCHK(c, hipMemcpyAsync(&nc, c->count.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (nc == 0) return FM3D_OK;
    HIPCHK(c, c->orbKp.ensure((size_t)(nc + 1) * sizeof(fm3d_keypoint)));
    fm3d::launch_orb_fast_scatter(c->orbMap.as<uint16_t>(), c->orbLev.as<fm3d::OrbLevel>(), 1, total,
                                  c->orbFlag.as<int>(), c->orbPos.as<int>(), c->orbKp.as<fm3d_keypoint>(), c->stream);
    k.resize(nc);
    HIPCHK(c, hipMemcpyAsync(k.data(), c->orbKp.p, (size_t)nc * sizeof(fm3d_keypoint), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (!nonmax)
        for (auto& q : k) q.response = 0.f;
    return FM3D_OK;
}

// StarDetector(maxSize, response, lineProj, lineBin, supp)(img) (features2d/src/stardetector.cpp):
// the pattern set on the host (StarDetectorComputeResponses' loop), the integrals, responses and tile
// suppression on the GPU (fm3d_star.hip), keypoints in tile order.  Undefined in OpenCV (and
// FM3D_ERR_INVALID here): min(w, h) <= 6, maxSize > 128; a suppression window wider than the border
// (the reference reads outside the image) too.
int star_patterns(int w, int h, int maxSize, fm3d::StarPat& P) {
    static const int sizes0[17] = {1, 2, 3, 4, 6, 8, 11, 12, 16, 22, 23, 32, 45, 46, 64, 90, 128};
    static const int pairs[12][2] = {{1, 0}, {3, 1}, {4, 2}, {5, 3}, {7, 4}, {8, 5},
                                     {9, 6}, {11, 8}, {13, 10}, {14, 11}, {15, 12}, {16, 14}};
    const int st = w + 1, mn = std::min(w, h);
    if (maxSize > 128 || mn <= 6) return 0;
    int np = 0;
    while (np < 12 && !(sizes0[pairs[np][0]] >= maxSize ||
                        sizes0[pairs[np + 1][0]] + sizes0[pairs[np + 1][0]] / 2 >= mn))
        np++;
    if (np == 0) return 0;
    np = std::min(np + 1, 12);  // the first pattern past the range stays, for the size rejection
    memset(&P, 0, sizeof(P));
    P.np = np;
    P.maxIdx = pairs[np - 1][0];
    int area[17];
    for (int i = 0; i <= P.maxIdx; i++) {
        const int u = sizes0[i], t = u + u / 2;
        int* o = P.ofs + 8 * i;
        o[0] = (u + 1) * st + u + 1;
        o[1] = -u * st + u + 1;
        o[2] = (u + 1) * st - u;
        o[3] = -u * st - u;
        o[4] = (t + 1) * st + 1;
        o[5] = -t;
        o[6] = t + 1;
        o[7] = -t * st + 1;
        area[i] = (2 * u + 1) * (2 * u + 1) + t * t + (t + 1) * (t + 1);
        P.sizes1[i] = u;
    }
    P.sizes1[0] = -P.sizes1[0];
    P.sizes1[1] = -P.sizes1[1];
    P.sizes1[P.maxIdx] = -P.sizes1[P.maxIdx];
    P.border = sizes0[P.maxIdx] + sizes0[P.maxIdx] / 2;
    P.nsimd = w - 2 * P.border >= 0 ? 4 * ((w - 2 * P.border) / 4) : 0;
    for (int i = 0; i < np; i++) {
        const int inner = area[pairs[i][1]], outer = area[pairs[i][0]] - inner;
        P.inv[2 * i] = 1.f / (float)outer;
        P.inv[2 * i + 1] = 1.f / (float)inner;
    }
    return np;
}

// the image, its integrals and StarDetectorComputeResponses' maps on the device (starR, starZ)
int star_responses(fm3d_ctx* c, const uint8_t* img, int w, int h, int maxSize, fm3d::StarPat& P) {
    if (!star_patterns(w, h, maxSize, P))
        return fail(c, FM3D_ERR_INVALID, "STAR: undefined for min(w, h) <= 6 or MaxSize > 128");
    // FM3D_STAR_TILT=rows: the one-workgroup row walk (A/B knob); default: the diagonal scans
    const char* tilt = getenv("FM3D_STAR_TILT");
    const bool rows = tilt && std::string(tilt) == "rows";
    if (rows && (w > fm3d::star_tilted_max_width() || fm3d::star_tilted_lds_bytes(w) > 160 * 1024))
        return fail(c, FM3D_ERR_INVALID, "STAR: image wider than 6,000 pixels for the row walk");
    const long long W1H1 = (long long)(w + 1) * (h + 1), WH = (long long)w * h;
    if (W1H1 > INT32_MAX / 4) return fail(c, FM3D_ERR_INVALID, "image too large for STAR");
    HIPCHK(c, c->starImg.ensure((size_t)WH));
    HIPCHK(c, c->starS.ensure((size_t)W1H1 * sizeof(int)));
    HIPCHK(c, c->starT.ensure((size_t)W1H1 * sizeof(int)));
    HIPCHK(c, c->starF.ensure((size_t)W1H1 * sizeof(int)));
    HIPCHK(c, c->starR.ensure((size_t)WH * sizeof(float)));
    HIPCHK(c, c->starZ.ensure((size_t)WH * sizeof(short)));
    HIPCHK(c, hipMemcpyAsync(c->starImg.p, img, (size_t)WH, hipMemcpyHostToDevice, c->stream));
    fm3d::launch_integral(c->starImg.as<uint8_t>(), w, h, c->starS.as<int>(), c->stream);
    if (rows) {
        fm3d::launch_star_tilted(c->starImg.as<uint8_t>(), w, h, c->starT.as<int>(), c->starF.as<int>(), c->stream);
    } else {
        HIPCHK(c, c->starWork.ensure(fm3d::star_diag_bytes(w, h)));
        fm3d::launch_star_tilted_diag(c->starImg.as<uint8_t>(), w, h, c->starWork.p, c->starT.as<int>(),
                                      c->starF.as<int>(), c->stream);
    }
    fm3d::launch_star_resp(c->starS.as<int>(), c->starT.as<int>(), c->starF.as<int>(), w, h, P, c->starR.as<float>(),
                           c->starZ.as<short>(), c->stream);
    HIPCHK(c, hipGetLastError());
    return FM3D_OK;
}

int star_detect(fm3d_ctx* c, const uint8_t* img, int w, int h, int maxSize, int respThr, int lineProj, int lineBin,
                int supp, std::vector<fm3d_keypoint>& k) {
    k.clear();
    fm3d::StarPat P;
    if (!star_patterns(w, h, maxSize, P))
        return fail(c, FM3D_ERR_INVALID, "STAR: undefined for min(w, h) <= 6 or MaxSize > 128");
    const int delta = supp / 2;
    if (delta < 0 || delta > P.border) return fail(c, FM3D_ERR_INVALID, "STAR: Suppression wider than the border");
    fm3d::StarNms N{P.border, delta, 0, 0, respThr, lineProj, lineBin};
    if (h - 2 * P.border > 0 && w - 2 * P.border > 0) {
        N.ny = (h - 2 * P.border + delta) / (delta + 1);
        N.nx = (w - 2 * P.border + delta) / (delta + 1);
    }
    const int nslot = 2 * N.nx * N.ny;
    int r;
    if ((r = ensure_scan_tmp(c, std::max(nslot, 1)))) return r;
    HIPCHK(c, c->starKp.ensure((size_t)(nslot + 1) * sizeof(fm3d_keypoint)));
    HIPCHK(c, c->starFlag.ensure((size_t)(nslot + 1) * sizeof(int)));
    HIPCHK(c, c->starPos.ensure((size_t)(nslot + 1) * sizeof(int)));
    if ((r = star_responses(c, img, w, h, maxSize, P))) return r;
    if (nslot == 0) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        return FM3D_OK;
    }
    fm3d::launch_star_nms(c->starR.as<float>(), c->starZ.as<short>(), w, h, N, c->starKp.as<fm3d_keypoint>(),
                          c->starFlag.as<int>(), c->stream);
    fm3d::launch_exclusive_scan(c->starFlag.as<int>(), nslot, c->starPos.as<int>(), c->count.as<int>(), c->scanTmp.p,
                                c->stream);
    HIPCHK(c, hipGetLastError());
    int nk = 0;
    HIPCHK(c, hipMemcpyAsync(&nk, c->count.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (nk == 0) return FM3D_OK;
    HIPCHK(c, c->starOut.ensure((size_t)nk * sizeof(fm3d_keypoint)));
    fm3d::launch_star_scatter(c->starKp.as<fm3d_keypoint>(), c->starFlag.as<int>(), c->starPos.as<int>(), nslot,
                              c->starOut.as<fm3d_keypoint>(), c->stream);
    HIPCHK(c, hipGetLastError());
    k.resize(nk);
    HIPCHK(c, hipMemcpyAsync(k.data(), c->starOut.p, (size_t)nk * sizeof(fm3d_keypoint), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return FM3D_OK;
}

int surf_upload_image(fm3d_ctx* c, const uint8_t* img, int w, int h) {
    HIPCHK(c, c->sfImg.ensure((size_t)w * h));
    HIPCHK(c, hipMemcpyAsync(c->sfImg.p, img, (size_t)w * h, hipMemcpyHostToDevice, c->stream));
    if (c->sfDW.bytes == 0) {
        const std::vector<float> dw = surf_dw();
        HIPCHK(c, c->sfDW.ensure(400 * sizeof(float)));
        HIPCHK(c, hipMemcpyAsync(c->sfDW.p, dw.data(), 400 * sizeof(float), hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));  // dw leaves scope
    }
    return FM3D_OK;
}

}  // namespace

extern "C" {

const char* fm3d_version(void) { return "fm3d 0.1 (gfx950)"; }

int fm3d_ctx_create(const fm3d_settings* s, int device, fm3d_ctx** out) {
    if (!s || !out) return FM3D_ERR_INVALID;
    *out = nullptr;
    if (s->dltSolver != 0 && s->dltSolver != 1) return FM3D_ERR_INVALID;  // cvSVD or the legacy Jacobi
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return FM3D_ERR_HIP;
    if (device < 0 || device >= n) return FM3D_ERR_INVALID;
    if (hipSetDevice(device) != hipSuccess) return FM3D_ERR_HIP;
    fm3d_ctx* c = new fm3d_ctx();
    c->s = *s;
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return FM3D_ERR_HIP;
    }
    c->ownStream = true;
    // test hook: the look-back tag to start from (tests/test_gpu_c2_pipeline.py runs across its wrap)
    if (const char* le = getenv("FM3D_DEBUG_LB_EPOCH")) c->lbEpoch = (unsigned)strtoul(le, nullptr, 0);
    for (auto& e : c->ev) hipEventCreate(&e);
    hipEventCreateWithFlags(&c->evStage, hipEventDisableTiming);
    hipEventCreateWithFlags(&c->evProj, hipEventDisableTiming);
    hipEventCreateWithFlags(&c->evFront, hipEventDisableTiming);
    hipEventCreateWithFlags(&c->evLm, hipEventDisableTiming);
    c->cam.fx = s->Fx;
    c->cam.fy = s->Fy;
    c->cam.cx = s->Cx;
    c->cam.cy = s->Cy;
    c->cam.k[0] = s->k0;
    c->cam.k[1] = s->k1;
    c->cam.k[2] = s->p1;
    c->cam.k[3] = s->p2;
    c->cam.k[4] = s->k2;
    *out = c;
    return FM3D_OK;
}

void fm3d_ctx_destroy(fm3d_ctx* c) {
    if (!c) return;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    DevBuf* bufs[] = {&c->lvlDesc, &c->offsets, &c->A, &c->B, &c->cqA, &c->ctB, &c->idx, &c->key, &c->fkey,
                      &c->knnOut, &c->cand, &c->flag, &c->matches, &c->count, &c->scanTmp, &c->kp1, &c->kp2,
                      &c->triPts, &c->triMask, &c->triMask8, &c->pts, &c->srcIdx, &c->lmNormals, &c->lmStatus,
                      &c->lmInfo, &c->lmNfev, &c->lmMdat, &c->lmQueue, &c->lmStat,
                      &c->slab, &c->slabI1,
                      &c->records, &c->recTmp, &c->recFlag, &c->lmProj, &c->partIdx, &c->partKey, &c->bPairs, &c->f32Work, &c->A8, &c->B8, &c->u8Flag,
                      &c->sfImg, &c->sfSum, &c->sfDet, &c->sfTr, &c->sfLayers, &c->sfMids, &c->sfCand, &c->sfCount,
                      &c->sfSortTmp, &c->sfFlag, &c->sfPos, &c->sfKp, &c->sfKin, &c->sfSrc, &c->sfDesc, &c->sfDW, &c->sfAng,
                      &c->orbPyr, &c->orbTab, &c->orbLev, &c->orbMap, &c->orbFlag, &c->orbPos, &c->orbKp, &c->orbR,
                      &c->orbBlur, &c->orbDesc, &c->orbPat, &c->siftImg, &c->siftBase, &c->siftG, &c->siftD,
                      &c->siftGL, &c->siftDL, &c->siftTaps, &c->siftScan, &c->siftFlag, &c->siftPos, &c->siftCand,
                      &c->siftAng, &c->siftNpk, &c->siftKp, &c->siftDesc, &c->brImg, &c->brSum, &c->brKp,
                      &c->brIdx, &c->brPat, &c->brPairs, &c->brDesc, &c->starImg, &c->starS, &c->starT, &c->starF,
                      &c->starR, &c->starZ, &c->starKp, &c->starFlag, &c->starPos, &c->starOut, &c->starWork,
                      &c->nccS, &c->nccN, &c->nccB, &c->pcnt, &c->frImg, &c->frSum, &c->frKp, &c->frScale,
                      &c->frLut, &c->frOp, &c->frPairs, &c->frAng, &c->frDesc, &c->msImg, &c->msWork,
                      &c->msHeap, &c->msNode, &c->msHist, &c->msReg, &c->msCnt, &c->msOff, &c->msXY, &c->msScr, &c->msRank,
                      &c->msKp, &c->msFlag, &c->msPos, &c->msOut, &c->msPad, &c->msRegC};
    for (DevBuf* b : bufs) b->release();
    HostBuf* hbufs[] = {&c->hA, &c->hB, &c->hK1, &c->hK2, &c->hImg, &c->hTab, &c->hProj, &c->hSmall, &c->hFlag};
    for (HostBuf* b : hbufs) b->release();
    hipEventDestroy(c->evStage);
    hipEventDestroy(c->evProj);
    hipEventDestroy(c->evFront);
    hipEventDestroy(c->evLm);
    if (c->linkLeader) {
        auto& v = c->linkLeader->linkMembers;
        v.erase(std::remove(v.begin(), v.end(), c), v.end());
    }
    for (fm3d_ctx* m : c->linkMembers) m->linkLeader = nullptr;
    for (auto& b : c->pyr1) b.release();
    for (auto& b : c->pyr2) b.release();
    for (auto& e : c->ev) hipEventDestroy(e);
    if (c->ownStream) hipStreamDestroy(c->stream);
    delete c;
}

const char* fm3d_last_error(const fm3d_ctx* c) { return c ? c->err.c_str() : "null context"; }

int fm3d_ctx_set_stream(fm3d_ctx* c, void* stream) {
    if (!c) return FM3D_ERR_INVALID;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    if (c->ownStream) hipStreamDestroy(c->stream);
    if (stream) {
        c->stream = (hipStream_t)stream;
        c->ownStream = false;
    } else {
        HIPCHK(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        c->ownStream = true;
    }
    return FM3D_OK;
}

int fm3d_knn2(fm3d_ctx* c, const void* descA, int nA, const void* descB, int nB, int dim, int type, fm3d_dmatch* out) {
    if (!c || (!descA && nA) || (!descB && nB) || (!out && nA)) return fail(c, FM3D_ERR_INVALID, "null argument");
    hipSetDevice(c->device);
    int t, dp, r;
    if ((r = stage_descriptors(c, descA, nA, descB, nB, dim, type, &t, &dp))) return r;
    if ((r = run_match(c, nA, nB, t, dp, 0.0, 0, true))) return r;
    if (nA) HIPCHK(c, hipMemcpyAsync(out, c->knnOut.p, (size_t)nA * 2 * sizeof(fm3d_dmatch), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return FM3D_OK;
}

int fm3d_match_nndr(fm3d_ctx* c, const void* descA, int nA, const void* descB, int nB, int dim, int type,
                    double epsilon, fm3d_dmatch* matches, int* nMatches) {
    if (!c || !nMatches || (!descA && nA) || (!descB && nB) || (!matches && nA))
        return fail(c, FM3D_ERR_INVALID, "null argument");
    hipSetDevice(c->device);
    int t, dp, r;
    if ((r = stage_descriptors(c, descA, nA, descB, nB, dim, type, &t, &dp))) return r;
    if ((r = run_match(c, nA, nB, t, dp, epsilon, 0, false))) return r;
    if ((r = ensure_scan_tmp(c, nA))) return r;
    HIPCHK(c, c->matches.ensure((size_t)(nA + 1) * sizeof(fm3d_dmatch)));
    fm3d::launch_compact_dmatch(c->cand.as<fm3d_dmatch>(), c->flag.as<int>(), nA, c->matches.as<fm3d_dmatch>(),
                                c->count.as<int>(), c->scanTmp.p, c->stream);
    HIPCHK(c, hipGetLastError());
    int n = 0;
    HIPCHK(c, hipMemcpyAsync(&n, c->count.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (n) HIPCHK(c, hipMemcpy(matches, c->matches.p, (size_t)n * sizeof(fm3d_dmatch), hipMemcpyDeviceToHost));
    *nMatches = n;
    return FM3D_OK;
}

int fm3d_g12_from_poses(const fm3d_settings* s, const double T1[3], const double T2[3], const double r1[3],
                        const double r2[3], double g[16]) {
    if (!s || !T1 || !T2 || !r1 || !r2 || !g) return FM3D_ERR_INVALID;
    double RIC[9], R1[9], R2[9], gIC[16], g1[16], g2[16], a[16], b[16], cc[16], d[16];
    rodrigues_v2m(s->rodriguesIC, RIC);  // SingleCameraTriangulator ctor (:42-65)
    compose(RIC, s->translationIC, gIC);
    rodrigues_v2m(r1, R1);
    rodrigues_v2m(r2, R2);
    compose(R1, T1, g1);
    compose(R2, T2, g2);
    inv4(gIC, a);
    inv4(g2, b);
    mul4(a, b, cc);
    mul4(cc, g1, d);
    mul4(d, gIC, g);
    return FM3D_OK;
}

int fm3d_camera2_from_g12(const double g12[16], double R2[9], double t2[3]) {
    if (!g12 || !R2 || !t2) return FM3D_ERR_INVALID;
    camera2_from_g12(g12, R2, t2);
    return FM3D_OK;
}

int fm3d_setg12(fm3d_ctx* c, const double T1[3], const double T2[3], const double r1[3], const double r2[3],
                double g12[16]) {
    if (!c || !T1 || !T2 || !r1 || !r2) return fail(c, FM3D_ERR_INVALID, "null argument");
    double g[16];
    fm3d_g12_from_poses(&c->s, T1, T2, r1, r2, g);
    install_g12(c, g);
    if (g12) std::memcpy(g12, g, sizeof(g));
    return FM3D_OK;
}

int fm3d_set_g12(fm3d_ctx* c, const double g12[16]) {
    if (!c || !g12) return fail(c, FM3D_ERR_INVALID, "null argument");
    install_g12(c, g12);
    return FM3D_OK;
}

int fm3d_get_camera2(const fm3d_ctx* c, double R2[9], double t2[3]) {
    if (!c || !c->haveG12) return FM3D_ERR_INVALID;
    std::memcpy(R2, c->R2, sizeof(c->R2));
    std::memcpy(t2, c->t2, sizeof(c->t2));
    return FM3D_OK;
}

int fm3d_triangulate(fm3d_ctx* c, const fm3d_point2f* kpts1, int n1, const fm3d_point2f* kpts2, int n2,
                     const fm3d_dmatch* matches, int K, double* points, uint8_t* inlierMask, int* nPoints) {
    if (!c || !nPoints || K < 0) return fail(c, FM3D_ERR_INVALID, "bad argument");
    if (!c->haveG12) return fail(c, FM3D_ERR_INVALID, "g12 not set (SingleCameraTriangulator::setg12)");
    hipSetDevice(c->device);
    for (int i = 0; i < K; i++)
        if (matches[i].queryIdx < 0 || matches[i].queryIdx >= n1 || matches[i].trainIdx < 0 || matches[i].trainIdx >= n2)
            return fail(c, FM3D_ERR_INVALID, "match index out of range");  // std::vector::at would throw
    int r;
    if ((r = upload(c, c->kp1, kpts1, (size_t)n1 * sizeof(fm3d_point2f)))) return r;
    if ((r = upload(c, c->kp2, kpts2, (size_t)n2 * sizeof(fm3d_point2f)))) return r;
    if ((r = upload(c, c->matches, matches, (size_t)K * sizeof(fm3d_dmatch)))) return r;
    HIPCHK(c, c->triPts.ensure((size_t)(K + 1) * 3 * sizeof(double)));
    HIPCHK(c, c->triMask.ensure((size_t)(K + 1) * sizeof(int)));
    HIPCHK(c, c->triMask8.ensure((size_t)(K + 1)));
    HIPCHK(c, c->pts.ensure((size_t)(K + 1) * 3 * sizeof(double)));
    HIPCHK(c, c->srcIdx.ensure((size_t)(K + 1) * sizeof(int)));
    if ((r = ensure_scan_tmp(c, K))) return r;
    fm3d::TriParams p{};
    p.cam = c->cam;
    std::memcpy(p.g12, c->g12, sizeof(p.g12));
    p.zmin = c->s.zThresholdMin;
    p.zmax = c->s.zThresholdMax;
    p.kp1 = c->kp1.as<fm3d_point2f>();
    p.kp2 = c->kp2.as<fm3d_point2f>();
    p.matches = c->matches.as<fm3d_dmatch>();
    p.K = K;
    p.queryOffset = 0;
    p.pts = c->triPts.as<double>();
    p.mask = c->triMask.as<int>();
    p.mask8 = c->triMask8.as<uint8_t>();
    p.dltSolver = c->s.dltSolver;
    fm3d::launch_triangulate(p, c->stream);
    fm3d::launch_compact_points(c->triPts.as<double>(), c->triMask.as<int>(), K, nullptr, c->pts.as<double>(),
                                c->count.as<int>(), c->srcIdx.as<int>(), c->scanTmp.p, c->stream);
    HIPCHK(c, hipGetLastError());
    int n = 0;
    HIPCHK(c, hipMemcpyAsync(&n, c->count.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    if (inlierMask && K) HIPCHK(c, hipMemcpyAsync(inlierMask, c->triMask8.p, K, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (n && points) HIPCHK(c, hipMemcpy(points, c->pts.p, (size_t)n * 3 * sizeof(double), hipMemcpyDeviceToHost));
    *nPoints = n;
    return FM3D_OK;
}

int fm3d_set_images(fm3d_ctx* c, const uint8_t* img1, const uint8_t* img2, int width, int height, int stride) {
    if (!c) return FM3D_ERR_INVALID;
    hipSetDevice(c->device);
    return set_images_impl(c, img1, img2, width, height, stride);
}

int fm3d_get_pyramid_level(const fm3d_ctx* cc, int which, int level, uint8_t* out, int* w, int* h) {
    fm3d_ctx* c = const_cast<fm3d_ctx*>(cc);
    if (!c || level < 0 || level >= (int)c->pyr1.size() || (which != 1 && which != 2)) return FM3D_ERR_INVALID;
    hipSetDevice(c->device);
    if (w) *w = c->lw[level];
    if (h) *h = c->lh[level];
    if (out) {
        const DevBuf& b = which == 1 ? c->pyr1[level] : c->pyr2[level];
        HIPCHK(c, hipMemcpy(out, b.p, (size_t)c->lw[level] * c->lh[level], hipMemcpyDeviceToHost));
    }
    return FM3D_OK;
}

int fm3d_optimize_normals(fm3d_ctx* c, double* points, int P, double* normals, int32_t* status, int32_t* info,
                          int32_t* nfev, int* nKept, fm3d_lm_stats* stats) {
    if (!c || !nKept || P < 0 || (P && (!points || !normals))) return fail(c, FM3D_ERR_INVALID, "bad argument");
    hipSetDevice(c->device);
    int r;
    if ((r = upload(c, c->pts, points, (size_t)P * 3 * sizeof(double)))) return r;
    if ((r = run_lm(c, P, nullptr, stats, c->ev[0], c->ev[1]))) return r;
    std::vector<double> nrm((size_t)P * 3);
    std::vector<int> st(P), inf((size_t)P * 8), nf((size_t)P * 8);
    unsigned long long cnt[26] = {};
    if (P) {
        HIPCHK(c, hipMemcpyAsync(nrm.data(), c->lmNormals.p, nrm.size() * sizeof(double), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipMemcpyAsync(st.data(), c->lmStatus.p, st.size() * sizeof(int), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipMemcpyAsync(inf.data(), c->lmInfo.p, inf.size() * sizeof(int), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipMemcpyAsync(nf.data(), c->lmNfev.p, nf.size() * sizeof(int), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipMemcpyAsync(cnt, c->lmStat.p, sizeof(cnt), hipMemcpyDeviceToHost, c->stream));
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    int overflow = 0;  // lmStat is reset by run_lm for every call (P == 0 included)
    HIPCHK(c, hipMemcpy(&overflow, c->lmStat.as<unsigned long long>() + 2, sizeof(int), hipMemcpyDeviceToHost));
    if (overflow) return fail(c, FM3D_ERR_HIP, "LM kernel iteration guard tripped (internal error)");
    float ms = 0.f;
    if (P) hipEventElapsedTime(&ms, c->ev[0], c->ev[1]);
    // erase semantics (normaloptimizer.cpp:366,378): stable compaction, input order kept
    int kept = 0;
    bool nanPlane = false;
    for (int i = 0; i < P; i++) {
        if (status) status[i] = st[i];
        if (info) std::memcpy(&info[(size_t)8 * i], &inf[(size_t)8 * i], 8 * sizeof(int));
        if (nfev) std::memcpy(&nfev[(size_t)8 * i], &nf[(size_t)8 * i], 8 * sizeof(int));
        if (st[i] == FM3D_ST_NAN_PLANE) nanPlane = true;
        if (st[i] == FM3D_ST_OK) {
            for (int k = 0; k < 3; k++) {
                points[3 * kept + k] = points[3 * i + k];
                normals[3 * kept + k] = nrm[3 * i + k];
            }
            kept++;
        }
    }
    *nKept = kept;
    if (stats) {
        stats->points_in = P;
        stats->points_kept = kept;
        stats->evaluations = (int64_t)cnt[0];
        stats->pixel_evaluations = (int64_t)cnt[1];
        for (int i = 0; i < P; i++)
            if (st[i] >= 0 && st[i] < 8) stats->drops[st[i]]++;
        stats->kernel_ms = ms;
        fill_lm_cycles(c, cnt, stats);
    }
    if (nanPlane && c->s.strictNanExit)
        return fail(c, FM3D_ERR_NAN_PLANE, "projectPointToPlane hit NaN (reference: exit(-6))");
    return FM3D_OK;
}

// ---------------- whole pipeline, device resident ----------------
}  // extern "C"
namespace {
#define PENDING_CHECK(c)                                                                            \
    do {                                                                                            \
        if ((c)->pending)                                                                           \
            return fail((c), FM3D_ERR_INVALID, "a submitted frame pair is pending: fm3d_pipeline_wait first"); \
    } while (0)

// the inputs of one frame pair into HBM on the context stream (pinned staging, asynchronous):
// descriptors, keypoints, both images and their pyramids (a6, normaloptimizer.cpp:206-221)
int stage_pipeline(fm3d_ctx* c, const void* descA, int nA, const void* descB, int nB, int dim, int type,
                   const fm3d_point2f* kpts1, const fm3d_point2f* kpts2, const uint8_t* img1, const uint8_t* img2,
                   int width, int height, int queryOffset, bool speculate = false) {
    if (!kpts1 || !kpts2) return fail(c, FM3D_ERR_INVALID, "null argument");
    int t, dp, r;
    // the previous pair's copies out of the staging buffers have run: one wait, then every H2D of
    // this pair is queued without another (the call returns before they execute)
    if ((r = staging_wait(c))) return r;
    if ((r = stage_descriptors(c, descA, nA, descB, nB, dim, type, &t, &dp, false, speculate))) return r;
    if ((r = upload_pinned(c, c->kp1, c->hK1, kpts1, (size_t)nA * sizeof(fm3d_point2f)))) return r;
    if ((r = upload_pinned(c, c->kp2, c->hK2, kpts2, (size_t)nB * sizeof(fm3d_point2f)))) return r;
    if (img1 || img2) {
        if ((r = set_images_impl(c, img1, img2, width, height, width, false, false))) return r;  // records evStage
    } else {  // no images (C2's match + DLT needs none): the context keeps the ones it has, if any
        HIPCHK(c, hipEventRecord(c->evStage, c->stream));
    }
    if (!c->haveG12) {
        double g[16];
        if ((r = fm3d_setg12(c, c->s.pos1, c->s.pos2, c->s.pos1 + 3, c->s.pos2 + 3, g))) return r;
    }
    if ((r = ensure_offsets(c))) return r;
    c->stNA = nA;
    c->stNB = nB;
    c->stDim = dim;
    c->stType = t;
    c->stDimPad = dp;
    c->stQueryOffset = queryOffset;
    c->staged = true;
    return FM3D_OK;
}

// match -> NNDR -> compaction -> DLT triangulation -> compaction on the staged inputs (ev[2..5]),
// sized by the query count: the match count K and the inlier count P stay on the device
// (c->pcnt[0], [1]) and bound nothing the host launches, so the stages queue without a host
// round trip (c->matches, c->pts, c->srcIdx hold K / P entries)
int pipeline_front(fm3d_ctx* c) {
    const int nA = c->stNA, nB = c->stNB;
    int r;
    hipEvent_t* ev = c->ev;
    HIPCHK(c, c->pcnt.ensure(64));
    int* cnt = c->pcnt.as<int>();
    HIPCHK(c, hipEventRecord(ev[2], c->stream));
    // a1: match + NNDR (+ the stable compaction of the kept matches, fused into the NNDR launch)
    if ((r = ensure_scan_tmp(c, nA))) return r;
    HIPCHK(c, c->matches.ensure((size_t)(nA + 1) * sizeof(fm3d_dmatch)));
    if ((r = run_match(c, nA, nB, c->stType, c->stDimPad, c->s.nndrEpsilon, c->stQueryOffset, false,
                       c->matches.as<fm3d_dmatch>(), cnt + 0)))
        return r;
    // the stage boundaries (ev[3]: match + NNDR done, ev[5]: DLT done) only when asked for: a timed
    // event between two launches costs the C2 step 4-10 us of gap (rocprofv3 trace, round 5);
    // FM3D_STAGE_EVENTS=0 leaves only the step's own ev[2] / ev[1]
    c->stageEv = stage_events();
    if (c->stageEv) HIPCHK(c, hipEventRecord(ev[3], c->stream));
    // a4, a5: triangulate (matches are device resident; K <= nA)
    HIPCHK(c, c->triPts.ensure((size_t)(nA + 1) * 3 * sizeof(double)));
    HIPCHK(c, c->triMask.ensure((size_t)(nA + 1) * sizeof(int)));
    HIPCHK(c, c->pts.ensure((size_t)(nA + 1) * 3 * sizeof(double)));
    HIPCHK(c, c->srcIdx.ensure((size_t)(nA + 1) * sizeof(int)));
    fm3d::TriParams tp{};
    tp.cam = c->cam;
    std::memcpy(tp.g12, c->g12, sizeof(tp.g12));
    tp.zmin = c->s.zThresholdMin;
    tp.zmax = c->s.zThresholdMax;
    tp.kp1 = c->kp1.as<fm3d_point2f>();
    tp.kp2 = c->kp2.as<fm3d_point2f>();
    tp.matches = c->matches.as<fm3d_dmatch>();
    tp.K = nA;
    tp.Kdev = cnt + 0;
    tp.queryOffset = c->stQueryOffset;
    tp.pts = c->triPts.as<double>();
    tp.mask = c->triMask.as<int>();
    tp.mask8 = nullptr;
    tp.dltSolver = c->s.dltSolver;
    {   // DLT with the inliers' compaction fused (launch_triangulate_compact)
        fm3d::LookBack lb;
        if ((r = make_lookback(c, fm3d::triangulate_compact_blocks(nA), &lb))) return r;
        fm3d::launch_triangulate_compact(tp, c->pts.as<double>(), c->srcIdx.as<int>(), cnt + 1, lb, c->stream,
                                         c->frontHostCnt);
    }
    HIPCHK(c, hipGetLastError());
    if (c->stageEv) HIPCHK(c, hipEventRecord(ev[5], c->stream));
    return FM3D_OK;
}

// the survivor records of c's pair (after its LM normals, in stream order), then one D2H of the
// counts, the pair's LM counters and the LM launch's counters (lmStat: the launching context's)
int enqueue_epilogue(fm3d_ctx* c, fm3d_record* out, const void* lmStat) {
    const int nA = c->stNA;
    int* cnt = c->pcnt.as<int>();
    HIPCHK(c, c->recTmp.ensure((size_t)(nA + 1) * sizeof(fm3d_record)));
    HIPCHK(c, c->recFlag.ensure((size_t)(nA + 1) * sizeof(int)));
    if (!out) {
        HIPCHK(c, c->records.ensure((size_t)(nA + 1) * sizeof(fm3d_record)));
        out = c->records.as<fm3d_record>();
    }
    c->pendOut = out;
    fm3d::launch_make_records(c->matches.as<fm3d_dmatch>(), c->srcIdx.as<int>(), nA, cnt + 1, c->pts.as<double>(),
                              c->lmNormals.as<double>(), c->lmStatus.as<int>(), c->recTmp.as<fm3d_record>(),
                              c->recFlag.as<int>(), c->stream);
    fm3d::launch_compact_records(c->recTmp.as<fm3d_record>(), c->recFlag.as<int>(), nA, cnt + 1, out, cnt + 2,
                                 c->scanTmp.p, c->stream);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, c->hSmall.ensure(sizeof(PipeSmall)));
    PipeSmall* hs = c->hSmall.as<PipeSmall>();
    HIPCHK(c, hipMemcpyAsync(hs->cnt, cnt, sizeof(hs->cnt) + sizeof(hs->prob), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(hs->lm, lmStat, sizeof(hs->lm), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipEventRecord(c->ev[1], c->stream));
    return FM3D_OK;
}

// the whole path on the staged inputs, queued on the context stream: front half, LM normals over
// the device-counted inliers (a6-a15; the pyramids were built at staging: images are inputs of the
// path), survivor records (compacted into out, or the internal buffer), then one D2H of the counts
// and the LM counters into pinned memory.  Nothing here waits for the device.
int enqueue_full(fm3d_ctx* c, fm3d_record* out, fm3d_lm_stats* ls) {
    int r;
    if ((r = pipeline_front(c))) return r;
    if ((r = run_lm(c, c->stNA, c->pcnt.as<int>() + 1, ls, c->ev[6], c->ev[7]))) return r;
    return enqueue_epilogue(c, out, c->lmStat.p);
}

// the leader's pair with its members' queued front halves: ONE LM launch over all these pairs'
// points on the leader's stream (after every member's front half), then each pair's records on
// its own stream
int enqueue_linked(fm3d_ctx* c, const std::vector<fm3d_ctx*>& ms, fm3d_lm_stats* ls) {
    int r;
    if ((r = pipeline_front(c))) return r;
    std::vector<LMSrc> src;
    for (fm3d_ctx* m : ms) {
        HIPCHK(c, hipStreamWaitEvent(c->stream, m->evFront, 0));
        src.push_back({m, m->stNA, m->pcnt.as<int>() + 1});
        HIPCHK(c, hipEventRecord(m->ev[6], c->stream));
    }
    src.push_back({c, c->stNA, c->pcnt.as<int>() + 1});
    if ((r = run_lm_multi(c, src.data(), (int)src.size(), ls, c->ev[6], c->ev[7]))) return r;
    // each member gets its own copy of the launch's counters (on this stream, before evLm): the
    // leader's next run_lm_multi resets c->lmStat, possibly before a member's epilogue has read it
    for (fm3d_ctx* m : ms) {
        HIPCHK(m, m->lmStat.ensure(256));
        HIPCHK(c, hipMemcpyAsync(m->lmStat.p, c->lmStat.p, sizeof(PipeSmall::lm), hipMemcpyDeviceToDevice, c->stream));
    }
    HIPCHK(c, hipEventRecord(c->evLm, c->stream));
    if ((r = enqueue_epilogue(c, c->subOut, c->lmStat.p))) return r;
    for (fm3d_ctx* m : ms) {
        HIPCHK(c, hipEventRecord(m->ev[7], c->stream));
        m->subLm = *ls;
        m->lmGroups = c->lmGroups;
        m->wallKhz = c->wallKhz;
        hipSetDevice(m->device);
        HIPCHK(m, hipStreamWaitEvent(m->stream, c->evLm, 0));
        if ((r = enqueue_epilogue(m, m->subOut, m->lmStat.p))) return r;
        m->frontOnly = false;
    }
    return FM3D_OK;
}

// after the stream ran enqueue_full: guards, counts and stats (t0: the event the total starts at)
int finalize_full(fm3d_ctx* c, const fm3d_lm_stats& ls, hipEvent_t t0, bool staged_in_step, int* nKept,
                  fm3d_pipeline_stats* stats) {
    hipEvent_t* ev = c->ev;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const PipeSmall* hs = c->hSmall.as<PipeSmall>();
    const int K = hs->cnt[0], P = hs->cnt[1], kept = hs->cnt[2];
    c->stK = K;
    c->stP = P;
    // the LM watchdog (maxIter / FM3D_LM_MAX_SECONDS) leaves points in kLMRunning: an error, not drops
    if (hs->lm[2]) return fail(c, FM3D_ERR_HIP, "LM kernel iteration guard tripped (internal error)");
    if (c->s.strictNanExit && P > 0) {  // reference exit(-6) on a NaN plane hit (:465-469)
        std::vector<int> st(P);
        HIPCHK(c, hipMemcpy(st.data(), c->lmStatus.p, (size_t)P * sizeof(int), hipMemcpyDeviceToHost));
        for (int i = 0; i < P; i++)
            if (st[i] == FM3D_ST_NAN_PLANE)
                return fail(c, FM3D_ERR_NAN_PLANE, "projectPointToPlane hit NaN (reference: exit(-6))");
    }
    if (nKept) *nKept = kept;
    if (stats) {
        std::memset(stats, 0, sizeof(*stats));
        stats->queries = c->stNA;
        stats->trains = c->stNB;
        stats->matches = K;
        stats->inliers = P;
        stats->kept = kept;
        float ms;
        stage_times(c, stats);
        ms = 0;
        if (staged_in_step) hipEventElapsedTime(&ms, ev[8], ev[2]);
        stats->pyramid_ms = ms;  // the inputs' H2D + pyramids (fm3d_pipeline_submit only)
        ms = 0;
        hipEventElapsedTime(&ms, ev[6], ev[7]);
        stats->lm_ms = ms;
        hipEventElapsedTime(&ms, t0, ev[1]);
        stats->total_ms = ms;
        stats->lm = ls;
        stats->lm.points_in = P;
        stats->lm.points_kept = kept;
        stats->lm.evaluations = (int64_t)hs->prob[0];  // this pair's (a launch may hold two)
        stats->lm.pixel_evaluations = (int64_t)hs->prob[1];
        stats->lm.kernel_ms = stats->lm_ms;
        fill_lm_cycles(c, hs->lm, &stats->lm);
    }
    return FM3D_OK;
}
}  // namespace
extern "C" {

int fm3d_pipeline_upload(fm3d_ctx* c, const void* descA, int nA, const void* descB, int nB, int dim, int type,
                         const fm3d_point2f* kpts1, const fm3d_point2f* kpts2, const uint8_t* img1, const uint8_t* img2,
                         int width, int height, int queryOffset) {
    if (!c) return FM3D_ERR_INVALID;
    PENDING_CHECK(c);
    hipSetDevice(c->device);
    int r;
    if ((r = stage_pipeline(c, descA, nA, descB, nB, dim, type, kpts1, kpts2, img1, img2, width, height, queryOffset)))
        return r;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return FM3D_OK;
}

int fm3d_pipeline_run(fm3d_ctx* c, fm3d_record* recordsDev, int* nKept, fm3d_pipeline_stats* stats) {
    if (!c || !c->staged) return fail(c, FM3D_ERR_INVALID, "fm3d_pipeline_upload not called");
    PENDING_CHECK(c);
    hipSetDevice(c->device);
    fm3d_lm_stats ls{};
    int r;
    if ((r = enqueue_full(c, recordsDev, &ls))) return r;
    return finalize_full(c, ls, c->ev[2], false, nKept, stats);
}

}  // extern "C"
namespace {
// one frame pair staged and queued on c's stream (records into out: device, or null = internal);
// a link member queues its front half only, a leader joins its queued members' pairs
int submit_impl(fm3d_ctx* c, const void* descA, int nA, const void* descB, int nB, int dim, int type,
                const fm3d_point2f* kpts1, const fm3d_point2f* kpts2, const uint8_t* img1, const uint8_t* img2,
                int width, int height, int queryOffset, fm3d_record* out) {
    PENDING_CHECK(c);
    hipSetDevice(c->device);
    HIPCHK(c, hipEventRecord(c->ev[8], c->stream));
    int r;
    if ((r = stage_pipeline(c, descA, nA, descB, nB, dim, type, kpts1, kpts2, img1, img2, width, height, queryOffset)))
        return r;
    c->subLm = fm3d_lm_stats{};
    c->subOut = out;
    if (c->linkLeader) {  // member: the front half now, the LM with the leader's next pair
        if ((r = pipeline_front(c))) return r;
        HIPCHK(c, hipEventRecord(c->evFront, c->stream));
        c->frontOnly = true;
    } else if (!c->linkMembers.empty()) {
        std::vector<fm3d_ctx*> ms;  // the members with a pair queued since this leader's last launch
        for (fm3d_ctx* m : c->linkMembers)
            if (m->frontOnly) ms.push_back(m);
        if ((r = ms.empty() ? enqueue_full(c, out, &c->subLm) : enqueue_linked(c, ms, &c->subLm))) return r;
    } else {
        if ((r = enqueue_full(c, out, &c->subLm))) return r;
    }
    c->pending = true;
    return FM3D_OK;
}

// a member whose leader took no pair since its submit: its LM alone, on its own stream
int flush_member(fm3d_ctx* c) {
    if (!c->frontOnly) return FM3D_OK;
    hipSetDevice(c->device);
    int r;
    if ((r = run_lm(c, c->stNA, c->pcnt.as<int>() + 1, &c->subLm, c->ev[6], c->ev[7]))) return r;
    if ((r = enqueue_epilogue(c, c->subOut, c->lmStat.p))) return r;
    c->frontOnly = false;
    return FM3D_OK;
}
}  // namespace
extern "C" {

int fm3d_pipeline_submit(fm3d_ctx* c, const void* descA, int nA, const void* descB, int nB, int dim, int type,
                         const fm3d_point2f* kpts1, const fm3d_point2f* kpts2, const uint8_t* img1, const uint8_t* img2,
                         int width, int height, int queryOffset) {
    if (!c) return FM3D_ERR_INVALID;
    return submit_impl(c, descA, nA, descB, nB, dim, type, kpts1, kpts2, img1, img2, width, height, queryOffset,
                       nullptr);
}

int fm3d_pipeline_link(fm3d_ctx* member, fm3d_ctx* leader) {
    if (!member || !leader || member == leader) return FM3D_ERR_INVALID;
    if (member->pending || leader->pending) return fail(member, FM3D_ERR_INVALID, "a submitted frame pair is pending");
    if (member->linkLeader || !member->linkMembers.empty() || leader->linkLeader)
        return fail(member, FM3D_ERR_INVALID, "a context is linked already");
    if ((int)leader->linkMembers.size() + 1 >= fm3d::kLMMaxProblems)
        return fail(member, FM3D_ERR_INVALID, "a leader takes at most 3 members");
    if (member->device != leader->device) return fail(member, FM3D_ERR_INVALID, "linked contexts need one device");
    member->linkLeader = leader;
    leader->linkMembers.push_back(member);
    return FM3D_OK;
}

int fm3d_pipeline_wait(fm3d_ctx* c, fm3d_record* out, int cap, int* nKept, fm3d_pipeline_stats* stats) {
    if (!c) return FM3D_ERR_INVALID;
    if (!c->pending) return fail(c, FM3D_ERR_INVALID, "no frame pair submitted (fm3d_pipeline_submit)");
    if (c->pendingDlt) return fail(c, FM3D_ERR_INVALID, "a front half is pending: fm3d_pipeline_wait_dlt");
    if (c->pendingNcc) return fail(c, FM3D_ERR_INVALID, "an NCC scoring is pending: fm3d_pipeline_wait_ncc");
    hipSetDevice(c->device);
    int r;
    if ((r = flush_member(c))) return r;
    c->pending = false;
    int kept = 0;
    if ((r = finalize_full(c, c->subLm, c->ev[8], true, &kept, stats))) return r;
    if (out && kept > cap) return fail(c, FM3D_ERR_INVALID, "record buffer too small");
    if (out && kept)
        HIPCHK(c, hipMemcpy(out, c->pendOut, (size_t)kept * sizeof(fm3d_record), hipMemcpyDeviceToHost));
    if (nKept) *nKept = kept;
    return FM3D_OK;
}

}  // extern "C"

// ---- internal entry points of the multi-GPU host (fm3d_mgpu.cpp; fm3d_internal.h, not the C ABI)
int fm3d_internal_submit_to(fm3d_ctx* c, const void* descA, int nA, const void* descB, int nB, int dim, int type,
                            const fm3d_point2f* kpts1, const fm3d_point2f* kpts2, const uint8_t* img1,
                            const uint8_t* img2, int width, int height, fm3d_record* recordsDev) {
    if (!c) return FM3D_ERR_INVALID;
    return submit_impl(c, descA, nA, descB, nB, dim, type, kpts1, kpts2, img1, img2, width, height, 0, recordsDev);
}

int fm3d_internal_flush(fm3d_ctx* c) { return c ? flush_member(c) : FM3D_ERR_INVALID; }
bool fm3d_internal_front_only(const fm3d_ctx* c) { return c && c->frontOnly; }

int fm3d_internal_enqueue(fm3d_ctx* c, fm3d_record* recordsDev) {
    if (!c || !c->staged) return fail(c, FM3D_ERR_INVALID, "fm3d_pipeline_upload not called");
    PENDING_CHECK(c);
    hipSetDevice(c->device);
    HIPCHK(c, hipEventRecord(c->ev[8], c->stream));
    c->subLm = fm3d_lm_stats{};
    int r;
    if ((r = enqueue_full(c, recordsDev, &c->subLm))) return r;
    c->pending = true;
    return FM3D_OK;
}

int fm3d_internal_finish(fm3d_ctx* c, int* nKept, fm3d_pipeline_stats* stats) {
    if (!c || !c->pending) return fail(c, FM3D_ERR_INVALID, "nothing pending");
    hipSetDevice(c->device);
    c->pending = false;
    return finalize_full(c, c->subLm, c->ev[8], true, nKept, stats);
}

const int* fm3d_internal_kept_dev(fm3d_ctx* c) { return c->pcnt.as<int>() + 2; }
hipStream_t fm3d_internal_stream(fm3d_ctx* c) { return c->stream; }
int fm3d_internal_device(fm3d_ctx* c) { return c->device; }
// the device memory one context may take: its largest LM launch's slabs (every CU filled) plus the
// per-pair buffers of nA queries against nB train rows of dim elements (a conservative estimate of
// what the pipeline's DevBufs grow to: descriptors, their u8 / unpacked copies, per-query match,
// triangulation, LM and record arrays, the matchers' part lists, pyramids)
int fm3d_internal_memory_need(fm3d_ctx* c, int64_t nA, int64_t nB, int dim, int type, int width, int height,
                              size_t* bytes) {
    hipSetDevice(c->device);
    int r;
    if ((r = ensure_offsets(c))) return r;
    const bool tree = c->s.lmReduction != 0;
    const int slots = fm3d::kLM2Slots + (tree ? 1 : 0);
    const void* kptr = tree ? reinterpret_cast<const void*>(fm3d::lm2_kernel<true, true>)
                            : reinterpret_cast<const void*>(fm3d::lm2_kernel<true, false>);
    long groups = 0;
    if ((r = lm_groups(c, kptr, slots, -1, &groups))) return r;
    const size_t ents = (size_t)c->nOffPad * slots;
    size_t need = ents * (2 * sizeof(double) + 5 * 4) * groups + 32768;
    const size_t rowIn = type == FM3D_DESC_F32 ? (size_t)dim * 4 : (size_t)dim;
    const size_t rowWork = 256 + (type == FM3D_DESC_F32 ? (size_t)dim * 4 : 0);  // u8 / unpacked / pair copies
    need += (size_t)(nA + nB) * (rowIn + rowWork) + (size_t)nB * 64;
    need += (size_t)nA * 1536;  // per query: top-2 lists + 16 parts, matches, points, masks, LM arrays, records
    need += (size_t)width * height * 4 + ((size_t)16 << 20);  // pyramids with guards, small buffers
    *bytes = need;
    return FM3D_OK;
}

int fm3d_internal_prepare(fm3d_ctx* c) {  // the device count buffer, before a collective names it
    hipSetDevice(c->device);
    HIPCHK(c, c->pcnt.ensure(64));
    return FM3D_OK;
}

extern "C" {

}  // extern "C"
namespace {
// the staged pair's front half with its counts written to page-locked memory by the DLT kernel
int queue_front_counts(fm3d_ctx* c) {
    int r;
    HIPCHK(c, c->hSmall.ensure(sizeof(PipeSmall)));
    PipeSmall* hs = c->hSmall.as<PipeSmall>();
    // the counts reach the page-locked buffer from the DLT kernel itself (no copy launch)
    void* dcnt = nullptr;
    HIPCHK(c, hipHostGetDevicePointer(&dcnt, hs->cnt, 0));
    c->frontHostCnt = (int*)dcnt;
    r = pipeline_front(c);
    c->frontHostCnt = nullptr;
    if (r) return r;
    HIPCHK(c, hipEventRecord(c->ev[1], c->stream));
    return FM3D_OK;
}

// after a speculative front half (stage_descriptors' speculate): when the pack kernel flagged an
// element that is not an integer in [0, 255], the float rows (still on the device) go through the
// float matchers and the front half runs again, as the non-speculative staging would have run it
int redo_float_front(fm3d_ctx* c) {
    if (!c->specU8) return FM3D_OK;
    c->specU8 = false;
    const int flag = *c->hFlag.as<int>();
    if (flag == 0) return FM3D_OK;
    if (flag < 0) return fail(c, FM3D_ERR_HIP, "the float rows' flag never arrived");
    std::swap(c->A, c->A8);
    std::swap(c->B, c->B8);
    c->stType = FM3D_DESC_F32;
    c->stDimPad = c->stDim;
    int r;
    if ((r = queue_front_counts(c))) return r;
    HIPCHK(c, hipEventSynchronize(c->ev[1]));
    return FM3D_OK;
}
}  // namespace
extern "C" {

int fm3d_pipeline_submit_dlt(fm3d_ctx* c) {
    if (!c || !c->staged) return fail(c, FM3D_ERR_INVALID, "fm3d_pipeline_upload not called");
    PENDING_CHECK(c);
    hipSetDevice(c->device);
    int r;
    if ((r = queue_front_counts(c))) return r;
    c->pending = true;
    c->pendingDlt = true;
    return FM3D_OK;
}

int fm3d_pipeline_submit_dlt_pair(fm3d_ctx* c, const void* descA, int nA, const void* descB, int nB, int dim,
                                  int type, const fm3d_point2f* kpts1, const fm3d_point2f* kpts2, int queryOffset) {
    if (!c) return FM3D_ERR_INVALID;
    PENDING_CHECK(c);
    hipSetDevice(c->device);
    int r;
    if ((r = stage_pipeline(c, descA, nA, descB, nB, dim, type, kpts1, kpts2, nullptr, nullptr, 0, 0, queryOffset,
                            true)))
        return r;
    if ((r = queue_front_counts(c))) return r;
    c->pending = true;
    c->pendingDlt = true;
    return FM3D_OK;
}

int fm3d_pipeline_wait_dlt(fm3d_ctx* c, int* nInliers, fm3d_pipeline_stats* stats) {
    if (!c) return FM3D_ERR_INVALID;
    if (!c->pendingDlt) return fail(c, FM3D_ERR_INVALID, "no front half submitted (fm3d_pipeline_submit_dlt)");
    hipSetDevice(c->device);
    hipEvent_t* ev = c->ev;
    c->pending = false;
    c->pendingDlt = false;
    HIPCHK(c, hipEventSynchronize(ev[1]));
    int r;
    if ((r = redo_float_front(c))) return r;
    const PipeSmall* hs = c->hSmall.as<PipeSmall>();
    const int K = hs->cnt[0], P = hs->cnt[1];
    c->stK = K;
    c->stP = P;
    if (nInliers) *nInliers = P;
    if (stats) {
        std::memset(stats, 0, sizeof(*stats));
        stats->queries = c->stNA;
        stats->trains = c->stNB;
        stats->matches = K;
        stats->inliers = P;
        float ms;
        stage_times(c, stats);
        hipEventElapsedTime(&ms, ev[2], ev[1]);
        stats->total_ms = ms;
    }
    return FM3D_OK;
}

int fm3d_pipeline_run_dlt(fm3d_ctx* c, int* nInliers, fm3d_pipeline_stats* stats) {
    int r;
    if ((r = fm3d_pipeline_submit_dlt(c))) return r;
    return fm3d_pipeline_wait_dlt(c, nInliers, stats);
}

int fm3d_pipeline_submit_ncc(fm3d_ctx* c, int Hphi, int Htheta, double span) {
    if (!c || !c->staged) return fail(c, FM3D_ERR_INVALID, "fm3d_pipeline_upload not called");
    PENDING_CHECK(c);
    if (Hphi <= 0 || Htheta <= 0 || Hphi * Htheta > 32) return fail(c, FM3D_ERR_INVALID, "1 <= Hphi * Htheta <= 32");
    if (!c->haveG12) return fail(c, FM3D_ERR_INVALID, "fm3d_set_g12 / fm3d_setg12 not called");
    hipSetDevice(c->device);
    hipEvent_t* ev = c->ev;
    int r;
    c->nccP = 0;
    if ((r = pipeline_front(c))) return r;
    const int nA = c->stNA;
    const int H = Hphi * Htheta;
    HIPCHK(c, hipEventRecord(ev[6], c->stream));
    if (nA > 0) {
        if ((r = ensure_offsets(c))) return r;
        HIPCHK(c, c->nccS.ensure((size_t)nA * H * sizeof(double)));
        HIPCHK(c, c->nccN.ensure((size_t)nA * 3 * sizeof(double)));
        HIPCHK(c, c->nccB.ensure((size_t)nA * sizeof(int)));
        fm3d::NccParams p{};
        p.points = c->pts.as<double>();
        p.P = nA;  // the bound; the inlier count is on the device
        p.Pdev = c->pcnt.as<int>() + 1;
        p.cam = lm_camera(c->cam);  // the kernel's bit-pattern isPixelGood (fm3d_ncc.hip ncc_geometry)
        std::memcpy(p.R2, c->R2, sizeof(p.R2));
        std::memcpy(p.t2, c->t2, sizeof(p.t2));
        p.img1 = c->pyr1[0].as<uint8_t>();
        p.img2 = c->pyr2[0].as<uint8_t>();
        p.w = c->lw[0];
        p.h = c->lh[0];
        p.offsets = c->offsets.as<int2>();
        p.nOff = c->nOff;
        p.nOffPad = c->nOffPad;
        p.boundW = c->s.boundWidth;
        p.boundH = c->s.boundHeight;
        p.cmax = (int)(2 * c->s.zThresholdMax);
        p.Hphi = Hphi;
        p.Htheta = Htheta;
        p.span = span;
        p.scores = c->nccS.as<double>();
        p.normals = c->nccN.as<double>();
        p.best = c->nccB.as<int>();
        fm3d::launch_ncc_hypotheses(p, c->stream);
        HIPCHK(c, hipGetLastError());
    }
    HIPCHK(c, hipEventRecord(ev[7], c->stream));
    HIPCHK(c, c->hSmall.ensure(sizeof(PipeSmall)));
    PipeSmall* hs = c->hSmall.as<PipeSmall>();
    HIPCHK(c, hipMemcpyAsync(hs->cnt, c->pcnt.p, sizeof(hs->cnt), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipEventRecord(ev[1], c->stream));
    c->pending = true;
    c->pendingNcc = true;
    c->nccHPending = H;
    return FM3D_OK;
}

int fm3d_pipeline_wait_ncc(fm3d_ctx* c, int* nPoints, fm3d_pipeline_stats* stats) {
    if (!c) return FM3D_ERR_INVALID;
    if (!c->pendingNcc) return fail(c, FM3D_ERR_INVALID, "no NCC scoring submitted (fm3d_pipeline_submit_ncc)");
    hipSetDevice(c->device);
    hipEvent_t* ev = c->ev;
    c->pending = false;
    c->pendingNcc = false;
    HIPCHK(c, hipEventSynchronize(ev[1]));
    const PipeSmall* hs = c->hSmall.as<PipeSmall>();
    const int K = hs->cnt[0], P = hs->cnt[1];
    c->stK = K;
    c->stP = P;
    c->nccH = c->nccHPending;
    c->nccP = P;  // the score rows fm3d_pipeline_ncc_download returns (set only by a successful run)
    if (nPoints) *nPoints = P;
    if (stats) {
        std::memset(stats, 0, sizeof(*stats));
        stats->queries = c->stNA;
        stats->trains = c->stNB;
        stats->matches = K;
        stats->inliers = P;
        stats->kept = P;
        float ms;
        stage_times(c, stats);
        hipEventElapsedTime(&ms, ev[6], ev[7]);
        stats->lm_ms = ms;  // the normal stage: here the NCC scoring
        hipEventElapsedTime(&ms, ev[2], ev[1]);
        stats->total_ms = ms;
    }
    return FM3D_OK;
}

int fm3d_pipeline_run_ncc(fm3d_ctx* c, int Hphi, int Htheta, double span, int* nPoints, fm3d_pipeline_stats* stats) {
    int r;
    if ((r = fm3d_pipeline_submit_ncc(c, Hphi, Htheta, span))) return r;
    return fm3d_pipeline_wait_ncc(c, nPoints, stats);
}

int fm3d_pipeline_ncc_download(fm3d_ctx* c, double* scores, double* normals, int32_t* best) {
    if (!c || !c->staged) return FM3D_ERR_INVALID;
    PENDING_CHECK(c);
    hipSetDevice(c->device);
    // the rows of the last successful fm3d_pipeline_run_ncc (a later run / run_dlt does not resize them)
    const size_t P = (size_t)c->nccP;
    if (P && scores) HIPCHK(c, hipMemcpy(scores, c->nccS.p, P * c->nccH * sizeof(double), hipMemcpyDeviceToHost));
    if (P && normals) HIPCHK(c, hipMemcpy(normals, c->nccN.p, P * 3 * sizeof(double), hipMemcpyDeviceToHost));
    if (P && best) HIPCHK(c, hipMemcpy(best, c->nccB.p, P * sizeof(int), hipMemcpyDeviceToHost));
    return FM3D_OK;
}

int fm3d_pipeline_dlt_download(fm3d_ctx* c, fm3d_dmatch* matches, double* points, int32_t* matchIdx) {
    if (!c || !c->staged) return FM3D_ERR_INVALID;
    PENDING_CHECK(c);
    hipSetDevice(c->device);
    if (matches && c->stK) HIPCHK(c, hipMemcpy(matches, c->matches.p, (size_t)c->stK * sizeof(fm3d_dmatch), hipMemcpyDeviceToHost));
    if (points && c->stP) HIPCHK(c, hipMemcpy(points, c->pts.p, (size_t)c->stP * 3 * sizeof(double), hipMemcpyDeviceToHost));
    if (matchIdx && c->stP) HIPCHK(c, hipMemcpy(matchIdx, c->srcIdx.p, (size_t)c->stP * sizeof(int), hipMemcpyDeviceToHost));
    return FM3D_OK;
}

int fm3d_records_download(fm3d_ctx* c, const fm3d_record* recordsDev, int n, fm3d_record* out) {
    if (!c || n < 0 || (n && !out)) return FM3D_ERR_INVALID;
    hipSetDevice(c->device);
    const void* src = recordsDev ? (const void*)recordsDev : c->records.p;
    if (n) HIPCHK(c, hipMemcpy(out, src, (size_t)n * sizeof(fm3d_record), hipMemcpyDeviceToHost));
    return FM3D_OK;
}

int fm3d_gravity(const fm3d_settings* s, double g[3]) {
    // NormalOptimizer ctor (normaloptimizer.cpp:160-178): Rodrigues(rodriguesIC).inv() * (0,0,-1),
    // OpenCV 2.4's closed-form 3x3 Matx inverse, Matx * Vec accumulated from 0 in index order
    if (!s || !g) return FM3D_ERR_INVALID;
    double a[9], b[9];
    rodrigues_v2m(s->rodriguesIC, a);
#define A(i, j) a[(i)*3 + (j)]
    double d = A(0, 0) * (A(1, 1) * A(2, 2) - A(2, 1) * A(1, 2)) - A(0, 1) * (A(1, 0) * A(2, 2) - A(2, 0) * A(1, 2)) +
               A(0, 2) * (A(1, 0) * A(2, 1) - A(2, 0) * A(1, 1));
    if (d == 0) return FM3D_ERR_INVALID;
    d = 1 / d;
    b[0] = (A(1, 1) * A(2, 2) - A(1, 2) * A(2, 1)) * d;
    b[1] = (A(0, 2) * A(2, 1) - A(0, 1) * A(2, 2)) * d;
    b[2] = (A(0, 1) * A(1, 2) - A(0, 2) * A(1, 1)) * d;
    b[3] = (A(1, 2) * A(2, 0) - A(1, 0) * A(2, 2)) * d;
    b[4] = (A(0, 0) * A(2, 2) - A(0, 2) * A(2, 0)) * d;
    b[5] = (A(0, 2) * A(1, 0) - A(0, 0) * A(1, 2)) * d;
    b[6] = (A(1, 0) * A(2, 1) - A(1, 1) * A(2, 0)) * d;
    b[7] = (A(0, 1) * A(2, 0) - A(0, 0) * A(2, 1)) * d;
    b[8] = (A(0, 0) * A(1, 1) - A(0, 1) * A(1, 0)) * d;
#undef A
    const double v[3] = {0, 0, -1};
    for (int i = 0; i < 3; i++) {
        double acc = 0;
        for (int k = 0; k < 3; k++) acc += b[i * 3 + k] * v[k];
        g[i] = acc;
    }
    return FM3D_OK;
}

int fm3d_features_frames(fm3d_ctx* c, const double* points, const double* normals, int P, double* frames) {
    if (!c || P < 0 || (P && (!points || !normals || !frames))) return FM3D_ERR_INVALID;
    if (P == 0) return FM3D_OK;
    hipSetDevice(c->device);
    double g[3];
    int r;
    if ((r = fm3d_gravity(&c->s, g))) return fail(c, r, "gravity: singular rodriguesIC rotation");
    DevBuf a, b, f;
    HIPCHK(c, a.ensure((size_t)P * 3 * sizeof(double)));
    HIPCHK(c, b.ensure((size_t)P * 3 * sizeof(double)));
    HIPCHK(c, f.ensure((size_t)P * 16 * sizeof(double)));
    HIPCHK(c, hipMemcpyAsync(a.p, points, (size_t)P * 3 * sizeof(double), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(b.p, normals, (size_t)P * 3 * sizeof(double), hipMemcpyHostToDevice, c->stream));
    fm3d::launch_features_frames(a.as<double>(), b.as<double>(), P, g, f.as<double>(), c->stream);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(frames, f.p, (size_t)P * 16 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return FM3D_OK;
}

int fm3d_patch_size(const fm3d_settings* s) {
    if (!s) return FM3D_ERR_INVALID;
    // numberOfPointsPerEdge (neighborhoodsgenerator.cpp:136-137)
    return 2 * ((int)floor(s->neighEpsilon / (0.01 * s->cmPerPixel)));
}

int fm3d_export_patches(fm3d_ctx* c, const double* frames, int P, uint8_t* patches, double* imagePoints) {
    if (!c || P < 0 || (P && (!frames || !patches))) return FM3D_ERR_INVALID;
    if (c->pyr1.empty()) return fail(c, FM3D_ERR_INVALID, "fm3d_set_images not called");
    const int size = fm3d_patch_size(&c->s);
    if (size <= 0) return fail(c, FM3D_ERR_INVALID, "patch size <= 0 (Neighborhoods.epsilon / cmPerPixel)");
    if (P == 0) return FM3D_OK;
    hipSetDevice(c->device);
    const size_t per = (size_t)size * size;
    DevBuf f, rt, out, pts;
    HIPCHK(c, f.ensure((size_t)P * 16 * sizeof(double)));
    HIPCHK(c, rt.ensure((size_t)P * 12 * sizeof(double)));
    HIPCHK(c, out.ensure((size_t)P * per));
    if (imagePoints) HIPCHK(c, pts.ensure((size_t)P * per * 2 * sizeof(double)));
    HIPCHK(c, hipMemcpyAsync(f.p, frames, (size_t)P * 16 * sizeof(double), hipMemcpyHostToDevice, c->stream));
    fm3d::launch_export_patches(f.as<double>(), P, size, c->s.neighEpsilon, c->s.cmPerPixel * 0.01, c->cam,
                                c->pyr1[0].as<uint8_t>(), c->lw[0], c->lh[0], rt.as<double>(), out.as<uint8_t>(),
                                imagePoints ? pts.as<double>() : nullptr, c->stream);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(patches, out.p, (size_t)P * per, hipMemcpyDeviceToHost, c->stream));
    if (imagePoints)
        HIPCHK(c, hipMemcpyAsync(imagePoints, pts.p, (size_t)P * per * 2 * sizeof(double), hipMemcpyDeviceToHost,
                                 c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return FM3D_OK;
}

int fm3d_square_neighborhoods(fm3d_ctx* c, const double* frames, int P, double* out) {
    if (!c || P < 0 || (P && (!frames || !out))) return FM3D_ERR_INVALID;
    const int size = fm3d_patch_size(&c->s);
    if (size <= 0) return fail(c, FM3D_ERR_INVALID, "neighbourhood size <= 0 (Neighborhoods.epsilon / cmPerPixel)");
    if (P == 0) return FM3D_OK;
    hipSetDevice(c->device);
    // chunks of frames bound the device buffer (~512 MB of points); the copy of chunk k overlaps
    // nothing here -- the host buffer is the boundary
    const size_t perFrame = (size_t)size * size * 3 * sizeof(double);
    const int chunk = (int)std::max<size_t>(1, std::min<size_t>((size_t)P, ((size_t)512 << 20) / perFrame));
    DevBuf f, o;
    HIPCHK(c, f.ensure((size_t)chunk * 16 * sizeof(double)));
    HIPCHK(c, o.ensure((size_t)chunk * perFrame));
    for (int p0 = 0; p0 < P; p0 += chunk) {
        const int n = std::min(chunk, P - p0);
        HIPCHK(c, hipMemcpyAsync(f.p, frames + (size_t)16 * p0, (size_t)n * 16 * sizeof(double),
                                 hipMemcpyHostToDevice, c->stream));
        fm3d::launch_square_neighborhoods(f.as<double>(), n, size, c->s.neighEpsilon, c->s.cmPerPixel * 0.01,
                                          o.as<double>(), c->stream);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipMemcpyAsync(out + (size_t)p0 * size * size * 3, o.p, (size_t)n * perFrame,
                                 hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    return FM3D_OK;
}

int fm3d_circular_neighborhoods(fm3d_ctx* c, const double* points, const double* normals, int P, double* out) {
    if (!c || P < 0 || (P && (!points || !out))) return FM3D_ERR_INVALID;
    if (c->s.neighMethod != 1) return fail(c, FM3D_ERR_INVALID, "Neighborhoods.method is not circular");
    const int T = c->s.neighThetas, Rn = c->s.neighRays;
    if (T <= 0 || Rn <= 0) return fail(c, FM3D_ERR_INVALID, "Neighborhoods.thetas / rays <= 0");
    if (P == 0) return FM3D_OK;
    hipSetDevice(c->device);
    // the constructor's lookup table (neighborhoodsgenerator.cpp:50-64), libm sin as the reference
    const double eps = c->s.neighEpsilon;
    const double rayIncrement = eps / Rn, thetaIncrement = 2 * M_PI / T;
    const int S = T * Rn;
    std::vector<double> lut((size_t)S * 3);
    for (int i = 1; i <= Rn; i++)
        for (int j = 0; j < T; j++) {
            const double t = j * thetaIncrement;
            double* e = &lut[3 * ((size_t)(i - 1) * T + j)];
            e[0] = (double)i * rayIncrement;
            e[1] = std::sin(t);
            e[2] = 2 * (std::sin(t / 2)) * (std::sin(t / 2));
        }
    // chunks of points bound the device buffer (~512 MB of samples)
    const size_t perPoint = (size_t)S * 3 * sizeof(double);
    const int chunk = (int)std::max<size_t>(1, std::min<size_t>((size_t)P, ((size_t)512 << 20) / perPoint));
    DevBuf L, X, N, O;
    HIPCHK(c, L.ensure(lut.size() * sizeof(double)));
    HIPCHK(c, X.ensure((size_t)chunk * 3 * sizeof(double)));
    if (normals) HIPCHK(c, N.ensure((size_t)chunk * 3 * sizeof(double)));
    HIPCHK(c, O.ensure((size_t)chunk * perPoint));
    HIPCHK(c, hipMemcpyAsync(L.p, lut.data(), lut.size() * sizeof(double), hipMemcpyHostToDevice, c->stream));
    for (int p0 = 0; p0 < P; p0 += chunk) {
        const int n = std::min(chunk, P - p0);
        HIPCHK(c, hipMemcpyAsync(X.p, points + (size_t)3 * p0, (size_t)n * 3 * sizeof(double), hipMemcpyHostToDevice,
                                 c->stream));
        if (normals)
            HIPCHK(c, hipMemcpyAsync(N.p, normals + (size_t)3 * p0, (size_t)n * 3 * sizeof(double),
                                     hipMemcpyHostToDevice, c->stream));
        fm3d::launch_circular_neighborhoods(X.as<double>(), normals ? N.as<double>() : nullptr, n, S, L.as<double>(),
                                            eps, O.as<double>(), c->stream);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipMemcpyAsync(out + (size_t)p0 * S * 3, O.p, (size_t)n * perPoint, hipMemcpyDeviceToHost,
                                 c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    return FM3D_OK;
}

int fm3d_surf_detect(fm3d_ctx* c, const uint8_t* img, int w, int h, fm3d_keypoint* kpts, int cap, int* n,
                     float* desc) {
    if (!c || !img || !n || w <= 0 || h <= 0 || cap < 0 || (cap > 0 && !kpts)) return FM3D_ERR_INVALID;
    const fm3d_settings& S = c->s;
    if (S.detectorType != FM3D_FEAT_SURF || (desc && S.extractorType != FM3D_FEAT_SURF))
        return fail(c, FM3D_ERR_UNSUPPORTED, "only the STATIC SURF detector / extractor runs on the GPU");
    if (S.surfOctaves < 1 || S.surfOctaveLayers < 1 || S.surfHessianThreshold < 0)
        return fail(c, FM3D_ERR_INVALID, "SURF NumOctaves / NumOctaveLayers / HessianThreshold out of range");
    hipSetDevice(c->device);
    int r;
    if ((r = surf_upload_image(c, img, w, h))) return r;
    const SurfPlan P = surf_plan(w, h, S.surfOctaves, S.surfOctaveLayers);
    HIPCHK(c, c->sfSum.ensure((size_t)(w + 1) * (h + 1) * sizeof(int)));
    HIPCHK(c, c->sfDet.ensure(P.detFloats * sizeof(float) + 16));
    HIPCHK(c, c->sfTr.ensure(P.detFloats * sizeof(float) + 16));
    HIPCHK(c, c->sfLayers.ensure(P.L.size() * sizeof(fm3d::SurfLayer)));
    HIPCHK(c, c->sfMids.ensure(P.M.size() * sizeof(fm3d::SurfMid)));
    HIPCHK(c, c->sfCand.ensure((size_t)P.candCap * sizeof(fm3d::SurfCand)));
    HIPCHK(c, c->sfCount.ensure(64));
    HIPCHK(c, hipMemcpyAsync(c->sfLayers.p, P.L.data(), P.L.size() * sizeof(fm3d::SurfLayer), hipMemcpyHostToDevice,
                             c->stream));
    HIPCHK(c, hipMemcpyAsync(c->sfMids.p, P.M.data(), P.M.size() * sizeof(fm3d::SurfMid), hipMemcpyHostToDevice,
                             c->stream));
    HIPCHK(c, hipMemsetAsync(c->sfDet.p, 0, P.detFloats * sizeof(float), c->stream));
    HIPCHK(c, hipMemsetAsync(c->sfTr.p, 0, P.detFloats * sizeof(float), c->stream));
    HIPCHK(c, hipMemsetAsync(c->sfCount.p, 0, 64, c->stream));
    fm3d::launch_integral(c->sfImg.as<uint8_t>(), w, h, c->sfSum.as<int>(), c->stream);
    fm3d::launch_surf_hessian(c->sfSum.as<int>(), w, c->sfLayers.as<fm3d::SurfLayer>(), (int)P.L.size(), P.hTotal,
                              c->sfDet.as<float>(), c->sfTr.as<float>(), c->stream);
    fm3d::launch_surf_maxima(c->sfDet.as<float>(), c->sfTr.as<float>(), c->sfLayers.as<fm3d::SurfLayer>(),
                             c->sfMids.as<fm3d::SurfMid>(), (int)P.M.size(), P.mTotal, (float)S.surfHessianThreshold,
                             c->sfCand.as<fm3d::SurfCand>(), c->sfCount.as<int>(), (int)P.candCap, c->stream);
    HIPCHK(c, hipGetLastError());
    int nc = 0;
    HIPCHK(c, hipMemcpyAsync(&nc, c->sfCount.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (nc > P.candCap) return fail(c, FM3D_ERR_HIP, "SURF candidate buffer overflow");
    const size_t sortBytes = fm3d::surf_sort_tmp_bytes(nc);
    HIPCHK(c, c->sfSortTmp.ensure(sortBytes + 16));
    fm3d::launch_surf_sort(c->sfCand.as<fm3d::SurfCand>(), nc, c->sfSortTmp.p, sortBytes, c->stream);
    if ((r = ensure_scan_tmp(c, nc))) return r;
    HIPCHK(c, c->sfFlag.ensure((size_t)(nc + 1) * sizeof(int)));
    HIPCHK(c, c->sfPos.ensure((size_t)(nc + 1) * sizeof(int)));
    HIPCHK(c, c->sfKp.ensure((size_t)(nc + 1) * sizeof(fm3d_keypoint)));
    int nk = 0;
    if (nc > 0) {
        const float* ang = nullptr;
        if (!S.surfUpright) {  // SURFInvoker's orientation; keypoints without a sample are removed
            HIPCHK(c, c->sfAng.ensure((size_t)(nc + 1) * sizeof(float)));
            fm3d::launch_surf_orient(c->sfCand.p, sizeof(fm3d::SurfCand), nc, c->sfSum.as<int>(), 0, w, h, surf_ori(),
                                     c->sfFlag.as<int>(), c->sfAng.as<float>(), c->stream);
            ang = c->sfAng.as<float>();
        }
        fm3d::launch_surf_upright(c->sfCand.as<fm3d::SurfCand>(), c->sfCount.as<int>(), nc, w, h, c->sfFlag.as<int>(),
                                  c->sfPos.as<int>(), c->count.as<int>(), c->scanTmp.p, c->sfKp.as<fm3d_keypoint>(),
                                  nullptr, ang, c->stream);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipMemcpyAsync(&nk, c->count.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    const int nw = std::min(nk, cap);
    const int dsize = S.surfExtended ? 128 : 64;
    if (desc && nw > 0) {
        HIPCHK(c, c->sfDesc.ensure((size_t)nw * dsize * sizeof(float)));
        fm3d::launch_surf_describe(c->sfImg.as<uint8_t>(), 0, w, h, c->sfKp.as<fm3d_keypoint>(), nw, c->sfDW.as<float>(),
                                   S.surfExtended, S.surfUpright, c->sfDesc.as<float>(), c->stream);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipMemcpyAsync(desc, c->sfDesc.p, (size_t)nw * dsize * sizeof(float), hipMemcpyDeviceToHost,
                                 c->stream));
    }
    if (nw > 0)
        HIPCHK(c, hipMemcpyAsync(kpts, c->sfKp.p, (size_t)nw * sizeof(fm3d_keypoint), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    *n = nk;
    return FM3D_OK;
}

int fm3d_surf_compute(fm3d_ctx* c, const uint8_t* img, int w, int h, const fm3d_keypoint* kpts, int n,
                      fm3d_keypoint* kout, int32_t* kept, int* nOut, float* desc) {
    if (!c || !img || !nOut || w <= 0 || h <= 0 || n < 0 || (n > 0 && (!kpts || !kout || !desc)))
        return FM3D_ERR_INVALID;
    const fm3d_settings& S = c->s;
    if (S.extractorType != FM3D_FEAT_SURF) return fail(c, FM3D_ERR_UNSUPPORTED, "only the SURF extractor runs on the GPU");
    *nOut = 0;
    if (n == 0) return FM3D_OK;
    // a kept keypoint of size < 0.36 has an empty window: OpenCV's resize asserts (a window narrower
    // than the 21 x 21 patch, size < 7.5, is enlarged by the kernel as OpenCV's INTER_AREA does)
    for (int q = 0; q < n; q++) {
        const float sz = kpts[q].size, s = sz * 1.2f / 9.0f;
        const int gws = 2 * (int)std::lrint(2 * s);
        if (!(sz >= FLT_EPSILON) || h + 1 < gws || w + 1 < gws) continue;  // dropped anyway
        if ((int)((20 + 1) * s) < 1)
            return fail(c, FM3D_ERR_INVALID, "SURF compute: keypoint size < 0.36 (an empty window; OpenCV asserts)");
    }
    hipSetDevice(c->device);
    int r;
    if ((r = surf_upload_image(c, img, w, h))) return r;
    if ((r = ensure_scan_tmp(c, n))) return r;
    HIPCHK(c, c->sfKin.ensure((size_t)n * sizeof(fm3d_keypoint)));
    HIPCHK(c, c->sfKp.ensure((size_t)n * sizeof(fm3d_keypoint)));
    HIPCHK(c, c->sfFlag.ensure((size_t)(n + 1) * sizeof(int)));
    HIPCHK(c, c->sfPos.ensure((size_t)(n + 1) * sizeof(int)));
    HIPCHK(c, c->sfSrc.ensure((size_t)(n + 1) * sizeof(int)));
    HIPCHK(c, hipMemcpyAsync(c->sfKin.p, kpts, (size_t)n * sizeof(fm3d_keypoint), hipMemcpyHostToDevice, c->stream));
    const float* ang = nullptr;
    if (!S.surfUpright) {  // the orientation needs the integral image (SURF::operator() computes it)
        HIPCHK(c, c->sfSum.ensure((size_t)(w + 1) * (h + 1) * sizeof(int)));
        HIPCHK(c, c->sfAng.ensure((size_t)(n + 1) * sizeof(float)));
        fm3d::launch_integral(c->sfImg.as<uint8_t>(), w, h, c->sfSum.as<int>(), c->stream);
        fm3d::launch_surf_orient(c->sfKin.p, sizeof(fm3d_keypoint), n, c->sfSum.as<int>(), 0, w, h, surf_ori(),
                                 c->sfFlag.as<int>(), c->sfAng.as<float>(), c->stream);
        ang = c->sfAng.as<float>();
    }
    fm3d::launch_surf_keep(c->sfKin.as<fm3d_keypoint>(), n, w, h, c->sfFlag.as<int>(), c->sfPos.as<int>(),
                           c->count.as<int>(), c->scanTmp.p, c->sfKp.as<fm3d_keypoint>(), c->sfSrc.as<int>(), ang,
                           c->stream);
    HIPCHK(c, hipGetLastError());
    int nk = 0;
    HIPCHK(c, hipMemcpyAsync(&nk, c->count.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const int dsize = S.surfExtended ? 128 : 64;
    if (nk > 0) {
        HIPCHK(c, c->sfDesc.ensure((size_t)nk * dsize * sizeof(float)));
        fm3d::launch_surf_describe(c->sfImg.as<uint8_t>(), 0, w, h, c->sfKp.as<fm3d_keypoint>(), nk, c->sfDW.as<float>(),
                                   S.surfExtended, S.surfUpright, c->sfDesc.as<float>(), c->stream);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipMemcpyAsync(desc, c->sfDesc.p, (size_t)nk * dsize * sizeof(float), hipMemcpyDeviceToHost,
                                 c->stream));
        HIPCHK(c, hipMemcpyAsync(kout, c->sfKp.p, (size_t)nk * sizeof(fm3d_keypoint), hipMemcpyDeviceToHost, c->stream));
        if (kept)
            HIPCHK(c, hipMemcpyAsync(kept, c->sfSrc.p, (size_t)nk * sizeof(int), hipMemcpyDeviceToHost, c->stream));
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    *nOut = nk;
    return FM3D_OK;
}

int fm3d_extract_descriptors_from_patches_any(fm3d_ctx* c, const uint8_t* patches, int P, int size, void* desc) {
    if (!c || P < 0 || size <= 0 || (P && (!patches || !desc))) return FM3D_ERR_INVALID;
    const int ex = c->s.extractorType;
    if (ex == FM3D_FEAT_SURF || ex == FM3D_FEAT_SIFT)
        return fm3d_extract_descriptors_from_patches(c, patches, P, size, static_cast<float*>(desc));
    if (ex != FM3D_FEAT_ORB && ex != FM3D_FEAT_BRISK && ex != FM3D_FEAT_FREAK)
        return fail(c, FM3D_ERR_UNSUPPORTED, "the settings' extractor type has no GPU implementation");
    // descriptorsmatcher.cpp:142-172: the centred keypoint per patch, compute on each patch; the rows
    // start as Mat::zeros and a dropped keypoint's empty row copies nothing
    const int cols = ex == FM3D_FEAT_ORB ? 32 : 64;
    uint8_t* d = static_cast<uint8_t*>(desc);
    std::memset(d, 0, (size_t)P * cols);
    const float center = (float)(int)std::floor(size / 2);
    const fm3d_keypoint k{center, center, (float)size, -1.f, 1.f, 0, 0};
    for (int p = 0; p < P; p++) {
        fm3d_keypoint ko;
        int m = 0, r;
        const uint8_t* img = patches + (size_t)p * size * size;
        r = ex == FM3D_FEAT_ORB     ? fm3d_orb_compute(c, img, size, size, &k, 1, &ko, nullptr, &m, d + (size_t)p * cols)
            : ex == FM3D_FEAT_BRISK ? fm3d_brisk_compute(c, img, size, size, &k, 1, &ko, nullptr, &m, d + (size_t)p * cols)
                                    : fm3d_freak_compute(c, img, size, size, &k, 1, &ko, nullptr, &m, d + (size_t)p * cols);
        if (r) return r;
        if (p == 0 && m == 0 && ex == FM3D_FEAT_ORB)
            return fail(c, FM3D_ERR_INVALID, "ORB drops the first patch's keypoint (the reference's rows would have 0 columns)");
    }
    return FM3D_OK;
}

int fm3d_extract_descriptors_from_patches(fm3d_ctx* c, const uint8_t* patches, int P, int size, float* desc) {
    if (!c || P < 0 || size <= 0 || (P && (!patches || !desc))) return FM3D_ERR_INVALID;
    const fm3d_settings& S = c->s;
    if (S.extractorType == FM3D_FEAT_SIFT) return sift_patches(c, patches, P, size, desc);
    if (S.extractorType != FM3D_FEAT_SURF)
        return fail(c, FM3D_ERR_UNSUPPORTED, "only the SURF and SIFT extractors describe patches on the GPU");
    if (P == 0) return FM3D_OK;
    // descriptorsmatcher.cpp:146-158: one keypoint per patch at (center, center), center =
    // (int)floor(size / 2), size = the patch edge, angle -1, response 1, octave 0, class_id 0
    const float center = (float)(int)std::floor(size / 2);
    fm3d_keypoint k{center, center, (float)size, -1.f, 1.f, 0, 0};
    const float s = k.size * 1.2f / 9.0f;
    const int gws = 2 * cv_round_h(2 * s);
    if (size + 1 < gws) return fail(c, FM3D_ERR_INVALID, "patch keypoint dropped by SURF (descriptor row missing)");
    if (S.surfUpright) k.angle = 360.f - 90.f;
    hipSetDevice(c->device);
    const size_t per = (size_t)size * size;
    const int dsize = S.surfExtended ? 128 : 64;
    std::vector<fm3d_keypoint> kp((size_t)P, k);
    HIPCHK(c, c->sfImg.ensure((size_t)P * per));
    HIPCHK(c, c->sfKp.ensure((size_t)P * sizeof(fm3d_keypoint)));
    HIPCHK(c, c->sfDesc.ensure((size_t)P * dsize * sizeof(float)));
    HIPCHK(c, hipMemcpyAsync(c->sfImg.p, patches, (size_t)P * per, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->sfKp.p, kp.data(), kp.size() * sizeof(fm3d_keypoint), hipMemcpyHostToDevice, c->stream));
    if (!S.surfUpright) {
        // every patch keypoint's orientation on that patch's integral image; a patch whose keypoint
        // has no orientation sample would lose its descriptor row (never for the centred keypoint
        // of a patch this size, but checked)
        const int r = ensure_scan_tmp(c, P);
        if (r) return r;
        const size_t sumPer = (size_t)(size + 1) * (size + 1);
        HIPCHK(c, c->sfSum.ensure((size_t)P * sumPer * sizeof(int)));
        HIPCHK(c, c->sfAng.ensure((size_t)(P + 1) * sizeof(float)));
        HIPCHK(c, c->sfFlag.ensure((size_t)(P + 1) * sizeof(int)));
        HIPCHK(c, c->sfPos.ensure((size_t)(P + 1) * sizeof(int)));
        HIPCHK(c, c->sfKin.ensure((size_t)P * sizeof(fm3d_keypoint)));
        HIPCHK(c, hipMemcpyAsync(c->sfKin.p, kp.data(), kp.size() * sizeof(fm3d_keypoint), hipMemcpyHostToDevice,
                                 c->stream));
        fm3d::launch_integral_batch(c->sfImg.as<uint8_t>(), size, size, P, c->sfSum.as<int>(), c->stream);
        fm3d::launch_surf_orient(c->sfKin.p, sizeof(fm3d_keypoint), P, c->sfSum.as<int>(), sumPer, size, size,
                                 surf_ori(), c->sfFlag.as<int>(), c->sfAng.as<float>(), c->stream);
        fm3d::launch_surf_keep(c->sfKin.as<fm3d_keypoint>(), P, size, size, c->sfFlag.as<int>(), c->sfPos.as<int>(),
                               c->count.as<int>(), c->scanTmp.p, c->sfKp.as<fm3d_keypoint>(), nullptr,
                               c->sfAng.as<float>(), c->stream);
        HIPCHK(c, hipGetLastError());
        int nk = 0;
        HIPCHK(c, hipMemcpyAsync(&nk, c->count.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (nk != P) return fail(c, FM3D_ERR_INVALID, "patch keypoint dropped by SURF (no orientation sample)");
    }
    if (c->sfDW.bytes == 0) {
        const std::vector<float> dw = surf_dw();
        HIPCHK(c, c->sfDW.ensure(400 * sizeof(float)));
        HIPCHK(c, hipMemcpyAsync(c->sfDW.p, dw.data(), 400 * sizeof(float), hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    fm3d::launch_surf_describe(c->sfImg.as<uint8_t>(), per, size, size, c->sfKp.as<fm3d_keypoint>(), P,
                               c->sfDW.as<float>(), S.surfExtended, S.surfUpright, c->sfDesc.as<float>(), c->stream);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(desc, c->sfDesc.p, (size_t)P * dsize * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return FM3D_OK;
}

int fm3d_orb_set_pattern(fm3d_ctx* c, const int32_t* xy, int npoints) {
    if (!c || (xy && npoints != 512)) return FM3D_ERR_INVALID;
    c->orbUserPattern.clear();
    if (xy) c->orbUserPattern.assign(xy, xy + 1024);
    return FM3D_OK;
}

int fm3d_orb_detect(fm3d_ctx* c, const uint8_t* img, int w, int h, fm3d_keypoint* kpts, int cap, int* n,
                    uint8_t* desc) {
    if (!c || !img || !n || w <= 0 || h <= 0 || cap < 0 || (cap > 0 && !kpts)) return FM3D_ERR_INVALID;
    const fm3d_settings& S = c->s;
    if (S.detectorType != FM3D_FEAT_ORB || (desc && S.extractorType != FM3D_FEAT_ORB))
        return fail(c, FM3D_ERR_UNSUPPORTED, "the settings' detector (extractor) is not ORB");
    int r;
    if ((r = orb_check_settings(c))) return r;
    hipSetDevice(c->device);
    const int nl = S.orbNumLevels, half = S.orbPatchSize / 2;
    // computeKeyPoints: features per level
    std::vector<int> nper(nl);
    {
        const float factor = (float)(1.0 / S.orbScaleFactor);
        float nd = S.orbNumFeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nl));
        int sum = 0;
        for (int l = 0; l < nl - 1; l++) {
            nper[l] = (int)std::lrint(nd);
            sum += nper[l];
            nd *= factor;
        }
        nper[nl - 1] = std::max(S.orbNumFeatures - sum, 0);
    }
    const OrbPlan P = orb_plan(w, h, S.orbScaleFactor, nl);
    if ((r = orb_build_pyramid(c, img, w, h, P))) return r;
    // FAST + non-max + border over all levels, compacted in level-major raster order
    if (P.total > INT32_MAX / 2) return fail(c, FM3D_ERR_INVALID, "image too large for the ORB pyramid");
    const int tot = (int)P.total;
    if ((r = ensure_scan_tmp(c, tot))) return r;
    HIPCHK(c, c->orbMap.ensure((size_t)tot * sizeof(uint16_t) + 64));
    HIPCHK(c, c->orbFlag.ensure((size_t)(tot + 1) * sizeof(int)));
    HIPCHK(c, c->orbPos.ensure((size_t)(tot + 1) * sizeof(int)));
    fm3d::launch_orb_fast(c->orbPyr.as<uint8_t>(), c->orbLev.as<fm3d::OrbLevel>(), nl, P.total, S.orbFastThreshold,
                          S.orbEdgeThreshold, 1, c->orbMap.as<uint16_t>(), c->orbFlag.as<int>(), c->stream);
    fm3d::launch_exclusive_scan(c->orbFlag.as<int>(), tot, c->orbPos.as<int>(), c->count.as<int>(), c->scanTmp.p,
                                c->stream);
    HIPCHK(c, hipGetLastError());
    int nc = 0;
    HIPCHK(c, hipMemcpyAsync(&nc, c->count.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, c->orbKp.ensure((size_t)(nc + 1) * sizeof(fm3d_keypoint)));
    fm3d::launch_orb_fast_scatter(c->orbMap.as<uint16_t>(), c->orbLev.as<fm3d::OrbLevel>(), nl, P.total,
                                  c->orbFlag.as<int>(), c->orbPos.as<int>(), c->orbKp.as<fm3d_keypoint>(), c->stream);
    std::vector<fm3d_keypoint> k((size_t)nc + 1);
    if (nc > 0)
        HIPCHK(c, hipMemcpyAsync(k.data(), c->orbKp.p, (size_t)nc * sizeof(fm3d_keypoint), hipMemcpyDeviceToHost,
                                 c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    // per level: retainBest(2 * n), Harris, retainBest(n)
    std::vector<int> start(nl + 1, 0);
    for (int i = 0; i < nc; i++) start[k[i].octave + 1]++;
    for (int l = 0; l < nl; l++) start[l + 1] += start[l];
    std::vector<fm3d_keypoint> kb;
    std::vector<int> bstart(nl + 1, 0);
    for (int l = 0; l < nl; l++) {
        const int m = orb_retain_best(k.data() + start[l], start[l + 1] - start[l], 2 * nper[l]);
        kb.insert(kb.end(), k.begin() + start[l], k.begin() + start[l] + m);
        bstart[l + 1] = (int)kb.size();
    }
    const int nb = (int)kb.size();
    if (nb > 0) {
        HIPCHK(c, hipMemcpyAsync(c->orbKp.p, kb.data(), (size_t)nb * sizeof(fm3d_keypoint), hipMemcpyHostToDevice,
                                 c->stream));
        fm3d::launch_orb_harris(c->orbPyr.as<uint8_t>(), c->orbLev.as<fm3d::OrbLevel>(), c->orbKp.as<fm3d_keypoint>(),
                                nb, c->stream);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipMemcpyAsync(kb.data(), c->orbKp.p, (size_t)nb * sizeof(fm3d_keypoint), hipMemcpyDeviceToHost,
                                 c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    std::vector<fm3d_keypoint> kf;
    for (int l = 0; l < nl; l++) {
        const int m = orb_retain_best(kb.data() + bstart[l], bstart[l + 1] - bstart[l], nper[l]);
        const float sf = orb_scale(S.orbScaleFactor, l);
        for (int i = 0; i < m; i++) {
            fm3d_keypoint q = kb[bstart[l] + i];
            q.octave = l;
            q.size = S.orbPatchSize * sf;
            kf.push_back(q);
        }
    }
    const int nf = (int)kf.size(), nw = std::min(nf, cap);
    if (nf > 0) {
        fm3d::OrbUmax um{};
        {  // computeKeyPoints' umax
            const int vmax = (int)std::floor(half * std::sqrt(2.f) / 2 + 1);
            const int vmin = (int)std::ceil(half * std::sqrt(2.f) / 2);
            for (int v = 0; v <= vmax; ++v) um.u[v] = (int)std::lrint(std::sqrt((double)half * half - v * v));
            for (int v = half, v0 = 0; v >= vmin; --v) {
                while (um.u[v0] == um.u[v0 + 1]) ++v0;
                um.u[v] = v0;
                ++v0;
            }
        }
        HIPCHK(c, hipMemcpyAsync(c->orbKp.p, kf.data(), (size_t)nf * sizeof(fm3d_keypoint), hipMemcpyHostToDevice,
                                 c->stream));
        fm3d::launch_orb_angle(c->orbPyr.as<uint8_t>(), c->orbLev.as<fm3d::OrbLevel>(), c->orbKp.as<fm3d_keypoint>(), nf,
                               half, um, c->stream);
        HIPCHK(c, hipGetLastError());
        if (desc && nw > 0 && (r = orb_describe(c, P, nw, desc))) return r;
        HIPCHK(c, hipMemcpyAsync(kf.data(), c->orbKp.p, (size_t)nf * sizeof(fm3d_keypoint), hipMemcpyDeviceToHost,
                                 c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    for (int i = 0; i < nw; i++) {
        fm3d_keypoint q = kf[i];
        if (q.octave != 0) {
            const float sf = orb_scale(S.orbScaleFactor, q.octave);
            q.x *= sf;
            q.y *= sf;
        }
        kpts[i] = q;
    }
    *n = nf;
    return FM3D_OK;
}

int fm3d_sift_detect(fm3d_ctx* c, const uint8_t* img, int w, int h, fm3d_keypoint* kpts, int cap, int* n,
                     float* desc) {
    if (!c || !img || !n || w <= 0 || h <= 0 || cap < 0 || (cap > 0 && !kpts)) return FM3D_ERR_INVALID;
    const fm3d_settings& S = c->s;
    if (S.detectorType != FM3D_FEAT_SIFT || (desc && S.extractorType != FM3D_FEAT_SIFT))
        return fail(c, FM3D_ERR_UNSUPPORTED, "the settings' detector (extractor) is not SIFT");
    int r;
    if ((r = sift_check_settings(c))) return r;
    hipSetDevice(c->device);
    const int L = S.siftOctaveLayers, firstOctave = -1;
    const int nOct = sift_num_octaves(w, h, firstOctave);
    std::vector<fm3d_keypoint> k;
    SiftPlan P;
    if (nOct >= 1) {
        if (!sift_plan(w, h, firstOctave, nOct, L, P))
            return fail(c, FM3D_ERR_INVALID, "SIFT: an octave of the image would be empty");
        if ((r = sift_build(c, img, w, h, P, true))) return r;
        // findScaleSpaceExtrema: flags over every (octave, layer 1..L, row, column), compacted in that order
        std::vector<fm3d::SiftScan> scan;
        long long total = 0;
        for (int o = 0; o < nOct; o++)
            for (int i = 1; i <= L; i++) {
                const fm3d::SiftLevel& d = P.D[o * (L + 2) + i];
                scan.push_back({total, o * (L + 2) + i, o, i, 0});
                total += (long long)d.w * d.h;
            }
        if (total > INT32_MAX / 2) return fail(c, FM3D_ERR_INVALID, "image too large for the SIFT scan");
        const int tot = (int)total;
        const int threshold = (int)std::floor(0.5 * S.siftContrastThreshold / L * 255 * 1);
        HIPCHK(c, c->siftScan.ensure(scan.size() * sizeof(fm3d::SiftScan)));
        HIPCHK(c, hipMemcpyAsync(c->siftScan.p, scan.data(), scan.size() * sizeof(fm3d::SiftScan), hipMemcpyHostToDevice,
                                 c->stream));
        if ((r = ensure_scan_tmp(c, tot))) return r;
        HIPCHK(c, c->siftFlag.ensure((size_t)(tot + 1) * sizeof(int)));
        HIPCHK(c, c->siftPos.ensure((size_t)(tot + 1) * sizeof(int)));
        fm3d::launch_sift_extrema(c->siftD.as<float>(), c->siftDL.as<fm3d::SiftLevel>(), c->siftScan.as<fm3d::SiftScan>(),
                                  (int)scan.size(), total, threshold, c->siftFlag.as<int>(), c->stream);
        fm3d::launch_exclusive_scan(c->siftFlag.as<int>(), tot, c->siftPos.as<int>(), c->count.as<int>(), c->scanTmp.p,
                                    c->stream);
        HIPCHK(c, hipGetLastError());
        int nc = 0;
        HIPCHK(c, hipMemcpyAsync(&nc, c->count.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (nc > 0) {
            HIPCHK(c, c->siftCand.ensure((size_t)nc * sizeof(fm3d::SiftCand)));
            HIPCHK(c, c->siftAng.ensure((size_t)nc * 36 * sizeof(float)));
            HIPCHK(c, c->siftNpk.ensure((size_t)nc * sizeof(int)));
            fm3d::launch_sift_cand_scatter(c->siftDL.as<fm3d::SiftLevel>(), c->siftScan.as<fm3d::SiftScan>(),
                                           (int)scan.size(), total, c->siftFlag.as<int>(), c->siftPos.as<int>(),
                                           c->siftCand.as<fm3d::SiftCand>(), c->stream);
            fm3d::launch_sift_adjust(c->siftD.as<float>(), c->siftDL.as<fm3d::SiftLevel>(), L,
                                     (float)S.siftContrastThreshold, (float)S.siftEdgeThreshold, (float)S.siftSigma,
                                     c->siftCand.as<fm3d::SiftCand>(), nc, c->stream);
            fm3d::launch_sift_orient(c->siftG.as<float>(), c->siftGL.as<fm3d::SiftLevel>(), L,
                                     c->siftCand.as<fm3d::SiftCand>(), nc, c->siftAng.as<float>(),
                                     c->siftNpk.as<int>(), c->stream);
            HIPCHK(c, hipGetLastError());
            std::vector<fm3d::SiftCand> cand(nc);
            std::vector<int> npk(nc);
            std::vector<float> ang((size_t)nc * 36);
            HIPCHK(c, hipMemcpyAsync(cand.data(), c->siftCand.p, (size_t)nc * sizeof(fm3d::SiftCand),
                                     hipMemcpyDeviceToHost, c->stream));
            HIPCHK(c, hipMemcpyAsync(npk.data(), c->siftNpk.p, (size_t)nc * sizeof(int), hipMemcpyDeviceToHost, c->stream));
            HIPCHK(c, hipMemcpyAsync(ang.data(), c->siftAng.p, ang.size() * sizeof(float), hipMemcpyDeviceToHost,
                                     c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
            for (int q = 0; q < nc; q++) {
                const fm3d::SiftCand& C = cand[q];
                if (!C.ok) continue;
                for (int p = 0; p < npk[q]; p++)
                    k.push_back({C.x, C.y, C.size, ang[(size_t)q * 36 + p], C.response, C.koct, -1});
            }
        }
        sift_remove_duplicated(k);
        if (S.siftNumFeatures > 0) k.resize(orb_retain_best(k.data(), (int)k.size(), S.siftNumFeatures));
        for (auto& q : k) {  // firstOctave -1: back to the image's coordinates
            const float scale = 1.f / (float)(1 << -firstOctave);
            q.octave = (q.octave & ~255) | ((q.octave + firstOctave) & 255);
            q.x *= scale;
            q.y *= scale;
            q.size *= scale;
        }
    }
    const int nf = (int)k.size(), nw = std::min(nf, cap);
    for (int i = 0; i < nw; i++) kpts[i] = k[i];
    *n = nf;
    if (desc && nw > 0) {
        // the reference's separate compute (runByKeypointSize keeps all: detected sizes are > 0)
        std::vector<fm3d_keypoint> kd(k.begin(), k.begin() + nw);
        if ((r = sift_describe(c, img, w, h, kd, desc, nOct >= 1 ? &P : nullptr))) return r;
    }
    return FM3D_OK;
}

int fm3d_sift_compute(fm3d_ctx* c, const uint8_t* img, int w, int h, const fm3d_keypoint* kpts, int n,
                      fm3d_keypoint* kout, int32_t* kept, int* nOut, float* desc) {
    if (!c || !img || !nOut || w <= 0 || h <= 0 || n < 0 || (n > 0 && (!kpts || !kout || !desc)))
        return FM3D_ERR_INVALID;
    if (c->s.extractorType != FM3D_FEAT_SIFT) return fail(c, FM3D_ERR_UNSUPPORTED, "the settings' extractor is not SIFT");
    int r;
    if ((r = sift_check_settings(c))) return r;
    hipSetDevice(c->device);
    // DescriptorExtractor::compute: runByKeypointSize(FLT_EPSILON) (runByImageBorder(0) keeps all)
    std::vector<fm3d_keypoint> k;
    std::vector<int> src;
    for (int i = 0; i < n; i++)
        if (!(kpts[i].size < FLT_EPSILON || kpts[i].size > FLT_MAX)) {
            k.push_back(kpts[i]);
            src.push_back(i);
        }
    if ((r = sift_describe(c, img, w, h, k, desc, nullptr))) return r;
    for (size_t i = 0; i < k.size(); i++) {
        kout[i] = k[i];
        if (kept) kept[i] = src[i];
    }
    *nOut = (int)k.size();
    return FM3D_OK;
}

int fm3d_sift_pyramid(fm3d_ctx* c, const uint8_t* img, int w, int h, int firstOctave, int nOctaves, int dog,
                      float* out, int32_t* sizes, int64_t* total) {
    if (!c || !img || !total || w <= 0 || h <= 0 || firstOctave < -1 || firstOctave > 0 || nOctaves < 1)
        return FM3D_ERR_INVALID;
    int r;
    if ((r = sift_check_settings(c))) return r;
    hipSetDevice(c->device);
    SiftPlan P;
    if (!sift_plan(w, h, firstOctave, nOctaves, c->s.siftOctaveLayers, P))
        return fail(c, FM3D_ERR_INVALID, "SIFT: an octave of the image would be empty");
    const std::vector<fm3d::SiftLevel>& Lv = dog ? P.D : P.G;
    *total = dog ? P.dTotal : P.gTotal;
    if (sizes)
        for (size_t i = 0; i < Lv.size(); i++) {
            sizes[2 * i] = Lv[i].w;
            sizes[2 * i + 1] = Lv[i].h;
        }
    if (!out) return FM3D_OK;
    if ((r = sift_build(c, img, w, h, P, dog != 0))) return r;
    HIPCHK(c, hipMemcpyAsync(out, dog ? c->siftD.p : c->siftG.p, (size_t)*total * sizeof(float), hipMemcpyDeviceToHost,
                             c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return FM3D_OK;
}

int fm3d_fast_detect(fm3d_ctx* c, const uint8_t* img, int w, int h, int threshold, int nonmax, fm3d_keypoint* kpts,
                     int cap, int* n) {
    if (!c || !img || !n || w <= 0 || h <= 0 || cap < 0 || (cap > 0 && !kpts)) return FM3D_ERR_INVALID;
    hipSetDevice(c->device);
    std::vector<fm3d_keypoint> k;
    int r;
    if ((r = fast_detect(c, img, w, h, threshold, nonmax != 0, k))) return r;
    for (int i = 0; i < (int)k.size() && i < cap; i++) kpts[i] = k[i];
    *n = (int)k.size();
    return FM3D_OK;
}

// ---------------------------------------------------------------- BRISK extractor
// cv::BRISK's descriptor on given keypoints (OpenCV 2.4.9 brisk.cpp; oracle/orc_brisk.c): what OpenCV's
// constructor precomputes (pattern points per scale and rotation, the short pairs, the size list) and
// its per-keypoint bookkeeping (scale, rotation bin, border filter) stay on the host, in the same
// float / double expressions and glibc calls; the intensities and bits run on the GPU.
}  // extern "C"
namespace brisk {
constexpr int kScales = 64, kRot = 1024, kPoints = 60;
const int kNum[5] = {1, 10, 14, 15, 20};
void radii(float* r) {
    const double f = 0.85 * 1.0;
    r[0] = (float)(f * 0.);
    r[1] = (float)(f * 2.9);
    r[2] = (float)(f * 4.9);
    r[3] = (float)(f * 7.4);
    r[4] = (float)(f * 10.8);
}
float scale_factor(int scale) {
    const float lb_scale = (float)(std::log(30.0) / std::log(2.0));
    const float step = lb_scale / kScales;
    return (float)std::pow(2.0, (double)(scale * step));
}
void point(int scale, int rot, int i, float& px, float& py, float& sg, int* ringOut = nullptr) {
    float r[5];
    radii(r);
    const float sc = scale_factor(scale);
    const double theta = (double)rot * 2 * M_PI / (double)kRot;
    int ring = 0, num = i;
    while (num >= kNum[ring]) num -= kNum[ring++];
    const double alpha = (double)num * 2 * M_PI / (double)kNum[ring];
    const float rr = sc * r[ring];
    px = (float)(rr * std::cos(alpha + theta));
    py = (float)(rr * std::sin(alpha + theta));
    sg = ring == 0 ? 1.3f * sc * 0.5f : (float)(1.3f * sc * (double)r[ring] * std::sin(M_PI / kNum[ring]));
    if (ringOut) *ringOut = ring;
}
int size_of(int scale) {
    float r[5];
    radii(r);
    const float sc = scale_factor(scale);
    int best = 0;
    for (int i = 0; i < kPoints; i++) {
        float x, y, sg;
        int ring;
        point(scale, 0, i, x, y, sg, &ring);
        best = std::max(best, (int)std::ceil(sc * r[ring] + sg) + 1);
    }
    return best;
}
int kscale(float size) {
    const float log2c = 0.693147180559945f;
    const float lb = (float)(logf(30.f) / log2c);
    const float b06 = 12.0f * 0.6f;
    int s = (int)(kScales / lb * (logf(size / b06) / log2c) + 0.5);
    return std::min(std::max(s, 0), kScales - 1);
}
int theta(float angle) {
    if (angle == -1) return 0;
    int t = (int)(kRot * (angle / 360.0) + 0.5);
    if (t < 0) t += kRot;
    if (t >= kRot) t -= kRot;
    return t;
}
std::vector<int> short_pairs() {  // (i, j) interleaved, in generation order
    const float dMin = (float)(8.2 * 1.0), dMax = (float)(5.85 * 1.0);
    const float dMin_sq = dMin * dMin, dMax_sq = dMax * dMax;
    float X[kPoints], Y[kPoints], sg;
    for (int i = 0; i < kPoints; i++) point(0, 0, i, X[i], Y[i], sg);
    std::vector<int> p;
    for (int i = 1; i < kPoints; i++)
        for (int j = 0; j < i; j++) {
            const float dx = X[j] - X[i], dy = Y[j] - Y[i];
            const float n2 = dx * dx + dy * dy;
            if (n2 > dMin_sq) continue;
            if (n2 < dMax_sq) {
                p.push_back(i);
                p.push_back(j);
            }
        }
    return p;
}
}  // namespace brisk

int brisk_compute(fm3d_ctx* c, const uint8_t* img, int w, int h, const fm3d_keypoint* kpts, int n, fm3d_keypoint* kout,
                  int32_t* kept, int* nOut, uint8_t* desc) {
    static const std::vector<int> pairs = brisk::short_pairs();
    static const std::vector<int> sizes = [] {
        std::vector<int> v(brisk::kScales);
        for (int s = 0; s < brisk::kScales; s++) v[s] = brisk::size_of(s);
        return v;
    }();
    *nOut = 0;
    // runByKeypointSize(FLT_EPSILON), then the scale-dependent border (RoiPredicate), order kept
    std::vector<fm3d_keypoint> K;
    std::vector<int> src, combo;
    std::vector<long> keys;
    for (int q = 0; q < n; q++) {
        const fm3d_keypoint& k = kpts[q];
        if (!(k.size >= FLT_EPSILON)) continue;
        const int sc = brisk::kscale(k.size), b = sizes[sc];
        if (k.x < (float)b || k.x >= (float)(w - b) || k.y < (float)b || k.y >= (float)(h - b)) continue;
        K.push_back(k);
        src.push_back(q);
        keys.push_back((long)sc * brisk::kRot + brisk::theta(k.angle));
    }
    const int m = (int)K.size();
    if (m == 0) return FM3D_OK;
    // the pattern rows in use
    std::vector<long> uniq(keys);
    std::sort(uniq.begin(), uniq.end());
    uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
    std::vector<float> pat(uniq.size() * brisk::kPoints * 4, 0.f);
    for (size_t u = 0; u < uniq.size(); u++)
        for (int i = 0; i < brisk::kPoints; i++) {
            float* p = &pat[(u * brisk::kPoints + i) * 4];
            brisk::point((int)(uniq[u] / brisk::kRot), (int)(uniq[u] % brisk::kRot), i, p[0], p[1], p[2]);
        }
    std::vector<int> pidx(m);
    for (int i = 0; i < m; i++) pidx[i] = (int)(std::lower_bound(uniq.begin(), uniq.end(), keys[i]) - uniq.begin());
    const long long W1H1 = (long long)(w + 1) * (h + 1);
    if (W1H1 > INT32_MAX / 4) return fail(c, FM3D_ERR_INVALID, "image too large for BRISK");
    HIPCHK(c, c->brImg.ensure((size_t)w * h));
    HIPCHK(c, c->brSum.ensure((size_t)W1H1 * sizeof(int)));
    HIPCHK(c, c->brKp.ensure((size_t)m * sizeof(fm3d_keypoint)));
    HIPCHK(c, c->brIdx.ensure((size_t)m * sizeof(int)));
    HIPCHK(c, c->brPat.ensure(pat.size() * sizeof(float)));
    HIPCHK(c, c->brPairs.ensure(pairs.size() * sizeof(int)));
    HIPCHK(c, c->brDesc.ensure((size_t)m * 64));
    HIPCHK(c, hipMemcpyAsync(c->brImg.p, img, (size_t)w * h, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->brKp.p, K.data(), (size_t)m * sizeof(fm3d_keypoint), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->brIdx.p, pidx.data(), (size_t)m * sizeof(int), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->brPat.p, pat.data(), pat.size() * sizeof(float), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->brPairs.p, pairs.data(), pairs.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
    fm3d::launch_integral(c->brImg.as<uint8_t>(), w, h, c->brSum.as<int>(), c->stream);
    fm3d::launch_brisk_desc(c->brImg.as<uint8_t>(), c->brSum.as<int>(), w, c->brKp.as<fm3d_keypoint>(),
                            c->brIdx.as<int>(), m, c->brPat.as<float4>(), c->brPairs.as<int2>(), (int)pairs.size() / 2,
                            c->brDesc.as<uint8_t>(), c->stream);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(desc, c->brDesc.p, (size_t)m * 64, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (int i = 0; i < m; i++) {
        kout[i] = K[i];
        if (kept) kept[i] = src[i];
    }
    *nOut = m;
    return FM3D_OK;
}

// ---------------------------------------------------------------- FREAK extractor
// cv::FREAK() on given keypoints (OpenCV 2.4.9 freak.cpp; oracle/orc_freak.c): FREAK::buildPattern's
// tables (the 43 points of each of the 64 scales and 256 orientations in glibc's double cos / sin, the
// pattern sizes, the orientation weights) and the per-keypoint scale and border filter stay on the
// host in the same float / double expressions and glibc calls; intensities, orientation and bits run
// on the GPU (fm3d_freak.hip).
namespace freak {
constexpr float kPatternScale = 22.0f;  // cv::FREAK() defaults
constexpr int kOctaves = 4;
struct Pattern {
    std::vector<float4> lut;  // (x, y, sigma, 0) per (scale, orientation, point)
    int sizes[fm3d::kFreakScales];
    int op[4 * fm3d::kFreakOrientPairs];  // (i, j, weight_dx, weight_dy)
};
const Pattern& pattern() {
    static const Pattern P = [] {
        Pattern p;
        const int n[8] = {6, 6, 6, 6, 6, 6, 6, 1};
        const double bigR = 2.0 / 3.0, smallR = 2.0 / 24.0;
        const double unitSpace = (bigR - smallR) / 21.0;
        const double radius[8] = {bigR, bigR - 6 * unitSpace, bigR - 11 * unitSpace, bigR - 15 * unitSpace,
                                  bigR - 18 * unitSpace, bigR - 20 * unitSpace, smallR, 0.0};
        const double sigma[8] = {radius[0] / 2.0, radius[1] / 2.0, radius[2] / 2.0, radius[3] / 2.0,
                                 radius[4] / 2.0, radius[5] / 2.0, radius[6] / 2.0, radius[6] / 2.0};
        const double scaleStep = std::pow(2.0, (double)kOctaves / fm3d::kFreakScales);
        p.lut.resize((size_t)fm3d::kFreakScales * fm3d::kFreakOrient * fm3d::kFreakPoints);
        for (int s = 0; s < fm3d::kFreakScales; s++) {
            const double scalingFactor = std::pow(scaleStep, (double)s);
            p.sizes[s] = 0;
            for (int r = 0; r < fm3d::kFreakOrient; r++) {
                const double theta = (double)r * 2 * M_PI / (double)fm3d::kFreakOrient;
                int q = 0;
                for (int i = 0; i < 8; i++)
                    for (int k = 0; k < n[i]; k++) {
                        const double beta = M_PI / n[i] * (i % 2);
                        const double alpha = (double)k * 2 * M_PI / (double)n[i] + beta + theta;
                        float4& pt = p.lut[((size_t)s * fm3d::kFreakOrient + r) * fm3d::kFreakPoints + q];
                        pt.x = (float)(radius[i] * std::cos(alpha) * scalingFactor * kPatternScale);
                        pt.y = (float)(radius[i] * std::sin(alpha) * scalingFactor * kPatternScale);
                        pt.z = (float)(sigma[i] * scalingFactor * kPatternScale);
                        pt.w = 0.f;
                        const int sizeMax = (int)std::ceil((radius[i] + sigma[i]) * scalingFactor * kPatternScale) + 1;
                        if (p.sizes[s] < sizeMax) p.sizes[s] = sizeMax;
                        q++;
                    }
            }
        }
        for (int m = fm3d::kFreakOrientPairs; m--;) {
            const int i = FM3D_FREAK_ORIENT_PAIRS[2 * m], j = FM3D_FREAK_ORIENT_PAIRS[2 * m + 1];
            const float dx = p.lut[i].x - p.lut[j].x, dy = p.lut[i].y - p.lut[j].y;
            const float norm_sq = dx * dx + dy * dy;
            p.op[4 * m] = i;
            p.op[4 * m + 1] = j;
            p.op[4 * m + 2] = (int)((dx / norm_sq) * 4096.0 + 0.5);
            p.op[4 * m + 3] = (int)((dy / norm_sq) * 4096.0 + 0.5);
        }
        return p;
    }();
    return P;
}
int kscale(float size) {
    const float sizeCst = (float)(fm3d::kFreakScales / (0.693147180559945 * kOctaves));
    int s = (int)(logf(size / 7) * sizeCst + 0.5);
    return std::min(std::max(s, 0), fm3d::kFreakScales - 1);
}
// the compressed pair index (FREAK::DEF_PAIRS) -> (i, j < i) of the 903 pairs in generation order
int2 pair_of(int k) {
    int a = 1;
    while (k >= a) k -= a++;
    return make_int2(a, k);
}
}  // namespace freak

int freak_compute(fm3d_ctx* c, const uint8_t* img, int w, int h, const fm3d_keypoint* kpts, int n, fm3d_keypoint* kout,
                  int32_t* kept, int* nOut, uint8_t* desc) {
    const freak::Pattern& P = freak::pattern();
    *nOut = 0;
    // runByKeypointSize(FLT_EPSILON) (NaN dropped), then FREAK's scale-dependent border, order kept
    std::vector<fm3d_keypoint> K;
    std::vector<int> src, scl;
    for (int q = 0; q < n; q++) {
        const fm3d_keypoint& k = kpts[q];
        if (!(k.size >= FLT_EPSILON && k.size <= FLT_MAX)) continue;
        const int s = freak::kscale(k.size);
        const float ps = (float)P.sizes[s];
        if (k.x <= ps || k.y <= ps || k.x >= w - ps || k.y >= h - ps) continue;
        K.push_back(k);
        src.push_back(q);
        scl.push_back(s);
    }
    const int m = (int)K.size();
    if (m == 0) return FM3D_OK;
    const long long W1H1 = (long long)(w + 1) * (h + 1);
    if (W1H1 > INT32_MAX / 4) return fail(c, FM3D_ERR_INVALID, "image too large for FREAK");
    std::vector<int2> pairs(FM3D_FREAK_NB_PAIRS);
    for (int k = 0; k < FM3D_FREAK_NB_PAIRS; k++)
        pairs[k] = freak::pair_of(c->freakUserPairs.empty() ? FM3D_FREAK_DEF_PAIRS[k] : c->freakUserPairs[k]);
    if (c->frLut.bytes == 0) {  // the whole pattern, once per context (8.4 MB)
        HIPCHK(c, c->frLut.ensure(P.lut.size() * sizeof(float4)));
        HIPCHK(c, c->frOp.ensure(sizeof(P.op)));
        HIPCHK(c, hipMemcpy(c->frLut.p, P.lut.data(), P.lut.size() * sizeof(float4), hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(c->frOp.p, P.op, sizeof(P.op), hipMemcpyHostToDevice));
    }
    HIPCHK(c, c->frImg.ensure((size_t)w * h));
    HIPCHK(c, c->frSum.ensure((size_t)W1H1 * sizeof(int)));
    HIPCHK(c, c->frKp.ensure((size_t)m * sizeof(fm3d_keypoint)));
    HIPCHK(c, c->frScale.ensure((size_t)m * sizeof(int)));
    HIPCHK(c, c->frPairs.ensure(pairs.size() * sizeof(int2)));
    HIPCHK(c, c->frAng.ensure((size_t)m * sizeof(float)));
    HIPCHK(c, c->frDesc.ensure((size_t)m * 64));
    HIPCHK(c, hipMemcpyAsync(c->frImg.p, img, (size_t)w * h, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->frKp.p, K.data(), (size_t)m * sizeof(fm3d_keypoint), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->frScale.p, scl.data(), (size_t)m * sizeof(int), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->frPairs.p, pairs.data(), pairs.size() * sizeof(int2), hipMemcpyHostToDevice, c->stream));
    fm3d::launch_integral(c->frImg.as<uint8_t>(), w, h, c->frSum.as<int>(), c->stream);
    fm3d::launch_freak_desc(c->frImg.as<uint8_t>(), c->frSum.as<int>(), w, c->frKp.as<fm3d_keypoint>(),
                            c->frScale.as<int>(), m, c->frLut.as<float4>(), c->frOp.as<int4>(), c->frPairs.as<int2>(),
                            c->frAng.as<float>(), c->frDesc.as<uint8_t>(), c->stream);
    HIPCHK(c, hipGetLastError());
    std::vector<float> ang(m);
    HIPCHK(c, hipMemcpyAsync(desc, c->frDesc.p, (size_t)m * 64, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(ang.data(), c->frAng.p, (size_t)m * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (int i = 0; i < m; i++) {
        kout[i] = K[i];
        kout[i].angle = ang[i];  // FREAK's orientation normalisation sets the keypoint angle
        if (kept) kept[i] = src[i];
    }
    *nOut = m;
    return FM3D_OK;
}

// MSER (fm3d_mser.hip): the floods of `count` images (two per image, slot = 2 * image + pass), then the
// regions' records and point offsets.  regs: every slot's regions in slot order ({colour, head node,
// count, slot}); off: their prefix (points before each).
int mser_flood(fm3d_ctx* c, const uint8_t* img, int count, int w, int h, const fm3d::MserParams& P,
               fm3d::MserLayout& L, std::vector<int4>& regs, std::vector<long long>& off) {
    if (w <= 0 || h <= 0 || count <= 0) return fail(c, FM3D_ERR_INVALID, "MSER: empty image");
    if ((long long)(w + 2) * (h + 2) >= (1LL << 28) - 1 || w > 65535 || h > 65535)
        return fail(c, FM3D_ERR_INVALID, "MSER: image too large");
    if ((long long)2 * count * w * h >= (1LL << 30)) return fail(c, FM3D_ERR_INVALID, "MSER: batch too large");
    const int slots = 2 * count;
    L = fm3d::mser_layout(w, h);
    HIPCHK(c, c->msImg.ensure((size_t)count * w * h));
    HIPCHK(c, c->msPad.ensure((size_t)slots * L.padBytes));
    HIPCHK(c, c->msWork.ensure(L.visInLds ? 16 : (size_t)slots * L.visWords * sizeof(unsigned)));
    HIPCHK(c, c->msHeap.ensure((size_t)slots * L.heapEntries * sizeof(int2)));
    HIPCHK(c, c->msNode.ensure((size_t)slots * L.nodes * sizeof(int2)));
    HIPCHK(c, c->msHist.ensure((size_t)slots * L.hists * sizeof(fm3d::MserHist)));
    HIPCHK(c, c->msReg.ensure((size_t)slots * L.regCap * sizeof(int4)));
    HIPCHK(c, c->msCnt.ensure((size_t)slots * sizeof(int)));
    HIPCHK(c, hipMemcpyAsync(c->msImg.p, img, (size_t)count * w * h, hipMemcpyHostToDevice, c->stream));
    fm3d::launch_mser_flood(c->msImg.as<uint8_t>(), count, L, P, c->msPad.as<uint8_t>(), c->msWork.as<unsigned>(),
                            c->msHeap.as<int2>(), c->msNode.as<int2>(), c->msHist.as<fm3d::MserHist>(),
                            c->msReg.as<int4>(), c->msCnt.as<int>(), c->stream);
    HIPCHK(c, hipGetLastError());
    std::vector<int> cnt(slots, 0);
    HIPCHK(c, hipMemcpyAsync(cnt.data(), c->msCnt.p, (size_t)slots * sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    long long total = 0;
    for (int k = 0; k < slots; k++) {
        if (cnt[k] < 0 || cnt[k] > L.regCap) return fail(c, FM3D_ERR_HIP, "MSER: region count out of range");
        total += cnt[k];
    }
    regs.resize((size_t)total);
    for (int k = 0, at = 0; k < slots; at += cnt[k], k++)
        if (cnt[k])
            HIPCHK(c, hipMemcpyAsync(regs.data() + at, c->msReg.as<int4>() + (size_t)k * L.regCap,
                                     (size_t)cnt[k] * sizeof(int4), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    off.assign(regs.size() + 1, 0);
    for (int k = 0, i = 0; k < slots; k++)
        for (int j = 0; j < cnt[k]; j++, i++) {
            if (regs[i].z <= 0 || regs[i].z > (long long)w * h) return fail(c, FM3D_ERR_HIP, "MSER: bad region size");
            regs[i].w = k;
            off[i + 1] = off[i] + regs[i].z;
        }
    return FM3D_OK;
}

// the region points (gathered from the ranked node lists) and each region's fitEllipse keypoint + kept flag
int mser_fit(fm3d_ctx* c, const fm3d::MserLayout& L, int count, const std::vector<int4>& regs,
             const std::vector<long long>& off) {
    const int n = (int)regs.size();
    if (n == 0) return FM3D_OK;
    const long long tot = off[n];
    HIPCHK(c, c->msOff.ensure((size_t)(n + 1) * sizeof(long long)));
    HIPCHK(c, c->msRegC.ensure((size_t)n * sizeof(int4)));
    HIPCHK(c, c->msXY.ensure((size_t)tot * sizeof(int2)));
    HIPCHK(c, c->msScr.ensure((size_t)tot * 5 * sizeof(double)));
    HIPCHK(c, c->msKp.ensure((size_t)(n + 1) * sizeof(fm3d_keypoint)));
    HIPCHK(c, c->msFlag.ensure((size_t)(n + 1) * sizeof(int)));
    HIPCHK(c, hipMemcpyAsync(c->msOff.p, off.data(), (size_t)(n + 1) * sizeof(long long), hipMemcpyHostToDevice,
                             c->stream));
    HIPCHK(c, hipMemcpyAsync(c->msRegC.p, regs.data(), (size_t)n * sizeof(int4), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, c->msRank.ensure(fm3d::mser_rank_bytes(L.nodes, 2 * count)));
    const fm3d::MserRank K =
        fm3d::launch_mser_rank(c->msNode.as<int2>(), L.nodes, 2 * count, c->msRank.as<int>(), c->stream);
    fm3d::launch_mser_fit(c->msRegC.as<int4>(), n, K, L.nodes, c->msOff.as<long long>(), L, c->msXY.as<int2>(),
                          c->msScr.as<double>(), c->msKp.as<fm3d_keypoint>(), c->msFlag.as<int>(), nullptr, c->stream);
    HIPCHK(c, hipGetLastError());
    return FM3D_OK;
}

fm3d::MserParams mser_params(int delta, int minArea, int maxArea, double maxVariation, double minDiversity) {
    fm3d::MserParams P;
    P.delta = delta;
    P.minArea = minArea;
    P.maxArea = maxArea;
    P.maxVariation = maxVariation;
    P.minDiversity = minDiversity;
    return P;
}

// MserFeatureDetector::detect: the kept keypoints in region order
// MserFeatureDetector::detect on `count` images: the kept keypoints of each image in region order,
// image after image; per[i] = image i's count
int mser_detect(fm3d_ctx* c, const uint8_t* img, int count, int w, int h, const fm3d::MserParams& P,
                std::vector<fm3d_keypoint>& k, std::vector<int>& per) {
    k.clear();
    per.assign(count, 0);
    fm3d::MserLayout L;
    std::vector<int4> regs;
    std::vector<long long> off;
    int r;
    if ((r = mser_flood(c, img, count, w, h, P, L, regs, off))) return r;
    const int n = (int)regs.size();
    for (int i = 0; i < n; i++)
        if (regs[i].z < 5) return fail(c, FM3D_ERR_INVALID, "MSER: a region under 5 points (fitEllipse throws)");
    if (n == 0) return FM3D_OK;
    if ((r = mser_fit(c, L, count, regs, off))) return r;
    if ((r = ensure_scan_tmp(c, n))) return r;
    HIPCHK(c, c->msPos.ensure((size_t)(n + 1) * sizeof(int)));
    fm3d::launch_exclusive_scan(c->msFlag.as<int>(), n, c->msPos.as<int>(), c->count.as<int>(), c->scanTmp.p, c->stream);
    HIPCHK(c, hipGetLastError());
    int nk = 0;
    std::vector<int> pos(n);
    HIPCHK(c, hipMemcpyAsync(&nk, c->count.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    if (count > 1) HIPCHK(c, hipMemcpyAsync(pos.data(), c->msPos.p, (size_t)n * sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (count == 1) {
        per[0] = nk;
    } else {  // image i's keypoints: the kept regions of slots 2i and 2i + 1
        std::vector<int> first(count + 1, n);  // image i's first region (n: past the end)
        for (int i = n - 1; i >= 0; i--) first[regs[i].w >> 1] = i;
        for (int i = count - 1; i >= 0; i--)
            if (first[i] == n) first[i] = first[i + 1];  // an image without regions
        auto at = [&](int f) { return f < n ? pos[f] : nk; };
        for (int i = 0; i < count; i++) per[i] = at(first[i + 1]) - at(first[i]);
    }
    if (nk == 0) return FM3D_OK;
    HIPCHK(c, c->msOut.ensure((size_t)nk * sizeof(fm3d_keypoint)));
    fm3d::launch_star_scatter(c->msKp.as<fm3d_keypoint>(), c->msFlag.as<int>(), c->msPos.as<int>(), n,
                              c->msOut.as<fm3d_keypoint>(), c->stream);
    HIPCHK(c, hipGetLastError());
    k.resize(nk);
    HIPCHK(c, hipMemcpyAsync(k.data(), c->msOut.p, (size_t)nk * sizeof(fm3d_keypoint), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return FM3D_OK;
}

extern "C" {
int fm3d_mser_detect(fm3d_ctx* c, const uint8_t* img, int w, int h, int delta, int minArea, int maxArea,
                     double maxVariation, double minDiversity, fm3d_keypoint* kpts, int cap, int* n) {
    if (!c || !img || !n || w <= 0 || h <= 0 || cap < 0 || (cap > 0 && !kpts)) return FM3D_ERR_INVALID;
    hipSetDevice(c->device);
    std::vector<fm3d_keypoint> k;
    std::vector<int> per;
    int r;
    if ((r = mser_detect(c, img, 1, w, h, mser_params(delta, minArea, maxArea, maxVariation, minDiversity), k, per)))
        return r;
    for (int i = 0; i < (int)k.size() && i < cap; i++) kpts[i] = k[i];
    *n = (int)k.size();
    return FM3D_OK;
}

int fm3d_mser_detect_batch(fm3d_ctx* c, const uint8_t* imgs, int count, int w, int h, int delta, int minArea,
                           int maxArea, double maxVariation, double minDiversity, fm3d_keypoint* kpts, int cap,
                           int32_t* counts, int* total) {
    if (!c || !imgs || !counts || !total || count <= 0 || w <= 0 || h <= 0 || cap < 0 || (cap > 0 && !kpts))
        return FM3D_ERR_INVALID;
    hipSetDevice(c->device);
    std::vector<fm3d_keypoint> k;
    std::vector<int> per;
    int r;
    if ((r = mser_detect(c, imgs, count, w, h, mser_params(delta, minArea, maxArea, maxVariation, minDiversity), k,
                         per)))
        return r;
    for (int i = 0; i < (int)k.size() && i < cap; i++) kpts[i] = k[i];
    for (int i = 0; i < count; i++) counts[i] = per[i];
    *total = (int)k.size();
    return FM3D_OK;
}

int fm3d_mser_regions(fm3d_ctx* c, const uint8_t* img, int w, int h, int delta, int minArea, int maxArea,
                      double maxVariation, double minDiversity, int32_t* color, int32_t* count, int cap, int32_t* pts,
                      int64_t ptsCap, int* nRegions, int64_t* nPoints) {
    if (!c || !img || !nRegions || !nPoints || w <= 0 || h <= 0 || cap < 0 || ptsCap < 0 ||
        (cap > 0 && (!color || !count)) || (ptsCap > 0 && !pts))
        return FM3D_ERR_INVALID;
    hipSetDevice(c->device);
    fm3d::MserLayout L;
    std::vector<int4> regs;
    std::vector<long long> off;
    int r;
    const fm3d::MserParams P = mser_params(delta, minArea, maxArea, maxVariation, minDiversity);
    if ((r = mser_flood(c, img, 1, w, h, P, L, regs, off))) return r;
    const int n = (int)regs.size();
    if ((r = mser_fit(c, L, 1, regs, off))) return r;  // gathers the region points into msXY
    const long long tot = off[n];
    for (int i = 0; i < n && i < cap; i++) {
        color[i] = regs[i].x;
        count[i] = regs[i].z;
    }
    const long long m = std::min<long long>(tot, ptsCap);
    if (m > 0)
        HIPCHK(c, hipMemcpyAsync(pts, c->msXY.p, (size_t)m * sizeof(int2), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    *nRegions = n;
    *nPoints = tot;
    return FM3D_OK;
}

int fm3d_freak_compute(fm3d_ctx* c, const uint8_t* img, int w, int h, const fm3d_keypoint* kpts, int n,
                       fm3d_keypoint* kout, int32_t* kept, int* nOut, uint8_t* desc) {
    if (!c || !img || !nOut || w <= 0 || h <= 0 || n < 0 || (n > 0 && (!kpts || !kout || !desc)))
        return FM3D_ERR_INVALID;
    hipSetDevice(c->device);
    return freak_compute(c, img, w, h, kpts, n, kout, kept, nOut, desc);
}

int fm3d_freak_set_pairs(fm3d_ctx* c, const int32_t* pairs, int n) {
    if (!c || (pairs && n != FM3D_FREAK_NB_PAIRS)) return FM3D_ERR_INVALID;
    if (pairs)
        for (int k = 0; k < n; k++)
            if (pairs[k] < 0 || pairs[k] >= 903) return fail(c, FM3D_ERR_INVALID, "a FREAK pair index outside [0, 903)");
    c->freakUserPairs.clear();
    if (pairs) c->freakUserPairs.assign(pairs, pairs + n);
    return FM3D_OK;
}

int fm3d_brisk_compute(fm3d_ctx* c, const uint8_t* img, int w, int h, const fm3d_keypoint* kpts, int n,
                       fm3d_keypoint* kout, int32_t* kept, int* nOut, uint8_t* desc) {
    if (!c || !img || !nOut || w <= 0 || h <= 0 || n < 0 || (n > 0 && (!kpts || !kout || !desc)))
        return FM3D_ERR_INVALID;
    hipSetDevice(c->device);
    return brisk_compute(c, img, w, h, kpts, n, kout, kept, nOut, desc);
}

int fm3d_star_responses(fm3d_ctx* c, const uint8_t* img, int w, int h, int maxSize, float* resp, int16_t* sizes,
                        int* border) {
    if (!c || !img || !resp || !sizes || !border || w <= 0 || h <= 0) return FM3D_ERR_INVALID;
    hipSetDevice(c->device);
    fm3d::StarPat P;
    int r;
    if ((r = star_responses(c, img, w, h, maxSize, P))) return r;
    HIPCHK(c, hipMemcpyAsync(resp, c->starR.p, (size_t)w * h * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(sizes, c->starZ.p, (size_t)w * h * sizeof(int16_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    *border = P.border;
    return FM3D_OK;
}

int fm3d_star_detect(fm3d_ctx* c, const uint8_t* img, int w, int h, int maxSize, int response, int lineThreshold,
                     int lineBinarized, int suppression, fm3d_keypoint* kpts, int cap, int* n) {
    if (!c || !img || !n || w <= 0 || h <= 0 || cap < 0 || (cap > 0 && !kpts)) return FM3D_ERR_INVALID;
    hipSetDevice(c->device);
    std::vector<fm3d_keypoint> k;
    int r;
    if ((r = star_detect(c, img, w, h, maxSize, response, lineThreshold, lineBinarized, suppression, k))) return r;
    for (int i = 0; i < (int)k.size() && i < cap; i++) kpts[i] = k[i];
    *n = (int)k.size();
    return FM3D_OK;
}

}  // extern "C"

namespace {
// one detector call into a host vector (the entries' cap / count protocol)
template <class F>
int detect_into(F&& f, std::vector<fm3d_keypoint>& k) {
    int cap = 4096, n = 0, r;
    for (;;) {
        k.resize(cap);
        if ((r = f(k.data(), cap, &n))) return r;
        if (n <= cap) break;
        cap = n;
    }
    k.resize(n);
    return FM3D_OK;
}

// the settings' detector as it stands (STATIC, or one ADAPTIVE detector call with threshold thr)
int detect_static(fm3d_ctx* c, const uint8_t* img, int w, int h, std::vector<fm3d_keypoint>& k) {
    const fm3d_settings& S = c->s;
    switch (S.detectorType) {
    case FM3D_FEAT_SURF:
        return detect_into([&](fm3d_keypoint* p, int cap, int* n) { return fm3d_surf_detect(c, img, w, h, p, cap, n, nullptr); }, k);
    case FM3D_FEAT_ORB:
        return detect_into([&](fm3d_keypoint* p, int cap, int* n) { return fm3d_orb_detect(c, img, w, h, p, cap, n, nullptr); }, k);
    case FM3D_FEAT_SIFT:
        return detect_into([&](fm3d_keypoint* p, int cap, int* n) { return fm3d_sift_detect(c, img, w, h, p, cap, n, nullptr); }, k);
    case FM3D_FEAT_FAST:
        return fast_detect(c, img, w, h, S.fastThreshold, S.fastNonmax != 0, k);
    case FM3D_FEAT_STAR:
        return star_detect(c, img, w, h, S.starMaxSize, S.starResponse, S.starLineThreshold, S.starLineBinarized,
                           S.starSuppression, k);
    case FM3D_FEAT_MSER:
    {
        std::vector<int> per;
        return mser_detect(c, img, 1, w, h,
                           mser_params(S.mserDelta, S.mserMinArea, S.mserMaxArea, S.mserMaxVariation,
                                       S.mserMinDiversity),
                           k, per);
    }
    default:
        return fail(c, FM3D_ERR_UNSUPPORTED, "the settings' detector type has no GPU implementation");
    }
}

// DynamicAdaptedFeatureDetector(AdjusterAdapter::create(type), min, max, iters)::detect
// (features2d/src/dynamic.cpp): detect, then raise / lower the adjuster's threshold until the count
// is in [min, max], the threshold leaves the adjuster's range, the iterations run out or it
// oscillates.  FastAdjuster(20, true, 1, 200): FastFeatureDetector(thresh, true), -- / ++ by one;
// SurfAdjuster(400, 2, 1000): the default SURF (4 octaves, 2 layers, not upright) at hessianThreshold
// thresh, * 0.9 (floored at 1.1) / * 1.1; StarAdjuster(30, 2, 200): StarFeatureDetector(16,
// cvRound(thresh), 10, 8, 3), the same scaling.  The keypoints are the last call's.
int detect_adaptive(fm3d_ctx* c, const uint8_t* img, int w, int h, std::vector<fm3d_keypoint>& k) {
    const fm3d_settings S = c->s;
    const bool fast = S.detectorType == FM3D_FEAT_FAST, star = S.detectorType == FM3D_FEAT_STAR;
    if (!fast && !star && S.detectorType != FM3D_FEAT_SURF)
        return fail(c, FM3D_ERR_UNSUPPORTED, "ADAPTIVE runs the FAST, SURF and STAR adjusters");
    double thresh = fast ? 20 : star ? 30 : 400;
    const double minT = fast ? 1 : 2, maxT = fast ? 200 : star ? 200 : 1000;
    bool down = false, up = false, good = false;
    int iters = S.adaptiveMaxIters, r = FM3D_OK;
    k.clear();
    while (iters > 0 && !(down && up) && !good && thresh > minT && thresh < maxT) {
        if (fast) {
            r = fast_detect(c, img, w, h, (int)thresh, true, k);
        } else if (star) {
            r = star_detect(c, img, w, h, 16, (int)std::nearbyint(thresh), 10, 8, 3, k);
        } else {
            fm3d_settings t = S;  // FeatureDetector::create("SURF") + set("hessianThreshold", thresh)
            t.detectorMode = 0;
            t.surfHessianThreshold = thresh;
            t.surfOctaves = 4;
            t.surfOctaveLayers = 2;
            t.surfExtended = 0;
            t.surfUpright = 0;
            c->s = t;
            r = detect_static(c, img, w, h, k);
            c->s = S;
        }
        if (r) return r;
        if ((int)k.size() < S.adaptiveMinFeatures) {
            down = true;
            if (fast)
                thresh -= 1;
            else if ((thresh *= 0.9) < 1.1)
                thresh = 1.1;
        } else if ((int)k.size() > S.adaptiveMaxFeatures) {
            up = true;
            if (fast)
                thresh += 1;
            else
                thresh *= 1.1;
        } else {
            good = true;
        }
        iters--;
    }
    return FM3D_OK;
}
}  // namespace

extern "C" {

int fm3d_detect(fm3d_ctx* c, const uint8_t* img, int w, int h, fm3d_keypoint* kpts, int cap, int* n) {
    if (!c || !img || !n || w <= 0 || h <= 0 || cap < 0 || (cap > 0 && !kpts)) return FM3D_ERR_INVALID;
    hipSetDevice(c->device);
    std::vector<fm3d_keypoint> k;
    int r = c->s.detectorMode == 1 ? detect_adaptive(c, img, w, h, k) : detect_static(c, img, w, h, k);
    if (r) return r;
    for (int i = 0; i < (int)k.size() && i < cap; i++) kpts[i] = k[i];
    *n = (int)k.size();
    return FM3D_OK;
}

int fm3d_descriptor_info(const fm3d_ctx* c, int* cols, int* type) {
    if (!c || !cols || !type) return FM3D_ERR_INVALID;
    switch (c->s.extractorType) {
    case FM3D_FEAT_SURF:
        *cols = c->s.surfExtended ? 128 : 64;
        *type = FM3D_DESC_F32;
        return FM3D_OK;
    case FM3D_FEAT_SIFT:
        *cols = 128;
        *type = FM3D_DESC_F32;
        return FM3D_OK;
    case FM3D_FEAT_ORB:
        *cols = 32;
        *type = FM3D_DESC_BITS;
        return FM3D_OK;
    case FM3D_FEAT_BRISK:
    case FM3D_FEAT_FREAK:
        *cols = 64;
        *type = FM3D_DESC_BITS;
        return FM3D_OK;
    default:
        return FM3D_ERR_UNSUPPORTED;
    }
}

int fm3d_compute(fm3d_ctx* c, const uint8_t* img, int w, int h, const fm3d_keypoint* kpts, int n, fm3d_keypoint* kout,
                 int32_t* kept, int* nOut, void* desc) {
    switch (c ? c->s.extractorType : FM3D_FEAT_OTHER) {
    case FM3D_FEAT_SURF:
        return fm3d_surf_compute(c, img, w, h, kpts, n, kout, kept, nOut, static_cast<float*>(desc));
    case FM3D_FEAT_SIFT:
        return fm3d_sift_compute(c, img, w, h, kpts, n, kout, kept, nOut, static_cast<float*>(desc));
    case FM3D_FEAT_ORB:
        return fm3d_orb_compute(c, img, w, h, kpts, n, kout, kept, nOut, static_cast<uint8_t*>(desc));
    case FM3D_FEAT_BRISK:
        return fm3d_brisk_compute(c, img, w, h, kpts, n, kout, kept, nOut, static_cast<uint8_t*>(desc));
    case FM3D_FEAT_FREAK:
        return fm3d_freak_compute(c, img, w, h, kpts, n, kout, kept, nOut, static_cast<uint8_t*>(desc));
    default:
        return c ? fail(c, FM3D_ERR_UNSUPPORTED, "the settings' extractor type has no GPU implementation")
                 : FM3D_ERR_INVALID;
    }
}

int fm3d_orb_compute(fm3d_ctx* c, const uint8_t* img, int w, int h, const fm3d_keypoint* kpts, int n,
                     fm3d_keypoint* kout, int32_t* kept, int* nOut, uint8_t* desc) {
    if (!c || !img || !nOut || w <= 0 || h <= 0 || n < 0 || (n > 0 && (!kpts || !kout || !desc)))
        return FM3D_ERR_INVALID;
    const fm3d_settings& S = c->s;
    if (S.extractorType != FM3D_FEAT_ORB) return fail(c, FM3D_ERR_UNSUPPORTED, "the settings' extractor is not ORB");
    int r;
    if ((r = orb_check_settings(c))) return r;
    *nOut = 0;
    if (n == 0) return FM3D_OK;
    const int b = S.orbEdgeThreshold;
    // runByKeypointSize(FLT_EPSILON) (NaN kept), runByImageBorder(edgeThreshold) on rounded positions
    std::vector<int> src;
    int L = 0;
    for (int i = 0; i < n; i++) {
        const float sz = kpts[i].size;
        if (sz < FLT_EPSILON || sz > FLT_MAX) continue;
        if (b > 0) {
            if (h <= 2 * b || w <= 2 * b) continue;
            const long ix = std::lrint(kpts[i].x), iy = std::lrint(kpts[i].y);
            if (!(ix >= b && ix < b + (w - 2 * b) && iy >= b && iy < b + (h - 2 * b))) continue;
        }
        if (kpts[i].octave < 0) return fail(c, FM3D_ERR_INVALID, "ORB compute: keypoint with a negative octave");
        if (kpts[i].octave >= 64) return fail(c, FM3D_ERR_INVALID, "ORB compute: keypoint octave >= 64");
        L = std::max(L, kpts[i].octave + 1);
        src.push_back(i);
    }
    if (src.empty()) return FM3D_OK;
    // grouped by octave (input order within a level), positions in level coordinates
    std::vector<fm3d_keypoint> k;
    std::vector<int> order;
    for (int l = 0; l < L; l++) {
        const float inv = 1 / orb_scale(S.orbScaleFactor, l);
        for (int i : src) {
            if (kpts[i].octave != l) continue;
            fm3d_keypoint q = kpts[i];
            if (l != 0) {
                q.x *= inv;
                q.y *= inv;
            }
            k.push_back(q);
            order.push_back(i);
        }
    }
    hipSetDevice(c->device);
    const OrbPlan P = orb_plan(w, h, S.orbScaleFactor, L);
    for (const fm3d_keypoint& q : k) {  // the descriptor's reads stay inside the level
        const fm3d::OrbLevel& lv = P.L[q.octave];
        const long ix = std::lrint(q.x), iy = std::lrint(q.y);
        const int reach = (int)std::ceil(S.orbPatchSize / 2 * 1.4143) + 4;
        if (ix < reach || iy < reach || ix >= lv.w - reach || iy >= lv.h - reach)
            return fail(c, FM3D_ERR_INVALID, "ORB compute: keypoint octave inconsistent with its position");
    }
    if ((r = orb_build_pyramid(c, img, w, h, P))) return r;
    const int m = (int)k.size();
    HIPCHK(c, c->orbKp.ensure((size_t)m * sizeof(fm3d_keypoint)));
    HIPCHK(c, hipMemcpyAsync(c->orbKp.p, k.data(), (size_t)m * sizeof(fm3d_keypoint), hipMemcpyHostToDevice, c->stream));
    if ((r = orb_describe(c, P, m, desc))) return r;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (int i = 0; i < m; i++) {
        fm3d_keypoint q = k[i];
        if (q.octave != 0) {
            const float sf = orb_scale(S.orbScaleFactor, q.octave);
            q.x *= sf;
            q.y *= sf;
        }
        kout[i] = q;
        if (kept) kept[i] = order[i];
    }
    *nOut = m;
    return FM3D_OK;
}

int fm3d_ncc_hypotheses(fm3d_ctx* c, const double* points, int P, int Hphi, int Htheta, double span, double* scores,
                        double* normals, int32_t* best) {
    if (!c || P < 0 || Hphi <= 0 || Htheta <= 0 || Hphi * Htheta > 32 || (P && (!points || !scores || !normals || !best)))
        return FM3D_ERR_INVALID;
    if (c->pyr1.empty()) return fail(c, FM3D_ERR_INVALID, "fm3d_set_images (NormalOptimizer::setImages) not called");
    if (!c->haveG12) return fail(c, FM3D_ERR_INVALID, "fm3d_set_g12 / fm3d_setg12 not called");
    if (P == 0) return FM3D_OK;
    hipSetDevice(c->device);
    int r;
    if ((r = ensure_offsets(c))) return r;
    const int H = Hphi * Htheta;
    DevBuf X, S, N, B;
    HIPCHK(c, X.ensure((size_t)P * 3 * sizeof(double)));
    HIPCHK(c, S.ensure((size_t)P * H * sizeof(double)));
    HIPCHK(c, N.ensure((size_t)P * 3 * sizeof(double)));
    HIPCHK(c, B.ensure((size_t)P * sizeof(int)));
    HIPCHK(c, hipMemcpyAsync(X.p, points, (size_t)P * 3 * sizeof(double), hipMemcpyHostToDevice, c->stream));
    fm3d::NccParams p{};
    p.points = X.as<double>();
    p.P = P;
    p.cam = lm_camera(c->cam);  // the kernel's bit-pattern isPixelGood (fm3d_ncc.hip ncc_geometry)
    std::memcpy(p.R2, c->R2, sizeof(p.R2));
    std::memcpy(p.t2, c->t2, sizeof(p.t2));
    p.img1 = c->pyr1[0].as<uint8_t>();
    p.img2 = c->pyr2[0].as<uint8_t>();
    p.w = c->lw[0];
    p.h = c->lh[0];
    p.offsets = c->offsets.as<int2>();
    p.nOff = c->nOff;
    p.nOffPad = c->nOffPad;
    p.boundW = c->s.boundWidth;
    p.boundH = c->s.boundHeight;
    p.cmax = (int)(2 * c->s.zThresholdMax);
    p.Hphi = Hphi;
    p.Htheta = Htheta;
    p.span = span;
    p.scores = S.as<double>();
    p.normals = N.as<double>();
    p.best = B.as<int>();
    fm3d::launch_ncc_hypotheses(p, c->stream);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(scores, S.p, (size_t)P * H * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(normals, N.p, (size_t)P * 3 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(best, B.p, (size_t)P * sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return FM3D_OK;
}

int fm3d_pyrdown(fm3d_ctx* c, const uint8_t* src, int width, int height, uint8_t* dst) {
    if (!c || !src || !dst || width <= 0 || height <= 0) return FM3D_ERR_INVALID;
    hipSetDevice(c->device);
    DevBuf a, b;
    HIPCHK(c, a.ensure((size_t)width * height));
    const int dw = (width + 1) / 2, dh = (height + 1) / 2;
    HIPCHK(c, b.ensure((size_t)dw * dh));
    HIPCHK(c, hipMemcpy(a.p, src, (size_t)width * height, hipMemcpyHostToDevice));
    fm3d::launch_pyrdown(a.as<uint8_t>(), width, height, b.as<uint8_t>(), c->stream);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(dst, b.p, (size_t)dw * dh, hipMemcpyDeviceToHost));
    a.release();
    b.release();
    return FM3D_OK;
}

int fm3d_neighborhood(fm3d_ctx* c, const double X[3], double* xy, int cap, int* m) {
    // host restatement of extractPixelsContour (used to cross-check the kernel's own)
    if (!c || !X || !m) return FM3D_ERR_INVALID;
    const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, Z[3] = {0, 0, 0};
    double cx, cy;
    fm3d::project1(c->cam, I, Z, X[0], X[1], X[2], cx, cy);
    const int R = c->s.pixelsRay;
    int n = 0;
    for (int i = -R; i <= R; i++)
        for (int j = -R; j <= R; j++)
            if (i * i + j * j <= R * R) {
                double px = cx + i, py = cy + j;
                if (px < 0 || py < 0 || px >= c->s.boundWidth || py >= c->s.boundHeight) continue;
                if (n < cap && xy) {
                    xy[2 * n] = px;
                    xy[2 * n + 1] = py;
                }
                n++;
            }
    *m = n;
    return FM3D_OK;
}

int fm3d_plane_to_image2(fm3d_ctx* c, const double X[3], const double n[3], double* xy, double* uv, int32_t* status,
                         int cap, int* m) {
    if (!c || !X || !n || !m || cap < 0) return FM3D_ERR_INVALID;
    if (!c->haveG12) return fail(c, FM3D_ERR_INVALID, "no camera-2 pose: call fm3d_setg12 / fm3d_set_g12 first");
    hipSetDevice(c->device);
    int r;
    if ((r = ensure_offsets(c))) return r;
    const int N = c->nOff;
    DevBuf bxy, buv, bkeep, bst;
    HIPCHK(c, bxy.ensure((size_t)N * 16));
    HIPCHK(c, buv.ensure((size_t)N * 16));
    HIPCHK(c, bkeep.ensure((size_t)N * 4));
    HIPCHK(c, bst.ensure((size_t)N * 4));
    fm3d::PlaneProjParams p{};
    p.cam = c->cam;
    std::memcpy(p.R2, c->R2, sizeof(p.R2));
    std::memcpy(p.t2, c->t2, sizeof(p.t2));
    for (int k = 0; k < 3; k++) {
        p.X[k] = X[k];
        p.n[k] = n[k];
    }
    p.cmax = (double)(int)(2 * c->s.zThresholdMax);
    p.offsets = c->offsets.as<int2>();
    p.nOff = N;
    p.boundW = c->s.boundWidth;
    p.boundH = c->s.boundHeight;
    p.w = c->w;  // isPixelGood bounds of the images set with fm3d_set_images (0: none)
    p.h = c->h;
    p.xy = bxy.as<double>();
    p.uv = buv.as<double>();
    p.keep = bkeep.as<int>();
    p.status = bst.as<int>();
    fm3d::launch_plane_project(p, c->stream);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(c->stream));
    std::vector<double> hxy((size_t)2 * N), huv((size_t)2 * N);
    std::vector<int> hk(N), hs(N);
    HIPCHK(c, hipMemcpy(hxy.data(), bxy.p, (size_t)N * 16, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(huv.data(), buv.p, (size_t)N * 16, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(hk.data(), bkeep.p, (size_t)N * 4, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(hs.data(), bst.p, (size_t)N * 4, hipMemcpyDeviceToHost));
    int k = 0;
    for (int t = 0; t < N; t++) {
        if (!hk[t]) continue;
        if (k < cap) {
            if (xy) { xy[2 * k] = hxy[2 * t]; xy[2 * k + 1] = hxy[2 * t + 1]; }
            if (uv) { uv[2 * k] = huv[2 * t]; uv[2 * k + 1] = huv[2 * t + 1]; }
            if (status) status[k] = hs[t];
        }
        k++;
    }
    *m = k;
    bxy.release();
    buv.release();
    bkeep.release();
    bst.release();
    return FM3D_OK;
}

int fm3d_undistort(fm3d_ctx* c, const double* xy, int n, double* out) {
    if (!c || n < 0 || (n && (!xy || !out))) return FM3D_ERR_INVALID;
    hipSetDevice(c->device);
    DevBuf a, b;
    HIPCHK(c, a.ensure((size_t)n * 16 + 16));
    HIPCHK(c, b.ensure((size_t)n * 16 + 16));
    HIPCHK(c, hipMemcpy(a.p, xy, (size_t)n * 16, hipMemcpyHostToDevice));
    fm3d::launch_undistort(c->cam, a.as<double>(), n, b.as<double>(), c->stream);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(out, b.p, (size_t)n * 16, hipMemcpyDeviceToHost));
    a.release();
    b.release();
    return FM3D_OK;
}

}  // extern "C"
