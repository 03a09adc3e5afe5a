// fm3d_misc.hip -- triangulation, pyramids, undistortion and stable compaction.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fm3d_kernels.h"

namespace fm3d {

namespace {

// ---------------- DLT triangulation ----------------
// The default null vector is cvTriangulatePoints' (OpenCV 2.4): the 6 x 4 matrA and JacobiSVD, as
// include/fm3d_cvsvd.h restates them (fm3d_cv::triangulate_point), bit for bit the oracle's
// orc_triangulate1.  dltSolver = 1 (opt-in) keeps the solver of rounds 1-5 below: the 4-row system
// and a one-sided (Hestenes) Jacobi SVD in the round-robin pair order (0,1)+(2,3), (0,2)+(1,3),
// (0,3)+(1,2), up to 30 sweeps (oracle ORC_GEOM_DLT_LEGACY).  The two rotations of a step touch
// disjoint columns: independent, so their dependent chains (three divisions and two square roots
// each) run side by side.  Its points leave OpenCV's by up to ~1e-12 relative.
template <int P, int Q>
__device__ __forceinline__ bool jacobi_pair(double* A, double* V) {
    double alpha = 0, beta = 0, gamma = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        double ap = A[i * 4 + P], aq = A[i * 4 + Q];
        alpha += ap * ap;
        beta += aq * aq;
        gamma += ap * aq;
    }
    if (gamma != 0. && fabs(gamma) > 1e-15 * sqrt(alpha * beta)) {
        double zeta = (beta - alpha) / (2. * gamma);
        double t = (zeta >= 0. ? 1. : -1.) / (fabs(zeta) + sqrt(1. + zeta * zeta));
        double cs = 1. / sqrt(1. + t * t);
        double sn = cs * t;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            double ap = A[i * 4 + P], aq = A[i * 4 + Q];
            A[i * 4 + P] = cs * ap - sn * aq;
            A[i * 4 + Q] = sn * ap + cs * aq;
            ap = V[i * 4 + P];
            aq = V[i * 4 + Q];
            V[i * 4 + P] = cs * ap - sn * aq;
            V[i * 4 + Q] = sn * ap + cs * aq;
        }
        return true;
    }
    return false;
}
__device__ inline void dlt_nullvec(double* A, double* v) {
    double V[16];
#pragma unroll
    for (int i = 0; i < 16; i++) V[i] = (i % 5 == 0) ? 1. : 0.;
    for (int sweep = 0; sweep < 30; sweep++) {
        bool rotated = jacobi_pair<0, 1>(A, V);
        rotated |= jacobi_pair<2, 3>(A, V);
        rotated |= jacobi_pair<0, 2>(A, V);
        rotated |= jacobi_pair<1, 3>(A, V);
        rotated |= jacobi_pair<0, 3>(A, V);
        rotated |= jacobi_pair<1, 2>(A, V);
        if (!rotated) break;
    }
    double nrm[4];
#pragma unroll
    for (int p = 0; p < 4; p++) {
        double s = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) s += A[i * 4 + p] * A[i * 4 + p];
        nrm[p] = s;
    }
    int best = 0;
#pragma unroll
    for (int p = 1; p < 4; p++)
        if (nrm[p] < nrm[best]) best = p;
#pragma unroll
    for (int i = 0; i < 4; i++) v[i] = best == 0 ? V[i * 4] : best == 1 ? V[i * 4 + 1] : best == 2 ? V[i * 4 + 2] : V[i * 4 + 3];
}

// setKeypoints (singlecameratriangulator.cpp:145-171) + triangulate (:173-230), one
// thread per match: gather, undistortPoints, cvTriangulatePoints, z filter.  A thread's A and V
// (32 doubles) and the sweep's temporaries need ~150 VGPRs: 64-thread workgroups (launch bound)
// give it the registers; under the default 1024-thread bound (128 VGPRs) the sweeps spilled to
// scratch and the kernel lasted 27-33 us at any match count (rocprofv3, round 3).
constexpr int kTriThreads = 64;
// match i: its homogeneous DLT point and whether it is an inlier (zThresholdMin <= Z/W < Max)
__device__ __forceinline__ bool tri_one(const TriParams& p, int i, double* X) {
    const fm3d_dmatch mt = p.matches[i];
    const fm3d_point2f k1 = p.kp1[mt.queryIdx - p.queryOffset];
    const fm3d_point2f k2 = p.kp2[mt.trainIdx];
    double u1x, u1y, u2x, u2y;
    undistort1(p.cam, (double)k1.x, (double)k1.y, u1x, u1y);
    undistort1(p.cam, (double)k2.x, (double)k2.y, u2x, u2y);
    // P1 = [I|0], P2 = [I|0] * g12 (rows 0..2 of g12)
    if (p.dltSolver == 0) {
        fm3d_cv::triangulate_point(p.g12, u1x, u1y, u2x, u2y, X);
    } else {  // rows x*P.row2 - P.row0, y*P.row2 - P.row1 per view
        double A[16];
        const double P1[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
        for (int k = 0; k < 4; k++) {
            A[0 * 4 + k] = u1x * P1[8 + k] - P1[0 + k];
            A[1 * 4 + k] = u1y * P1[8 + k] - P1[4 + k];
            A[2 * 4 + k] = u2x * p.g12[8 + k] - p.g12[0 + k];
            A[3 * 4 + k] = u2y * p.g12[8 + k] - p.g12[4 + k];
        }
        dlt_nullvec(A, X);
    }
    // Z/W < zThresholdMin || Z/W >= zThresholdMax -> outlier (:200-216)
    const bool out = (X[2] / X[3] < p.zmin || X[2] / X[3] >= p.zmax);
    p.mask[i] = out ? 0 : 1;
    if (p.mask8) p.mask8[i] = out ? 0 : 1;
    return !out;
}
__global__ __launch_bounds__(kTriThreads) void triangulate_kernel(TriParams p) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (p.Kdev ? *p.Kdev : p.K)) return;  // the match count on the device (grid: its bound)
    double X[4];
    tri_one(p, i, X);
    p.pts[3 * i + 0] = X[0] / X[3];
    p.pts[3 * i + 1] = X[1] / X[3];
    p.pts[3 * i + 2] = X[2] / X[3];
}
// the same with the inliers compacted in match order (fm3d_kernels.h LookBack): out, srcIdx, *count
// -- the pipeline's a4/a5 without compact<Point3>'s launch (12 us at C2, one workgroup)
// hostCnt (page-locked host memory, or null): the last block also stores (match count, inlier count)
// there with system-scope stores, so a caller that waits for the kernel reads them without a copy
// launch (fm3d_pipeline_submit_dlt; 3.4 us of copy kernel and a 6 us gap at C2)
__global__ __launch_bounds__(kTriThreads) void triangulate_compact_kernel(TriParams p, double* __restrict__ out,
                                                                          int* __restrict__ srcIdx,
                                                                          int* __restrict__ count, LookBack lb,
                                                                          int* hostCnt) {
    __shared__ int sBid;
    const int lane = threadIdx.x;
    if (lane == 0) sBid = lookback_block_id(lb);
    __syncthreads();
    const int bid = sBid;
    const int i = bid * kTriThreads + lane;
    double X[4];
    const bool inl = i < (p.Kdev ? *p.Kdev : p.K) && tri_one(p, i, X);
    const unsigned long long bal = __ballot(inl);
    const int ex = lookback_exclusive(lb.st, lb.epoch, bid, __popcll(bal));  // one wave: kTriThreads == 64
    const int o = ex + __popcll(bal & ((1ull << lane) - 1));
    if (inl) {
        out[3 * o + 0] = X[0] / X[3];
        out[3 * o + 1] = X[1] / X[3];
        out[3 * o + 2] = X[2] / X[3];
        srcIdx[o] = i;
    }
    if (lane == 0 && bid == (int)gridDim.x - 1) {
        const int total = ex + __popcll(bal);
        *count = total;
        if (hostCnt) {
            __hip_atomic_store(&hostCnt[0], p.Kdev ? *p.Kdev : p.K, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&hostCnt[1], total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// ---------------- the LM launch's resets (LMReset) ----------------
__global__ void lm_reset_kernel(LMReset r, int maxP) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < 32) r.stat[t] = t == 20 ? ~0ull : 0ull;
    if (r.queue && t < 64) r.queue[t] = 0;
    for (int j = 0; j < r.nProb; j++) {
        if (t < 4) r.pcnt16[j][t] = 0;
        if (t < r.P[j]) r.status[j][t] = kLMRunning;
        if (t < 8 * r.P[j]) {
            r.info[j][t] = 0;
            r.nfev[j][t] = 0;
        }
    }
    (void)maxP;
}

// ---------------- cv::pyrDown (8U) ----------------
__device__ inline int reflect101(int q, int len) {
    if (len == 1) return 0;
    while (q < 0 || q >= len) q = q < 0 ? -q : 2 * len - q - 2;
    return q;
}

__global__ void pyrdown_kernel(const uint8_t* __restrict__ src, int w, int h, uint8_t* __restrict__ dst) {
    const int dw = (w + 1) / 2, dh = (h + 1) / 2;
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y * blockDim.y + threadIdx.y;
    if (x >= dw || y >= dh) return;
    const int wt[5] = {1, 4, 6, 4, 1};
    int sx[5];
    for (int j = 0; j < 5; j++) sx[j] = reflect101(2 * x + j - 2, w);
    int s = 0;
    for (int i = 0; i < 5; i++) {
        const uint8_t* row = src + (size_t)reflect101(2 * y + i - 2, h) * w;
        int rs = 0;
        for (int j = 0; j < 5; j++) rs += wt[j] * row[sx[j]];
        s += wt[i] * rs;
    }
    dst[(size_t)y * dw + x] = (uint8_t)((s + 128) >> 8);
}

__global__ void undistort_kernel(Camera cam, const double* __restrict__ xy, int n, double* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    undistort1(cam, xy[2 * i], xy[2 * i + 1], out[2 * i], out[2 * i + 1]);
}

// extractPixelsContour(X) (singlecameratriangulator.cpp:341-397) and, for every kept pixel,
// get3dPointsFromImage1Pixels (:530-574: undistortPoints, projectPointToPlane :421-470,
// isInBoundingBox :646-655) + projectPointsToImage2 (:591-626) at scale 1 through the plane (X, n):
// one thread per circle offset (reference order).  keep[t] = 1 for pixels inside the bound
// (compacted on the host in offset order), status[t] 0 / 5 NaN plane / 2 bounding box / 4 image-2
// pixel outside isPixelGood(.., 1.0) of a w x h image (w = 0: not tested).
__global__ void plane_project_kernel(PlaneProjParams p) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= p.nOff) return;
    const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, Z[3] = {0, 0, 0};
    double cx, cy;
    project1(p.cam, I, Z, p.X[0], p.X[1], p.X[2], cx, cy);
    const int2 o = p.offsets[t];
    const double px = cx + o.x, py = cy + o.y;
    const int keep = !(px < 0 || py < 0 || px >= p.boundW || py >= p.boundH);
    p.keep[t] = keep;
    p.xy[2 * t] = px;
    p.xy[2 * t + 1] = py;
    if (!keep) return;
    double ux, uy;
    undistort1(p.cam, px, py, ux, uy);
    const double mm = p.n[0] * p.X[0] + p.n[1] * p.X[1] + p.n[2] * p.X[2];
    const double nn = p.n[0] * ux + p.n[1] * uy + p.n[2] * 1.;
    const double k = mm / nn;
    const double P0 = k * ux, P1 = k * uy, P2 = k * 1.;
    const double cm = p.cmax;
    int st = 0;
    if (P0 != P0 || P1 != P1 || P2 != P2) st = 5;
    else if (!((P0 > -cm && P0 < cm) && (P1 > -cm && P1 < cm) && (P2 > 0. && P2 < cm))) st = 2;
    double u, v;
    project1(p.cam, p.R2, p.t2, P0, P1, P2, u, v);
    if (!st && p.w > 0 && !pixel_good(u, v, 1.0, p.w, p.h)) st = 4;
    p.uv[2 * t] = u;
    p.uv[2 * t + 1] = v;
    p.status[t] = st;
}

// ---------------- stable compaction (three-phase scan) ----------------
constexpr int kScanBlock = 1024;  // items per block (256 threads x 4)

// n: the item count, or its bound when nDev holds the count on the device (the grid is sized by
// the bound; items past the count read as unflagged, so the extra blocks count 0)
__device__ __forceinline__ int dev_count(const int* nDev, int n) {
    if (!nDev) return n;
    const int d = *nDev;
    return d < n ? d : n;
}

__global__ void scan_count_kernel(const int* __restrict__ flag, int n, const int* __restrict__ nDev,
                                  int* __restrict__ blockSums) {
    __shared__ int red[256];
    n = dev_count(nDev, n);
    const int base = blockIdx.x * kScanBlock;
    int c = 0;
    for (int k = 0; k < 4; k++) {
        int i = base + threadIdx.x * 4 + k;
        c += (i < n && flag[i]) ? 1 : 0;
    }
    red[threadIdx.x] = c;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) blockSums[blockIdx.x] = red[0];
}

// exclusive scan of nb block sums in one workgroup of 1024 threads (chunked)
__global__ void scan_blocks_kernel(int* __restrict__ blockSums, int nb, int* __restrict__ total) {
    __shared__ int buf[1024];
    __shared__ int carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int c0 = 0; c0 < nb; c0 += 1024) {
        const int i = c0 + threadIdx.x;
        int v = (i < nb) ? blockSums[i] : 0;
        buf[threadIdx.x] = v;
        __syncthreads();
        for (int off = 1; off < 1024; off <<= 1) {
            int t = (int)threadIdx.x >= off ? buf[threadIdx.x - off] : 0;
            __syncthreads();
            buf[threadIdx.x] += t;
            __syncthreads();
        }
        const int incl = buf[threadIdx.x];
        if (i < nb) blockSums[i] = carry + incl - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry += incl;
        __syncthreads();
    }
    if (threadIdx.x == 0 && total) *total = carry;
}

// local exclusive offsets of a 1024-item block; returns the per-thread base
__device__ inline int block_local_offset(const int* flag, int n, int base, int* sh, int& c4, int f[4]) {
    c4 = 0;
    for (int k = 0; k < 4; k++) {
        int i = base + threadIdx.x * 4 + k;
        f[k] = (i < n && flag[i]) ? 1 : 0;
        c4 += f[k];
    }
    sh[threadIdx.x] = c4;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
        int t = (int)threadIdx.x >= off ? sh[threadIdx.x - off] : 0;
        __syncthreads();
        sh[threadIdx.x] += t;
        __syncthreads();
    }
    return sh[threadIdx.x] - c4;
}

template <typename T>
__global__ void scatter_kernel(const T* __restrict__ in, const int* __restrict__ flag, int n,
                               const int* __restrict__ nDev, const int* __restrict__ blockOff, T* __restrict__ out,
                               int* __restrict__ srcIndex) {
    __shared__ int sh[256];
    n = dev_count(nDev, n);
    const int base = blockIdx.x * kScanBlock;
    int c4, f[4];
    int o = blockOff[blockIdx.x] + block_local_offset(flag, n, base, sh, c4, f);
    for (int k = 0; k < 4; k++) {
        int i = base + threadIdx.x * 4 + k;
        if (f[k]) {
            out[o] = in[i];
            if (srcIndex) srcIndex[o] = i;
            o++;
        }
    }
}

struct Point3 {
    double v[3];
};

__global__ void offsets_kernel(const int* __restrict__ flag, int n, const int* __restrict__ blockOff,
                               int* __restrict__ offsets) {
    __shared__ int sh[256];
    const int base = blockIdx.x * kScanBlock;
    int c4, f[4];
    int o = blockOff[blockIdx.x] + block_local_offset(flag, n, base, sh, c4, f);
    for (int k = 0; k < 4; k++) {
        int i = base + threadIdx.x * 4 + k;
        if (i < n) offsets[i] = o;
        o += f[k];
    }
}

// up to kSmallCompact items: one workgroup of 1024 threads, item i = 1024 * it + thread (coalesced,
// every flag loaded at once), the (iteration, wave) counts by ballots, their exclusive scan over 256
// entries in (iteration, wave) order by the first four waves -- one launch instead of three.  With
// offsets the per-item exclusive offsets are written, with out the flagged items (and srcIndex)
// scattered in order.  count: the total.
constexpr int kSmallCompact = 16384;

template <typename T>
__global__ __launch_bounds__(1024) void compact_small_kernel(const T* __restrict__ in, const int* __restrict__ flag,
                                                             int n, const int* __restrict__ nDev, T* __restrict__ out,
                                                             int* __restrict__ count, int* __restrict__ srcIndex,
                                                             int* __restrict__ offsets) {
    __shared__ int wt[256];
    __shared__ int ws4[4];
    __shared__ int totS;
    n = dev_count(nDev, n);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int ipt = (n + 1023) >> 10;  // iterations, <= 16
    bool f[16];
#pragma unroll
    for (int it = 0; it < 16; it++) {
        const int i = it * 1024 + tid;
        f[it] = it < ipt && i < n && flag[i] != 0;
    }
    const unsigned long long below = (1ull << lane) - 1ull;
    int pre[16];
#pragma unroll
    for (int it = 0; it < 16; it++) {
        const unsigned long long b = __ballot(f[it]);
        pre[it] = __popcll(b & below);
        if (lane == 0) wt[it * 16 + wid] = __popcll(b);
    }
    __syncthreads();
    int v = 0, x = 0;
    if (tid < 256) {
        v = wt[tid];
        x = v;
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) ws4[wid] = x;
    }
    __syncthreads();
    if (tid < 256) {
        int add = 0;
        for (int w = 0; w < wid; w++) add += ws4[w];
        wt[tid] = add + x - v;  // exclusive
        if (tid == 255) totS = add + x;
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 16; it++) {
        const int i = it * 1024 + tid;
        if (it < ipt && i < n) {
            const int o = wt[it * 16 + wid] + pre[it];
            if (offsets) offsets[i] = o;
            if (f[it]) {
                if (out) out[o] = in[i];
                if (srcIndex) srcIndex[o] = i;
            }
        }
    }
    if (tid == 0 && count) *count = totS;
}

template <typename T>
void compact(const T* in, const int* flag, int n, const int* nDev, T* out, int* count, int* srcIndex, void* tmp,
             hipStream_t s) {
    const int nb = (n + kScanBlock - 1) / kScanBlock;
    int* blockSums = (int*)tmp;
    if (n <= 0) {
        hipMemsetAsync(count, 0, sizeof(int), s);
        return;
    }
    if (n <= kSmallCompact) {
        compact_small_kernel<T><<<1, 1024, 0, s>>>(in, flag, n, nDev, out, count, srcIndex, nullptr);
        return;
    }
    scan_count_kernel<<<nb, 256, 0, s>>>(flag, n, nDev, blockSums);
    scan_blocks_kernel<<<1, 1024, 0, s>>>(blockSums, nb, count);
    scatter_kernel<T><<<nb, 256, 0, s>>>(in, flag, n, nDev, blockSums, out, srcIndex);
}

__global__ void make_records_kernel(const fm3d_dmatch* __restrict__ matches, const int* __restrict__ inlierSrc,
                                    int nInl, const int* __restrict__ nDev, const double* __restrict__ pts,
                                    const double* __restrict__ normals, const int* __restrict__ status,
                                    fm3d_record* __restrict__ rec, int* __restrict__ flag) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= dev_count(nDev, nInl)) return;
    const fm3d_dmatch m = matches[inlierSrc[i]];
    fm3d_record r;
    r.queryIdx = m.queryIdx;
    r.trainIdx = m.trainIdx;
    r.distance = m.distance;
    r.status = status[i];
    for (int k = 0; k < 3; k++) {
        r.point[k] = pts[3 * i + k];
        r.normal[k] = normals[3 * i + k];
    }
    rec[i] = r;
    flag[i] = status[i] == FM3D_ST_OK ? 1 : 0;
}

}  // namespace

void launch_triangulate(const TriParams& p, hipStream_t s) {
    if (p.K <= 0) return;
    triangulate_kernel<<<(p.K + kTriThreads - 1) / kTriThreads, kTriThreads, 0, s>>>(p);
}

int triangulate_compact_blocks(int K) { return K > 0 ? (K + kTriThreads - 1) / kTriThreads : 1; }

void launch_triangulate_compact(const TriParams& p, double* out, int* srcIdx, int* count, const LookBack& lb,
                                hipStream_t s, int* hostCnt) {
    triangulate_compact_kernel<<<triangulate_compact_blocks(p.K), kTriThreads, 0, s>>>(p, out, srcIdx, count, lb,
                                                                                      hostCnt);
}

void launch_lm_reset(const LMReset& r, hipStream_t s) {
    int maxP = 0;
    for (int j = 0; j < r.nProb; j++) maxP = r.P[j] > maxP ? r.P[j] : maxP;
    const long n = 8L * maxP > 64 ? 8L * maxP : 64;
    lm_reset_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(r, maxP);
}

void launch_pyrdown(const uint8_t* src, int w, int h, uint8_t* dst, hipStream_t s) {
    const int dw = (w + 1) / 2, dh = (h + 1) / 2;
    dim3 blk(32, 8), grd((dw + 31) / 32, (dh + 7) / 8);
    pyrdown_kernel<<<grd, blk, 0, s>>>(src, w, h, dst);
}

void launch_plane_project(const PlaneProjParams& p, hipStream_t s) {
    if (p.nOff > 0) plane_project_kernel<<<(p.nOff + 255) / 256, 256, 0, s>>>(p);
}

void launch_undistort(const Camera& cam, const double* xy, int n, double* out, hipStream_t s) {
    if (n <= 0) return;
    undistort_kernel<<<(n + 255) / 256, 256, 0, s>>>(cam, xy, n, out);
}

size_t scan_tmp_bytes(int n) { return sizeof(int) * ((size_t)(n + kScanBlock - 1) / kScanBlock + 16); }

void launch_compact_dmatch(const fm3d_dmatch* in, const int* flag, int n, fm3d_dmatch* out, int* count, void* tmp,
                           hipStream_t s) {
    compact<fm3d_dmatch>(in, flag, n, nullptr, out, count, nullptr, tmp, s);
}

void launch_compact_points(const double* in, const int* flag, int n, const int* nDev, double* out, int* count,
                           int* srcIndex, void* tmp, hipStream_t s) {
    compact<Point3>((const Point3*)in, flag, n, nDev, (Point3*)out, count, srcIndex, tmp, s);
}

void launch_exclusive_scan(const int* flag, int n, int* offsets, int* total, void* tmp, hipStream_t s) {
    const int nb = (n + kScanBlock - 1) / kScanBlock;
    int* blockSums = (int*)tmp;
    if (n <= 0) {
        hipMemsetAsync(total, 0, sizeof(int), s);
        return;
    }
    if (n <= kSmallCompact) {
        compact_small_kernel<int><<<1, 1024, 0, s>>>(nullptr, flag, n, nullptr, nullptr, total, nullptr, offsets);
        return;
    }
    scan_count_kernel<<<nb, 256, 0, s>>>(flag, n, nullptr, blockSums);
    scan_blocks_kernel<<<1, 1024, 0, s>>>(blockSums, nb, total);
    offsets_kernel<<<nb, 256, 0, s>>>(flag, n, blockSums, offsets);
}

void launch_make_records(const fm3d_dmatch* matches, const int* inlierSrc, int nInl, const int* nDev, const double* pts,
                         const double* normals, const int* status, fm3d_record* rec, int* flag, hipStream_t s) {
    if (nInl <= 0) return;
    make_records_kernel<<<(nInl + 255) / 256, 256, 0, s>>>(matches, inlierSrc, nInl, nDev, pts, normals, status, rec,
                                                            flag);
}

void launch_compact_records(const fm3d_record* in, const int* flag, int n, const int* nDev, fm3d_record* out,
                            int* count, void* tmp, hipStream_t s) {
    compact<fm3d_record>(in, flag, n, nDev, out, count, nullptr, tmp, s);
}

}  // namespace fm3d
