// fm3d_star.hip -- the STAR (CenSurE) detector on gfx950.
//
// Reference: DescriptorsMatcher's DetectorType STAR (descriptorsmatcher.cpp:204-213,
// cv::StarFeatureDetector(MaxSize, Response, LineThreshold, LineBinarized, Suppression)) and the
// StarAdjuster of its ADAPTIVE mode (:185-200).  The algorithm is OpenCV 2.4.9's
// features2d/src/stardetector.cpp, restated in oracle/orc_star.c; the GPU equals that oracle bit for bit:
//   integral (fm3d_surf.hip)  the upright sum S
//   star_diag_*_kernel        the tilted sum T and the flat-tilted sum F from prefix sums down the
//                             diagonals of the row prefix sums (below): every diagonal an independent
//                             chunked scan, exact modulo 2^32
//   star_tilted_kernel        (FM3D_STAR_TILT=rows) the same T and F by OpenCV's row recursions, one
//                             workgroup walking the rows with the last three in an LDS ring
//   star_resp_kernel          a thread per pixel: every pattern's box sum from 8 integral reads (int),
//                             then the (inner, outer) pairs in OpenCV's order and float arithmetic, the
//                             SSE2 block's float(vals) - float(inner) on its columns and the scalar
//                             tail's int difference on the rest
//   star_nms_kernel           a thread per (Suppression/2 + 1)^2 tile and extremum: the tile's maximum
//                             or minimum, its window, the size and line tests; two slots per tile,
//                             compacted in tile order by a scan
// The L2-resident integrals (3 x 4 (w+1)(h+1) bytes) serve the responses' gathers.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "fm3d_kernels.h"

namespace fm3d {

namespace {

constexpr int kTiltThreads = 1024;
// (outer, inner) pattern pairs of StarDetectorComputeResponses (each inner pattern half its outer one)
__device__ constexpr int kStarPairs[12][2] = {{1, 0}, {3, 1}, {4, 2}, {5, 3}, {7, 4}, {8, 5},
                                              {9, 6}, {11, 8}, {13, 10}, {14, 11}, {15, 12}, {16, 14}};

// T and F, (h+1) x (w+1) int32.  LDS: the last three rows of each (row y written, y-1 and y-2 read)
// and the image rows of the current block of rows.  Per block of `bk` rows the workgroup first stages
// the bk + 1 image rows the block reads (one round trip to memory per block instead of one per row);
// then each row is a thread per column and a barrier that waits on LDS only: the row's global stores
// stay in flight (no load in the row loop waits behind them).
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__global__ __launch_bounds__(kTiltThreads) void star_tilted_kernel(const uint8_t* __restrict__ I, int w, int h,
                                                                   int bk, int* __restrict__ T, int* __restrict__ F) {
    extern __shared__ int ring[];  // [3][w+1] of T, [3][w+1] of F, then (bk + 1) x w image bytes
    const int st = w + 1, tid = threadIdx.x;
    int* RT = ring;
    int* RF = ring + 3 * st;
    uint8_t* G = reinterpret_cast<uint8_t*>(ring + 6 * st);
    // rows 0 and 1: zeros, then the top image row alone
    for (int x = tid; x <= w; x += kTiltThreads) {
        const int m1 = x >= 1 ? I[x - 1] : 0, z = x < w ? I[x] : 0;
        const int t = x == 0 ? 0 : m1;
        const int f = x == 0 ? z : x == w ? m1 : z + m1;
        T[x] = F[x] = 0;
        RT[x] = RF[x] = 0;
        T[st + x] = t;
        F[st + x] = f;
        RT[st + x] = t;
        RF[st + x] = f;
    }
    int* Trow = T + (size_t)2 * st;
    int* Frow = F + (size_t)2 * st;
    int cur = 2, q1 = 1, q2 = 0;  // ring slots of rows y, y-1, y-2
    for (int yb = 2; yb <= h; yb += bk) {
        // image rows yb-2 .. min(yb+bk-2, h-1) into G (row r at (r - (yb-2)) * w)
        const int nrow = min(bk + 1, h - (yb - 2));
        __syncthreads();  // the previous block's reads of G are done (and rows 0-1 are in the ring)
        for (int e = tid; e < nrow * w; e += kTiltThreads) G[e] = I[(size_t)(yb - 2) * w + e];
        __syncthreads();
        const int ye = min(yb + bk - 1, h);
        for (int y = yb; y <= ye; y++) {
            const int *t1 = RT + q1 * st, *t2 = RT + q2 * st, *f1 = RF + q1 * st, *f2 = RF + q2 * st;
            int *tc = RT + cur * st, *fc = RF + cur * st;
            const uint8_t *a = G + (y - yb + 1) * w, *b = a - w;  // image rows y-1 and y-2
            // branch-free (a divergent boundary wave would run every case's loads in turn and hold up
            // the barrier): OpenCV's column-0, 1 and w formulas as masked terms of the general one.
            // Column 1's F, f1[2] + b[0] + a[1] + a[0], equals the general form because
            // F(y-1, 0) - F(y-2, 1) = b[0] (both are sums of the same triangles bar that pixel).
            const int t1_2 = t1[2], a0 = a[0], b0 = b[0];
            for (int x = tid; x <= w; x += kTiltThreads) {
                const int xl = max(x - 1, 0), xr = min(x + 1, w);
                const int L = (x >= 2 || x == w) ? t1[xl] : 0, Rr = x < w ? t1[xr] : 0;
                const int M = (x >= 2 && x < w) ? t2[x] : 0;
                const int am = x >= 1 ? a[xl] : 0, bm = x >= 1 ? b[xl] : 0, az = x < w ? a[min(x, w - 1)] : 0;
                const int t = L + Rr - M + bm + am;
                const int fg = f1[xl] + f1[xr] - f2[x] + az + am;
                const int f = x == w ? t : (x == 0 ? t1_2 + b0 + a0 : fg);
                tc[x] = t;
                fc[x] = f;
                Trow[x] = t;
                Frow[x] = f;
            }
            Trow += st;
            Frow += st;
            const int nx = q2;
            q2 = q1;
            q1 = cur;
            cur = nx;
            lds_barrier();
        }
    }
}

// ---- the same T and F without the row chain.  With R(y', k) the sum of image row y''s first k pixels,
// clamped to k in [0, w] (Re), the zero-padded definitions give
//   T(y, x) = P(y, x + y - 1) - N(y, x - y),   F(y, x) = P(y, x + y) - N(y, x - y),
//   P(y, u) = sum_{y' < y} Re(y', u - y'),      N(y, v) = sum_{y' < y} Re(y', v + y'),
// prefix sums down the anti-diagonals (P) and diagonals (N) of Re: independent columns of a scan over
// y, done in chunks of kDiagRows rows (partial sums, a scan over the chunks, then the rows of each
// chunk).  Modulo-2^32 arithmetic: exact wherever OpenCV's int sums are.  Column j of P is u = j - 1,
// of N v = j - h; Wd = w + h + 2 columns.
constexpr int kDiagRows = 16;

__device__ __forceinline__ unsigned diag_re(const int* __restrict__ R, int w, int yp, int k) {
    return (unsigned)R[(size_t)(yp + 1) * (w + 1) + min(max(k, 0), w)];
}

// part[z][c][j]: the chunk's sum of Re over its source rows y' in [c*B, min(c*B + B, h))
__global__ __launch_bounds__(256) void star_diag_part_kernel(const int* __restrict__ R, int w, int h, int Wd, int C,
                                                             unsigned* __restrict__ part) {
    const int j = blockIdx.x * 256 + threadIdx.x, c = blockIdx.y, z = blockIdx.z;
    if (j >= Wd) return;
    const int y0 = c * kDiagRows, y1 = min(y0 + kDiagRows, h);
    unsigned acc = 0;
    for (int yp = y0; yp < y1; yp++) acc += diag_re(R, w, yp, z == 0 ? (j - 1) - yp : (j - h) + yp);
    part[((size_t)z * C + c) * Wd + j] = acc;
}

// part -> exclusive prefix over the chunks, in place
__global__ __launch_bounds__(256) void star_diag_scan_kernel(int Wd, int C, unsigned* __restrict__ part) {
    const int j = blockIdx.x * 256 + threadIdx.x, z = blockIdx.y;
    if (j >= Wd) return;
    unsigned run = 0;
    for (int c = 0; c < C; c++) {
        unsigned* p = part + ((size_t)z * C + c) * Wd + j;
        const unsigned v = *p;
        *p = run;
        run += v;
    }
}

// PN[z][y][j] for the rows y in [c*B, min(c*B + B, h + 1))
__global__ __launch_bounds__(256) void star_diag_emit_kernel(const int* __restrict__ R, int w, int h, int Wd, int C,
                                                             const unsigned* __restrict__ base,
                                                             unsigned* __restrict__ PN) {
    const int j = blockIdx.x * 256 + threadIdx.x, c = blockIdx.y, z = blockIdx.z;
    if (j >= Wd) return;
    unsigned acc = base[((size_t)z * C + c) * Wd + j];
    const int y0 = c * kDiagRows, y1 = min(y0 + kDiagRows, h + 1);
    unsigned* out = PN + (size_t)z * (h + 1) * Wd + j;
    for (int y = y0; y < y1; y++) {
        out[(size_t)y * Wd] = acc;
        if (y < h) acc += diag_re(R, w, y, z == 0 ? (j - 1) - y : (j - h) + y);
    }
}

__global__ __launch_bounds__(256) void star_diag_final_kernel(const unsigned* __restrict__ PN, int w, int h, int Wd,
                                                              int* __restrict__ T, int* __restrict__ F) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63), y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x > w || y > h) return;
    const unsigned* P = PN + (size_t)y * Wd;
    const unsigned* N = PN + ((size_t)(h + 1) + y) * Wd;
    const unsigned n = N[x - y + h];
    T[(size_t)y * (w + 1) + x] = (int)(P[x + y] - n);
    F[(size_t)y * (w + 1) + x] = (int)(P[x + y + 1] - n);
}

__global__ __launch_bounds__(256) void star_resp_kernel(const int* __restrict__ S, const int* __restrict__ T,
                                                        const int* __restrict__ F, int w, int h, StarPat P,
                                                        float* __restrict__ resp, short* __restrict__ sizes) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63), y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= w || y >= h) return;
    float best = 0.f;
    int bestSize = 0;
    const int B = P.border;
    if (y >= B && y < h - B && x >= B && x < w - B) {
        const int o = y * (w + 1) + x;
        const bool simd = x - B < P.nsimd;
        int vals[17];
#pragma unroll
        for (int i = 0; i < 17; i++) {
            if (i > P.maxIdx) break;
            const int* p = P.ofs + 8 * i;
            vals[i] = S[o + p[0]] - S[o + p[1]] - S[o + p[2]] + S[o + p[3]] + T[o + p[4]] - F[o + p[5]] -
                      F[o + p[6]] + T[o + p[7]];
        }
#pragma unroll
        for (int i = 0; i < 12; i++) {
            if (i >= P.np) break;
            const int in = vals[kStarPairs[i][1]], ov = vals[kStarPairs[i][0]];
            const float outer = simd ? __fsub_rn((float)ov, (float)in) : (float)(ov - in);
            const float r = __fsub_rn(__fmul_rn((float)in, P.inv[2 * i + 1]), __fmul_rn(outer, P.inv[2 * i]));
            if (fabsf(r) > fabsf(best)) {
                best = r;
                bestSize = P.sizes1[kStarPairs[i][0]];
            }
        }
    }
    resp[(size_t)y * w + x] = best;
    sizes[(size_t)y * w + x] = (short)bestSize;
}

// StarDetectorSuppressLines: true = reject
__device__ bool star_lines(const float* __restrict__ R, const short* __restrict__ Z, int w, int x0, int y0, int sz,
                           int lineProj, int lineBin) {
    const int d = sz / 4, rad = d * 4;
    float Lxx = 0.f, Lyy = 0.f, Lxy = 0.f;
    for (int y = y0 - rad; y <= y0 + rad; y += d)
        for (int x = x0 - rad; x <= x0 + rad; x += d) {
            const float Lx = __fsub_rn(R[(size_t)y * w + x + 1], R[(size_t)y * w + x - 1]);
            const float Ly = __fsub_rn(R[(size_t)(y + 1) * w + x], R[(size_t)(y - 1) * w + x]);
            Lxx = __fadd_rn(Lxx, __fmul_rn(Lx, Lx));
            Lyy = __fadd_rn(Lyy, __fmul_rn(Ly, Ly));
            Lxy = __fadd_rn(Lxy, __fmul_rn(Lx, Ly));
        }
    const float tr = __fadd_rn(Lxx, Lyy);
    if (__fmul_rn(tr, tr) >= __fmul_rn((float)lineProj, __fsub_rn(__fmul_rn(Lxx, Lyy), __fmul_rn(Lxy, Lxy))))
        return true;
    int Bxx = 0, Byy = 0, Bxy = 0;
    for (int y = y0 - rad; y <= y0 + rad; y += d)
        for (int x = x0 - rad; x <= x0 + rad; x += d) {
            const int bx = (Z[(size_t)y * w + x + 1] == sz) - (Z[(size_t)y * w + x - 1] == sz);
            const int by = (Z[(size_t)(y + 1) * w + x] == sz) - (Z[(size_t)(y - 1) * w + x] == sz);
            Bxx += bx * bx;
            Byy += by * by;
            Bxy += bx * by;
        }
    return (Bxx + Byy) * (Bxx + Byy) >= lineBin * (Bxx * Byy - Bxy * Bxy);
}

// a thread per (tile, extremum): slot 2t the tile's maximum, 2t + 1 its minimum
__global__ __launch_bounds__(64) void star_nms_kernel(const float* __restrict__ R, const short* __restrict__ Z, int w,
                                                      int h, StarNms N, fm3d_keypoint* __restrict__ kp,
                                                      int* __restrict__ flag) {
    const int slot = blockIdx.x * 64 + threadIdx.x, t = slot >> 1, pass = slot & 1;
    if (t >= N.nx * N.ny) return;
    const int B = N.border, delta = N.delta;
    const int y = B + (t / N.nx) * (delta + 1), x = B + (t % N.nx) * (delta + 1);
    float maxR = (float)N.respThr, minR = (float)-N.respThr;
    int mx = -1, my = -1, nx = -1, ny = -1;
    const int ey = min(y + delta, h - B - 1), ex = min(x + delta, w - B - 1);
    for (int y1 = y; y1 <= ey; y1++)
        for (int x1 = x; x1 <= ex; x1++) {
            const float v = R[(size_t)y1 * w + x1];
            if (maxR < v) {
                maxR = v;
                mx = x1;
                my = y1;
            } else if (minR > v) {
                minR = v;
                nx = x1;
                ny = y1;
            }
        }
    const int px = pass ? nx : mx, py = pass ? ny : my;
    bool ok = px >= 0;
    for (int y1 = py - delta; ok && y1 <= py + delta; y1++)
        for (int x1 = px - delta; x1 <= px + delta; x1++) {
            const float v = R[(size_t)y1 * w + x1];
            if ((pass ? v <= minR : v >= maxR) && (y1 != py || x1 != px)) {
                ok = false;
                break;
            }
        }
    if (ok) {
        const int sz = Z[(size_t)py * w + px];
        ok = sz >= 4 && !star_lines(R, Z, w, px, py, sz, N.lineProj, N.lineBin);
        if (ok) {
            fm3d_keypoint k;
            k.x = (float)px;
            k.y = (float)py;
            k.size = (float)sz;
            k.angle = -1.f;
            k.response = maxR;  // OpenCV 2.4.9 gives the minimum's keypoint the tile's maxResponse too
            k.octave = 0;
            k.class_id = -1;
            kp[slot] = k;
        }
    }
    flag[slot] = ok ? 1 : 0;
}

__global__ __launch_bounds__(256) void star_scatter_kernel(const fm3d_keypoint* __restrict__ kp, const int* __restrict__ flag,
                                                           const int* __restrict__ pos, int n,
                                                           fm3d_keypoint* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n && flag[i]) out[pos[i]] = kp[i];
}

}  // namespace

// the rows per staged block: as many as fit the LDS beside the two 3-row rings, at most 32
static int star_tilted_block(int w) {
    const long ring = 6L * (w + 1) * sizeof(int), room = 160L * 1024 - ring;
    return (int)std::min<long>(32, room / w - 1);
}

size_t star_tilted_lds_bytes(int w) {
    const int bk = star_tilted_block(w);
    return (size_t)6 * (w + 1) * sizeof(int) + (size_t)(bk + 1) * w;
}
int star_tilted_max_width() { return 6000; }  // staged blocks of >= 2 rows

void launch_star_tilted(const uint8_t* img, int w, int h, int* T, int* F, hipStream_t s) {
    if (w <= 0 || h <= 0) return;
    const int bk = star_tilted_block(w);
    const size_t lds = star_tilted_lds_bytes(w);
    if (lds > 64 * 1024)
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&star_tilted_kernel),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    star_tilted_kernel<<<1, kTiltThreads, lds, s>>>(img, w, h, bk, T, F);
}

size_t star_diag_bytes(int w, int h) {
    const size_t Wd = (size_t)w + h + 2, C = (size_t)(h + 1 + kDiagRows - 1) / kDiagRows;
    return ((size_t)(h + 1) * (w + 1) + 2 * C * Wd + 2 * (size_t)(h + 1) * Wd) * 4 + 256;
}

void launch_star_tilted_diag(const uint8_t* img, int w, int h, void* work, int* T, int* F, hipStream_t s) {
    if (w <= 0 || h <= 0) return;
    const int Wd = w + h + 2, C = (h + 1 + kDiagRows - 1) / kDiagRows;
    int* R = static_cast<int*>(work);
    unsigned* part = reinterpret_cast<unsigned*>(R + (size_t)(h + 1) * (w + 1));
    unsigned* PN = part + 2 * (size_t)C * Wd;
    launch_integral_rows(img, w, h, R, s);
    const unsigned gx = (unsigned)((Wd + 255) / 256);
    star_diag_part_kernel<<<dim3(gx, C, 2), 256, 0, s>>>(R, w, h, Wd, C, part);
    star_diag_scan_kernel<<<dim3(gx, 2), 256, 0, s>>>(Wd, C, part);
    star_diag_emit_kernel<<<dim3(gx, C, 2), 256, 0, s>>>(R, w, h, Wd, C, part, PN);
    star_diag_final_kernel<<<dim3((w + 1 + 63) / 64, (h + 1 + 3) / 4), 256, 0, s>>>(PN, w, h, Wd, T, F);
}

void launch_star_resp(const int* S, const int* T, const int* F, int w, int h, const StarPat& P, float* resp,
                      short* sizes, hipStream_t s) {
    if (w <= 0 || h <= 0) return;
    star_resp_kernel<<<dim3((w + 63) / 64, (h + 3) / 4), 256, 0, s>>>(S, T, F, w, h, P, resp, sizes);
}

void launch_star_nms(const float* resp, const short* sizes, int w, int h, const StarNms& N, fm3d_keypoint* kp, int* flag,
                     hipStream_t s) {
    const int n = 2 * N.nx * N.ny;
    if (n <= 0) return;
    star_nms_kernel<<<(n + 63) / 64, 64, 0, s>>>(resp, sizes, w, h, N, kp, flag);
}

void launch_star_scatter(const fm3d_keypoint* kp, const int* flag, const int* pos, int n, fm3d_keypoint* out,
                         hipStream_t s) {
    if (n <= 0) return;
    star_scatter_kernel<<<(n + 255) / 256, 256, 0, s>>>(kp, flag, pos, n, out);
}

}  // namespace fm3d
