// fm3d_star.hip -- the STAR (CenSurE) detector on gfx950.
//
// Reference: DescriptorsMatcher's DetectorType STAR (descriptorsmatcher.cpp:204-213,
// cv::StarFeatureDetector(MaxSize, Response, LineThreshold, LineBinarized, Suppression)) and the
// StarAdjuster of its ADAPTIVE mode (:185-200).  The algorithm is OpenCV 2.4.9's
// features2d/src/stardetector.cpp, restated in oracle/orc_star.c; the GPU equals that oracle bit for bit:
//   integral (fm3d_surf.hip)  the upright sum S
//   star_tilted_kernel        the tilted sum T and the flat-tilted sum F: one workgroup walks the rows
//                             (each row needs the two above it at x-1, x, x+1), a thread per column,
//                             the last three rows of each in an LDS ring, separate waves storing the
//                             finished rows; OpenCV's row recursions with its own formulas at columns
//                             0, 1 and w.  Integer adds: exact.
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

#include "fm3d_kernels.h"

namespace fm3d {

namespace {

constexpr int kTiltThreads = 1024;
// (outer, inner) pattern pairs of StarDetectorComputeResponses (each inner pattern half its outer one)
__device__ constexpr int kStarPairs[12][2] = {{1, 0}, {3, 1}, {4, 2}, {5, 3}, {7, 4}, {8, 5},
                                              {9, 6}, {11, 8}, {13, 10}, {14, 11}, {15, 12}, {16, 14}};

// T and F, (h+1) x (w+1) int32.  LDS: the last three rows of each (row y written, y-1 and y-2 read).
// Waves 0-11 compute, a thread per column (the image bytes of the next row loaded one row ahead);
// waves 12-15 copy the finished row y-1 from LDS to global memory while row y is computed, so the
// computing waves never issue a store and their per-row barrier waits on LDS only (s_waitcnt is per
// wave: a store would make the next image load's wait cover it).
constexpr int kTiltCompute = 768, kTiltMaxCols = 6;  // columns per computing thread: w + 1 <= 4608

__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__global__ __launch_bounds__(kTiltThreads) void star_tilted_kernel(const uint8_t* __restrict__ I, int w, int h,
                                                                   int* __restrict__ T, int* __restrict__ F) {
    extern __shared__ int ring[];  // [3][w+1] of T, then [3][w+1] of F
    const int st = w + 1, tid = threadIdx.x;
    int* RT = ring;
    int* RF = ring + 3 * st;
    const bool compute = tid < kTiltCompute;
    // image bytes per column slot: I(r, x-1) and I(r, x) of rows y-1 (c), y-2 (p) and y (n, prefetch)
    int cm1[kTiltMaxCols], c0[kTiltMaxCols], pm1[kTiltMaxCols], p0[kTiltMaxCols];
    auto ld = [&](int r, int x, int& m1, int& z) {
        const uint8_t* row = I + (size_t)r * w;
        m1 = x >= 1 && x <= w ? row[x - 1] : 0;
        z = x < w ? row[x] : 0;
    };
    if (compute) {
#pragma unroll
        for (int j = 0; j < kTiltMaxCols; j++) {
            const int x = tid + j * kTiltCompute;
            if (x > w) break;
            ld(0, x, pm1[j], p0[j]);
            // row 0: zeros; row 1: the top image row alone
            const int t = x == 0 ? 0 : pm1[j];
            const int f = x == 0 ? p0[j] : x == w ? pm1[j] : p0[j] + pm1[j];
            T[x] = F[x] = 0;
            RT[x] = RF[x] = 0;
            T[st + x] = t;
            F[st + x] = f;
            RT[st + x] = t;
            RF[st + x] = f;
            if (h >= 2) ld(1, x, cm1[j], c0[j]);
        }
    }
    __syncthreads();
    for (int y = 2; y <= h; y++) {
        const int cur = y % 3, q1 = (y - 1) % 3, q2 = (y - 2) % 3;
        if (compute) {
            const int *t1 = RT + q1 * st, *t2 = RT + q2 * st, *f1 = RF + q1 * st, *f2 = RF + q2 * st;
            int *tc = RT + cur * st, *fc = RF + cur * st;
#pragma unroll
            for (int j = 0; j < kTiltMaxCols; j++) {
                const int x = tid + j * kTiltCompute;
                if (x > w) break;
                int nm1 = 0, n0 = 0;
                if (y < h) ld(y, x, nm1, n0);  // the next row's bytes, in flight over this row
                // a = image row y-1 (cm1 = a[x-1], c0 = a[x]), b = row y-2 (pm1 = b[x-1], p0 = b[x])
                int t, f;
                if (x >= 2 && x < w) {
                    t = t1[x - 1] + t1[x + 1] - t2[x] + pm1[j] + cm1[j];
                    f = f1[x - 1] + f1[x + 1] - f2[x] + c0[j] + cm1[j];
                } else if (x == w) {
                    t = f = t1[w - 1] + pm1[j] + cm1[j];
                } else if (x == 1) {
                    t = t1[2] + pm1[j] + cm1[j];
                    f = f1[2] + pm1[j] + c0[j] + cm1[j];
                } else {  // x == 0: T[0] = T(y-1, 1), F[0] = T[1] of this row = T(y-1, 2) + b[0] + a[0]
                    t = t1[1];
                    f = t1[2] + p0[j] + c0[j];
                }
                tc[x] = t;
                fc[x] = f;
                pm1[j] = cm1[j];
                p0[j] = c0[j];
                cm1[j] = nm1;
                c0[j] = n0;
            }
        } else {  // copy the finished row y-1 (read-only during this row) to global memory
            const int r = (y - 1) % 3;
            for (int x = tid - kTiltCompute; x <= w; x += kTiltThreads - kTiltCompute) {
                T[(size_t)(y - 1) * st + x] = RT[r * st + x];
                F[(size_t)(y - 1) * st + x] = RF[r * st + x];
            }
        }
        lds_barrier();
    }
    if (!compute && h >= 2) {  // the last row
        const int r = h % 3;
        for (int x = tid - kTiltCompute; x <= w; x += kTiltThreads - kTiltCompute) {
            T[(size_t)h * st + x] = RT[r * st + x];
            F[(size_t)h * st + x] = RF[r * st + x];
        }
    }
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

size_t star_tilted_lds_bytes(int w) { return (size_t)6 * (w + 1) * sizeof(int); }
int star_tilted_max_width() { return kTiltCompute * kTiltMaxCols - 1; }

void launch_star_tilted(const uint8_t* img, int w, int h, int* T, int* F, hipStream_t s) {
    if (w <= 0 || h <= 0) return;
    star_tilted_kernel<<<1, kTiltThreads, star_tilted_lds_bytes(w), s>>>(img, w, h, T, F);
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
