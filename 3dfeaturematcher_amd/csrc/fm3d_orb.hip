// fm3d_orb.hip -- ORB feature detection + description on gfx950 (the detectors
// beside the settings' SURF).
//
// Reference: FeatureOptions DetectorType / ExtractorType ORB (descriptorsmatcher.cpp:273-279,
// 336-341): cv::ORB(NumFeatures, ScaleFactor, NumLevels) of OpenCV 2.4.9, restated operation for
// operation in oracle/orc_orb.c (the GPU equals that oracle bit for bit).  Pixel work runs here; the
// two KeyPointsFilter::retainBest selections run on the host with libstdc++'s own std::nth_element /
// std::partition (fm3d_host.cpp), whose exact reordering decides which tied keypoints survive.
//   orb_resize_kernel   a pyramid level from the previous one (resize INTER_LINEAR, 8U): a thread per
//                       destination pixel, the host's fixed-point tables, the horizontal taps in int,
//                       the vertical pass as SSE2's VResizeLinearVec_32s8u on its columns and as the
//                       scalar FixedPtCast on the rest;
//   orb_fast_kernel     FAST-9 over every level at once (a thread per pixel): the 9-of-16 arc test and
//                       cornerScore<16>, into a corner|score map;
//   orb_nms_kernel      3x3 non-maximum suppression + the edge border, flags for the ordered
//                       compaction (level-major raster order = FAST's output order);
//   orb_harris_kernel   HarrisResponses (7x7, k 0.04): a thread per keypoint, int sums, float score;
//   orb_angle_kernel    IC_Angle: a wave per keypoint, lane = column of the circular patch, integer
//                       moments (exact in any order), fastAtan2;
//   orb_blur_rows/cols  GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101): int rows with the x256 kernel,
//                       the columns as SSE2's SymmColumnVec_32s8u (float) on the first floor(w/4)*4
//                       columns and fixed point on the rest;
//   orb_desc_kernel     computeOrbDescriptor (WTA_K 2): a thread per descriptor byte, 8 comparisons of
//                       the rotated pattern points.
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include "fm3d_device.h"
#include "fm3d_kernels.h"

namespace fm3d {

namespace {

__device__ __forceinline__ int cv_roundf(float v) { return (int)rintf(v); }
__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// ---------------------------------------------------------------- pyramid
__global__ __launch_bounds__(256) void orb_resize_kernel(const uint8_t* __restrict__ src, int sw, int sh,
                                                         uint8_t* __restrict__ dst, int dw, int dh,
                                                         const int* __restrict__ xofs, const short* __restrict__ alpha,
                                                         const int* __restrict__ yofs, const short* __restrict__ beta,
                                                         int xmax, int xs) {
    const int dx = blockIdx.x * 256 + threadIdx.x, dy = blockIdx.y;
    if (dx >= dw) return;
    const uint8_t* S0 = src + (size_t)clampi(yofs[dy], 0, sh - 1) * sw;
    const uint8_t* S1 = src + (size_t)clampi(yofs[dy] + 1, 0, sh - 1) * sw;
    const int sx = xofs[dx];
    int D0, D1;
    if (dx < xmax) {
        const int a0 = alpha[2 * dx], a1 = alpha[2 * dx + 1];
        D0 = S0[sx] * a0 + S0[sx + 1] * a1;
        D1 = S1[sx] * a0 + S1[sx + 1] * a1;
    } else {
        D0 = S0[sx] * 2048;
        D1 = S1[sx] * 2048;
    }
    const int b0 = beta[2 * dy], b1 = beta[2 * dy + 1];
    int v;
    if (dx < xs) {  // SSE2: (D >> 4) as int16, _mm_mulhi_epi16 by beta, (+2) >> 2
        v = (((D0 >> 4) * b0) >> 16) + (((D1 >> 4) * b1) >> 16);
        v = (v + 2) >> 2;
    } else {
        v = (b0 * D0 + b1 * D1 + (1 << 21)) >> 22;
    }
    dst[(size_t)dy * dw + dx] = (uint8_t)clampi(v, 0, 255);
}

// ---------------------------------------------------------------- FAST
__constant__ int kCircle[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},   {3, 0},  {3, -1}, {2, -2}, {1, -3},
                                   {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

__device__ __forceinline__ int level_of(const OrbLevel* L, int nL, long long t) {
    int l = 0;
    while (l + 1 < nL && t >= L[l + 1].first) l++;
    return l;
}

// map[pixel] = 0x100 | cornerScore for a corner, 0 elsewhere (the scanned area is 3 <= x < w-3,
// 3 <= y < h-3, as FAST_t's loops)
__global__ __launch_bounds__(256) void orb_fast_kernel(const uint8_t* __restrict__ pyr, const OrbLevel* __restrict__ L,
                                                       int nL, long long total, int thr, uint16_t* __restrict__ map) {
    const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
    if (t >= total) return;
    const int l = level_of(L, nL, t);
    const OrbLevel lv = L[l];
    const int p = (int)(t - lv.first), y = p / lv.w, x = p - y * lv.w;
    uint16_t out = 0;
    if (x >= 3 && x < lv.w - 3 && y >= 3 && y < lv.h - 3) {
        const uint8_t* c = pyr + lv.first + (size_t)y * lv.w + x;
        const int v = c[0];
        int d[25], cd = 0, cb = 0;
        bool dark = false, bright = false;
#pragma unroll
        for (int k = 0; k < 25; k++) {
            const int q = c[kCircle[k & 15][0] + kCircle[k & 15][1] * lv.w];
            d[k] = v - q;
            if (q < v - thr) {
                if (++cd > 8) dark = true;
            } else {
                cd = 0;
            }
            if (q > v + thr) {
                if (++cb > 8) bright = true;
            } else {
                cb = 0;
            }
        }
        if (dark || bright) {
            int a0 = -1000, b0 = 1000;
#pragma unroll
            for (int k = 0; k < 16; k++) {
                int mn = d[k], mx = d[k];
#pragma unroll
                for (int j = 1; j <= 8; j++) {
                    mn = min(mn, d[k + j]);
                    mx = max(mx, d[k + j]);
                }
                a0 = max(a0, mn);
                b0 = min(b0, mx);
            }
            out = (uint16_t)(0x100 | ((max(a0, -b0) - 1) & 0xff));
        }
    }
    map[t] = out;
}

// flag = a corner whose score beats its 8 neighbours' (0 for non-corners), inside the edge border
// (runByImageBorder on the level: Rect(b, b, w - 2b, h - 2b))
__global__ __launch_bounds__(256) void orb_nms_kernel(const uint16_t* __restrict__ map, const OrbLevel* __restrict__ L,
                                                      int nL, long long total, int border, int nonmax,
                                                      int* __restrict__ flag) {
    const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
    if (t >= total) return;
    const int l = level_of(L, nL, t);
    const OrbLevel lv = L[l];
    const int p = (int)(t - lv.first), y = p / lv.w, x = p - y * lv.w;
    const uint16_t m = map[t];
    int f = 0;
    if ((m & 0x100) && lv.w > 2 * border && lv.h > 2 * border && x >= border && x < lv.w - border && y >= border &&
        y < lv.h - border) {
        const int s = m & 0xff, w = lv.w;
        const uint16_t* c = map + t;
        f = !nonmax || (s > (c[-1] & 0xff) && s > (c[1] & 0xff) && s > (c[-w - 1] & 0xff) && s > (c[-w] & 0xff) &&
            s > (c[-w + 1] & 0xff) && s > (c[w - 1] & 0xff) && s > (c[w] & 0xff) && s > (c[w + 1] & 0xff));
    }
    flag[t] = f;
}

__global__ __launch_bounds__(256) void orb_fast_scatter_kernel(const uint16_t* __restrict__ map,
                                                               const OrbLevel* __restrict__ L, int nL, long long total,
                                                               const int* __restrict__ flag, const int* __restrict__ pos,
                                                               fm3d_keypoint* __restrict__ out) {
    const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
    if (t >= total || !flag[t]) return;
    const int l = level_of(L, nL, t);
    const OrbLevel lv = L[l];
    const int p = (int)(t - lv.first), y = p / lv.w, x = p - y * lv.w;
    fm3d_keypoint k;
    k.x = (float)x;
    k.y = (float)y;
    k.size = 7.f;
    k.angle = -1.f;
    k.response = (float)(map[t] & 0xff);
    k.octave = l;
    k.class_id = -1;
    out[pos[t]] = k;
}

// ---------------------------------------------------------------- Harris, IC_Angle
__global__ __launch_bounds__(256) void orb_harris_kernel(const uint8_t* __restrict__ pyr, const OrbLevel* __restrict__ L,
                                                         fm3d_keypoint* __restrict__ kp, int n) {
    const int q = blockIdx.x * 256 + threadIdx.x;
    if (q >= n) return;
    const fm3d_keypoint k = kp[q];
    const OrbLevel lv = L[k.octave];
    const int w = lv.w;
    const int x0 = cv_roundf(k.x - 3), y0 = cv_roundf(k.y - 3);
    const uint8_t* img = pyr + lv.first;
    int a = 0, b = 0, c = 0;
    for (int i = 0; i < 7; i++)
        for (int j = 0; j < 7; j++) {
            const uint8_t* p = img + (size_t)(y0 + i) * w + x0 + j;
            const int Ix = (p[1] - p[-1]) * 2 + (p[-w + 1] - p[-w - 1]) + (p[w + 1] - p[w - 1]);
            const int Iy = (p[w] - p[-w]) * 2 + (p[w - 1] - p[-w - 1]) + (p[w + 1] - p[-w + 1]);
            a += Ix * Ix;
            b += Iy * Iy;
            c += Ix * Iy;
        }
    float scale = (1 << 2) * 7 * 255.0f;
    scale = 1.0f / scale;
    const float sq = scale * scale * scale * scale;
    kp[q].response = ((float)a * b - (float)c * c - 0.04f * ((float)a + b) * ((float)a + b)) * sq;
}

// a wave per keypoint: lane l < 2*half+1 takes column u = l - half of the circular patch
__global__ __launch_bounds__(256) void orb_angle_kernel(const uint8_t* __restrict__ pyr, const OrbLevel* __restrict__ L,
                                                        fm3d_keypoint* __restrict__ kp, int n, int half, OrbUmax um) {
    const int lane = threadIdx.x & 63;
    const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= n) return;
    const fm3d_keypoint k = kp[q];
    const OrbLevel lv = L[k.octave];
    const int w = lv.w;
    const uint8_t* c = pyr + lv.first + (size_t)cv_roundf(k.y) * w + cv_roundf(k.x);
    int m10 = 0, m01 = 0;
    const int u = lane - half;
    if (lane <= 2 * half) {
        m10 = u * c[u];
        for (int v = 1; v <= half; v++) {
            const int d = um.u[v];
            if (u >= -d && u <= d) {
                const int vp = c[u + v * w], vm = c[u - v * w];
                m01 += v * (vp - vm);
                m10 += u * (vp + vm);
            }
        }
    }
    for (int off = 32; off >= 1; off >>= 1) {
        m10 += __shfl_xor(m10, off);
        m01 += __shfl_xor(m01, off);
    }
    if (lane == 0) kp[q].angle = fast_atan2f((float)m01, (float)m10);
}

// ---------------------------------------------------------------- blur + descriptors
__device__ __forceinline__ int reflect101(int p, int n) {
    if (n == 1) return 0;
    while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
    return p;
}

__global__ __launch_bounds__(256) void orb_blur_rows_kernel(const uint8_t* __restrict__ pyr,
                                                            const OrbLevel* __restrict__ L, int nL, long long total,
                                                            OrbBlurK bk, int* __restrict__ R) {
    const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
    if (t >= total) return;
    const int l = level_of(L, nL, t);
    const OrbLevel lv = L[l];
    const int p = (int)(t - lv.first), y = p / lv.w, x = p - y * lv.w;
    const uint8_t* row = pyr + lv.first + (size_t)y * lv.w;
    int s = 0;
#pragma unroll
    for (int k = 0; k < 7; k++) s += bk.ik[k] * row[reflect101(x + k - 3, lv.w)];
    R[t] = s;
}

__global__ __launch_bounds__(256) void orb_blur_cols_kernel(const int* __restrict__ R, const OrbLevel* __restrict__ L,
                                                            int nL, long long total, OrbBlurK bk,
                                                            uint8_t* __restrict__ out) {
    const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
    if (t >= total) return;
    const int l = level_of(L, nL, t);
    const OrbLevel lv = L[l];
    const int p = (int)(t - lv.first), y = p / lv.w, x = p - y * lv.w;
    const int* col = R + lv.first + x;
    const int w = lv.w, h = lv.h;
    int v;
    if (x < (w / 4) * 4) {  // SymmColumnVec_32s8u (SSE2): float
        float s = (float)col[(size_t)y * w] * bk.fk[0] + 0.f;
#pragma unroll
        for (int k = 1; k <= 3; k++)
            s = s + (float)(col[(size_t)reflect101(y + k, h) * w] + col[(size_t)reflect101(y - k, h) * w]) * bk.fk[k];
        v = (int)rintf(s);
    } else {  // FixedPtCastEx<int, uchar>(16)
        int s = bk.ik[3] * col[(size_t)y * w];
#pragma unroll
        for (int k = 1; k <= 3; k++)
            s += bk.ik[3 + k] * (col[(size_t)reflect101(y + k, h) * w] + col[(size_t)reflect101(y - k, h) * w]);
        v = (s + (1 << 15)) >> 16;
    }
    out[lv.first + (size_t)y * w + x] = (uint8_t)clampi(v, 0, 255);
}

// a thread per descriptor byte: bit j = I(rot p[16i+2j]) < I(rot p[16i+2j+1]) on the blurred level
__global__ __launch_bounds__(256) void orb_desc_kernel(const uint8_t* __restrict__ blur, const OrbLevel* __restrict__ L,
                                                       const fm3d_keypoint* __restrict__ kp, int n,
                                                       const int* __restrict__ pattern, uint8_t* __restrict__ desc) {
    const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
    if (t >= (long long)n * 32) return;
    const int q = (int)(t >> 5), i = (int)(t & 31);
    const fm3d_keypoint k = kp[q];
    const OrbLevel lv = L[k.octave];
    float angle = k.angle;
    angle *= (float)(M_PI / 180.f);
    const float a = (float)fm3d_cos((double)angle), b = (float)fm3d_sin((double)angle);
    const int w = lv.w;
    const uint8_t* c = blur + lv.first + (size_t)cv_roundf(k.y) * w + cv_roundf(k.x);
    int val = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const int* p0 = pattern + (i * 16 + 2 * j) * 2;
        const float x0 = p0[0] * a - p0[1] * b, y0 = p0[0] * b + p0[1] * a;
        const float x1 = p0[2] * a - p0[3] * b, y1 = p0[2] * b + p0[3] * a;
        const int t0 = c[cv_roundf(y0) * w + cv_roundf(x0)], t1 = c[cv_roundf(y1) * w + cv_roundf(x1)];
        val |= (t0 < t1) << j;
    }
    desc[t] = (uint8_t)val;
}

inline unsigned blocks(long long n) { return (unsigned)((n + 255) / 256); }

}  // namespace

void launch_orb_resize(const uint8_t* src, int sw, int sh, uint8_t* dst, int dw, int dh, const int* xofs,
                       const short* alpha, const int* yofs, const short* beta, int xmax, int xs, hipStream_t s) {
    if (dw <= 0 || dh <= 0) return;
    orb_resize_kernel<<<dim3((dw + 255) / 256, dh), 256, 0, s>>>(src, sw, sh, dst, dw, dh, xofs, alpha, yofs, beta,
                                                                  xmax, xs);
}

void launch_orb_fast(const uint8_t* pyr, const OrbLevel* L, int nL, long long total, int thr, int border, int nonmax,
                     uint16_t* map, int* flag, hipStream_t s) {
    if (total <= 0) return;
    orb_fast_kernel<<<blocks(total), 256, 0, s>>>(pyr, L, nL, total, thr, map);
    orb_nms_kernel<<<blocks(total), 256, 0, s>>>(map, L, nL, total, border, nonmax, flag);
}

void launch_orb_fast_scatter(const uint16_t* map, const OrbLevel* L, int nL, long long total, const int* flag,
                             const int* pos, fm3d_keypoint* out, hipStream_t s) {
    if (total <= 0) return;
    orb_fast_scatter_kernel<<<blocks(total), 256, 0, s>>>(map, L, nL, total, flag, pos, out);
}

void launch_orb_harris(const uint8_t* pyr, const OrbLevel* L, fm3d_keypoint* kp, int n, hipStream_t s) {
    if (n <= 0) return;
    orb_harris_kernel<<<blocks(n), 256, 0, s>>>(pyr, L, kp, n);
}

void launch_orb_angle(const uint8_t* pyr, const OrbLevel* L, fm3d_keypoint* kp, int n, int half, const OrbUmax& um,
                      hipStream_t s) {
    if (n <= 0) return;
    orb_angle_kernel<<<(n + 3) / 4, 256, 0, s>>>(pyr, L, kp, n, half, um);
}

void launch_orb_blur(const uint8_t* pyr, const OrbLevel* L, int nL, long long total, const OrbBlurK& bk, int* R,
                     uint8_t* out, hipStream_t s) {
    if (total <= 0) return;
    orb_blur_rows_kernel<<<blocks(total), 256, 0, s>>>(pyr, L, nL, total, bk, R);
    orb_blur_cols_kernel<<<blocks(total), 256, 0, s>>>(R, L, nL, total, bk, out);
}

void launch_orb_desc(const uint8_t* blur, const OrbLevel* L, const fm3d_keypoint* kp, int n, const int* pattern,
                     uint8_t* desc, hipStream_t s) {
    if (n <= 0) return;
    orb_desc_kernel<<<blocks((long long)n * 32), 256, 0, s>>>(blur, L, kp, n, pattern, desc);
}

}  // namespace fm3d
