// fm3d_surf.hip -- SURF feature detection + description on gfx950.
//
// Reference: the detector / extractor DescriptorsMatcher builds from build/settings.yml:37-49
// (descriptorsmatcher.cpp:176-359: SURF, HessianThreshold 400, NumOctaves 4, NumOctaveLayers 2,
// Extended 1, Upright 1), called by compareWithNNDR (:110-115) and extractDescriptorsFromPatches
// (:133-174).  The algorithm is OpenCV 2.4's nonfree SURF (restated operation for operation in
// oracle/orc_surf.c; the GPU equals that oracle bit for bit):
//   integral_rows_kernel / integral_cols_kernel  integral(img, sum, CV_32S): exact int32 prefix sums
//                        (a wave per row with shuffle scans, then banded column scans);
//   hessian_kernel       calcLayerDetAndTrace for every layer at once: one thread per layer sample,
//                        10 box sums of the resized Haar patterns (40 integral reads, L2-resident),
//                        float det / trace;
//   maxima_kernel        findMaximaInLayer: one thread per middle-layer sample, threshold, 3x3x3
//                        non-maximum suppression, interpolateKeypoint (Cramer's rule in float),
//                        appended through an atomic counter; then a device merge sort by
//                        KeypointGreater (discovery order breaks ties) and the upright pass;
//   orient_kernel        SURFInvoker's dominant orientation (Upright 0): a wave per keypoint, the
//                        113 disc samples' Haar responses compacted in sample order by ballot, the
//                        72 sliding 60-degree windows one lane each (each lane sums its window in
//                        the reference's sample order), the first largest window by a wave argmax;
//   describe_kernel      SURFInvoker: one workgroup per keypoint.  The 21x21 INTER_AREA patch comes
//                        straight from the image (the border-replicated upright window or the
//                        bilinear rotated one is never materialised): OpenCV's row buffers, one per
//                        window row, in LDS,
//                        then the beta-weighted rows per destination row, both in OpenCV's order;
//                        then the 2x2 Haar gradients with the Gaussian weights, the 4x4 subregion
//                        sums (one lane each, OpenCV's sample order) and the unit-length scale.
// Everything is integer or float/double work without reductions across lanes except the
// descriptor's squared magnitude, summed by lane 0 in the reference's order.
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include <hipcub/hipcub.hpp>

#include "fm3d_kernels.h"
#include "fm3d_device.h"

namespace fm3d {

namespace {

// cvRound of a float (round to nearest, ties to even)
__device__ __forceinline__ int cv_roundf(float v) { return (int)rintf(v); }
__device__ __forceinline__ int cv_round(double v) { return (int)rint(v); }

// ---------------------------------------------------------------- integral image
// sum: (h+1) x (w+1) int32, row 0 and column 0 zero.  Pass 1: row prefix sums (a wave per row).
// blockIdx.y: image of a batch (image b at img + b*w*h, its sum at sum + b*(w+1)*(h+1))
__global__ __launch_bounds__(64) void integral_rows_kernel(const uint8_t* __restrict__ img, int w, int h,
                                                            int* __restrict__ sum) {
    const int y = blockIdx.x, lane = threadIdx.x;
    img += (size_t)blockIdx.y * w * h;
    sum += (size_t)blockIdx.y * (w + 1) * (h + 1);
    int* row = sum + (size_t)(y + 1) * (w + 1);
    if (lane == 0) row[0] = 0;
    int carry = 0;
    for (int x0 = 0; x0 < w; x0 += 64) {
        const int x = x0 + lane;
        int v = x < w ? img[(size_t)y * w + x] : 0;
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(v, o);
            if (lane >= o) v += t;
        }
        if (x < w) row[x + 1] = carry + v;
        carry += __shfl(v, 63);
    }
}
// pass 2: column sums down the rows.  A workgroup takes 64 columns and its 16 waves 16 bands of
// rows: each band's column sums first (independent loads), then each band's running sums from the
// bands above it.  Exact: 32-bit wrap-around adds in any order.
constexpr int kIntBands = 16;
__global__ __launch_bounds__(64 * kIntBands) void integral_cols_kernel(int w, int h, int* __restrict__ sum) {
    __shared__ unsigned bandSum[kIntBands][64];
    const int lane = threadIdx.x & 63, band = threadIdx.x >> 6;
    sum += (size_t)blockIdx.y * (w + 1) * (h + 1);
    const int x = blockIdx.x * 64 + lane;
    const int rows = (h + kIntBands - 1) / kIntBands;
    const int y0 = 1 + band * rows, y1 = min(h + 1, y0 + rows);
    const bool ok = x <= w;
    const size_t ld = (size_t)w + 1;
    unsigned t = 0;
    if (ok)
        for (int y = y0; y < y1; y++) t += (unsigned)sum[(size_t)y * ld + x];
    bandSum[band][lane] = t;
    __syncthreads();
    if (!ok) return;
    unsigned acc = 0;
    for (int b = 0; b < band; b++) acc += bandSum[b][lane];
    if (band == 0) sum[x] = 0;
    constexpr int kU = 8;  // loads of a batch issued before its dependent adds
    for (int y = y0; y < y1; y += kU) {
        unsigned v[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) v[u] = y + u < y1 ? (unsigned)sum[(size_t)(y + u) * ld + x] : 0u;
#pragma unroll
        for (int u = 0; u < kU; u++) {
            acc += v[u];
            if (y + u < y1) sum[(size_t)(y + u) * ld + x] = (int)acc;
        }
    }
}

// ---------------------------------------------------------------- Hessian layers
__device__ __forceinline__ float haar_sum(const int* __restrict__ o, const SurfHF* f, int n) {
    double d = 0;
    for (int k = 0; k < n; k++) d += (o[f[k].p0] + o[f[k].p3] - o[f[k].p1] - o[f[k].p2]) * f[k].w;
    return (float)d;
}

__global__ __launch_bounds__(256) void hessian_kernel(const int* __restrict__ sum, int w,
                                                      const SurfLayer* __restrict__ layers, int nL,
                                                      float* __restrict__ det, float* __restrict__ tr) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    int l = 0;
    while (l + 1 < nL && t >= layers[l + 1].first) l++;
    const SurfLayer& ly = layers[l];
    const long long u = t - ly.first;
    if (u >= (long long)ly.si * ly.sj) return;
    const int i = (int)(u / ly.sj), j = (int)(u - (long long)i * ly.sj);
    const int* o = sum + (size_t)i * ly.step * (w + 1) + (size_t)j * ly.step;
    const float dx = haar_sum(o, ly.hf, 3), dy = haar_sum(o, ly.hf + 3, 3), dxy = haar_sum(o, ly.hf + 6, 4);
    const size_t at = ly.off + (size_t)(i + ly.margin) * ly.cols + j + ly.margin;
    det[at] = dx * dy - 0.81f * dxy * dxy;
    tr[at] = dx + dy;
}

// ---------------------------------------------------------------- maxima + interpolation
__device__ bool interpolate_kp(const float N9[3][9], int dxs, int dys, int ds, SurfCand& k) {
    const float b0 = -(N9[1][5] - N9[1][3]) / 2, b1 = -(N9[1][7] - N9[1][1]) / 2, b2 = -(N9[2][4] - N9[0][4]) / 2;
    const float dxx = N9[1][3] - 2 * N9[1][4] + N9[1][5];
    const float dxy = (N9[1][8] - N9[1][6] - N9[1][2] + N9[1][0]) / 4;
    const float dxsv = (N9[2][5] - N9[2][3] - N9[0][5] + N9[0][3]) / 4;
    const float dyy = N9[1][1] - 2 * N9[1][4] + N9[1][7];
    const float dysv = (N9[2][7] - N9[2][1] - N9[0][7] + N9[0][1]) / 4;
    const float dss = N9[0][4] - 2 * N9[1][4] + N9[2][4];
    // Matx33f::solve (Matx_FastSolveOp<float, 3, 1>): Cramer's rule with the float determinant
    const float a00 = dxx, a01 = dxy, a02 = dxsv, a10 = dxy, a11 = dyy, a12 = dysv, a20 = dxsv, a21 = dysv, a22 = dss;
    float d = a00 * (a11 * a22 - a21 * a12) - a01 * (a10 * a22 - a20 * a12) + a02 * (a10 * a21 - a20 * a11);
    float x0 = 0, x1 = 0, x2 = 0;
    if (d != 0) {
        d = 1 / d;
        x0 = d * (b0 * (a11 * a22 - a12 * a21) - a01 * (b1 * a22 - a12 * b2) + a02 * (b1 * a21 - a11 * b2));
        x1 = d * (a00 * (b1 * a22 - a12 * b2) - b0 * (a10 * a22 - a12 * a20) + a02 * (a10 * b2 - b1 * a20));
        x2 = d * (a00 * (a11 * b2 - b1 * a21) - a01 * (a10 * b2 - b1 * a20) + b0 * (a10 * a21 - a11 * a20));
    }
    const bool ok = (x0 != 0 || x1 != 0 || x2 != 0) && fabsf(x0) <= 1 && fabsf(x1) <= 1 && fabsf(x2) <= 1;
    if (ok) {
        k.x += x0 * dxs;
        k.y += x1 * dys;
        k.size = (float)cv_roundf(k.size + x2 * ds);
    }
    return ok;
}

__global__ __launch_bounds__(256) void maxima_kernel(const float* __restrict__ det, const float* __restrict__ tr,
                                                     const SurfLayer* __restrict__ layers,
                                                     const SurfMid* __restrict__ mids, int nM, float thr,
                                                     SurfCand* __restrict__ out, int* __restrict__ count, int cap) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    int m = 0;
    while (m + 1 < nM && t >= mids[m + 1].first) m++;
    const SurfMid& md = mids[m];
    const long long u = t - md.first;
    if (u >= (long long)md.rows * md.cols) return;
    const int i = (int)(u / md.cols), j = (int)(u - (long long)i * md.cols);
    if (i < md.margin || i >= md.rows - md.margin || j < md.margin || j >= md.cols - md.margin) return;
    const SurfLayer& ly = layers[md.layer];
    const float* D1 = det + layers[md.layer - 1].off;
    const float* D2 = det + ly.off;
    const float* D3 = det + layers[md.layer + 1].off;
    const int cols = md.cols;
    const float val0 = D2[(size_t)i * cols + j];
    if (!(val0 > thr)) return;
    float N9[3][9];
    const float* Ds[3] = {D1, D2, D3};
    for (int a = 0; a < 3; a++)
        for (int b = -1; b <= 1; b++)
            for (int c = -1; c <= 1; c++) N9[a][(b + 1) * 3 + c + 1] = Ds[a][(size_t)(i + b) * cols + j + c];
    for (int a = 0; a < 3; a++)
        for (int b = 0; b < 9; b++)
            if (!(a == 1 && b == 4) && !(val0 > N9[a][b])) return;
    const int size = ly.size, step = ly.step;
    const int sum_i = step * (i - (size / 2) / step), sum_j = step * (j - (size / 2) / step);
    const float t2 = tr[ly.off + (size_t)i * cols + j];
    SurfCand k;
    k.y = sum_i + (size - 1) * 0.5f;
    k.x = sum_j + (size - 1) * 0.5f;
    k.size = (float)size;
    k.response = val0;
    k.octave = md.octave;
    k.class_id = (t2 > 0) - (t2 < 0);
    k.seq = ((long long)md.layer << 42) | ((long long)i << 21) | j;
    if (!interpolate_kp(N9, step, step, size - layers[md.layer - 1].size, k)) return;
    const int slot = atomicAdd(count, 1);
    if (slot < cap) out[slot] = k;
}

// KeypointGreater (surf.cpp): response, size, octave descending, then y, x descending; ties in
// discovery order (the sequential (layer, row, column) scan)
struct KpGreater {
    __host__ __device__ bool operator()(const SurfCand& a, const SurfCand& b) const {
        if (a.response != b.response) return a.response > b.response;
        if (a.size != b.size) return a.size > b.size;
        if (a.octave != b.octave) return a.octave > b.octave;
        if (a.y != b.y) return a.y > b.y;
        if (a.x != b.x) return a.x > b.x;
        return a.seq < b.seq;
    }
};

// the detect-time SURFInvoker pass (upright): flag = the gradient wavelet fits the integral image
__global__ void upright_flag_kernel(const SurfCand* __restrict__ c, const int* __restrict__ count, int cap, int w,
                                    int h, int* __restrict__ flag) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    const int n = min(*count, cap);
    if (q >= cap) return;
    if (q >= n) {
        flag[q] = 0;
        return;
    }
    const float s = c[q].size * 1.2f / 9.0f;
    const int gws = 2 * cv_roundf(2 * s);
    flag[q] = (h + 1 < gws || w + 1 < gws) ? 0 : 1;
}
__global__ void keypoint_scatter_kernel(const SurfCand* __restrict__ c, const int* __restrict__ flag,
                                        const int* __restrict__ pos, const float* __restrict__ angle, int cap,
                                        fm3d_keypoint* __restrict__ out, int* __restrict__ src) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= cap || !flag[q]) return;
    fm3d_keypoint k;
    k.x = c[q].x;
    k.y = c[q].y;
    k.size = c[q].size;
    k.angle = angle ? angle[q] : 360.f - 90.f;
    k.response = c[q].response;
    k.octave = c[q].octave;
    k.class_id = c[q].class_id;
    out[pos[q]] = k;
    if (src) src[pos[q]] = q;
}

// SURF::operator() with provided keypoints: the SURFInvoker drop (wavelet larger than the integral
// image), compacted with their input index; angle = the upright 270
__global__ void keep_flag_kernel(const fm3d_keypoint* __restrict__ k, int n, int w, int h, int* __restrict__ flag) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    // DescriptorExtractor::compute runs KeyPointsFilter::runByKeypointSize(FLT_EPSILON) first
    // (runByImageBorder(0) removes nothing); then SURFInvoker's drop of wavelets larger than the image
    const float s = k[q].size * 1.2f / 9.0f;
    const int gws = 2 * cv_roundf(2 * s);
    flag[q] = (!(k[q].size >= 1.19209290e-07f) || h + 1 < gws || w + 1 < gws) ? 0 : 1;
}
__global__ void keep_scatter_kernel(const fm3d_keypoint* __restrict__ k, const int* __restrict__ flag,
                                    const int* __restrict__ pos, const float* __restrict__ angle, int n,
                                    fm3d_keypoint* __restrict__ out, int* __restrict__ src) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n || !flag[q]) return;
    fm3d_keypoint o = k[q];
    o.angle = angle ? angle[q] : 360.f - 90.f;
    out[pos[q]] = o;
    if (src) src[pos[q]] = q;
}


// ---------------------------------------------------------------- orientation (Upright 0)
// resizeHaarPattern of SURFInvoker's 4x4 orientation wavelets (dx_s / dy_s) to size gws
__device__ inline void ori_haar(int gws, int W1, SurfHF* dx, SurfHF* dy) {
    const int DXO[2][5] = {{0, 0, 2, 4, -1}, {2, 0, 4, 4, 1}};
    const int DYO[2][5] = {{0, 0, 4, 2, 1}, {0, 2, 4, 4, -1}};
    const float ratio = (float)gws / 4;
    for (int t = 0; t < 2; t++)
        for (int k = 0; k < 2; k++) {
            const int(*src)[5] = t ? DYO : DXO;
            SurfHF& d = t ? dy[k] : dx[k];
            const int dx1 = cv_roundf(ratio * src[k][0]), dy1 = cv_roundf(ratio * src[k][1]);
            const int dx2 = cv_roundf(ratio * src[k][2]), dy2 = cv_roundf(ratio * src[k][3]);
            d.p0 = dy1 * W1 + dx1;
            d.p1 = dy2 * W1 + dx1;
            d.p2 = dy1 * W1 + dx2;
            d.p3 = dy2 * W1 + dx2;
            d.w = src[k][4] / ((float)(dx2 - dx1) * (dy2 - dy1));
        }
}

constexpr int kOriWaves = 4;
// keypoint q = (x, y, size) at kp + q * kstride (SurfCand and fm3d_keypoint both start with them);
// its integral image at sum + q * sumStride (0: one image).  flag[q] = the keypoint survives
// SURFInvoker (size >= FLT_EPSILON -- DescriptorExtractor::compute's runByKeypointSize --, the
// wavelet fits, at least one orientation sample inside); angle[q] = its dominant orientation.
__global__ __launch_bounds__(64 * kOriWaves) void orient_kernel(const char* __restrict__ kp, size_t kstride, int n,
                                                              const int* __restrict__ sum, size_t sumStride, int w,
                                                              int h, SurfOri ori, int* __restrict__ flag,
                                                              float* __restrict__ angle) {
    __shared__ float SXs[kOriWaves][kOriMax], SYs[kOriWaves][kOriMax];
    __shared__ int SAs[kOriWaves][kOriMax];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int q = blockIdx.x * kOriWaves + wv;
    if (q >= n) return;  // a whole wave; the waves share no barrier
    float* SX = SXs[wv];
    float* SY = SYs[wv];
    int* SA = SAs[wv];
    const float* k = reinterpret_cast<const float*>(kp + (size_t)q * kstride);
    const float kx = k[0], ky = k[1], ksize = k[2];
    const int W1 = w + 1, H1 = h + 1;
    const float s = ksize * 1.2f / 9.0f;
    const int gws = 2 * cv_roundf(2 * s);
    if (!(ksize >= FLT_EPSILON) || H1 < gws || W1 < gws) {
        if (lane == 0) flag[q] = 0;
        return;
    }
    sum += (size_t)q * sumStride;
    SurfHF dxt[2], dyt[2];
    ori_haar(gws, W1, dxt, dyt);
    // the disc samples inside the integral image, compacted in sample order
    int nangle = 0;
    for (int base = 0; base < ori.n; base += 64) {
        const int kk = base + lane;
        bool in = false;
        float X = 0, Y = 0;
        if (kk < ori.n) {
            const int x = cv_roundf(kx + ori.ax[kk] * s - (float)(gws - 1) / 2);
            const int y = cv_roundf(ky + ori.ay[kk] * s - (float)(gws - 1) / 2);
            in = !(y < 0 || y >= H1 - gws || x < 0 || x >= W1 - gws);
            if (in) {
                const int* o = sum + (size_t)y * W1 + x;
                X = haar_sum(o, dxt, 2) * ori.w[kk];
                Y = haar_sum(o, dyt, 2) * ori.w[kk];
            }
        }
        const unsigned long long m = __ballot(in);
        if (in) {
            const int at = nangle + __popcll(m & ((1ull << lane) - 1));
            SX[at] = X;
            SY[at] = Y;
            SA[at] = cv_roundf(fast_atan2f(Y, X));
        }
        nangle += __popcll(m);
    }
    if (nangle == 0) {  // kp.size = -1: removed
        if (lane == 0) flag[q] = 0;
        return;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // windows i = 0, 5, ..., 355: lane l takes 5l and (l < 8) 5(l + 64); sequential sums as the source
    const int i0 = 5 * lane, i1 = 5 * (lane + 64);
    const bool two = lane < 72 - 64;
    float sx0 = 0, sy0 = 0, sx1 = 0, sy1 = 0;
    for (int j = 0; j < nangle; j++) {
        const float X = SX[j], Y = SY[j];
        const int a = SA[j];
        const int d0 = abs(a - i0);
        if (d0 < 30 || d0 > 360 - 30) {
            sx0 += X;
            sy0 += Y;
        }
        const int d1 = abs(a - i1);
        if (two && (d1 < 30 || d1 > 360 - 30)) {
            sx1 += X;
            sy1 += Y;
        }
    }
    // descriptor_mod: the first window of the largest sumx^2 + sumy^2 (strictly above 0)
    float bm = sx0 * sx0 + sy0 * sy0, bx = sx0, by = sy0;
    int bi = i0;
    if (two) {
        const float m1 = sx1 * sx1 + sy1 * sy1;
        if (m1 > bm) {
            bm = m1;
            bx = sx1;
            by = sy1;
            bi = i1;
        }
    }
    for (int off = 32; off >= 1; off >>= 1) {
        const float om = __shfl_xor(bm, off), ox = __shfl_xor(bx, off), oy = __shfl_xor(by, off);
        const int oi = __shfl_xor(bi, off);
        if (om > bm || (om == bm && oi < bi)) {
            bm = om;
            bx = ox;
            by = oy;
            bi = oi;
        }
    }
    if (!(bm > 0)) bx = by = 0;
    if (lane == 0) {
        flag[q] = 1;
        angle[q] = fast_atan2f(-by, bx);
    }
}

// ---------------------------------------------------------------- descriptors
__device__ __forceinline__ uint8_t sat_u8(float v) {
    const int iv = cv_roundf(v);
    return (uint8_t)(iv < 0 ? 0 : (iv > 255 ? 255 : iv));
}

// computeResizeAreaTab (OpenCV 2.4 imgproc/resize.cpp) of destination index d: the partial first
// cell, the whole cells, the partial last cell, in that order
struct AreaTab {
    int s1, cnt, pre, full;  // first whole cell, entries, partial first cell (0/1), whole cells
    float apre, afull, apost;
};
__device__ inline AreaTab area_tab(int d, double scale, int W) {
    AreaTab t;
    const double fs1 = d * scale;
    const double fs2 = fs1 + scale;
    const double cw = scale < W - fs1 ? scale : W - fs1;
    int s1 = (int)ceil(fs1);
    int s2 = (int)floor(fs2);
    s2 = s2 < W - 1 ? s2 : W - 1;
    s1 = s1 < s2 ? s1 : s2;
    t.s1 = s1;
    t.pre = (s1 - fs1 > 1e-3) ? 1 : 0;
    const int post = (fs2 - s2 > 1e-3) ? 1 : 0;
    t.full = s2 - s1;
    t.cnt = t.pre + t.full + post;
    t.apre = (float)((s1 - fs1) / cw);
    t.afull = (float)(1.0 / cw);
    double a = fs2 - s2;
    a = a < 1. ? a : 1.;
    a = a < cw ? a : cw;
    t.apost = (float)(a / cw);
    return t;
}
// the m-th entry of a tab: source index and weight
__device__ __forceinline__ int area_entry(const AreaTab& t, int m, float& alpha) {
    if (t.pre && m == 0) {
        alpha = t.apre;
        return t.s1 - 1;
    }
    const int r = m - t.pre;
    if (r < t.full) {
        alpha = t.afull;
        return t.s1 + r;
    }
    alpha = t.apost;
    return t.s1 + t.full;
}

// start + j * step (j < W) of a float start and a float step, summed into a double one step at a
// time, equals the closed form when every partial sum is a double exactly: all are multiples of
// g = 2^(min exponent - 23) (the coarser of the two float ulps, conservatively) and below
// |start| + W |step| in magnitude, so exact when that bound is under 2^53 g
__device__ inline bool seq_exact(float start, float step, int W) {
    if (step == 0.f) return true;
    int e = ilogbf(step);
    if (start != 0.f) e = min(e, ilogbf(start));
    const double M = fabs((double)start) + (double)W * fabs((double)step);
    return M * (1 + 1e-12) < ldexp(1.0, 53 + e - 23);
}

constexpr int kDescThreads = 256;
constexpr int kDescMaxW = 640;  // window edge whose row buffers fit the LDS of one workgroup

// keypoint q's descriptor (the list is compacted: every wavelet fits); one workgroup per keypoint.
// imgStride: keypoint q reads image img + q * imgStride (0: one shared image; the patch batch of
// extractDescriptorsFromPatches: one patch per keypoint).
//
// The W x W window is resized to 21 x 21 with INTER_AREA in OpenCV's two steps: a row buffer per
// source row (the horizontal weighted sum of that row, in the x-tab's order), then per destination
// row the beta-weighted rows in the y-tab's order.  A source row's buffer does not depend on the
// destination row, so each is computed once (all W of them, by the whole workgroup, lanes on
// consecutive window rows = consecutive image columns, so the byte loads coalesce) and kept in LDS.
// Windows wider than kDescMaxW take the per-output-pixel path (the same sums, recomputed).
__global__ __launch_bounds__(kDescThreads) void describe_kernel(const uint8_t* __restrict__ img, size_t imgStride,
                                                                int w, int h, const fm3d_keypoint* __restrict__ kp,
                                                                int n, const float* __restrict__ DW, int extended,
                                                                int upright, float* __restrict__ desc) {
    const int q = blockIdx.x, tid = threadIdx.x;
    if (q >= n) return;
    img += (size_t)q * imgStride;
    __shared__ float H[kDescMaxW * 21];  // row buffers [window row][destination column]
    __shared__ AreaTab T[21];
    __shared__ uint8_t P[21 * 21];
    __shared__ float DX[400], DY[400], V[128];
    __shared__ float sc;
    __shared__ float RSX[kDescMaxW], RSY[kDescMaxW];
    __shared__ bool RX[kDescMaxW];
    const fm3d_keypoint k = kp[q];
    const float s = k.size * 1.2f / 9.0f;
    const int gws = 2 * cv_roundf(2 * s);
    if (h + 1 < gws || w + 1 < gws) return;  // uniform over the workgroup
    const int W = (int)((20 + 1) * s);
    const float win_offset = -(float)(W - 1) / 2;
    const int start_x = cv_roundf(k.x + win_offset), start_y = cv_roundf(k.y - win_offset);
    // rotated window (Upright 0): row r starts at (RSX[r], RSY[r]), accumulated in float row after
    // row as the source does; along a row the source steps a double by cos_dir / -sin_dir.  RX[r]:
    // every such partial sum of row r is a double exactly (seq_exact), so start + c * step is the
    // same number; else the row is stepped sequentially
    float sin_dir = 0.f, cos_dir = 0.f, rsx0 = 0.f, rsy0 = 0.f;
    const bool rot = !upright;
    if (rot) {
        const float dir = k.angle * (float)(M_PI / 180);
        sin_dir = -(float)fm3d_sin((double)dir);
        cos_dir = (float)fm3d_cos((double)dir);
        rsx0 = k.x + win_offset * cos_dir + win_offset * sin_dir;
        rsy0 = k.y - win_offset * sin_dir + win_offset * cos_dir;
        if (W <= kDescMaxW) {
            if (tid < 2) {  // lane 0 the x starts, lane 1 the y starts
                float v = tid ? rsy0 : rsx0;
                const float st = tid ? cos_dir : sin_dir;
                float* R = tid ? RSY : RSX;
                for (int r = 0; r < W; r++, v += st) R[r] = v;
            }
            __syncthreads();
            for (int r = tid; r < W; r += kDescThreads)
                RX[r] = seq_exact(RSX[r], cos_dir, W) && seq_exact(RSY[r], -sin_dir, W);
            __syncthreads();
        }
    }
    // window pixel (row r, column c): upright = img(clamp(start_y - c), clamp(start_x + r))
    auto WIN = [&](int r, int c) -> int {
        if (!rot) {
            int x = start_x + r, y = start_y - c;
            x = x > 0 ? x : 0;
            y = y > 0 ? y : 0;
            x = x < w - 1 ? x : w - 1;
            y = y < h - 1 ? y : h - 1;
            return img[(size_t)y * w + x];
        }
        float sx, sy;
        bool exact;
        if (W <= kDescMaxW) {
            sx = RSX[r];
            sy = RSY[r];
            exact = RX[r];
        } else {
            sx = rsx0;
            sy = rsy0;
            for (int i = 0; i < r; i++) {
                sx += sin_dir;
                sy += cos_dir;
            }
            exact = seq_exact(sx, cos_dir, W) && seq_exact(sy, -sin_dir, W);
        }
        double px, py;
        if (exact) {
            px = (double)sx + (double)c * (double)cos_dir;
            py = (double)sy - (double)c * (double)sin_dir;
        } else {
            px = sx;
            py = sy;
            for (int j = 0; j < c; j++) {
                px += cos_dir;
                py -= sin_dir;
            }
        }
        const int ix = (int)floor(px), iy = (int)floor(py);
        if ((unsigned)ix < (unsigned)(w - 1) && (unsigned)iy < (unsigned)(h - 1)) {
            const float a = (float)(px - ix), b = (float)(py - iy);
            const uint8_t* p = img + (size_t)iy * w + ix;
            return (uint8_t)cv_roundf(p[0] * (1.f - a) * (1.f - b) + p[1] * a * (1.f - b) + p[w] * (1.f - a) * b +
                                      p[w + 1] * a * b);
        }
        int x = cv_round(px), y = cv_round(py);
        x = x > 0 ? x : 0;
        y = y > 0 ? y : 0;
        x = x < w - 1 ? x : w - 1;
        y = y < h - 1 ? y : h - 1;
        return img[(size_t)y * w + x];
    };
    const double scale = 1. / (21.0 / W);
    const int iscale = cv_round(scale);
    const bool fast = fabs(scale - iscale) < DBL_EPSILON;
    if (W < 21) {
        // a window narrower than the patch (size < 7.5): INTER_AREA enlarges by OpenCV's linear
        // emulation (oracle orc_resize_area_up): area-mode coefficients in 11-bit fixed point, the
        // horizontal pass in int (nearest from xmax on), the vertical one as VResizeLinearVec_32s8u on
        // columns 0..19 and FixedPtCast on column 20.  The window first goes to LDS.
        __shared__ uint8_t Wn[20 * 20];
        for (int e = tid; e < W * W; e += kDescThreads) Wn[e] = (uint8_t)WIN(e / W, e - (e / W) * W);
        __syncthreads();
        const double inv = 21.0 / W;
        auto tab = [&](int d, bool col, int& sx, int& a0, int& a1, bool& lin) {
            sx = (int)floor(d * scale);
            float f = (float)((d + 1) - (sx + 1) * inv);
            f = f <= 0 ? 0.f : f - floorf(f);
            lin = sx + 1 < W;  // columns: d < xmax
            if (col && sx >= W - 1) {
                f = 0.f;
                sx = W - 1;
            }
            a0 = (int)rintf(__fmul_rn(__fsub_rn(1.f, f), 2048.f));
            a1 = (int)rintf(__fmul_rn(f, 2048.f));
        };
        for (int pix = tid; pix < 441; pix += kDescThreads) {
            const int dy = pix / 21, dx = pix - dy * 21;
            int sx, a0, a1, sy, b0, b1;
            bool lin, lin_y;
            tab(dx, true, sx, a0, a1, lin);
            tab(dy, false, sy, b0, b1, lin_y);
            const int r0 = min(max(sy, 0), W - 1), r1 = min(max(sy + 1, 0), W - 1);
            const uint8_t *S0 = Wn + r0 * W, *S1 = Wn + r1 * W;
            const int h0 = lin ? S0[sx] * a0 + S0[sx + 1] * a1 : S0[sx] * 2048;
            const int h1 = lin ? S1[sx] * a0 + S1[sx + 1] * a1 : S1[sx] * 2048;
            int v = dx < 20 ? ((((h0 >> 4) * b0) >> 16) + (((h1 >> 4) * b1) >> 16) + 2) >> 2
                            : (b0 * h0 + b1 * h1 + (1 << 21)) >> 22;
            P[pix] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
        }
    } else if (fast) {
        // integer scale: exact integer block sums (any order), then OpenCV's rounding:
        // (sum + 2) >> 2 on the SIMD columns of the 2x2 case, cvRound(sum / iscale^2) elsewhere
        int* HI = reinterpret_cast<int*>(H);
        const bool rows = W <= kDescMaxW;
        if (rows) {
            for (int e = tid; e < W * 21; e += kDescThreads) {
                const int dx = e / W, a = e - dx * W;
                int sm = 0;
                for (int b = 0; b < iscale; b++) sm += WIN(a, dx * iscale + b);
                HI[a * 21 + dx] = sm;
            }
            __syncthreads();
        }
        for (int pix = tid; pix < 441; pix += kDescThreads) {
            const int dy = pix / 21, dx = pix - dy * 21;
            int sm = 0;
            for (int a = 0; a < iscale; a++) {
                if (rows) {
                    sm += HI[(dy * iscale + a) * 21 + dx];
                } else {
                    for (int b = 0; b < iscale; b++) sm += WIN(dy * iscale + a, dx * iscale + b);
                }
            }
            P[pix] = (iscale == 2 && dx < 16) ? (uint8_t)((sm + 2) >> 2) : sat_u8(sm * (1.f / (iscale * iscale)));
        }
    } else {
        if (tid < 21) T[tid] = area_tab(tid, scale, W);
        __syncthreads();
        if (W <= kDescMaxW) {
            // row buffers: H[a][dx] = sum over the x-tab entries of dx of WIN(a, sx) * alpha
            for (int e = tid; e < W * 21; e += kDescThreads) {
                const int dx = e / W, a = e - dx * W;
                const AreaTab tx = T[dx];
                float buf = 0.f;
                for (int b = 0; b < tx.cnt; b++) {
                    float alpha;
                    const int sx = area_entry(tx, b, alpha);
                    buf += WIN(a, sx) * alpha;
                }
                H[a * 21 + dx] = buf;
            }
            __syncthreads();
            for (int pix = tid; pix < 441; pix += kDescThreads) {
                const int dy = pix / 21, dx = pix - dy * 21;
                const AreaTab ty = T[dy];
                float acc = 0.f;
                for (int a = 0; a < ty.cnt; a++) {
                    float beta;
                    const int sy = area_entry(ty, a, beta);
                    const float buf = H[sy * 21 + dx];
                    acc = a == 0 ? beta * buf : acc + beta * buf;
                }
                P[pix] = sat_u8(acc);
            }
        } else {
            for (int pix = tid; pix < 441; pix += kDescThreads) {
                const int dy = pix / 21, dx = pix - dy * 21;
                const AreaTab ty = T[dy], tx = T[dx];
                float acc = 0.f;
                for (int a = 0; a < ty.cnt; a++) {
                    float beta;
                    const int sy = area_entry(ty, a, beta);
                    float buf = 0.f;
                    for (int b = 0; b < tx.cnt; b++) {
                        float alpha;
                        const int sx = area_entry(tx, b, alpha);
                        buf += WIN(sy, sx) * alpha;
                    }
                    acc = a == 0 ? beta * buf : acc + beta * buf;
                }
                P[pix] = sat_u8(acc);
            }
        }
    }
    __syncthreads();
    for (int e = tid; e < 400; e += kDescThreads) {
        const int i = e / 20, j = e - i * 20;
        const float dw = DW[e];
        DX[e] = (P[i * 21 + j + 1] - P[i * 21 + j] + P[(i + 1) * 21 + j + 1] - P[(i + 1) * 21 + j]) * dw;
        DY[e] = (P[(i + 1) * 21 + j] - P[i * 21 + j] + P[(i + 1) * 21 + j + 1] - P[i * 21 + j + 1]) * dw;
    }
    __syncthreads();
    const int per = extended ? 8 : 4, dsize = extended ? 128 : 64;
    if (tid < 16) {
        const int i = tid >> 2, j = tid & 3;
        float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int y = i * 5; y < i * 5 + 5; y++)
            for (int x = j * 5; x < j * 5 + 5; x++) {
                const float tx = DX[y * 20 + x], ty = DY[y * 20 + x];
                if (extended) {
                    if (ty >= 0) {
                        v[0] += tx;
                        v[1] += fabsf(tx);
                    } else {
                        v[2] += tx;
                        v[3] += fabsf(tx);
                    }
                    if (tx >= 0) {
                        v[4] += ty;
                        v[5] += fabsf(ty);
                    } else {
                        v[6] += ty;
                        v[7] += fabsf(ty);
                    }
                } else {
                    v[0] += tx;
                    v[1] += ty;
                    v[2] += fabsf(tx);
                    v[3] += fabsf(ty);
                }
            }
        for (int kk = 0; kk < per; kk++) V[tid * per + kk] = v[kk];
    }
    __syncthreads();
    if (tid == 0) {
        double sq = 0;
        for (int kk = 0; kk < dsize; kk++) sq += V[kk] * V[kk];
        sc = (float)(1. / (sqrt(sq) + DBL_EPSILON));
    }
    __syncthreads();
    float* o = desc + (size_t)q * dsize;
    for (int kk = tid; kk < dsize; kk += kDescThreads) o[kk] = V[kk] * sc;
}

}  // namespace

void launch_integral(const uint8_t* img, int w, int h, int* sum, hipStream_t s) {
    if (w <= 0 || h <= 0) return;
    integral_rows_kernel<<<h, 64, 0, s>>>(img, w, h, sum);
    integral_cols_kernel<<<(w + 1 + 63) / 64, 64 * kIntBands, 0, s>>>(w, h, sum);
}

void launch_integral_rows(const uint8_t* img, int w, int h, int* rows, hipStream_t s) {
    if (w <= 0 || h <= 0) return;
    integral_rows_kernel<<<h, 64, 0, s>>>(img, w, h, rows);
}

void launch_surf_hessian(const int* sum, int w, const SurfLayer* layers, int nL, long long total, float* det,
                         float* tr, hipStream_t s) {
    if (total <= 0) return;
    hessian_kernel<<<(unsigned)((total + 255) / 256), 256, 0, s>>>(sum, w, layers, nL, det, tr);
}

void launch_surf_maxima(const float* det, const float* tr, const SurfLayer* layers, const SurfMid* mids, int nM,
                        long long total, float thr, SurfCand* cand, int* count, int cap, hipStream_t s) {
    if (nM <= 0 || total <= 0) return;
    maxima_kernel<<<(unsigned)((total + 255) / 256), 256, 0, s>>>(det, tr, layers, mids, nM, thr, cand, count, cap);
}

size_t surf_sort_tmp_bytes(int n) {
    size_t bytes = 0;
    hipcub::DeviceMergeSort::SortKeys(nullptr, bytes, (SurfCand*)nullptr, n, KpGreater(), (hipStream_t)0);
    return bytes;
}

void launch_surf_sort(SurfCand* cand, int n, void* tmp, size_t tmpBytes, hipStream_t s) {
    if (n <= 1) return;
    hipcub::DeviceMergeSort::SortKeys(tmp, tmpBytes, cand, n, KpGreater(), s);
}

void launch_integral_batch(const uint8_t* img, int w, int h, int nb, int* sum, hipStream_t s) {
    if (w <= 0 || h <= 0 || nb <= 0) return;
    integral_rows_kernel<<<dim3(h, nb), 64, 0, s>>>(img, w, h, sum);
    integral_cols_kernel<<<dim3((w + 1 + 63) / 64, nb), 64 * kIntBands, 0, s>>>(w, h, sum);
}

void launch_surf_orient(const void* kp, size_t kstride, int n, const int* sum, size_t sumStride, int w, int h,
                        const SurfOri& ori, int* flag, float* angle, hipStream_t s) {
    if (n <= 0) return;
    orient_kernel<<<(n + kOriWaves - 1) / kOriWaves, 64 * kOriWaves, 0, s>>>(
        static_cast<const char*>(kp), kstride, n, sum, sumStride, w, h, ori, flag, angle);
}

void launch_surf_upright(const SurfCand* cand, const int* count, int n, int w, int h, int* flag, int* pos, int* total,
                         void* scanTmp, fm3d_keypoint* out, int* src, const float* angle, hipStream_t s) {
    if (n <= 0) return;
    if (!angle) upright_flag_kernel<<<(n + 255) / 256, 256, 0, s>>>(cand, count, n, w, h, flag);
    launch_exclusive_scan(flag, n, pos, total, scanTmp, s);
    keypoint_scatter_kernel<<<(n + 255) / 256, 256, 0, s>>>(cand, flag, pos, angle, n, out, src);
}

void launch_surf_keep(const fm3d_keypoint* in, int n, int w, int h, int* flag, int* pos, int* total, void* scanTmp,
                      fm3d_keypoint* out, int* src, const float* angle, hipStream_t s) {
    if (n <= 0) return;
    if (!angle) keep_flag_kernel<<<(n + 255) / 256, 256, 0, s>>>(in, n, w, h, flag);
    launch_exclusive_scan(flag, n, pos, total, scanTmp, s);
    keep_scatter_kernel<<<(n + 255) / 256, 256, 0, s>>>(in, flag, pos, angle, n, out, src);
}

void launch_surf_describe(const uint8_t* img, size_t imgStride, int w, int h, const fm3d_keypoint* kp, int n,
                          const float* DW, int extended, int upright, float* desc, hipStream_t s) {
    if (n <= 0) return;
    describe_kernel<<<n, kDescThreads, 0, s>>>(img, imgStride, w, h, kp, n, DW, extended, upright, desc);
}

}  // namespace fm3d
