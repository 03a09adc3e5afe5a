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
//   describe_kernel      SURFInvoker (upright): one workgroup per keypoint.  The 21x21 INTER_AREA
//                        patch comes straight from the image (the rotated, border-replicated window
//                        is never materialised): OpenCV's row buffers, one per window row, in LDS,
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

namespace fm3d {

namespace {

// cvRound of a float (round to nearest, ties to even)
__device__ __forceinline__ int cv_roundf(float v) { return (int)rintf(v); }
__device__ __forceinline__ int cv_round(double v) { return (int)rint(v); }

// ---------------------------------------------------------------- integral image
// sum: (h+1) x (w+1) int32, row 0 and column 0 zero.  Pass 1: row prefix sums (a wave per row).
__global__ __launch_bounds__(64) void integral_rows_kernel(const uint8_t* __restrict__ img, int w, int h,
                                                            int* __restrict__ sum) {
    const int y = blockIdx.x, lane = threadIdx.x;
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
                                        const int* __restrict__ pos, int cap, fm3d_keypoint* __restrict__ out,
                                        int* __restrict__ src) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= cap || !flag[q]) return;
    fm3d_keypoint k;
    k.x = c[q].x;
    k.y = c[q].y;
    k.size = c[q].size;
    k.angle = 360.f - 90.f;
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
                                    const int* __restrict__ pos, int n, fm3d_keypoint* __restrict__ out,
                                    int* __restrict__ src) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n || !flag[q]) return;
    fm3d_keypoint o = k[q];
    o.angle = 360.f - 90.f;
    out[pos[q]] = o;
    if (src) src[pos[q]] = q;
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
                                                                float* __restrict__ desc) {
    const int q = blockIdx.x, tid = threadIdx.x;
    if (q >= n) return;
    img += (size_t)q * imgStride;
    __shared__ float H[kDescMaxW * 21];  // row buffers [window row][destination column]
    __shared__ AreaTab T[21];
    __shared__ uint8_t P[21 * 21];
    __shared__ float DX[400], DY[400], V[128];
    __shared__ float sc;
    const fm3d_keypoint k = kp[q];
    const float s = k.size * 1.2f / 9.0f;
    const int gws = 2 * cv_roundf(2 * s);
    if (h + 1 < gws || w + 1 < gws) return;  // uniform over the workgroup
    const int W = (int)((20 + 1) * s);
    const float win_offset = -(float)(W - 1) / 2;
    const int start_x = cv_roundf(k.x + win_offset), start_y = cv_roundf(k.y - win_offset);
    // window pixel (row r, column c) = img(clamp(start_y - c), clamp(start_x + r))
    auto WIN = [&](int r, int c) -> int {
        int x = start_x + r, y = start_y - c;
        x = x > 0 ? x : 0;
        y = y > 0 ? y : 0;
        x = x < w - 1 ? x : w - 1;
        y = y < h - 1 ? y : h - 1;
        return img[(size_t)y * w + x];
    };
    const double scale = 1. / (21.0 / W);
    const int iscale = cv_round(scale);
    const bool fast = fabs(scale - iscale) < DBL_EPSILON;
    if (fast) {
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

void launch_surf_upright(const SurfCand* cand, const int* count, int n, int w, int h, int* flag, int* pos, int* total,
                         void* scanTmp, fm3d_keypoint* out, int* src, hipStream_t s) {
    if (n <= 0) return;
    upright_flag_kernel<<<(n + 255) / 256, 256, 0, s>>>(cand, count, n, w, h, flag);
    launch_exclusive_scan(flag, n, pos, total, scanTmp, s);
    keypoint_scatter_kernel<<<(n + 255) / 256, 256, 0, s>>>(cand, flag, pos, n, out, src);
}

void launch_surf_keep(const fm3d_keypoint* in, int n, int w, int h, int* flag, int* pos, int* total, void* scanTmp,
                      fm3d_keypoint* out, int* src, hipStream_t s) {
    if (n <= 0) return;
    keep_flag_kernel<<<(n + 255) / 256, 256, 0, s>>>(in, n, w, h, flag);
    launch_exclusive_scan(flag, n, pos, total, scanTmp, s);
    keep_scatter_kernel<<<(n + 255) / 256, 256, 0, s>>>(in, flag, pos, n, out, src);
}

void launch_surf_describe(const uint8_t* img, size_t imgStride, int w, int h, const fm3d_keypoint* kp, int n,
                          const float* DW, int extended, float* desc, hipStream_t s) {
    if (n <= 0) return;
    describe_kernel<<<n, kDescThreads, 0, s>>>(img, imgStride, w, h, kp, n, DW, extended, desc);
}

}  // namespace fm3d
