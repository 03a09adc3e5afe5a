// fm3d_freak.hip -- the FREAK descriptor on gfx950.
//
// Reference: DescriptorsMatcher's ExtractorType FREAK (descriptorsmatcher.cpp:350-353: cv::FREAK() with
// OpenCV 2.4.9's defaults -- orientation and scale normalised, patternScale 22, 4 octaves), matched by
// Hamming distance like ORB and BRISK rows (:64-66).  The algorithm is restated in oracle/orc_freak.c;
// the GPU equals that oracle bit for bit.  The host keeps what FREAK::buildPattern precomputes (the 43
// pattern points of every scale and orientation in glibc's double cos / sin, the pattern sizes, the
// orientation weights, the 512 selected pairs) and the per-keypoint scale and border filter; the
// kernel does the per-keypoint work, one wave per keypoint:
//   * lanes 0..42: meanIntensity of the unrotated pattern points (the integral box mean, C integer
//     division of the exact int sum; below sigma 0.5 freak.cpp's 1024 fixed-point bilinear sample);
//   * lanes 0..44: the orientation pairs' (I_i - I_j) * weight / 2048 (int, truncating), summed over
//     the wave (integer sums: any order); lane 0: angle = (float)(atan2f(d1, d0) * 180 / pi) with the
//     correctly rounded atan2f of fm3d_cvmath.h, thetaIdx = int(256 * angle * (1 / 360.0) + 0.5)
//     wrapped to [0, 256);
//   * lanes 0..42: the intensities of the pattern rotated to thetaIdx;
//   * lane b of the 64: descriptor byte b, its 8 bits the comparisons I_i >= I_j of pairs
//     128q + 16t + 15 - (b % 16) (q = b / 16, t = bit): the SSE2 build's layout.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fm3d_cvmath.h"
#include "fm3d_kernels.h"

namespace fm3d {

namespace {

// meanIntensity (freak.cpp): the pattern point (px, py) of sigma `radius` around the keypoint
__device__ __forceinline__ int freak_intensity(const uint8_t* __restrict__ img, const int* __restrict__ sum, int w,
                                               float kx, float ky, float px, float py, float radius) {
    const float xf = __fadd_rn(px, kx), yf = __fadd_rn(py, ky);
    const int x = (int)xf, y = (int)yf;
    if (radius < 0.5) {  // not reached with patternScale 22 (the smallest sigma is 0.92)
        const int r_x = (int)__fmul_rn(__fsub_rn(xf, (float)x), 1024.f);
        const int r_y = (int)__fmul_rn(__fsub_rn(yf, (float)y), 1024.f);
        const int r_x_1 = 1024 - r_x, r_y_1 = 1024 - r_y;
        const uint8_t* p = img + x + (size_t)y * w;
        unsigned v = (unsigned)(r_x_1 * r_y_1 * (int)p[0]);
        v += (unsigned)(r_x * r_y_1 * (int)p[1]);
        v += (unsigned)(r_x * r_y * (int)p[w + 1]);
        v += (unsigned)(r_x_1 * r_y * (int)p[w]);
        v += 2 * 1024 * 1024;
        return (uint8_t)(v / (4 * 1024 * 1024));
    }
    const int x_left = (int)((double)__fsub_rn(xf, radius) + 0.5);
    const int y_top = (int)((double)__fsub_rn(yf, radius) + 0.5);
    const int x_right = (int)((double)__fadd_rn(xf, radius) + 1.5);
    const int y_bottom = (int)((double)__fadd_rn(yf, radius) + 1.5);
    const size_t W = (size_t)w + 1;
    int r = sum[y_bottom * W + x_right];
    r -= sum[y_bottom * W + x_left];
    r += sum[y_top * W + x_left];
    r -= sum[y_top * W + x_right];
    r = r / ((x_right - x_left) * (y_bottom - y_top));
    return (uint8_t)r;
}

__global__ __launch_bounds__(64) void freak_kernel(const uint8_t* __restrict__ img, const int* __restrict__ sum, int w,
                                                   const fm3d_keypoint* __restrict__ kp, const int* __restrict__ scale,
                                                   int n, const float4* __restrict__ lut, const int4* __restrict__ opairs,
                                                   const int2* __restrict__ pairs, float* __restrict__ angle,
                                                   uint8_t* __restrict__ desc) {
    const int q = blockIdx.x, lane = threadIdx.x;
    if (q >= n) return;  // the whole block
    __shared__ int v[64];
    const fm3d_keypoint k = kp[q];
    const float4* base = lut + (size_t)scale[q] * kFreakOrient * kFreakPoints;
    if (lane < kFreakPoints) {
        const float4 pt = base[lane];
        v[lane] = freak_intensity(img, sum, w, k.x, k.y, pt.x, pt.y, pt.z);
    }
    __syncthreads();
    int d0 = 0, d1 = 0;
    if (lane < kFreakOrientPairs) {
        const int4 o = opairs[lane];
        const int delta = v[o.x] - v[o.y];
        d0 = delta * o.z / 2048;
        d1 = delta * o.w / 2048;
    }
    for (int s = 32; s > 0; s >>= 1) {
        d0 += __shfl_xor(d0, s);
        d1 += __shfl_xor(d1, s);
    }
    const float a = (float)((double)fm3d_cv_atan2f((float)d1, (float)d0) * (180.0 / M_PI));
    int theta = (int)((double)__fmul_rn((float)kFreakOrient, a) * (1 / 360.0) + 0.5);
    if (theta < 0) theta += kFreakOrient;
    if (theta >= kFreakOrient) theta -= kFreakOrient;
    __syncthreads();
    if (lane < kFreakPoints) {
        const float4 pt = base[(size_t)theta * kFreakPoints + lane];
        v[lane] = freak_intensity(img, sum, w, k.x, k.y, pt.x, pt.y, pt.z);
    }
    __syncthreads();
    const int qq = lane >> 4, b = lane & 15;
    unsigned byte = 0;
#pragma unroll
    for (int t = 0; t < 8; t++) {
        const int2 pr = pairs[128 * qq + 16 * t + 15 - b];
        byte |= (v[pr.x] >= v[pr.y] ? 1u : 0u) << t;
    }
    desc[(size_t)q * 64 + lane] = (uint8_t)byte;
    if (lane == 0) angle[q] = a;
}

}  // namespace

void launch_freak_desc(const uint8_t* img, const int* sum, int w, const fm3d_keypoint* kp, const int* scale, int n,
                       const float4* lut, const int4* opairs, const int2* pairs, float* angle, uint8_t* desc,
                       hipStream_t s) {
    if (n <= 0) return;
    freak_kernel<<<n, 64, 0, s>>>(img, sum, w, kp, scale, n, lut, opairs, pairs, angle, desc);
}

}  // namespace fm3d
