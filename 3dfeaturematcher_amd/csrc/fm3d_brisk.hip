// fm3d_brisk.hip -- the BRISK descriptor on gfx950.
//
// Reference: DescriptorsMatcher's ExtractorType BRISK (descriptorsmatcher.cpp:343-348,
// cv::BRISK(BriskDetector.Threshold, BriskDetector.Octaves)), whose compute on the caller's keypoints is
// OpenCV 2.4.9's BRISK::computeDescriptorsAndOrOrientation without the orientation step (restated in
// oracle/orc_brisk.c; the GPU equals that oracle bit for bit).  The host keeps what OpenCV precomputes
// in its constructor and per keypoint -- the pattern points of each (scale, rotation) in use (glibc's
// cos / sin, as the constructor's table), the short pairs, the keypoint's scale and the border
// filter -- and the kernel does the per-keypoint work:
//   brisk_desc_kernel   a wave per keypoint: lanes 0..59 the smoothed intensities of the 60 rotated
//                       pattern points (a box of half width sigma whose border pixels carry their
//                       covered fraction, OpenCV's fixed point: corners from the image, edges and
//                       interior from the integral image, exact integers), then the 512 short-pair
//                       comparisons as 8 ballots of 64 bits, written as 64 bytes.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fm3d_kernels.h"

namespace fm3d {

namespace {

constexpr int kBriskWaves = 4;  // keypoints per workgroup

// smoothedIntensity (x 1024, as OpenCV returns it) at key (kx, ky) + point (px, py) of sigma sg
__device__ int brisk_intensity(const uint8_t* __restrict__ img, const int* __restrict__ II, int w, float kx, float ky,
                               float px, float py, float sg) {
    const float xf = __fadd_rn(px, kx), yf = __fadd_rn(py, ky);
    if (sg < 0.5f) {  // bilinear (not reached by the default pattern)
        const int x = (int)xf, y = (int)yf;
        const int r_x = (int)__fmul_rn(__fsub_rn(xf, (float)x), 1024.f), r_y = (int)__fmul_rn(__fsub_rn(yf, (float)y), 1024.f);
        const int r_x_1 = 1024 - r_x, r_y_1 = 1024 - r_y;
        const uint8_t* p = img + (size_t)y * w + x;
        const int v = r_x_1 * r_y_1 * p[0] + r_x * r_y_1 * p[1] + r_x * r_y * p[w] + r_x_1 * r_y * p[w + 1];
        return (v + 512) / 1024;
    }
    const float area = __fmul_rn(__fmul_rn(4.0f, sg), sg);
    const int scaling = (int)(4194304.0 / (double)area);
    const int scaling2 = (int)((double)__fmul_rn((float)scaling, area) / 1024.0);
    const float x_1 = __fsub_rn(xf, sg), x1 = __fadd_rn(xf, sg), y_1 = __fsub_rn(yf, sg), y1 = __fadd_rn(yf, sg);
    const int xl = (int)((double)x_1 + 0.5), yt = (int)((double)y_1 + 0.5);
    const int xr = (int)((double)x1 + 0.5), yb = (int)((double)y1 + 0.5);
    const float r_x_1 = __fadd_rn(__fsub_rn((float)xl, x_1), 0.5f), r_y_1 = __fadd_rn(__fsub_rn((float)yt, y_1), 0.5f);
    const float r_x1 = __fadd_rn(__fsub_rn(x1, (float)xr), 0.5f), r_y1 = __fadd_rn(__fsub_rn(y1, (float)yb), 0.5f);
    const float fs = (float)scaling;
    const int A = (int)__fmul_rn(__fmul_rn(r_x_1, r_y_1), fs), B = (int)__fmul_rn(__fmul_rn(r_x1, r_y_1), fs);
    const int C = (int)__fmul_rn(__fmul_rn(r_x1, r_y1), fs), D = (int)__fmul_rn(__fmul_rn(r_x_1, r_y1), fs);
    const int rx_1i = (int)__fmul_rn(r_x_1, fs), ry_1i = (int)__fmul_rn(r_y_1, fs);
    const int rx1i = (int)__fmul_rn(r_x1, fs), ry1i = (int)__fmul_rn(r_y1, fs);
    const int s1 = w + 1;
    auto ii = [&](int r, int c) -> long long { return II[(size_t)r * s1 + c]; };
    auto box = [&](int r0, int r1, int c0, int c1) -> long long {  // rows [r0, r1), columns [c0, c1)
        return ii(r1, c1) - ii(r0, c1) - ii(r1, c0) + ii(r0, c0);
    };
    long long ret = (long long)A * img[(size_t)yt * w + xl] + (long long)B * img[(size_t)yt * w + xr] +
                    (long long)C * img[(size_t)yb * w + xr] + (long long)D * img[(size_t)yb * w + xl];
    ret += ry_1i * box(yt, yt + 1, xl + 1, xr) + ry1i * box(yb, yb + 1, xl + 1, xr);
    ret += rx_1i * box(yt + 1, yb, xl, xl + 1) + rx1i * box(yt + 1, yb, xr, xr + 1);
    ret += (long long)scaling * box(yt + 1, yb, xl + 1, xr);
    return (int)((ret + scaling2 / 2) / scaling2);
}

__global__ __launch_bounds__(64 * kBriskWaves) void brisk_desc_kernel(const uint8_t* __restrict__ img,
                                                                      const int* __restrict__ II, int w,
                                                                      const fm3d_keypoint* __restrict__ kp,
                                                                      const int* __restrict__ pidx, int n,
                                                                      const float4* __restrict__ pat,
                                                                      const int2* __restrict__ pairs, int npairs,
                                                                      uint8_t* __restrict__ desc) {
    __shared__ int vals[kBriskWaves][64];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int q = blockIdx.x * kBriskWaves + wave;
    if (q >= n) return;  // whole waves
    const fm3d_keypoint k = kp[q];
    if (lane < 60) {
        const float4 p = pat[(size_t)pidx[q] * 60 + lane];
        vals[wave][lane] = brisk_intensity(img, II, w, k.x, k.y, p.x, p.y, p.z);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t word = 0;
#pragma unroll
    for (int c = 0; c < 8; c++) {
        const int e = c * 64 + lane;
        bool bit = false;
        if (e < npairs) {
            const int2 pr = pairs[e];
            bit = vals[wave][pr.x] > vals[wave][pr.y];
        }
        const unsigned long long b = __ballot(bit);
        if (lane == 2 * c) word = (uint32_t)b;
        if (lane == 2 * c + 1) word = (uint32_t)(b >> 32);
    }
    if (lane < 16) reinterpret_cast<uint32_t*>(desc + (size_t)q * 64)[lane] = word;
}

}  // namespace

void launch_brisk_desc(const uint8_t* img, const int* II, int w, const fm3d_keypoint* kp, const int* pidx, int n,
                       const float4* pat, const int2* pairs, int npairs, uint8_t* desc, hipStream_t s) {
    if (n <= 0) return;
    brisk_desc_kernel<<<(n + kBriskWaves - 1) / kBriskWaves, 64 * kBriskWaves, 0, s>>>(img, II, w, kp, pidx, n, pat,
                                                                                      pairs, npairs, desc);
}

}  // namespace fm3d
