// fm3d_device.h -- device-side arithmetic shared by the fm3d kernels.
//
// Every function restates one reference/OpenCV-2.4 operation with its exact
// IEEE operation order (the library is compiled with -ffp-contract=off, so no
// FMA contraction): results are bit-identical to the CPU oracle.
#pragma once

#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include "fm3d_detmath.h"
#include "fm3d_cvsvd.h"

namespace fm3d {

struct Camera {
    double fx, fy, cx, cy;
    double k[5];  // OpenCV order k1,k2,p1,p2,k3 (settings k0,k1,p1,p2,k2; singlecameratriangulator.cpp:99-105)
};

// 1 / d, correctly rounded.  On the device for 2^-700 <= |d| <= 2^700 the hardware reciprocal with
// Newton steps and one Markstein correction (the division operator's steps without its operand
// scaling and fix-up, which change nothing in that range; fm3d_fastdiv.h recip_fast, checked against
// the operator by tools/micro/div_check.hip), else the operator.
__host__ __device__ inline double recip_exact(double d) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double ad = fabs(d);
    if (ad >= 0x1p-700 && ad <= 0x1p700) {
        double r = __builtin_amdgcn_rcp(d);
        double e = __builtin_fma(-d, r, 1.0);
        r = __builtin_fma(r, e, r);
        e = __builtin_fma(-d, r, 1.0);
        r = __builtin_fma(r, e, r);
        const double rem = __builtin_fma(-d, r, 1.0);
        return __builtin_fma(rem, r, r);
    }
#endif
    return 1. / d;
}

// cv::undistortPoints (OpenCV 2.4 cvUndistortPoints), 5 iterations, R = I.
// Reference call sites: singlecameratriangulator.cpp:169-170 (keypoints), :542 (neighbourhood).
// OpenCV evaluates icdist = (1 + ((k7 r2 + k6) r2 + k5) r2) / (1 + ((k3 r2 + k2) r2 + k1) r2) with
// the rational coefficients k5..k7 = 0, and then applies R = I and the identity P as
// (1 x + 0 y + 0, 0 x + 1 y + 0) * 1 / (0 x + 0 y + 1).  For a finite r2 the numerator is exactly 1,
// and for finite x, y the transform is x + 0, y + 0 (which turns -0 into +0, as 1 x + 0 y + 0 does)
// times 1: the same bits with fewer operations.  A non-finite r2, x or y takes the literal forms.
__host__ __device__ inline void undistort1(const Camera& c, double x, double y, double& ox, double& oy) {
    const double ifx = 1. / c.fx, ify = 1. / c.fy;
    double x0, y0;
    x0 = x = (x - c.cx) * ifx;
    y0 = y = (y - c.cy) * ify;
    for (int j = 0; j < 5; j++) {
        double r2 = x * x + y * y;
        const double den = 1 + ((c.k[4] * r2 + c.k[1]) * r2 + c.k[0]) * r2;
        double icdist;
        if (r2 <= DBL_MAX)
            icdist = recip_exact(den);
        else
            icdist = (1 + ((0. * r2 + 0.) * r2 + 0.) * r2) / den;
        double deltaX = 2 * c.k[2] * x * y + c.k[3] * (r2 + 2 * x * x);
        double deltaY = c.k[2] * (r2 + 2 * y * y) + 2 * c.k[3] * x * y;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    if (fabs(x) <= DBL_MAX && fabs(y) <= DBL_MAX) {
        ox = x + 0.;
        oy = y + 0.;
        return;
    }
    double xx = 1. * x + 0. * y + 0.;
    double yy = 0. * x + 1. * y + 0.;
    double ww = 1. / (0. * x + 0. * y + 1.);
    ox = xx * ww;
    oy = yy * ww;
}

// cv::projectPoints (OpenCV 2.4 cvProjectPoints2) of one point, rotation matrix R
// (row-major) and translation t.  Call sites: :388 (R = I, t = 0), :602 (camera 2).
__host__ __device__ inline void project1(const Camera& c, const double* R, const double* t, double X, double Y,
                                         double Z, double& u, double& v) {
    double x = R[0] * X + R[1] * Y + R[2] * Z + t[0];
    double y = R[3] * X + R[4] * Y + R[5] * Z + t[1];
    double z = R[6] * X + R[7] * Y + R[8] * Z + t[2];
    z = z ? 1. / z : 1;
    x *= z;
    y *= z;
    double r2 = x * x + y * y;
    double r4 = r2 * r2;
    double r6 = r4 * r2;
    double a1 = 2 * x * y;
    double a2 = r2 + 2 * x * x;
    double a3 = r2 + 2 * y * y;
    double cdist = 1 + c.k[0] * r2 + c.k[1] * r4 + c.k[4] * r6;
    // OpenCV's icdist2 = 1 / (1 + 0*r2 + 0*r4 + 0*r6) with k3..k5 = 0: exactly 1 when
    // r6 (hence r2, r4 >= 0) is finite, NaN otherwise -- x*cdist*icdist2 without the division
    double xc = x * cdist, yc = y * cdist;
    if (!(r6 - r6 == 0.)) xc = yc = __builtin_nan("");
    double xd = xc + c.k[2] * a1 + c.k[3] * a2;
    double yd = yc + c.k[2] * a3 + c.k[3] * a1;
    u = xd * c.fx + c.cx;
    v = yd * c.fy + c.cy;
}

// getBilinearInterpPix32f (tools.cpp:129-142) on a continuous 8-bit image that is
// followed by >= 2*w+2 zero bytes (the reference reads unchecked one row/col past
// the image when isPixelGood admits x == cols or y == rows).
__device__ inline float bilinear(const uint8_t* __restrict__ img, int w, float x, float y) {
    int x0 = (int)floor((double)x), y0 = (int)floor((double)y);
    const uint8_t* p0 = img + (long)y0 * w + x0;
    const uint8_t* p1 = p0 + w;
    float b00 = (float)p0[0], b10 = (float)p1[0], b01 = (float)p0[1], b11 = (float)p1[1];
    float xm0 = 1.0f - (x - (float)x0), xm1 = (x - (float)x0);
    float ym0 = 1.0f - (y - (float)y0), ym1 = (y - (float)y0);
    return xm0 * (b00 * ym0 + b10 * ym1) + xm1 * (b01 * ym0 + b11 * ym1);
}

// isPixelGood (singlecameratriangulator.cpp:657-665).  NaN coordinates are bad
// (the reference has undefined behaviour for them).
__host__ __device__ inline bool pixel_good(double x, double y, double scale, int cols, int rows) {
    if (x != x || y != y) return false;
    if ((x < 0) || (x > ((1 / scale) * cols)) || (y < 0) || (y > ((1 / scale) * rows))) return false;
    return true;
}
// the same test with the per-level bounds (1/scale)*cols, (1/scale)*rows precomputed
__host__ __device__ inline bool pixel_good_b(double x, double y, double xmax, double ymax) {
    if (x != x || y != y) return false;
    if ((x < 0) || (x > xmax) || (y < 0) || (y > ymax)) return false;
    return true;
}

// MINPACK enorm, accumulated element by element in index order (lmfit lm_enorm).
struct Enorm {
    double s1, s2, s3, x1max, x3max, agiant;
    __host__ __device__ inline void init(int n) {
        s1 = s2 = s3 = x1max = x3max = 0.;
        agiant = 1.304e19 / (double)n;
    }
    __host__ __device__ inline void add(double x) {
        const double rdwarf = 3.834e-20;
        double xabs = fabs(x), temp;
        if (xabs > rdwarf && xabs < agiant) {
            s2 += xabs * xabs;
        } else if (xabs > rdwarf) {
            if (xabs > x1max) {
                temp = x1max / xabs;
                s1 = 1 + s1 * temp * temp;
                x1max = xabs;
            } else {
                temp = xabs / x1max;
                s1 += temp * temp;
            }
        } else {
            if (xabs > x3max) {
                temp = x3max / xabs;
                s3 = 1 + s3 * temp * temp;
                x3max = xabs;
            } else if (xabs != 0.) {
                temp = xabs / x3max;
                s3 += temp * temp;
            }
        }
    }
    __host__ __device__ inline double finish() const {
        if (s1 != 0) return x1max * sqrt(s1 + (s2 / x1max) / x1max);
        if (s2 != 0) {
            if (s2 >= x3max) return sqrt(s2 * (1 + (x3max / s2) * (x3max * s3)));
            return sqrt(x3max * ((s2 / x3max) + (x3max * s3)));
        }
        return x3max * sqrt(s3);
    }
};

__host__ __device__ inline double enorm2(const double* x) {
    Enorm e;
    e.init(2);
    e.add(x[0]);
    e.add(x[1]);
    return e.finish();
}

// cv::fastAtan2 / phase(..., true) of OpenCV 2.4.9+ (core/mathfuncs.cpp, the polynomial; degrees in
// [0, 360)); SURF's orientation and ORB's IC_Angle.  Needs the correctly rounded float division
// (-fhip-fp32-correctly-rounded-divide-sqrt)
__device__ __forceinline__ float fast_atan2f(float y, float x) {
    constexpr float P1 = 0.9997878412794807f * (float)(180 / M_PI);
    constexpr float P3 = -0.3258083974640975f * (float)(180 / M_PI);
    constexpr float P5 = 0.1555786518463281f * (float)(180 / M_PI);
    constexpr float P7 = -0.04432655554792128f * (float)(180 / M_PI);
    const float ax = fabsf(x), ay = fabsf(y);
    float a;
    if (ax >= ay) {
        const float c = ay / (ax + (float)DBL_EPSILON), c2 = c * c;
        a = (((P7 * c2 + P5) * c2 + P3) * c2 + P1) * c;
    } else {
        const float c = ax / (ay + (float)DBL_EPSILON), c2 = c * c;
        a = 90.f - (((P7 * c2 + P5) * c2 + P3) * c2 + P1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// The decoupled look-back of one block (LookBack in fm3d_kernels.h), called by all 64 lanes of ONE wave
// of the block: lane 0 publishes the block's count ("aggregate", flag 1); then the wave reads the
// status words of its 64 nearest predecessors at once (one per lane), finds the nearest inclusive
// prefix (flag 2) with a ballot, and -- once every word up to it carries this launch's epoch -- adds
// the counts up to it; with no inclusive prefix in the window it moves 64 blocks further back.  Lane 0
// publishes the block's inclusive prefix.  Returns (on every lane) the number of items of all earlier
// blocks.  Status words are device-scope RELAXED atomics (vector memory, past the per-XCD caches): a
// word carries everything a successor needs (count, flag, epoch), and no block reads another's
// other outputs, so nothing has to be ordered around them -- release / acquire would add an L2
// writeback and invalidate per access (about 3.5 us each, MI355X_MICROARCH.md).  A walk of one
// word per step cost a memory round trip per predecessor (triangulate_compact 51 us at C2).
__device__ inline int lookback_exclusive(unsigned long long* st, unsigned epoch, int bid, int agg) {
    const int lane = (int)(threadIdx.x & 63);
    const unsigned long long tag = (unsigned long long)epoch << 32;
    if (bid == 0) {
        if (lane == 0)
            __hip_atomic_store(&st[0], tag | (2ull << 30) | (unsigned)agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    if (lane == 0)
        __hip_atomic_store(&st[bid], tag | (1ull << 30) | (unsigned)agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int ex = 0;
    for (int base = bid - 1;;) {
        const int b = base - lane;
        // below block 0 (never reached: block 0's word is inclusive) reads as an empty inclusive prefix
        const unsigned long long w =
            b >= 0 ? __hip_atomic_load(&st[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : (tag | (2ull << 30));
        const bool ready = (unsigned)(w >> 32) == epoch;
        const unsigned long long incl = __ballot(ready && ((w >> 30) & 3u) == 2u);
        const unsigned long long notReady = __ballot(!ready);
        const int l0 = incl ? __ffsll((long long)incl) - 1 : 63;
        const unsigned long long need = l0 == 63 ? ~0ull : ((1ull << (l0 + 1)) - 1);
        if (notReady & need) {
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        int v = lane <= l0 ? (int)(w & 0x3fffffffu) : 0;
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        ex += v;
        if (incl) break;
        base -= 64;
    }
    if (lane == 0)
        __hip_atomic_store(&st[bid], tag | (2ull << 30) | (unsigned)(ex + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return ex;
}

}  // namespace fm3d
