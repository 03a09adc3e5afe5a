// fm3d_fastdiv.h -- divisions with IEEE results at fewer VALU instructions (gfx950).
//
// The compiler's fp64 division is v_div_scale x2, v_rcp, two Newton steps, a multiply,
// one Markstein correction, v_div_fmas and v_div_fixup (11 instructions).  Where the
// operands need no scaling and no special-case fix-up, the same steps without
// v_div_scale / v_div_fmas / v_div_fixup produce the same bits; outside the guarded
// ranges these helpers fall back to the division operator.  tools/micro/div_check.hip
// compares every helper with the division operator on random operands.
#pragma once
#include <hip/hip_runtime.h>

namespace fm3d {

// a / d with y = RN(1/d) precomputed (pass-uniform d): q0 = RN(a*y) is within one ulp of
// a/d, and one Markstein step q0 + (a - d*q0)*y (residual exact by FMA) rounds correctly.
// mok (pass-uniform) requires 1e-200 < |d| < 1e200; |a| < 1e100 keeps the quotient normal
// for the operands the LM passes divide (|a| is 0 or above 1e-60: products of float
// intensity differences and O(1) weights).  a = -0 with d > 0 gives +0 (IEEE: -0); the
// passes never divide -0: their numerators are differences, +0 when the operands are equal.
// The fast sequence runs on every lane; the division operator only on the lanes outside the
// guard, inside a branch taken when any lane of the wave is (rare): no exec-mask juggling on
// the common path.
__device__ __forceinline__ double mdiv(double a, double d, double y, bool mok) {
    const double q0 = a * y;
    const double r = __builtin_fma(-d, q0, a);
    double q = __builtin_fma(r, y, q0);
    const bool ok = mok && fabs(a) < 1e100;
    if (__builtin_expect(__ballot(!ok) != 0, 0)) {
        if (!ok) q = a / d;
    }
    return q;
}
// the same sequence without the guard: for callers that have bounded |a| < 1e100 and checked
// mdiv_ok(d) for the whole pass
__device__ __forceinline__ double mdiv_fast(double a, double d, double y) {
    const double q0 = a * y;
    const double r = __builtin_fma(-d, q0, a);
    return __builtin_fma(r, y, q0);
}
__device__ __forceinline__ bool mdiv_ok(double d) { return fabs(d) > 1e-200 && fabs(d) < 1e200; }

// z ? 1/z : 1 (cvProjectPoints2).  For 2^-700 <= |z| <= 2^700 the hardware sequence
// scales nothing (exponent gap < 768, 1/z normal) and fixes nothing up.  recip_z_lo
// tests only the lower bound: for plane points inside the bounding box |z| is far below
// 2^700, and the other entries do not use the value.
__device__ __forceinline__ double recip_fast(double z) {
    double r = __builtin_amdgcn_rcp(z);
    double e = __builtin_fma(-z, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-z, r, 1.0);
    r = __builtin_fma(r, e, r);
    const double rem = __builtin_fma(-z, r, 1.0);
    return __builtin_fma(rem, r, r);
}
__device__ __forceinline__ double recip_z(double z) {
    const double az = fabs(z);
    if (az >= 0x1p-700 && az <= 0x1p700) return recip_fast(z);
    return z ? 1. / z : 1.;
}
__device__ __forceinline__ double recip_z_lo(double z) {
    double q = recip_fast(z);
    const bool ok = fabs(z) >= 0x1p-700;
    if (__builtin_expect(__ballot(!ok) != 0, 0)) {
        if (!ok) q = z ? 1. / z : 1.;
    }
    return q;
}

// mm / nn with a numerator in [2^-600, 2^60] (mok = div_nn_ok(mm), pass-uniform) and
// |nn| <= 2^60 (a unit normal times a ray (x, y, 1) of bounded x, y).  The sequence
// scales nothing unless |nn| < 2^-600, and the exponent gap reaches 768, or nn is
// denormal, only when |mm / nn| > 2^400.  So the result equals mm / nn whenever
// |mm / nn| < 2^100, and is NaN or at least 2^100 in magnitude otherwise: the ray-plane
// point falls outside the bounding box (|P| < 4) exactly when it does for the IEEE quotient.
__device__ __forceinline__ bool div_nn_ok(double mm) { return fabs(mm) >= 0x1p-600 && fabs(mm) <= 0x1p60; }
__device__ __forceinline__ double div_nn(double mm, double nn, bool mok) {
    if (mok) {
        double r = __builtin_amdgcn_rcp(nn);
        double e = __builtin_fma(-nn, r, 1.0);
        r = __builtin_fma(r, e, r);
        e = __builtin_fma(-nn, r, 1.0);
        r = __builtin_fma(r, e, r);
        const double q = mm * r;
        const double rem = __builtin_fma(-nn, q, mm);
        return __builtin_fma(rem, r, q);
    }
    return mm / nn;
}

}  // namespace fm3d
