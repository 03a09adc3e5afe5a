/*
 * fm3d_cvmath.h -- OpenCV 2.4.9 core float primitives the SIFT detector / extractor calls, restated
 * once for the CPU oracle (oracle/orc_sift.c, gcc -ffp-contract=off) and the HIP kernels
 * (3dfeaturematcher_amd/csrc/fm3d_sift.hip, -ffp-contract=off), so that both evaluate the same
 * IEEE operations in the same order:
 *
 *   cv::exp(const float*, float*, n)        core/mathfuncs.cpp Exp_32f: a 64-entry 2^(k/64) table
 *                                           and a degree-4 polynomial.  An x86-64 build runs the
 *                                           SSE2 loop on the first 8*floor(n/8) elements (polynomial
 *                                           in float) and the scalar loop on the rest (polynomial in
 *                                           double): which one an element takes depends on its index
 *                                           in the array, so fm3d_cv_exp_at takes (k, n).
 *   cv::fastAtan2 (float arrays, degrees)   FastAtan2_32f: the degree-7 odd polynomial (its SSE2 and
 *                                           scalar loops compute the same float operations)
 *   cv::magnitude                           sqrt(x*x + y*y) in float (SSE2 and scalar alike)
 *   cvRound / cvFloor                       round half to even (cvtss2si / cvtsd2si), floor
 *   cosf / sinf / powf(2, y)                libm in the reference; here (float) of the deterministic
 *                                           double functions of fm3d_detmath.h (the float results
 *                                           equal glibc's wherever the double value is not within
 *                                           ~1e-9 ulp of a float rounding boundary; measured in
 *                                           tests/test_sift_oracle.py)
 *
 * The expTab values are 2^(k/64) correctly rounded to double (Python decimal, 80 digits) times
 * EXPPOLY_32F_A0 in double, which is what the compiler folds OpenCV's `2^(k/64) literal *
 * EXPPOLY_32F_A0` initialisers to.
 *
 * TEST INFRASTRUCTURE + PRODUCT: plain arithmetic shared by both sides, no oracle logic.
 */
#ifndef FM3D_CVMATH_H
#define FM3D_CVMATH_H

#include "fm3d_detmath.h"

#if defined(__HIPCC__)
#define FM3D_CVC __device__ __constant__ static const
#define FM3D_RINTF(v) __builtin_rintf(v)
#define FM3D_RINT(v) __builtin_rint(v)
#else
#define FM3D_CVC static const
#define FM3D_RINTF(v) rintf(v)
#define FM3D_RINT(v) rint(v)
#endif

#define FM3D_EXPTAB_SCALE 6
#define FM3D_EXPTAB_MASK 63
#define FM3D_EXPPOLY_32F_A0 .9670371139572337719125840413672004409288e-2
#define FM3D_EXP_PRESCALE (1.4426950408889634073599246810019 * (1 << FM3D_EXPTAB_SCALE))
#define FM3D_EXP_POSTSCALE (1. / (1 << FM3D_EXPTAB_SCALE))
#define FM3D_EXP_MAX_VAL (3000. * (1 << FM3D_EXPTAB_SCALE))
#define FM3D_EXP_A4 ((float)(1.000000000000002438532970795181890933776 / FM3D_EXPPOLY_32F_A0))
#define FM3D_EXP_A3 ((float)(.6931471805521448196800669615864773144641 / FM3D_EXPPOLY_32F_A0))
#define FM3D_EXP_A2 ((float)(.2402265109513301490103372422686535526573 / FM3D_EXPPOLY_32F_A0))
#define FM3D_EXP_A1 ((float)(.5550339366753125211915322047004666939128e-1 / FM3D_EXPPOLY_32F_A0))

/* expTab[k] = 2^(k/64) * EXPPOLY_32F_A0 */
FM3D_CVC double fm3d_cv_exptab[64] = {
    0x1.3ce0f3e46f431p-7, 0x1.40544d4d75547p-7, 0x1.43d1453011896p-7, 0x1.4757f65ccd1f0p-7,
    0x1.4ae87beef14bap-7, 0x1.4e82f14d579f8p-7, 0x1.5227722b3ca9dp-7, 0x1.55d61a8914e9dp-7,
    0x1.598f06b56410cp-7, 0x1.5d52534d969c3p-7, 0x1.61201d3eddcf1p-7, 0x1.64f881c70e0fbp-7,
    0x1.68db9e757fb1ap-7, 0x1.6cc9912bf2329p-7, 0x1.70c2781f71f03p-7, 0x1.74c671d9405eep-7,
    0x1.78d59d37bec71p-7, 0x1.7cf0196f5b91cp-7, 0x1.8116060b822a4p-7, 0x1.854782ef8d7c0p-7,
    0x1.8984b057bd157p-7, 0x1.8dcdaeda2cf5ap-7, 0x1.92229f67d00c5p-7, 0x1.9683a34d6d757p-7,
    0x1.9af0dc34a0755p-7, 0x1.9f6a6c24db3f1p-7, 0x1.a3f075846c8c7p-7, 0x1.a8831b19880ecp-7,
    0x1.ad22800b51c0fp-7, 0x1.b1cec7e2ec22bp-7, 0x1.b688168c89657p-7, 0x1.bb4e90587f922p-7,
    0x1.c02259fc5fb16p-7, 0x1.c50398940ffd7p-7, 0x1.c9f271a2e9275p-7, 0x1.ceef0b14d6b67p-7,
    0x1.d3f98b3f7a8ccp-7, 0x1.d91218e353972p-7, 0x1.de38db2ce7b3ep-7, 0x1.e36df9b5f0d69p-7,
    0x1.e8b19c868d747p-7, 0x1.ee03ec1674412p-7, 0x1.f365114e2b44dp-7, 0x1.f8d535884255fp-7,
    0x1.fe54829290ff9p-7, 0x1.01f19157bbef2p-6, 0x1.04c0a04b92bdfp-6, 0x1.079783bc6f5adp-6,
    0x1.0a76517e255b1p-6, 0x1.0d5d1fa16145cp-6, 0x1.104c047452330p-6, 0x1.1343168355441p-6,
    0x1.16426c99a2f97p-6, 0x1.194a1dc1fe6bep-6, 0x1.1c5a4147666e5p-6, 0x1.1f72eeb5c89d0p-6,
    0x1.22943ddab6608p-6, 0x1.25be46c61be8ep-6, 0x1.28f121caf926dp-6, 0x1.2c2ce7801cc88p-6,
    0x1.2f71b0c0e1405p-6, 0x1.32bf96adebd97p-6, 0x1.3616b2adede21p-6, 0x1.39771e6e67ef9p-6,
};

FM3D_HD float fm3d_cv_bits2f(unsigned u)
{
    union {
        unsigned u;
        float f;
    } c;
    c.u = u;
    return c.f;
}

FM3D_HD unsigned fm3d_cv_f2bits(float f)
{
    union {
        unsigned u;
        float f;
    } c;
    c.f = f;
    return c.u;
}

/* cvRound(float) / cvRound(double): round half to even */
FM3D_HD int fm3d_cv_roundf(float v) { return (int)FM3D_RINTF(v); }
FM3D_HD int fm3d_cv_round(double v) { return (int)FM3D_RINT(v); }
FM3D_HD int fm3d_cv_floorf(float v) { return (int)floorf(v); }

/* Exp_32f, one lane of the SSE2 loop: the argument clamped in float, scaled and rounded in double,
   the fraction back to float, the table entry to float times 2^e built in the exponent bits
   (16-bit saturating pack, >> 6, + 127, clamped to [0, 255]), the polynomial in float */
FM3D_HD float fm3d_cv_exp_sse(float x)
{
    const float maxv = (float)(FM3D_EXP_MAX_VAL / FM3D_EXP_PRESCALE);
    const float minv = (float)(-FM3D_EXP_MAX_VAL / FM3D_EXP_PRESCALE);
    float xf = x < minv ? minv : x; /* _mm_max_ps(x, minval) */
    double xd;
    int xi, e, idx;
    float yf, z;
    xf = xf > maxv ? maxv : xf;     /* _mm_min_ps(., maxval) */
    xd = (double)xf * FM3D_EXP_PRESCALE;
    xi = (int)FM3D_RINT(xd);        /* _mm_cvtpd_epi32 */
    xd = xd - (double)xi;
    xf = (float)xd * (float)FM3D_EXP_POSTSCALE;
    xi = xi < -32768 ? -32768 : (xi > 32767 ? 32767 : xi); /* _mm_packs_epi32 */
    idx = xi & FM3D_EXPTAB_MASK;
    e = (xi >> FM3D_EXPTAB_SCALE) + 127;
    e = e < 0 ? 0 : (e > 255 ? 255 : e);
    yf = (float)fm3d_cv_exptab[idx] * fm3d_cv_bits2f((unsigned)e << 23);
    z = xf + FM3D_EXP_A1;
    z = z * xf + FM3D_EXP_A2;
    z = z * xf + FM3D_EXP_A3;
    z = z * xf + FM3D_EXP_A4;
    return z * yf;
}

/* Exp_32f, the scalar loops: in double, exponents >= 2^11 mapped to +-exp_max_val */
FM3D_HD float fm3d_cv_exp_scalar(float x)
{
    const unsigned b = fm3d_cv_f2bits(x);
    double x0 = (double)x * FM3D_EXP_PRESCALE;
    int val0, t;
    if (((b >> 23) & 255) > 127 + 10) x0 = (b >> 31) ? -FM3D_EXP_MAX_VAL : FM3D_EXP_MAX_VAL;
    val0 = (int)FM3D_RINT(x0);
    t = (val0 >> FM3D_EXPTAB_SCALE) + 127;
    t = !(t & ~255) ? t : (t < 0 ? 0 : 255);
    x0 = (x0 - val0) * FM3D_EXP_POSTSCALE;
    return (float)((double)fm3d_cv_bits2f((unsigned)t << 23) * fm3d_cv_exptab[val0 & FM3D_EXPTAB_MASK] *
                   ((((x0 + (double)FM3D_EXP_A1) * x0 + (double)FM3D_EXP_A2) * x0 + (double)FM3D_EXP_A3) * x0 +
                    (double)FM3D_EXP_A4));
}

/* element k of cv::exp over an array of n floats */
FM3D_HD float fm3d_cv_exp_at(float x, int k, int n)
{
    return (n >= 8 && k < (n & ~7)) ? fm3d_cv_exp_sse(x) : fm3d_cv_exp_scalar(x);
}

/* fastAtan2 in degrees, [0, 360) */
#define FM3D_ATAN2_P1 (0.9997878412794807f * (float)(180 / 3.141592653589793238462643383279502884))
#define FM3D_ATAN2_P3 (-0.3258083974640975f * (float)(180 / 3.141592653589793238462643383279502884))
#define FM3D_ATAN2_P5 (0.1555786518463281f * (float)(180 / 3.141592653589793238462643383279502884))
#define FM3D_ATAN2_P7 (-0.04432655554792128f * (float)(180 / 3.141592653589793238462643383279502884))
FM3D_HD float fm3d_cv_atan2_deg(float y, float x)
{
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)2.2204460492503131e-16);
        c2 = c * c;
        a = (((FM3D_ATAN2_P7 * c2 + FM3D_ATAN2_P5) * c2 + FM3D_ATAN2_P3) * c2 + FM3D_ATAN2_P1) * c;
    } else {
        c = ax / (ay + (float)2.2204460492503131e-16);
        c2 = c * c;
        a = 90.f - (((FM3D_ATAN2_P7 * c2 + FM3D_ATAN2_P5) * c2 + FM3D_ATAN2_P3) * c2 + FM3D_ATAN2_P1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

/* the reference's cosf / sinf / powf(2.f, y), deterministic */
FM3D_HD float fm3d_cv_cosf(float x) { return (float)fm3d_cos((double)x); }
FM3D_HD float fm3d_cv_sinf(float x) { return (float)fm3d_sin((double)x); }
/* atan2f (FREAK's orientation): the float of the deterministic double atan2 */
FM3D_HD float fm3d_cv_atan2f(float y, float x) { return (float)fm3d_atan2((double)y, (double)x); }
FM3D_HD float fm3d_cv_exp2f(float y)
{
    const float k = floorf(y);
    const double f = (double)(y - k); /* exact */
    return (float)ldexp(fm3d_exp(f * 0.69314718055994530942), (int)k);
}

/* borderInterpolate(p, len, BORDER_REFLECT_101) */
FM3D_HD int fm3d_cv_reflect101(int p, int len)
{
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0)
            p = -p;
        else
            p = len - 1 - (p - len) - 1;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

#endif /* FM3D_CVMATH_H */
