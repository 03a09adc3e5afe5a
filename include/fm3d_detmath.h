/*
 * fm3d_detmath.h -- deterministic double-precision transcendentals.
 *
 * The LM normal optimiser evaluates sph2car / car2sph (tools.cpp:767-777 of the
 * reference) and the exp() penalty weight (normaloptimizer.cpp:131-142) on every
 * residual evaluation.  glibc and the ROCm device library (ocml) may round these
 * differently in the last bit, which would make a bitwise GPU-vs-CPU comparison
 * of the LM trajectory impossible.  This header defines one implementation that
 * uses only IEEE +,-,*,/ , floor, ldexp and sqrt, with every operation order
 * written out, so that:
 *   - the HIP kernels (compiled with -ffp-contract=off), and
 *   - the oracle's "canonical" mode (compiled with gcc -ffp-contract=off)
 * produce bit-identical results.  Accuracy is ~1 ulp over the ranges the LM
 * sees; the oracle's "strict" mode keeps using libm, and the two are compared
 * at the north_star tolerance.
 *
 * Plain C99 + HIP: no overloading, no C++ features.
 */
#ifndef FM3D_DETMATH_H
#define FM3D_DETMATH_H

#include <math.h>

#if defined(__HIPCC__)
#define FM3D_HD __host__ __device__ static inline
#else
#define FM3D_HD static inline
#endif

/* pi/2 split in three parts (33 + 33 + 53 bits) for Cody-Waite reduction */
#define FM3D_PIO2_1 1.5707963267341256
#define FM3D_PIO2_2 6.077100506303966e-11
#define FM3D_PIO2_3 2.0222662487959506e-21
#define FM3D_TWO_OVER_PI 0.6366197723675814
#define FM3D_PIO2_HI 1.5707963267948966
#define FM3D_PIO2_LO 6.123233995736766e-17
#define FM3D_PI_HI 3.141592653589793
#define FM3D_PI_LO 1.2246467991473532e-16
#define FM3D_LN2_HI 0.6931471803691238
#define FM3D_LN2_LO 1.9082149292705877e-10
#define FM3D_INV_LN2 1.4426950408889634

/* Taylor polynomial of sin on |r| <= pi/4, terms through r^17. */
FM3D_HD double fm3d_sin_kernel(double r)
{
    double r2 = r * r;
    double p = 1.0 / 355687428096000.0;           /*  1/17! */
    p = -1.0 / 1307674368000.0 + r2 * p;          /* -1/15! */
    p = 1.0 / 6227020800.0 + r2 * p;              /*  1/13! */
    p = -1.0 / 39916800.0 + r2 * p;               /* -1/11! */
    p = 1.0 / 362880.0 + r2 * p;                  /*  1/9!  */
    p = -1.0 / 5040.0 + r2 * p;                   /* -1/7!  */
    p = 1.0 / 120.0 + r2 * p;                     /*  1/5!  */
    p = -1.0 / 6.0 + r2 * p;                      /* -1/3!  */
    return r + (r * r2) * p;
}

/* Taylor polynomial of cos on |r| <= pi/4, terms through r^18. */
FM3D_HD double fm3d_cos_kernel(double r)
{
    double r2 = r * r;
    double p = -1.0 / 6402373705728000.0;         /* -1/18! */
    p = 1.0 / 20922789888000.0 + r2 * p;          /*  1/16! */
    p = -1.0 / 87178291200.0 + r2 * p;            /* -1/14! */
    p = 1.0 / 479001600.0 + r2 * p;               /*  1/12! */
    p = -1.0 / 3628800.0 + r2 * p;                /* -1/10! */
    p = 1.0 / 40320.0 + r2 * p;                   /*  1/8!  */
    p = -1.0 / 720.0 + r2 * p;                    /* -1/6!  */
    p = 1.0 / 24.0 + r2 * p;                      /*  1/4!  */
    p = -0.5 + r2 * p;                            /* -1/2!  */
    return 1.0 + r2 * p;
}

/* reduce x to r in [-pi/4, pi/4] and quadrant q = k mod 4 */
FM3D_HD double fm3d_reduce_pio2(double x, int *q)
{
    double k = floor(x * FM3D_TWO_OVER_PI + 0.5);
    double r = ((x - k * FM3D_PIO2_1) - k * FM3D_PIO2_2) - k * FM3D_PIO2_3;
    double km = k - 4.0 * floor(k * 0.25);        /* k mod 4 in {0,1,2,3}, exact for |k| < 2^52 */
    *q = (int)km;
    return r;
}

FM3D_HD double fm3d_sin(double x)
{
    int q;
    double r;
    if (x != x) return x;
    if (x - x != 0.0) return (x - x) / (x - x);   /* +-inf -> NaN */
    r = fm3d_reduce_pio2(x, &q);
    if (q == 0) return fm3d_sin_kernel(r);
    if (q == 1) return fm3d_cos_kernel(r);
    if (q == 2) return -fm3d_sin_kernel(r);
    return -fm3d_cos_kernel(r);
}

FM3D_HD double fm3d_cos(double x)
{
    int q;
    double r;
    if (x != x) return x;
    if (x - x != 0.0) return (x - x) / (x - x);
    r = fm3d_reduce_pio2(x, &q);
    if (q == 0) return fm3d_cos_kernel(r);
    if (q == 1) return -fm3d_sin_kernel(r);
    if (q == 2) return -fm3d_cos_kernel(r);
    return fm3d_sin_kernel(r);
}

/* atan series for |u| <= 7/16: sum_{n=0..24} (-1)^n u^(2n+1)/(2n+1) */
FM3D_HD double fm3d_atan_series(double u)
{
    double u2 = u * u;
    double p = 1.0 / 49.0;
    p = -1.0 / 47.0 + u2 * p;
    p = 1.0 / 45.0 + u2 * p;
    p = -1.0 / 43.0 + u2 * p;
    p = 1.0 / 41.0 + u2 * p;
    p = -1.0 / 39.0 + u2 * p;
    p = 1.0 / 37.0 + u2 * p;
    p = -1.0 / 35.0 + u2 * p;
    p = 1.0 / 33.0 + u2 * p;
    p = -1.0 / 31.0 + u2 * p;
    p = 1.0 / 29.0 + u2 * p;
    p = -1.0 / 27.0 + u2 * p;
    p = 1.0 / 25.0 + u2 * p;
    p = -1.0 / 23.0 + u2 * p;
    p = 1.0 / 21.0 + u2 * p;
    p = -1.0 / 19.0 + u2 * p;
    p = 1.0 / 17.0 + u2 * p;
    p = -1.0 / 15.0 + u2 * p;
    p = 1.0 / 13.0 + u2 * p;
    p = -1.0 / 11.0 + u2 * p;
    p = 1.0 / 9.0 + u2 * p;
    p = -1.0 / 7.0 + u2 * p;
    p = 1.0 / 5.0 + u2 * p;
    p = -1.0 / 3.0 + u2 * p;
    return u + (u * u2) * p;
}

/* atan(t) for t in [0, 1] */
FM3D_HD double fm3d_atan01(double t)
{
    if (t < 0.4375) return fm3d_atan_series(t);
    if (t < 0.6875) {
        double u = (t - 0.5) / (1.0 + t * 0.5);
        return 0.4636476090008061 + (2.2698777452961687e-17 + fm3d_atan_series(u));
    }
    {
        double u = (t - 1.0) / (t + 1.0);
        return 0.7853981633974483 + (3.061616997868383e-17 + fm3d_atan_series(u));
    }
}

FM3D_HD double fm3d_atan2(double y, double x)
{
    double ax, ay, a;
    if (x != x || y != y) return x + y;
    ax = fabs(x);
    ay = fabs(y);
    if (ay == 0.0) {
        if (x > 0.0 || (x == 0.0 && 1.0 / x > 0.0)) return y;          /* +-0 */
        return y < 0.0 || (y == 0.0 && 1.0 / y < 0.0) ? -FM3D_PI_HI : FM3D_PI_HI;
    }
    if (ax == 0.0) return y < 0.0 ? -FM3D_PIO2_HI : FM3D_PIO2_HI;
    if (ax - ax != 0.0 || ay - ay != 0.0) {                            /* infinities */
        if (ax - ax != 0.0 && ay - ay != 0.0)
            a = x > 0.0 ? 0.7853981633974483 : 2.356194490192345;
        else if (ax - ax != 0.0)
            a = x > 0.0 ? 0.0 : FM3D_PI_HI;
        else
            a = FM3D_PIO2_HI;
        return y < 0.0 ? -a : a;
    }
    if (ay <= ax) {
        a = fm3d_atan01(ay / ax);
    } else {
        a = FM3D_PIO2_HI - (fm3d_atan01(ax / ay) - FM3D_PIO2_LO);
    }
    if (x < 0.0) a = FM3D_PI_HI - (a - FM3D_PI_LO);
    return y < 0.0 ? -a : a;
}

/* acos(c) for c in [-1, 1] (cvRodrigues2, matrix -> vector) */
FM3D_HD double fm3d_acos(double c)
{
    return fm3d_atan2(sqrt((1.0 - c) * (1.0 + c)), c);
}

FM3D_HD double fm3d_exp(double x)
{
    double k, r, p;
    if (x != x) return x;
    if (x > 709.782712893384) return 1.0 / 0.0 * 1.0;
    if (x < -745.1332191019412) return 0.0;
    k = floor(x * FM3D_INV_LN2 + 0.5);
    r = (x - k * FM3D_LN2_HI) - k * FM3D_LN2_LO;
    p = 1.0 / 6227020800.0;                       /* 1/13! */
    p = 1.0 / 479001600.0 + r * p;
    p = 1.0 / 39916800.0 + r * p;
    p = 1.0 / 3628800.0 + r * p;
    p = 1.0 / 362880.0 + r * p;
    p = 1.0 / 40320.0 + r * p;
    p = 1.0 / 5040.0 + r * p;
    p = 1.0 / 720.0 + r * p;
    p = 1.0 / 120.0 + r * p;
    p = 1.0 / 24.0 + r * p;
    p = 1.0 / 6.0 + r * p;
    p = 0.5 + r * p;
    p = 1.0 + r * p;
    p = 1.0 + r * p;
    /* two-step scaling keeps ldexp exact for k near the over/underflow edges */
    if (k > 1000.0) return ldexp(ldexp(p, 1000), (int)k - 1000);
    if (k < -1000.0) return ldexp(ldexp(p, -1000), (int)k + 1000);
    return ldexp(p, (int)k);
}

#endif /* FM3D_DETMATH_H */
