/*
 * fm3d_crmath.h -- correctly rounded sin / cos / atan2 / exp for the LM path.
 *
 * The reference evaluates sph2car / car2sph (tools.cpp:767-777) and the exp() penalty weight
 * (normaloptimizer.cpp:131-142) with the host libm.  The LM decides its steps at rounding-noise
 * level, so every last-bit difference of these functions can move a trajectory
 * (DESIGN.md §4).  Measured on the LM's arguments (tools/full_parity.py, profiles/r05_*):
 * this image's glibc 2.35 returns the correctly rounded double on ~99.8 % of them; the 1-ulp
 * polynomials of fm3d_detmath.h on only 80-90 %.  The functions here evaluate in double-double
 * arithmetic (error below 2^-90 relative, so a misrounding needs the true value within 2^-37 ulp
 * of a rounding boundary) and round once: the correctly rounded result for all practical
 * purposes, and therefore glibc's result wherever glibc is correctly rounded.
 *
 * Only IEEE +, -, *, /, floor, ldexp and sqrt, every operation order written out (the
 * products are exact through Veltkamp/Dekker splitting, no FMA), so the HIP kernels
 * (-ffp-contract=off) and the oracle (gcc -ffp-contract=off) produce the same bits.
 * Arguments beyond the double-double reductions' range (|x| >= 2^19 for sin/cos) take the
 * fm3d_detmath.h functions.  Plain C99 + HIP.
 */
#ifndef FM3D_CRMATH_H
#define FM3D_CRMATH_H

#include "fm3d_detmath.h"

typedef struct {
    double hi, lo;
} fm3d_dd;

FM3D_HD fm3d_dd fm3d_dd_make(double hi, double lo)
{
    fm3d_dd r;
    r.hi = hi;
    r.lo = lo;
    return r;
}
/* a + b exactly (Knuth) */
FM3D_HD fm3d_dd fm3d_two_sum(double a, double b)
{
    double s = a + b, bb = s - a;
    return fm3d_dd_make(s, (a - (s - bb)) + (b - bb));
}
/* a + b exactly when |a| >= |b| (Dekker) */
FM3D_HD fm3d_dd fm3d_quick_two_sum(double a, double b)
{
    double s = a + b;
    return fm3d_dd_make(s, b - (s - a));
}
/* a * b exactly (Dekker; |a|, |b| < 2^995) */
FM3D_HD fm3d_dd fm3d_two_prod(double a, double b)
{
    double p = a * b, t, ah, al, bh, bl;
    t = 134217729.0 * a;
    ah = t - (t - a);
    al = a - ah;
    t = 134217729.0 * b;
    bh = t - (t - b);
    bl = b - bh;
    return fm3d_dd_make(p, ((ah * bh - p) + ah * bl + al * bh) + al * bl);
}
FM3D_HD fm3d_dd fm3d_dd_add(fm3d_dd a, fm3d_dd b)
{
    fm3d_dd s = fm3d_two_sum(a.hi, b.hi), t = fm3d_two_sum(a.lo, b.lo);
    s.lo += t.hi;
    s = fm3d_quick_two_sum(s.hi, s.lo);
    s.lo += t.lo;
    return fm3d_quick_two_sum(s.hi, s.lo);
}
FM3D_HD fm3d_dd fm3d_dd_neg(fm3d_dd a) { return fm3d_dd_make(-a.hi, -a.lo); }
FM3D_HD fm3d_dd fm3d_dd_sub(fm3d_dd a, fm3d_dd b) { return fm3d_dd_add(a, fm3d_dd_neg(b)); }
FM3D_HD fm3d_dd fm3d_dd_add_d(fm3d_dd a, double b)
{
    fm3d_dd s = fm3d_two_sum(a.hi, b);
    s.lo += a.lo;
    return fm3d_quick_two_sum(s.hi, s.lo);
}
FM3D_HD fm3d_dd fm3d_dd_mul(fm3d_dd a, fm3d_dd b)
{
    fm3d_dd p = fm3d_two_prod(a.hi, b.hi);
    p.lo += a.hi * b.lo + a.lo * b.hi;
    return fm3d_quick_two_sum(p.hi, p.lo);
}
FM3D_HD fm3d_dd fm3d_dd_mul_d(fm3d_dd a, double b)
{
    fm3d_dd p = fm3d_two_prod(a.hi, b);
    p.lo += a.lo * b;
    return fm3d_quick_two_sum(p.hi, p.lo);
}
FM3D_HD fm3d_dd fm3d_dd_div(fm3d_dd a, fm3d_dd b)
{
    double q1 = a.hi / b.hi, q2, q3;
    fm3d_dd r = fm3d_dd_sub(a, fm3d_dd_mul_d(b, q1));
    q2 = r.hi / b.hi;
    r = fm3d_dd_sub(r, fm3d_dd_mul_d(b, q2));
    q3 = r.hi / b.hi;
    return fm3d_dd_add_d(fm3d_quick_two_sum(q1, q2), q3);
}
/* the double nearest the double-double value (a normalised pair: hi is already RN(hi + lo)) */
FM3D_HD double fm3d_dd_round(fm3d_dd a) { return a.hi + a.lo; }

/* pi/2 = FM3D_CR_P1 + FM3D_CR_P2 + FM3D_CR_P3 + O(1e-37): 33 + 33 + 53 bits (k*P1, k*P2 exact for
   |k| < 2^20) */
#define FM3D_CR_P1 1.5707963267341256
#define FM3D_CR_P2 6.077100506303966e-11
#define FM3D_CR_P3 2.0222662487959506e-21
#define FM3D_CR_RANGE 524288.0 /* 2^19 */

/* x - k*pi/2 as a double-double, k = nearest integer of x*2/pi, *q = k mod 4 */
FM3D_HD fm3d_dd fm3d_cr_reduce(double x, int *q)
{
    double k = floor(x * FM3D_TWO_OVER_PI + 0.5), km;
    fm3d_dd r = fm3d_two_sum(x, -(k * FM3D_CR_P1));
    r = fm3d_dd_add_d(r, -(k * FM3D_CR_P2));
    r = fm3d_dd_sub(r, fm3d_two_prod(k, FM3D_CR_P3));
    km = k - 4.0 * floor(k * 0.25);
    *q = (int)km;
    return r;
}
/* sin(r) for |r| <= pi/4 (+ the rounding slack of the reduction): r + r^3 P(r^2), Taylor terms
   through r^23; the first six coefficients double-double, the rest double (their rounding
   errors stay below 2^-80 of the result) */
FM3D_HD fm3d_dd fm3d_cr_sin_kernel(fm3d_dd r)
{
    static const double S[12][2] = {
        {-0.16666666666666666, -9.25185853854297e-18},   {0.008333333333333333, 1.1564823173178714e-19},
        {-0.0001984126984126984, -1.7209558293420705e-22}, {2.7557319223985893e-06, -1.858393274046472e-22},
        {-2.505210838544172e-08, 1.448814070935912e-24},  {1.6059043836821613e-10, 1.2585294588752098e-26},
        {-7.647163731819816e-13, 0},                      {2.8114572543455206e-15, 0},
        {-8.22063524662433e-18, 0},                       {1.9572941063391263e-20, 0},
        {-3.868170170630684e-23, 0},                      {6.446950284384474e-26, 0}};
    fm3d_dd r2 = fm3d_dd_mul(r, r), P;
    double p = S[11][0];
    int n;
    for (n = 10; n >= 6; n--) p = S[n][0] + r2.hi * p;
    P = fm3d_dd_make(p, 0.);
    for (n = 5; n >= 0; n--) P = fm3d_dd_add(fm3d_dd_make(S[n][0], S[n][1]), fm3d_dd_mul(r2, P));
    return fm3d_dd_add(r, fm3d_dd_mul(fm3d_dd_mul(r, r2), P));
}
/* cos(r) for |r| <= pi/4: 1 + r^2 Q(r^2), Taylor terms through r^24 */
FM3D_HD fm3d_dd fm3d_cr_cos_kernel(fm3d_dd r)
{
    static const double C[12][2] = {
        {-0.5, 0},                                         {0.041666666666666664, 2.3129646346357427e-18},
        {-0.001388888888888889, 5.300543954373577e-20},    {2.48015873015873e-05, 2.1511947866775882e-23},
        {-2.755731922398589e-07, -2.3767714622250297e-23}, {2.08767569878681e-09, -1.20734505911326e-25},
        {-1.1470745597729725e-11, 0},                      {4.779477332387385e-14, 0},
        {-1.5619206968586225e-16, 0},                      {4.110317623312165e-19, 0},
        {-8.896791392450574e-22, 0},                       {1.6117375710961184e-24, 0}};
    fm3d_dd r2 = fm3d_dd_mul(r, r), Q;
    double p = C[11][0];
    int n;
    for (n = 10; n >= 6; n--) p = C[n][0] + r2.hi * p;
    Q = fm3d_dd_make(p, 0.);
    for (n = 5; n >= 0; n--) Q = fm3d_dd_add(fm3d_dd_make(C[n][0], C[n][1]), fm3d_dd_mul(r2, Q));
    return fm3d_dd_add_d(fm3d_dd_mul(r2, Q), 1.0);
}

FM3D_HD double fm3d_sin_cr(double x)
{
    int q;
    fm3d_dd r, v;
    if (!(fabs(x) < FM3D_CR_RANGE)) return fm3d_sin(x); /* NaN, infinities, huge arguments */
    if (x == 0.0) return x;                              /* +-0 */
    r = fm3d_cr_reduce(x, &q);
    v = (q & 1) ? fm3d_cr_cos_kernel(r) : fm3d_cr_sin_kernel(r);
    if (q & 2) v = fm3d_dd_neg(v);
    return fm3d_dd_round(v);
}
FM3D_HD double fm3d_cos_cr(double x)
{
    int q;
    fm3d_dd r, v;
    if (!(fabs(x) < FM3D_CR_RANGE)) return fm3d_cos(x);
    r = fm3d_cr_reduce(x, &q);
    v = (q & 1) ? fm3d_cr_sin_kernel(r) : fm3d_cr_cos_kernel(r);
    if (q == 1 || q == 2) v = fm3d_dd_neg(v);
    return fm3d_dd_round(v);
}

/* fm3d_sin_cr(x) (cosine 0) or fm3d_cos_cr(x) (cosine 1), the same operations and so the same bits:
   cos(x) = sin(x + pi/2) takes the quadrant q + 1 of the same reduction.  For a wave whose lanes
   compute different ones side by side (the LM kernel's sph2car of an evaluation: four lanes) */
FM3D_HD double fm3d_sincos_sel_cr(double x, int cosine)
{
    int q;
    fm3d_dd r, v;
    if (!(fabs(x) < FM3D_CR_RANGE)) return cosine ? fm3d_cos(x) : fm3d_sin(x);
    if (!cosine && x == 0.0) return x;
    r = fm3d_cr_reduce(x, &q);
    q += cosine;
    v = (q & 1) ? fm3d_cr_cos_kernel(r) : fm3d_cr_sin_kernel(r);
    if (q & 2) v = fm3d_dd_neg(v);
    return fm3d_dd_round(v);
}

/* atan(t) for a double-double t in [0, 1]: atan(c) + atan((t - c) / (1 + t c)), c = j/16 the
   nearest sixteenth (|u| <= 1/32), the series through u^19 (double-double through u^5) */
FM3D_HD fm3d_dd fm3d_cr_atan01(fm3d_dd t)
{
    static const double A[17][2] = {
        {0, 0},
        {0.06241880999595735, -1.5490756308295046e-18}, {0.12435499454676144, -3.1253241424539383e-18},
        {0.18534794999569476, 4.180692268843079e-18},   {0.24497866312686414, 1.0698755618734451e-17},
        {0.3028848683749714, -1.1010827903001369e-17},  {0.35877067027057225, -2.4623815582638635e-17},
        {0.4124104415973873, -1.587652227770689e-17},   {0.4636476090008061, 2.2698777452961687e-17},
        {0.5123894603107377, -2.5462781472855804e-17},  {0.5585993153435624, -5.4556305485916264e-18},
        {0.6022873461349642, 2.950430737228402e-17},    {0.6435011087932844, 1.5834785051444286e-17},
        {0.6823165548747481, 6.943223671560008e-18},    {0.7188299996216245, -2.1478388444456983e-17},
        {0.7531512809621944, -2.4256934659182068e-17},  {0.7853981633974483, 3.061616997868383e-17}};
    static const double T[9][2] = {
        {-0.3333333333333333, -1.850371707708594e-17}, {0.2, -1.1102230246251566e-17},
        {-0.14285714285714285, 0}, {0.1111111111111111, 0}, {-0.09090909090909091, 0},
        {0.07692307692307693, 0}, {-0.06666666666666667, 0}, {0.058823529411764705, 0},
        {-0.05263157894736842, 0}};
    double c, p;
    int j = (int)floor(t.hi * 16.0 + 0.5), n;
    fm3d_dd u, u2, P;
    if (j > 16) j = 16;
    c = (double)j * 0.0625;
    u = j ? fm3d_dd_div(fm3d_dd_add_d(t, -c), fm3d_dd_add_d(fm3d_dd_mul_d(t, c), 1.0)) : t;
    u2 = fm3d_dd_mul(u, u);
    p = T[8][0];
    for (n = 7; n >= 2; n--) p = T[n][0] + u2.hi * p;
    P = fm3d_dd_make(p, 0.);
    for (n = 1; n >= 0; n--) P = fm3d_dd_add(fm3d_dd_make(T[n][0], T[n][1]), fm3d_dd_mul(u2, P));
    return fm3d_dd_add(fm3d_dd_make(A[j][0], A[j][1]), fm3d_dd_add(u, fm3d_dd_mul(fm3d_dd_mul(u, u2), P)));
}

FM3D_HD double fm3d_atan2_cr(double y, double x)
{
    double ax, ay;
    fm3d_dd a;
    if (x != x || y != y) return x + y;
    ax = fabs(x);
    ay = fabs(y);
    /* zeros and infinities: fm3d_detmath.h's exact special values */
    if (ay == 0.0 || ax == 0.0 || ax - ax != 0.0 || ay - ay != 0.0) return fm3d_atan2(y, x);
    if (ay <= ax) {
        a = fm3d_cr_atan01(fm3d_dd_div(fm3d_dd_make(ay, 0.), fm3d_dd_make(ax, 0.)));
    } else {
        a = fm3d_dd_sub(fm3d_dd_make(FM3D_PIO2_HI, FM3D_PIO2_LO),
                        fm3d_cr_atan01(fm3d_dd_div(fm3d_dd_make(ax, 0.), fm3d_dd_make(ay, 0.))));
    }
    if (x < 0.0) a = fm3d_dd_sub(fm3d_dd_make(FM3D_PI_HI, FM3D_PI_LO), a);
    return y < 0.0 ? -fm3d_dd_round(a) : fm3d_dd_round(a);
}

/* ln 2 = FM3D_CR_L1 + FM3D_CR_L2 + O(2e-31); L1 has 40 bits (k * L1 exact for |k| < 2^13) */
#define FM3D_CR_L1 0.6931471805601177
#define FM3D_CR_L2 -1.7239444525614835e-13

/* exp(x) = 2^k e^r, r = x - k ln 2; e^r = (1 + e(s))^256, s = r / 256, e(s) = expm1(s) by its
   series through s^9, then eight exact-form squarings e <- 2e + e^2 (double-double) */
FM3D_HD double fm3d_exp_cr(double x)
{
    static const double E[8][2] = {
        {0.5, 0}, {0.16666666666666666, 9.25185853854297e-18}, {0.041666666666666664, 2.3129646346357427e-18},
        {0.008333333333333333, 0}, {0.001388888888888889, 0}, {0.0001984126984126984, 0},
        {2.48015873015873e-05, 0}, {2.7557319223985893e-06, 0}};
    double k, p;
    fm3d_dd r, s, e, P;
    int n;
    if (x != x) return x;
    if (x > 709.782712893384 || x < -708.0) return fm3d_exp(x); /* overflow, subnormal results */
    k = floor(x * FM3D_INV_LN2 + 0.5);
    r = fm3d_two_sum(x, -(k * FM3D_CR_L1));
    r = fm3d_dd_sub(r, fm3d_two_prod(k, FM3D_CR_L2));
    s = fm3d_dd_make(r.hi * (1.0 / 256.0), r.lo * (1.0 / 256.0));
    p = E[7][0];
    for (n = 6; n >= 3; n--) p = E[n][0] + s.hi * p;
    P = fm3d_dd_make(p, 0.);
    for (n = 2; n >= 0; n--) P = fm3d_dd_add(fm3d_dd_make(E[n][0], E[n][1]), fm3d_dd_mul(s, P));
    e = fm3d_dd_add(s, fm3d_dd_mul(fm3d_dd_mul(s, s), P));
    for (n = 0; n < 8; n++) e = fm3d_dd_add(fm3d_dd_make(2.0 * e.hi, 2.0 * e.lo), fm3d_dd_mul(e, e));
    e = fm3d_dd_add_d(e, 1.0);
    return ldexp(fm3d_dd_round(e), (int)k);
}

/* hypot(x, y), the function OpenCV 2.4's JacobiSVDImpl_ forms each rotation with
   (include/fm3d_cvsvd.h).  x^2 + y^2 in double-double (exact products, one double-double add:
   relative error below 2^-104), r = sqrt of its high part (correctly rounded), one Newton correction
   (s - r^2) / 2r from the double-double residual, rounded once: correctly rounded unless the exact
   value lies within ~2^-50 ulp of a rounding boundary (tests/test_crmath.py: every case of its
   random and hard-case sets equals mpmath's).  |y| <= 2^-60 |x| returns |x|, which is the correctly
   rounded value there. */
FM3D_HD double fm3d_hypot_cr(double x, double y)
{
    double ax = fabs(x), ay = fabs(y), t, r, c;
    int e = 0;
    fm3d_dd s, d;
    if (ax == INFINITY || ay == INFINITY) return INFINITY;
    if (ax != ax || ay != ay) return ax + ay;
    if (ax < ay) {
        t = ax;
        ax = ay;
        ay = t;
    }
    if (ay <= ax * 0x1p-60) return ax;
    if (ax > 0x1p+500) {
        ax *= 0x1p-600;
        ay *= 0x1p-600;
        e = 600;
    } else if (ax < 0x1p-500) {
        ax *= 0x1p+600;
        ay *= 0x1p+600;
        e = -600;
    }
    s = fm3d_dd_add(fm3d_two_prod(ax, ax), fm3d_two_prod(ay, ay));
    r = sqrt(s.hi);
    d = fm3d_dd_sub(s, fm3d_two_prod(r, r));
    c = d.hi / (2.0 * r);
    return e ? ldexp(r + c, e) : r + c;
}

#endif /* FM3D_CRMATH_H */
