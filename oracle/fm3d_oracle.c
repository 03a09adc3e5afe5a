/*
 * fm3d_oracle.c -- CPU ORACLE for the 3DFeatureMatcher hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * or the timed CPU baseline.  The product (3dfeaturematcher_amd/libfm3d.so)
 * never links, loads or calls it.
 *
 * It is a plain-C restatement of the reference algorithm, following the
 * reference sources (paths relative to caomw/3DFeatureMatcher):
 *   DescriptorsMatcher/descriptorsmatcher.cpp:107-131   knnMatch(k=2) + NNDR
 *   Triangulator/singlecameratriangulator.cpp:123-230   setg12, setKeypoints, triangulate
 *   Triangulator/singlecameratriangulator.cpp:341-397   extractPixelsContour
 *   Triangulator/singlecameratriangulator.cpp:421-470   projectPointToPlane
 *   Triangulator/singlecameratriangulator.cpp:530-665   get3dPoints / intensities / projection / bounds
 *   Triangulator/normaloptimizer.cpp:65-149             evaluateNormal (LM residual)
 *   Triangulator/normaloptimizer.cpp:206-292            pyramids, optimize_pyramid, optimize
 *   Triangulator/normaloptimizer.cpp:321-452            computeOptimizedNormals (erase semantics)
 *   tools.cpp:87-142, 767-777                           compose/decompose, bilinear, sph<->car
 * and the third-party arithmetic the reference calls (not vendored in the
 * reference, versions unpinned; restated from their published algorithms):
 *   OpenCV 2.4.x: undistortPoints, projectPoints, Rodrigues, triangulatePoints,
 *                 Matx44d::inv (LU), pyrDown, FLANN L2/Hamming distances
 *   lmfit ~3.x/4.0 lmmin == MINPACK lmdif/qrfac/lmpar/qrsolv with lmfit defaults
 *                 (ftol=xtol=gtol=30*DBL_EPSILON, stepbound 100, patience 100)
 *
 * Parity pinning: the reference has no tests and no golden
 * vectors, and cannot be built here (OpenCV/PCL/lmfit absent).  The oracle is
 * pinned by tests/golden fixtures produced by independent numpy/scipy code
 * (numpy brute force, numpy.linalg.svd DLT, scipy.optimize.leastsq = MINPACK
 * lmdif driving a numpy evaluateNormal).  Exact lmfit trajectories are
 * "parity unpinned".
 *
 * Two LM modes, both MINPACK lmdif with Householder qrfac and every m_dat-long
 * sum in pixel (index) order:
 *   ORC_LM_STRICT  : libm transcendentals (sin/cos/atan2/exp) -- the reference's;
 *   ORC_LM_DETMATH : the correctly rounded transcendentals of include/fm3d_crmath.h (round 5;
 *                    before, the 1-ulp polynomials of include/fm3d_detmath.h, which the NCC
 *                    hypotheses keep: ORC_DET_1ULP).
 *                    THE GPU CONTRACT: the LM kernel (csrc/fm3d_lm2.hip) equals this
 *                    mode bit for bit (statuses, lmdif info / nfev per level, normals);
 *                    STRICT is the north_star's 1e-4 comparison.
 * Compiled with -ffp-contract=off (no FMA contraction), like the kernels.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include "fm3d_detmath.h"
#include "fm3d_crmath.h"

#define ORC_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------ */
/* camera model                                                        */
/* ------------------------------------------------------------------ */
typedef struct {
    double fx, fy, cx, cy;
    double k[5]; /* OpenCV order k1,k2,p1,p2,k3 == settings k0,k1,p1,p2,k2
                    (singlecameratriangulator.cpp:99-105) */
} orc_camera;

/* cvUndistortPoints (OpenCV 2.4), 5 fixed-point iterations, R = I, P = none.
   Call sites: singlecameratriangulator.cpp:169-170 and :542. */
static void orc_undistort1(const orc_camera *c, double x, double y, double *ox, double *oy)
{
    const double *k = c->k;
    double ifx = 1. / c->fx, ify = 1. / c->fy;
    double x0, y0;
    int j;
    x0 = x = (x - c->cx) * ifx;
    y0 = y = (y - c->cy) * ify;
    for (j = 0; j < 5; j++) {
        double r2 = x * x + y * y;
        /* rational-model numerator with k5..k7 = 0 evaluates to exactly 1 */
        double icdist = (1 + ((0. * r2 + 0.) * r2 + 0.) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
        double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x);
        double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    {   /* RR = identity */
        double xx = 1. * x + 0. * y + 0.;
        double yy = 0. * x + 1. * y + 0.;
        double ww = 1. / (0. * x + 0. * y + 1.);
        *ox = xx * ww;
        *oy = yy * ww;
    }
}

/* cvProjectPoints2 (OpenCV 2.4) for one point with rotation matrix R (row-major)
   and translation t.  Call sites: singlecameratriangulator.cpp:388 (R=I,t=0) and
   :602 (R = Rodrigues(decompose(g12))). */
/* cvProjectPoints2's distortion and intrinsics of a camera-frame point (x, y, z) */
static void orc_project_xyz(const orc_camera *c, double x, double y, double z, double *u, double *v)
{
    const double *k = c->k;
    double r2, r4, r6, a1, a2, a3, cdist, icdist2, xd, yd;
    z = z ? 1. / z : 1;
    x *= z;
    y *= z;
    r2 = x * x + y * y;
    r4 = r2 * r2;
    r6 = r4 * r2;
    a1 = 2 * x * y;
    a2 = r2 + 2 * x * x;
    a3 = r2 + 2 * y * y;
    cdist = 1 + k[0] * r2 + k[1] * r4 + k[4] * r6;
    icdist2 = 1. / (1 + 0. * r2 + 0. * r4 + 0. * r6);
    xd = x * cdist * icdist2 + k[2] * a1 + k[3] * a2;
    yd = y * cdist * icdist2 + k[2] * a3 + k[3] * a1;
    *u = xd * c->fx + c->cx;
    *v = yd * c->fy + c->cy;
}

/* the NCC kernel's camera-2 projection (csrc/fm3d_ncc.hip ncc_geometry_m): orc_project_xyz with every
   product-and-sum fused (C99 fma, one rounding, as the GPU's fma) -- the NCC hypotheses are an
   extension with no reference order to keep -- and 2 k xy as (2 k) RN(xy), the same bits as k RN(2 x y) */
static void orc_ncc_project(const orc_camera *c, double x, double y, double z, double *u, double *v)
{
    const double *k = c->k;
    double r2, r4, r6, xy, a2, a3, cdist, xd, yd;
    z = z ? 1. / z : 1;
    x *= z;
    y *= z;
    r2 = x * x + y * y;
    r4 = r2 * r2;
    r6 = r4 * r2;
    xy = x * y;
    a2 = fma(x * x, 2., r2);
    a3 = fma(y * y, 2., r2);
    cdist = fma(k[4], r6, fma(k[1], r4, fma(k[0], r2, 1.)));
    xd = fma(k[3], a2, fma(2. * k[2], xy, x * cdist));
    yd = fma(2. * k[3], xy, fma(k[2], a3, y * cdist));
    *u = fma(xd, c->fx, c->cx);
    *v = fma(yd, c->fy, c->cy);
}

static void orc_project1(const orc_camera *c, const double R[9], const double t[3],
                         double X, double Y, double Z, double *u, double *v)
{
    orc_project_xyz(c, R[0] * X + R[1] * Y + R[2] * Z + t[0], R[3] * X + R[4] * Y + R[5] * Z + t[1],
                    R[6] * X + R[7] * Y + R[8] * Z + t[2], u, v);
}

ORC_API void orc_undistort(const orc_camera *c, const double *xy, int n, double *out)
{
    int i;
    for (i = 0; i < n; i++) orc_undistort1(c, xy[2 * i], xy[2 * i + 1], &out[2 * i], &out[2 * i + 1]);
}

ORC_API void orc_project(const orc_camera *c, const double R[9], const double t[3],
                         const double *P, int n, double *out)
{
    int i;
    for (i = 0; i < n; i++)
        orc_project1(c, R, t, P[3 * i], P[3 * i + 1], P[3 * i + 2], &out[2 * i], &out[2 * i + 1]);
}

/* ------------------------------------------------------------------ */
/* Rodrigues / 4x4 transforms (host-side algebra, a3)                  */
/* ------------------------------------------------------------------ */
/* cvRodrigues2 vector -> matrix */
ORC_API void orc_rodrigues_v2m(const double r[3], double R[9])
{
    double rx = r[0], ry = r[1], rz = r[2];
    double theta = sqrt(rx * rx + ry * ry + rz * rz);
    int k;
    if (theta < DBL_EPSILON) {
        for (k = 0; k < 9; k++) R[k] = (k % 4 == 0) ? 1. : 0.;
        return;
    }
    {
        const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        double c = cos(theta), s = sin(theta), c1 = 1. - c;
        double itheta = theta ? 1. / theta : 0.;
        double rrt[9], rxm[9];
        rx *= itheta; ry *= itheta; rz *= itheta;
        rrt[0] = rx * rx; rrt[1] = rx * ry; rrt[2] = rx * rz;
        rrt[3] = rx * ry; rrt[4] = ry * ry; rrt[5] = ry * rz;
        rrt[6] = rx * rz; rrt[7] = ry * rz; rrt[8] = rz * rz;
        rxm[0] = 0; rxm[1] = -rz; rxm[2] = ry;
        rxm[3] = rz; rxm[4] = 0; rxm[5] = -rx;
        rxm[6] = -ry; rxm[7] = rx; rxm[8] = 0;
        for (k = 0; k < 9; k++) R[k] = c * I[k] + c1 * rrt[k] + s * rxm[k];
    }
}

/* ------------------------------------------------------------------ */
/* OpenCV 2.4's SVD (core/src/lapack.cpp), where the hot path calls it  */
/* ------------------------------------------------------------------ */
/* cvTriangulatePoints' null vector (singlecameratriangulator.cpp:186) and cvRodrigues2's
   orthonormalisation of R (decomposeTransformation, tools.cpp:110) both run cvSVD -> cv::SVD::compute
   -> _SVDcompute -> JacobiSVD(double) = JacobiSVDImpl_<double>(..., minval = DBL_MIN,
   eps = 10 DBL_EPSILON), restated below from OpenCV 2.4.9's published source.

   Geometry switches (measurement only: tools/dlt_parity.py):
     ORC_GEOM_DLT_LEGACY   the DLT of rounds 1-5: the 4-row system (no x P.row1 - y P.row0 rows), a
                           one-sided Jacobi in round-robin pair order with its own rotation formulas
                           and a 1e-15 threshold;
     ORC_GEOM_POLAR_NEWTON the polar factor of rounds 1-5: three Newton steps X <- (X + X^-T) / 2;
     ORC_GEOM_SVD_LANES    JacobiSVDImpl_'s dot product and rotated norms in VBLAS<double>'s two SSE2
                           lanes (VBLAS::dot / givensx, the accumulation order of the OpenCV releases
                           that kept W in _Tp) instead of 2.4.9's scalar double loops;
     ORC_GEOM_LIBM_HYPOT   libm's hypot for the rotation instead of fm3d_hypot_cr (the product's). */
enum { ORC_GEOM_DLT_LEGACY = 1, ORC_GEOM_POLAR_NEWTON = 2, ORC_GEOM_SVD_LANES = 4, ORC_GEOM_LIBM_HYPOT = 8 };
static int orc_geom_mode = 0;
ORC_API void orc_set_geometry_mode(int mode) { orc_geom_mode = mode; }
ORC_API int orc_get_geometry_mode(void) { return orc_geom_mode; }

#define ORC_SVD_MAXN 8
#define ORC_SVD_MAXM 8

/* cv::RNG (core.hpp): state = (uint64)(unsigned)state * CV_RNG_COEFF + (unsigned)(state >> 32) */
static unsigned orc_cv_rng_next(uint64_t *state)
{
    *state = (uint64_t)(unsigned)*state * 4164903690U + (unsigned)(*state >> 32);
    return (unsigned)*state;
}

/* VBLAS<double>::dot under SSE2: lanes (k, k+1) and (k+2, k+3) per step of 4, lane sums added
   pairwise, the low lane first; returns the elements consumed (0 when n < 4) */
static int orc_vblas_dot(const double *a, const double *b, int n, double *result)
{
    double s0[2] = {0, 0}, s1[2] = {0, 0};
    int k = 0;
    if (n < 4) return 0;
    for (; k <= n - 4; k += 4) {
        s0[0] = s0[0] + a[k] * b[k];
        s0[1] = s0[1] + a[k + 1] * b[k + 1];
        s1[0] = s1[0] + a[k + 2] * b[k + 2];
        s1[1] = s1[1] + a[k + 3] * b[k + 3];
    }
    s0[0] = s0[0] + s1[0];
    s0[1] = s0[1] + s1[1];
    *result = s0[0] + s0[1];
    return k;
}

/* VBLAS<double>::givensx under SSE2: the rotation two lanes at a time, the squared norms of the
   rotated rows per lane, the lanes added at the end */
static int orc_vblas_givensx(double *a, double *b, int n, double c, double s, double *anorm, double *bnorm)
{
    double sa[2] = {0, 0}, sb[2] = {0, 0};
    int k = 0, l;
    for (; k <= n - 2; k += 2)
        for (l = 0; l < 2; l++) {
            double t0 = a[k + l] * c + b[k + l] * s;
            double t1 = b[k + l] * c - a[k + l] * s;
            a[k + l] = t0;
            b[k + l] = t1;
            sa[l] = sa[l] + t0 * t0;
            sb[l] = sb[l] + t1 * t1;
        }
    *anorm = sa[0] + sa[1];
    *bnorm = sb[0] + sb[1];
    return k;
}

/* JacobiSVDImpl_<double>(At, astep, _W, Vt, vstep, m, n, n1, DBL_MIN, 10 DBL_EPSILON): At holds the n
   columns of A as rows of m (strides in elements); on return its first n1 rows are the left singular
   vectors, _W the singular values in descending order, Vt's rows the right singular vectors. */
static void orc_cv_jacobi_svd(double *At, int astep, double *_W, double *Vt, int vstep, int m, int n, int n1)
{
    const double minval = DBL_MIN, eps = DBL_EPSILON * 10;
    const int lanes = (orc_geom_mode & ORC_GEOM_SVD_LANES) != 0;
    double W[ORC_SVD_MAXN], c, s, sd;
    int i, j, k, iter, max_iter = m > 30 ? m : 30;
    uint64_t rng = 0x12345678;

    for (i = 0; i < n; i++) {
        for (k = 0, sd = 0; k < m; k++) {
            double t = At[i * astep + k];
            sd += t * t;
        }
        W[i] = sd;
        if (Vt) {
            for (k = 0; k < n; k++) Vt[i * vstep + k] = 0;
            Vt[i * vstep + i] = 1;
        }
    }

    for (iter = 0; iter < max_iter; iter++) {
        int changed = 0;
        for (i = 0; i < n - 1; i++)
            for (j = i + 1; j < n; j++) {
                double *Ai = At + i * astep, *Aj = At + j * astep;
                double a = W[i], p = 0, b = W[j], beta, gamma;
                k = lanes ? orc_vblas_dot(Ai, Aj, m, &p) : 0;
                for (; k < m; k++) p += Ai[k] * Aj[k];
                if (fabs(p) <= eps * sqrt(a * b)) continue;
                p *= 2;
                beta = a - b;
                gamma = (orc_geom_mode & ORC_GEOM_LIBM_HYPOT) ? hypot(p, beta) : fm3d_hypot_cr(p, beta);
                if (beta < 0) {
                    double delta = (gamma - beta) * 0.5;
                    s = sqrt(delta / gamma);
                    c = p / (gamma * s * 2);
                } else {
                    c = sqrt((gamma + beta) / (gamma * 2));
                    s = p / (gamma * c * 2);
                }
                a = b = 0;
                k = lanes ? orc_vblas_givensx(Ai, Aj, m, c, s, &a, &b) : 0;
                for (; k < m; k++) {
                    double t0 = c * Ai[k] + s * Aj[k];
                    double t1 = -s * Ai[k] + c * Aj[k];
                    Ai[k] = t0;
                    Aj[k] = t1;
                    a += t0 * t0;
                    b += t1 * t1;
                }
                W[i] = a;
                W[j] = b;
                changed = 1;
                if (Vt) {
                    /* VBLAS<double>::givens (SSE2, two lanes: Vi c + Vj s, Vj c - Vi s) and the
                       scalar tail give the scalar loop's bits: no FMA, and -(s Vi) + c Vj is
                       c Vj - s Vi exactly */
                    double *Vi = Vt + i * vstep, *Vj = Vt + j * vstep;
                    for (k = 0; k < n; k++) {
                        double t0 = c * Vi[k] + s * Vj[k];
                        double t1 = -s * Vi[k] + c * Vj[k];
                        Vi[k] = t0;
                        Vj[k] = t1;
                    }
                }
            }
        if (!changed) break;
    }

    for (i = 0; i < n; i++) {
        for (k = 0, sd = 0; k < m; k++) {
            double t = At[i * astep + k];
            sd += t * t;
        }
        W[i] = sqrt(sd);
    }

    for (i = 0; i < n - 1; i++) {
        j = i;
        for (k = i + 1; k < n; k++)
            if (W[j] < W[k]) j = k;
        if (i != j) {
            double t = W[i];
            W[i] = W[j];
            W[j] = t;
            if (Vt) {
                for (k = 0; k < m; k++) {
                    t = At[i * astep + k];
                    At[i * astep + k] = At[j * astep + k];
                    At[j * astep + k] = t;
                }
                for (k = 0; k < n; k++) {
                    t = Vt[i * vstep + k];
                    Vt[i * vstep + k] = Vt[j * vstep + k];
                    Vt[j * vstep + k] = t;
                }
            }
        }
    }

    for (i = 0; i < n; i++) _W[i] = W[i];
    if (!Vt) return;

    for (i = 0; i < n1; i++) {
        sd = i < n ? W[i] : 0;
        while (sd <= minval) {
            /* a zero singular value: a random +-1/m vector, twice orthogonalised against the
               previous left vectors and l1-normalised */
            const double val0 = 1. / m;
            for (k = 0; k < m; k++) At[i * astep + k] = (orc_cv_rng_next(&rng) & 256) != 0 ? val0 : -val0;
            for (iter = 0; iter < 2; iter++)
                for (j = 0; j < i; j++) {
                    double asum = 0;
                    sd = 0;
                    for (k = 0; k < m; k++) sd += At[i * astep + k] * At[j * astep + k];
                    for (k = 0; k < m; k++) {
                        double t = At[i * astep + k] - sd * At[j * astep + k];
                        At[i * astep + k] = t;
                        asum += fabs(t);
                    }
                    asum = asum ? 1 / asum : 0;
                    for (k = 0; k < m; k++) At[i * astep + k] *= asum;
                }
            sd = 0;
            for (k = 0; k < m; k++) {
                double t = At[i * astep + k];
                sd += t * t;
            }
            sd = sqrt(sd);
        }
        s = 1 / sd;
        for (k = 0; k < m; k++) At[i * astep + k] *= s;
    }
}

/* cv::SVD::compute (_SVDcompute) of an m x n row-major double matrix with m >= n and no FULL_UV:
   temp_a = A^T, JacobiSVD(temp_a, m, n, n1 = n); w (n), u (m x n, may be NULL) = temp_u^T,
   vt (n x n) = temp_v */
static void orc_cv_svd(const double *A, int m, int n, double *w, double *u, double *vt)
{
    double At[ORC_SVD_MAXN * ORC_SVD_MAXM];
    int i, k;
    for (i = 0; i < n; i++)
        for (k = 0; k < m; k++) At[i * m + k] = A[k * n + i];
    orc_cv_jacobi_svd(At, m, w, vt, n, m, n, n);
    if (u)
        for (k = 0; k < m; k++)
            for (i = 0; i < n; i++) u[k * n + i] = At[i * m + k];
}

/* elementwise SVD entry for the tests (tests/test_cvsvd.py): A (m x n, m >= n, n, m <= 8) -> w, u, vt */
ORC_API int orc_cv_svd_eval(const double *A, int m, int n, double *w, double *u, double *vt)
{
    if (m < n || n < 1 || m > ORC_SVD_MAXM || n > ORC_SVD_MAXN) return -1;
    orc_cv_svd(A, m, n, w, u, vt);
    return 0;
}

/* 3x3 inverse transpose via adjugate (the legacy Newton polar iteration, ORC_GEOM_POLAR_NEWTON) */
static void orc_inv_t3(const double A[9], double out[9])
{
    double c00 = A[4] * A[8] - A[5] * A[7];
    double c01 = A[5] * A[6] - A[3] * A[8];
    double c02 = A[3] * A[7] - A[4] * A[6];
    double c10 = A[2] * A[7] - A[1] * A[8];
    double c11 = A[0] * A[8] - A[2] * A[6];
    double c12 = A[1] * A[6] - A[0] * A[7];
    double c20 = A[1] * A[5] - A[2] * A[4];
    double c21 = A[2] * A[3] - A[0] * A[5];
    double c22 = A[0] * A[4] - A[1] * A[3];
    double det = A[0] * c00 + A[1] * c01 + A[2] * c02;
    double id = 1. / det;
    /* inverse transpose = cofactor matrix / det */
    out[0] = c00 * id; out[1] = c01 * id; out[2] = c02 * id;
    out[3] = c10 * id; out[4] = c11 * id; out[5] = c12 * id;
    out[6] = c20 * id; out[7] = c21 * id; out[8] = c22 * id;
}

/* cvRodrigues2's orthonormalisation of a 3x3 R (OpenCV 2.4 calib3d/src/calibration.cpp):
   cvSVD(R, W, U, V, CV_SVD_MODIFY_A + CV_SVD_U_T + CV_SVD_V_T), then
   cvGEMM(U, V, 1, 0, 0, R, CV_GEMM_A_T) = U V^T, which takes GEMMSingleMul's generic loop
   (flags != 0): s = 0; s += U(i,k) Vt(k,j) for k = 0..2; s * alpha */
ORC_API void orc_cv_polar3(const double R[9], double Rp[9])
{
    int i, j, k;
    if (orc_geom_mode & ORC_GEOM_POLAR_NEWTON) {
        double Y[9];
        memcpy(Rp, R, 9 * sizeof(double));
        for (i = 0; i < 3; i++) {
            orc_inv_t3(Rp, Y);
            for (k = 0; k < 9; k++) Rp[k] = 0.5 * (Rp[k] + Y[k]);
        }
        return;
    }
    {
        double W[3], U[9], Vt[9];
        orc_cv_svd(R, 3, 3, W, U, Vt);
        for (i = 0; i < 3; i++)
            for (j = 0; j < 3; j++) {
                double s = 0;
                for (k = 0; k < 3; k++) s += U[i * 3 + k] * Vt[k * 3 + j];
                Rp[i * 3 + j] = s * 1.;
            }
    }
}

/* cvRodrigues2 matrix -> vector (OpenCV 2.4): R replaced by its polar factor U V^T (above), then
   the rotation vector from its skew part and trace; acos from libm, or fm3d_acos (cr: 1) */
static void orc_rodrigues_m2v_acos(const double Rin[9], double r[3], int detacos)
{
    double R[9];
    double rx, ry, rz, s, c, theta;
    orc_cv_polar3(Rin, R);
    rx = R[7] - R[5];
    ry = R[2] - R[6];
    rz = R[3] - R[1];
    s = sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    theta = detacos ? fm3d_acos(c) : acos(c);
    if (s < 1e-5) {
        double t;
        if (c > 0)
            rx = ry = rz = 0;
        else {
            t = (R[0] + 1) * 0.5;
            rx = sqrt(t > 0. ? t : 0.);
            t = (R[4] + 1) * 0.5;
            ry = sqrt(t > 0. ? t : 0.) * (R[1] < 0 ? -1. : 1.);
            t = (R[8] + 1) * 0.5;
            rz = sqrt(t > 0. ? t : 0.) * (R[2] < 0 ? -1. : 1.);
            if (fabs(rx) < fabs(ry) && fabs(rx) < fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
            theta /= sqrt(rx * rx + ry * ry + rz * rz);
            rx *= theta; ry *= theta; rz *= theta;
        }
    } else {
        double vth = 1 / (2 * s);
        vth *= theta;
        rx *= vth; ry *= vth; rz *= vth;
    }
    r[0] = rx; r[1] = ry; r[2] = rz;
}

ORC_API void orc_rodrigues_m2v(const double Rin[9], double r[3])
{
    orc_rodrigues_m2v_acos(Rin, r, 0);
}

/* composeTransformation, tools.cpp:87-99 */
static void orc_compose(const double R[9], const double T[3], double G[16])
{
    G[0] = R[0]; G[1] = R[1]; G[2] = R[2]; G[3] = T[0];
    G[4] = R[3]; G[5] = R[4]; G[6] = R[5]; G[7] = T[1];
    G[8] = R[6]; G[9] = R[7]; G[10] = R[8]; G[11] = T[2];
    G[12] = 0; G[13] = 0; G[14] = 0; G[15] = 1;
}

/* Matx44d::inv() == OpenCV LU with partial pivoting (DECOMP_LU) */
static void orc_inv4(const double Ain[16], double B[16])
{
    double A[16];
    int i, j, k;
    memcpy(A, Ain, sizeof(A));
    for (i = 0; i < 16; i++) B[i] = (i % 5 == 0) ? 1. : 0.;
    for (i = 0; i < 4; i++) {
        double d;
        k = i;
        for (j = i + 1; j < 4; j++)
            if (fabs(A[j * 4 + i]) > fabs(A[k * 4 + i])) k = j;
        if (k != i) {
            for (j = i; j < 4; j++) { double t = A[i * 4 + j]; A[i * 4 + j] = A[k * 4 + j]; A[k * 4 + j] = t; }
            for (j = 0; j < 4; j++) { double t = B[i * 4 + j]; B[i * 4 + j] = B[k * 4 + j]; B[k * 4 + j] = t; }
        }
        d = -1 / A[i * 4 + i];
        for (j = i + 1; j < 4; j++) {
            double alpha = A[j * 4 + i] * d;
            for (k = i + 1; k < 4; k++) A[j * 4 + k] += alpha * A[i * 4 + k];
            for (k = 0; k < 4; k++) B[j * 4 + k] += alpha * B[i * 4 + k];
        }
        A[i * 4 + i] = -d;
    }
    for (i = 3; i >= 0; i--)
        for (j = 0; j < 4; j++) {
            double s = B[i * 4 + j];
            for (k = i + 1; k < 4; k++) s -= A[i * 4 + k] * B[k * 4 + j];
            B[i * 4 + j] = s * A[i * 4 + i];
        }
}

static void orc_mul4(const double a[16], const double b[16], double c[16])
{
    int i, j, k;
    for (i = 0; i < 4; i++)
        for (j = 0; j < 4; j++) {
            double s = 0;
            for (k = 0; k < 4; k++) s += a[i * 4 + k] * b[k * 4 + j];
            c[i * 4 + j] = s;
        }
}

/* SingleCameraTriangulator ctor (:42-65) + setg12 (:123-143):
   g12 = gIC^-1 * g2^-1 * g1 * gIC */
ORC_API void orc_setg12(const double rIC[3], const double tIC[3], const double T1[3], const double T2[3],
                        const double r1[3], const double r2[3], double g12[16])
{
    double RIC[9], R1[9], R2[9], gIC[16], g1[16], g2[16], a[16], b[16], c[16], d[16];
    orc_rodrigues_v2m(rIC, RIC);
    orc_compose(RIC, tIC, gIC);
    orc_rodrigues_v2m(r1, R1);
    orc_rodrigues_v2m(r2, R2);
    orc_compose(R1, T1, g1);
    orc_compose(R2, T2, g2);
    orc_inv4(gIC, a);
    orc_inv4(g2, b);
    orc_mul4(a, b, c);
    orc_mul4(c, g1, d);
    orc_mul4(d, gIC, g12);
}

/* decomposeTransformation (tools.cpp:101-114) followed by the Rodrigues
   vector->matrix that cvProjectPoints2 applies to r2: the exact R2,t2 that
   projectPointsToImage2 (singlecameratriangulator.cpp:591-602) projects with. */
ORC_API void orc_camera2_from_g12(const double g12[16], double R2[9], double t2[3])
{
    double R[9], r[3];
    R[0] = g12[0]; R[1] = g12[1]; R[2] = g12[2];
    R[3] = g12[4]; R[4] = g12[5]; R[5] = g12[6];
    R[6] = g12[8]; R[7] = g12[9]; R[8] = g12[10];
    orc_rodrigues_m2v(R, r);
    orc_rodrigues_v2m(r, R2);
    t2[0] = g12[3]; t2[1] = g12[7]; t2[2] = g12[11];
}

/* ------------------------------------------------------------------ */
/* DLT triangulation (a4, a5)                                          */
/* ------------------------------------------------------------------ */
/* ORC_GEOM_DLT_LEGACY (rounds 1-5): one Jacobi rotation of columns (p, q) of the 4x4 A (and V)
   unless they are orthogonal to 1e-15 */
static int orc_jacobi_pair(double A[16], double V[16], int p, int q)
{
    double alpha = 0, beta = 0, gamma = 0;
    int i;
    for (i = 0; i < 4; i++) {
        double ap = A[i * 4 + p], aq = A[i * 4 + q];
        alpha += ap * ap;
        beta += aq * aq;
        gamma += ap * aq;
    }
    if (gamma != 0. && fabs(gamma) > 1e-15 * sqrt(alpha * beta)) {
        double zeta = (beta - alpha) / (2. * gamma);
        double t = (zeta >= 0. ? 1. : -1.) / (fabs(zeta) + sqrt(1. + zeta * zeta));
        double cs = 1. / sqrt(1. + t * t);
        double sn = cs * t;
        for (i = 0; i < 4; i++) {
            double ap = A[i * 4 + p], aq = A[i * 4 + q];
            A[i * 4 + p] = cs * ap - sn * aq;
            A[i * 4 + q] = sn * ap + cs * aq;
            ap = V[i * 4 + p];
            aq = V[i * 4 + q];
            V[i * 4 + p] = cs * ap - sn * aq;
            V[i * 4 + q] = sn * ap + cs * aq;
        }
        return 1;
    }
    return 0;
}

/* ORC_GEOM_DLT_LEGACY: null vector of the 4-row system by the round-robin one-sided Jacobi
   ((0,1)+(2,3), (0,2)+(1,3), (0,3)+(1,2), up to 30 sweeps), the smallest column norm's V column */
static void orc_dlt_nullvec_legacy(double A[16], double v[4])
{
    static const int PQ[6][2] = {{0, 1}, {2, 3}, {0, 2}, {1, 3}, {0, 3}, {1, 2}};
    double V[16];
    int sweep, p, i, k, best;
    for (i = 0; i < 16; i++) V[i] = (i % 5 == 0) ? 1. : 0.;
    for (sweep = 0; sweep < 30; sweep++) {
        int rotated = 0;
        for (k = 0; k < 6; k++) rotated |= orc_jacobi_pair(A, V, PQ[k][0], PQ[k][1]);
        if (!rotated) break;
    }
    {
        double nrm[4];
        for (p = 0; p < 4; p++) {
            double s = 0;
            for (i = 0; i < 4; i++) s += A[i * 4 + p] * A[i * 4 + p];
            nrm[p] = s;
        }
        best = 0;
        for (p = 1; p < 4; p++)
            if (nrm[p] < nrm[best]) best = p;
    }
    for (i = 0; i < 4; i++) v[i] = V[i * 4 + best];
}

/* cv::triangulatePoints (OpenCV 2.4 cvTriangulatePoints, calib3d/src/triangulate.cpp) for one pair of
   undistorted points, P1 = [I|0], P2 = the first 3 rows of g12 (singlecameratriangulator.cpp:179-186):
   the 6 x 4 matrA, per view j rows 3j..3j+2 = x P.row2 - P.row0, y P.row2 - P.row1,
   x P.row1 - y P.row0; cvSVD(matrA, matrW, 0, matrV, CV_SVD_V_T); X = matrV's row 3 (the right singular
   vector of the smallest singular value after JacobiSVD's descending sort).  Returns homogeneous X. */
ORC_API void orc_triangulate1(const double g12[16], const double u1[2], const double u2[2], double X[4])
{
    double P1[12], P2[12];
    int j, k;
    for (k = 0; k < 12; k++) P1[k] = (k == 0 || k == 5 || k == 10) ? 1. : 0.;
    for (k = 0; k < 12; k++) P2[k] = g12[k];
    if (orc_geom_mode & ORC_GEOM_DLT_LEGACY) {
        double A[16];
        for (j = 0; j < 2; j++) {
            const double *P = j == 0 ? P1 : P2;
            double x = j == 0 ? u1[0] : u2[0];
            double y = j == 0 ? u1[1] : u2[1];
            for (k = 0; k < 4; k++) {
                A[(j * 2 + 0) * 4 + k] = x * P[8 + k] - P[0 + k];
                A[(j * 2 + 1) * 4 + k] = y * P[8 + k] - P[4 + k];
            }
        }
        orc_dlt_nullvec_legacy(A, X);
        return;
    }
    {
        double A[24], W[4], Vt[16];
        for (j = 0; j < 2; j++) {
            const double *P = j == 0 ? P1 : P2;
            double x = j == 0 ? u1[0] : u2[0];
            double y = j == 0 ? u1[1] : u2[1];
            for (k = 0; k < 4; k++) {
                A[(j * 3 + 0) * 4 + k] = x * P[8 + k] - P[0 + k];
                A[(j * 3 + 1) * 4 + k] = y * P[8 + k] - P[4 + k];
                A[(j * 3 + 2) * 4 + k] = x * P[4 + k] - y * P[0 + k];
            }
        }
        orc_cv_svd(A, 6, 4, W, NULL, Vt);
        for (k = 0; k < 4; k++) X[k] = Vt[3 * 4 + k];
    }
}

/* setKeypoints (:145-171) + triangulate (:173-230).
   kp: float xy per keypoint (cv::KeyPoint::pt).  Outputs: inlier mask per
   match, compacted points (in match order).  Returns number of inliers. */
ORC_API int orc_triangulate(const orc_camera *c, const double g12[16], double zmin, double zmax,
                            const float *kp1, const float *kp2, const int *query, const int *train, int K,
                            uint8_t *mask, double *points)
{
    int i, n = 0;
    for (i = 0; i < K; i++) {
        double a1x = (double)kp1[2 * query[i]], a1y = (double)kp1[2 * query[i] + 1];
        double a2x = (double)kp2[2 * train[i]], a2y = (double)kp2[2 * train[i] + 1];
        double u1[2], u2[2], X[4];
        orc_undistort1(c, a1x, a1y, &u1[0], &u1[1]);
        orc_undistort1(c, a2x, a2y, &u2[0], &u2[1]);
        orc_triangulate1(g12, u1, u2, X);
        if (X[2] / X[3] < zmin || X[2] / X[3] >= zmax) {
            mask[i] = 0;
        } else {
            mask[i] = 1;
            points[3 * n + 0] = X[0] / X[3];
            points[3 * n + 1] = X[1] / X[3];
            points[3 * n + 2] = X[2] / X[3];
            n++;
        }
    }
    return n;
}

/* ------------------------------------------------------------------ */
/* descriptor matching (a1)                                            */
/* ------------------------------------------------------------------ */
enum { ORC_F32 = 0, ORC_U8 = 1, ORC_BITS = 2 };

/* FLANN L2<float>: groups of 4, result += d0*d0 + d1*d1 + d2*d2 + d3*d3, then tail */
static float orc_l2_flann(const float *a, const float *b, int n)
{
    float result = 0.f;
    int i = 0;
    for (; i + 3 < n; i += 4) {
        float d0 = a[i] - b[i], d1 = a[i + 1] - b[i + 1], d2 = a[i + 2] - b[i + 2], d3 = a[i + 3] - b[i + 3];
        result += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
    }
    for (; i < n; i++) {
        float d0 = a[i] - b[i];
        result += d0 * d0;
    }
    return result;
}

/* k=2 brute force with (distance, trainIdx) lexicographic order.  key2 is the
   ranking value: the squared L2 (float FLANN order or exact integer) or the
   Hamming count.  dist is what cv::DMatch::distance holds
   (FlannBasedMatcher::convertToDMatches: sqrt for L2, float(int) for Hamming). */
ORC_API void orc_knn2(int type, const void *A, int nA, const void *B, int nB, int dim,
                      int *idx /* nA*2, -1 if absent */, float *dist /* nA*2 */, int nthreads)
{
    int i;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 16)
#endif
    for (i = 0; i < nA; i++) {
        double k1 = INFINITY, k2 = INFINITY;
        int i1 = -1, i2 = -1, j;
        for (j = 0; j < nB; j++) {
            double key;
            if (type == ORC_F32) {
                key = (double)orc_l2_flann((const float *)A + (size_t)i * dim, (const float *)B + (size_t)j * dim, dim);
            } else if (type == ORC_U8) {
                const uint8_t *a = (const uint8_t *)A + (size_t)i * dim, *b = (const uint8_t *)B + (size_t)j * dim;
                int64_t s = 0;
                int d;
                for (d = 0; d < dim; d++) { int df = (int)a[d] - (int)b[d]; s += df * df; }
                key = (double)s;
            } else {
                const uint8_t *a = (const uint8_t *)A + (size_t)i * dim, *b = (const uint8_t *)B + (size_t)j * dim;
                int s = 0, d;
                for (d = 0; d < dim; d++) s += __builtin_popcount((unsigned)(a[d] ^ b[d]));
                key = (double)s;
            }
            /* candidates arrive in increasing j: strict < keeps the lowest index on ties */
            if (key < k1) { k2 = k1; i2 = i1; k1 = key; i1 = j; }
            else if (key < k2) { k2 = key; i2 = j; }
        }
        idx[2 * i] = i1;
        idx[2 * i + 1] = i2;
        if (type == ORC_BITS) {
            dist[2 * i] = (float)k1;
            dist[2 * i + 1] = (float)k2;
        } else {
            dist[2 * i] = sqrtf((float)k1);
            dist[2 * i + 1] = sqrtf((float)k2);
        }
    }
}

/* compareWithNNDR (descriptorsmatcher.cpp:117-129): keep m[0] iff the query has
   2 neighbours and m[0].distance <= epsilon * m[1].distance (double compare).
   Output in query order: (queryIdx, trainIdx, distance). Returns count. */
ORC_API int orc_nndr(const int *idx, const float *dist, int nA, double eps, int *q_out, int *t_out, float *d_out)
{
    int i, n = 0;
    for (i = 0; i < nA; i++) {
        if (idx[2 * i] < 0 || idx[2 * i + 1] < 0) continue;
        if ((double)dist[2 * i] <= eps * (double)dist[2 * i + 1]) {
            q_out[n] = i;
            t_out[n] = idx[2 * i];
            d_out[n] = dist[2 * i];
            n++;
        }
    }
    return n;
}

/* ------------------------------------------------------------------ */
/* images                                                              */
/* ------------------------------------------------------------------ */
static int orc_reflect101(int p, int len)
{
    if (len == 1) return 0;
    while (p < 0 || p >= len) {
        if (p < 0) p = -p;
        else p = 2 * len - p - 2;
    }
    return p;
}

/* cv::pyrDown 8U (normaloptimizer.cpp:216-217): 5x5 [1 4 6 4 1]^2 / 256 with
   BORDER_REFLECT_101, (sum + 128) >> 8, dst size ((w+1)/2, (h+1)/2). */
ORC_API void orc_pyrdown(const uint8_t *src, int w, int h, uint8_t *dst)
{
    static const int wt[5] = {1, 4, 6, 4, 1};
    int dw = (w + 1) / 2, dh = (h + 1) / 2, x, y, i, j;
    for (y = 0; y < dh; y++)
        for (x = 0; x < dw; x++) {
            int s = 0;
            for (i = 0; i < 5; i++) {
                int sy = orc_reflect101(2 * y + i - 2, h);
                int rs = 0;
                for (j = 0; j < 5; j++) {
                    int sx = orc_reflect101(2 * x + j - 2, w);
                    rs += wt[j] * src[sy * w + sx];
                }
                s += wt[i] * rs;
            }
            dst[y * dw + x] = (uint8_t)((s + 128) >> 8);
        }
}

/* getBilinearInterpPix32f (tools.cpp:129-142).  The reference reads
   (y0,x0),(y1,x0),(y0,x1),(y1,x1) with no bounds check; isPixelGood admits
   x == cols and y == rows, so the reference reads one element past a row (which
   lands in the next row of a continuous cv::Mat) or past the image.  We emulate
   a continuous buffer followed by zero bytes. */
static float orc_pix(const uint8_t *img, int w, int h, int y, int x)
{
    long idx = (long)y * w + x;
    if (idx < 0 || idx >= (long)w * h) return 0.f;
    return (float)img[idx];
}

static float orc_bilinear(const uint8_t *img, int w, int h, float x, float y)
{
    int x0 = (int)floor((double)x), y0 = (int)floor((double)y);
    int x1 = x0 + 1, y1 = y0 + 1;
    float b00 = orc_pix(img, w, h, y0, x0), b10 = orc_pix(img, w, h, y1, x0);
    float b01 = orc_pix(img, w, h, y0, x1), b11 = orc_pix(img, w, h, y1, x1);
    float xm0 = 1.0f - (x - (float)x0), xm1 = (x - (float)x0);
    float ym0 = 1.0f - (y - (float)y0), ym1 = (y - (float)y0);
    return xm0 * (b00 * ym0 + b10 * ym1) + xm1 * (b01 * ym0 + b11 * ym1);
}

ORC_API float orc_bilinear_sample(const uint8_t *img, int w, int h, float x, float y)
{
    return orc_bilinear(img, w, h, x, y);
}

/* ------------------------------------------------------------------ */
/* neighbourhood (a8)                                                  */
/* ------------------------------------------------------------------ */
/* extractPixelsContour(Vec3d) (:376-397) -> (Vec2d) (:341-374).  Writes the
   kept pixel coordinates (double xy) and returns m_dat. */
ORC_API int orc_neighborhood(const orc_camera *c, const double X[3], int ray, int boundW, int boundH,
                             double *out_xy, int cap)
{
    static const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    static const double Z[3] = {0, 0, 0};
    double cx, cy;
    int i, j, n = 0;
    orc_project1(c, I, Z, X[0], X[1], X[2], &cx, &cy);
    for (i = -ray; i <= ray; i++)
        for (j = -ray; j <= ray; j++) {
            if (i * i + j * j <= ray * ray) {
                double px = cx + i, py = cy + j;
                if (px < 0 || py < 0 || px >= boundW || py >= boundH) continue;
                if (n < cap) { out_xy[2 * n] = px; out_xy[2 * n + 1] = py; }
                n++;
            }
        }
    return n;
}

/* ------------------------------------------------------------------ */
/* LM normal optimisation (a7, a9-a15)                                 */
/* ------------------------------------------------------------------ */
enum {
    ORC_ST_OK = 0,
    ORC_ST_NO_PIXELS = 1,   /* normaloptimizer.cpp:364-369 */
    ORC_ST_ABORT_BBOX = 2,  /* isInBoundingBox failed (:557-560) */
    ORC_ST_ABORT_PIX1 = 3,  /* updateImage1PixelsIntensity (:580-584) */
    ORC_ST_ABORT_PIX2 = 4,  /* projectPointsToImage2 (:623-626) */
    ORC_ST_NAN_PLANE = 5,   /* projectPointToPlane exit(-6) (:465-469) */
    ORC_ST_NAN_NORMAL = 6   /* evaluateNormal NaN normal (:81-85) */
};
/* LM modes (mode bit 2: fm3d_detmath transcendentals instead of libm) */
enum { ORC_LM_STRICT = 0, ORC_LM_DETMATH = 2 };
/* lmfit variants (parity-risk study only, tools/parity_risk.py).  The reference calls
   lmfit's lmmin with the printout callback + lm_princon_struct signature and reads status.info
   (normaloptimizer.cpp:269-287): the lmfit 3.x API.  The restatement is MINPACK lmdif; where lmfit
   3.x's published lmmin.c is recalled to differ (not verifiable here: lmfit is not in the image),
   one mode bit switches to the lmfit form:
     ORC_LMV_FDFLOOR   forward-difference step MAX(eps*eps, eps*|x|)  (MINPACK: eps*|x|, eps if 0)
     ORC_LMV_ENORM     lm_enorm thresholds sqrt(DBL_MIN) / sqrt(DBL_MAX) (MINPACK: 3.834e-20 / 1.304e19)
     ORC_LMV_DWARFEXIT return at once with info 0 when the starting fnorm <= DBL_MIN (lmfit's
                       "sum of squares below underflow limit"; MINPACK goes on to a Jacobian)
     ORC_LMV_TOL1E14   ftol = xtol = gtol = 1e-14 (the LM_USERTOL of lmfit builds that use the
                       hard-coded "x86" constants instead of float.h's 30*DBL_EPSILON)
   The user-break mapping (evaluate sets *info < 0 -> lmdif returns -> status.info = 11) is the
   same in both. */
enum { ORC_LMV_FDFLOOR = 4, ORC_LMV_ENORM = 8, ORC_LMV_DWARFEXIT = 16, ORC_LMV_TOL1E14 = 32 };
/* Reduction modes.  Default: every m_dat-long sum in pixel order (MINPACK's, the
   reference's).  ORC_LM_TREE: every m_dat-long sum as the fixed blocked tree of orc_tree_finish.
   ORC_LM_GRAM (with TREE): the 2-column Householder QR from the tree sums of the Jacobian sweep
   (column norms, a_p.a_q, a_p.f, a_q.f) where it is well conditioned, the Householder passes with
   tree sums elsewhere (orc_qr_tree). */
enum { ORC_LM_TREE = 64, ORC_LM_GRAM = 128 };
/* the Gram form is used when ||a_q'||^2 = S_qq - r01^2 > ORC_GRAM_C * S_qq (relative cancellation error
   below 2 eps / ORC_GRAM_C) */
#define ORC_GRAM_C 1e-6
static int orc_lmv_enorm = 0; /* set from the mode before the (parallel) point loop; read-only after */

typedef struct {
    const uint8_t *img[2][8]; /* pyramid levels of image 1 and 2 */
    int w[8], h[8];
} orc_pyramid;

typedef struct {
    const orc_camera *cam;
    const double *R2, *t2;
    const orc_pyramid *pyr;
    int level;
    double scale;
    double X[3];
    int cmax;           /* int cMax = 2*zThresholdMax (truncating), :648 */
    int m;
    const double *ray;  /* m * 2 undistorted (x,y); z = 1 */
    const double *pix;  /* m * 2 image-1 pixel coordinates */
    float *I1;          /* m intensities of image 1 at the current level */
    int I1_ok;
    int mode;
    long nfev;          /* evaluations in the current lmdif call */
} orc_lmdata;

/* isPixelGood (:657-665); NaN coordinates count as bad (the reference then
   has undefined behaviour inside getBilinearInterpPix32f). */
static int orc_pixel_good(double x, double y, double scale, int cols, int rows)
{
    if (x != x || y != y) return 0;
    if ((x < 0) || (x > ((1 / scale) * cols)) || (y < 0) || (y > ((1 / scale) * rows))) return 0;
    return 1;
}

/* updateImage1PixelsIntensity (:576-589).  Its inputs do not change inside a
   pyramid level, so the values (and the abort) are computed once per level. */
static void orc_update_I1(orc_lmdata *D)
{
    int i, L = D->level;
    D->I1_ok = 1;
    for (i = 0; i < D->m; i++) {
        double x = D->pix[2 * i], y = D->pix[2 * i + 1];
        if (!orc_pixel_good(x, y, D->scale, D->pyr->w[L], D->pyr->h[L])) { D->I1_ok = 0; return; }
        D->I1[i] = orc_bilinear(D->pyr->img[0][L], D->pyr->w[L], D->pyr->h[L],
                                (float)(D->scale * x), (float)(D->scale * y));
    }
}

/* DETMATH takes the correctly rounded functions of fm3d_crmath.h (the LM kernel's), or with
   ORC_DET_1ULP the 1-ulp polynomials of fm3d_detmath.h (the NCC hypotheses: csrc/fm3d_ncc.hip).
   Attribution switches (tools/full_parity.py): with ORC_LM_DETMATH, libm's function
   for one transcendental at a time. */
enum { ORC_LIBM_SIN = 256, ORC_LIBM_COS = 512, ORC_LIBM_ATAN2 = 1024, ORC_LIBM_EXP = 2048, ORC_DET_1ULP = 4096 };
static double orc_fsin(int mode, double x)
{
    if (!(mode & ORC_LM_DETMATH) || (mode & ORC_LIBM_SIN)) return sin(x);
    return (mode & ORC_DET_1ULP) ? fm3d_sin(x) : fm3d_sin_cr(x);
}
static double orc_fcos(int mode, double x)
{
    if (!(mode & ORC_LM_DETMATH) || (mode & ORC_LIBM_COS)) return cos(x);
    return (mode & ORC_DET_1ULP) ? fm3d_cos(x) : fm3d_cos_cr(x);
}
static double orc_fatan2(int mode, double y, double x)
{
    if (!(mode & ORC_LM_DETMATH) || (mode & ORC_LIBM_ATAN2)) return atan2(y, x);
    return (mode & ORC_DET_1ULP) ? fm3d_atan2(y, x) : fm3d_atan2_cr(y, x);
}
static double orc_fexp(int mode, double x)
{
    if (!(mode & ORC_LM_DETMATH) || (mode & ORC_LIBM_EXP)) return exp(x);
    return (mode & ORC_DET_1ULP) ? fm3d_exp(x) : fm3d_exp_cr(x);
}
/* the four transcendentals elementwise in a mode (tests/test_crmath.py pins the correctly rounded
   ones against mpmath): fn 0 sin(x), 1 cos(x), 2 atan2(x, y), 3 exp(x), 4 hypot(x, y) (DETMATH:
   fm3d_hypot_cr, the SVD's; else libm) */
ORC_API void orc_math_eval(int fn, int mode, const double *x, const double *y, int n, double *out)
{
    int i;
    for (i = 0; i < n; i++)
        out[i] = fn == 0 ? orc_fsin(mode, x[i]) : fn == 1 ? orc_fcos(mode, x[i])
               : fn == 2 ? orc_fatan2(mode, x[i], y[i]) : fn == 3 ? orc_fexp(mode, x[i])
               : (mode & ORC_LM_DETMATH) ? fm3d_hypot_cr(x[i], y[i]) : hypot(x[i], y[i]);
}

static void orc_sph2car(int mode, double phi, double theta, double n[3])
{   /* tools.cpp:772-777 */
    n[0] = orc_fcos(mode, theta) * orc_fcos(mode, phi);
    n[1] = orc_fcos(mode, theta) * orc_fsin(mode, phi);
    n[2] = orc_fsin(mode, theta);
}

static void orc_car2sph(int mode, const double v[3], double *phi, double *theta)
{   /* tools.cpp:767-771 */
    *theta = orc_fatan2(mode, v[2], sqrt(v[0] * v[0] + v[1] * v[1]));
    *phi = orc_fatan2(mode, v[1], v[0]);
}

/* evaluateNormal (normaloptimizer.cpp:65-149).  Returns 0 or a status code. */
static int orc_eval(orc_lmdata *D, const double *par, double *fvec)
{
    double phi = par[0], theta = par[1];
    double n[3], mm, w_theta = 1.0, w_phi = 1.0, w;
    int i, L = D->level;
    const double cm = (double)D->cmax;
    D->nfev++;
    orc_sph2car(D->mode, phi, theta, n);
    if (n[2] != n[2] || n[1] != n[1] || n[0] != n[0]) return ORC_ST_NAN_NORMAL;
    /* get3dPointsFromImage1Pixels (:530-574): plane point per pixel, NaN ->
       exit(-6) (:465-469), outside isInBoundingBox (:646-655) -> abort */
    mm = n[0] * D->X[0] + n[1] * D->X[1] + n[2] * D->X[2];
    for (i = 0; i < D->m; i++) {
        double ux = D->ray[2 * i], uy = D->ray[2 * i + 1];
        double nn = n[0] * ux + n[1] * uy + n[2] * 1.;
        double k = mm / nn;
        double P0 = k * ux, P1 = k * uy, P2 = k * 1.;
        if (P0 != P0 || P1 != P1 || P2 != P2) return ORC_ST_NAN_PLANE;
        if (!((P0 > -cm && P0 < cm) && (P1 > -cm && P1 < cm) && (P2 > 0. && P2 < cm))) return ORC_ST_ABORT_BBOX;
    }
    if (!D->I1_ok) return ORC_ST_ABORT_PIX1;
    /* weight (:125-142); abs() is std::abs(double) under the reference's <cmath> */
    if (fabs(theta) - M_PI / 2 > 0 || fabs(phi) - M_PI > 0) {
        w_theta = orc_fexp(D->mode, fabs(theta) - M_PI / 2) + 1;
        w_phi = orc_fexp(D->mode, fabs(phi) - M_PI + 1) + 1;
    }
    w = w_phi * w_theta;
    /* projectPointsToImage2 (:591-644) and the residual (:145-148) */
    for (i = 0; i < D->m; i++) {
        double ux = D->ray[2 * i], uy = D->ray[2 * i + 1];
        double nn = n[0] * ux + n[1] * uy + n[2] * 1.;
        double k = mm / nn;
        double u, v;
        float I2;
        orc_project1(D->cam, D->R2, D->t2, k * ux, k * uy, k * 1., &u, &v);
        if (!orc_pixel_good(u, v, D->scale, D->pyr->w[L], D->pyr->h[L])) return ORC_ST_ABORT_PIX2;
        I2 = orc_bilinear(D->pyr->img[1][L], D->pyr->w[L], D->pyr->h[L], (float)(D->scale * u), (float)(D->scale * v));
        fvec[i] = w * (D->I1[i] - I2);
    }
    return 0;
}

/* The geometry of one evaluateNormal call without the intensities: image-1 pixels -> undistorted
   rays -> plane (X, n) -> camera-2 projection at pyramid level 0, i.e. get3dPointsFromImage1Pixels
   (singlecameratriangulator.cpp:530-574, projectPointToPlane :421-470, isInBoundingBox :646-655)
   followed by projectPointsToImage2 (:591-626) with scale 1.  This is what the reference's
   image2pixels drawing code paints (normaloptimizer.cpp:421-445: get3dPointsFromImage1Pixels +
   projectPointsToImage2(pointGroup, 1.0, ...) at the final normal).  uv: m x 2; status per pixel
   (0, ORC_ST_NAN_PLANE, ORC_ST_ABORT_BBOX, or ORC_ST_ABORT_PIX2 when w > 0 and the projection
   fails isPixelGood for a w x h image).  Returns the first non-zero status (the reference stops
   there), 0 if none. */
ORC_API int orc_plane_to_image2(const orc_camera *cam, const double R2[9], const double t2[3], const double X[3],
                                const double n[3], const double *pix, int m, double zmax, int w, int h, double *uv,
                                int *status)
{
    const double cm = (double)(int)(2 * zmax);
    double mm = n[0] * X[0] + n[1] * X[1] + n[2] * X[2];
    int i, first = 0;
    for (i = 0; i < m; i++) {
        double ux, uy, nn, k, P0, P1, P2;
        int st = 0;
        orc_undistort1(cam, pix[2 * i], pix[2 * i + 1], &ux, &uy);
        nn = n[0] * ux + n[1] * uy + n[2] * 1.;
        k = mm / nn;
        P0 = k * ux; P1 = k * uy; P2 = k * 1.;
        if (P0 != P0 || P1 != P1 || P2 != P2) st = ORC_ST_NAN_PLANE;
        else if (!((P0 > -cm && P0 < cm) && (P1 > -cm && P1 < cm) && (P2 > 0. && P2 < cm))) st = ORC_ST_ABORT_BBOX;
        orc_project1(cam, R2, t2, P0, P1, P2, &uv[2 * i], &uv[2 * i + 1]);
        if (!st && w > 0 && !orc_pixel_good(uv[2 * i], uv[2 * i + 1], 1.0, w, h)) st = ORC_ST_ABORT_PIX2;
        status[i] = st;
        if (st && !first) first = st;
    }
    return first;
}

/* The patch sample of projectPointsToImage / projectReferencePointsToImageWithFrame
   (singlecameratriangulator.cpp:737-766, :819-848): 0 where isPixelGood(p, 1.0) fails for a
   w x h image, else static_cast<uchar>(getBilinearInterpPix32f(img, x, y)) (truncation). */
ORC_API void orc_sample_points(const uint8_t *img, int w, int h, const double *uv, int n, uint8_t *out)
{
    int i;
    for (i = 0; i < n; i++) {
        double x = uv[2 * i], y = uv[2 * i + 1];
        out[i] = orc_pixel_good(x, y, 1.0, w, h) ? (uint8_t)orc_bilinear(img, w, h, (float)x, (float)y) : 0;
    }
}

/* ---- MINPACK building blocks (lmfit's lm_enorm/lm_qrfac/lm_lmpar/lm_qrsolv) ---- */
#define LM_EPSMCH DBL_EPSILON
#define LM_DWARF DBL_MIN

/* enorm: scaled Euclidean norm (MINPACK) */
static double orc_enorm(int n, const double *x)
{
    const double rdwarf = orc_lmv_enorm ? sqrt(DBL_MIN) : 3.834e-20, rgiant = orc_lmv_enorm ? sqrt(DBL_MAX) : 1.304e19;
    double s1 = 0, s2 = 0, s3 = 0, x1max = 0, x3max = 0, agiant = rgiant / (double)n, xabs, temp;
    int i;
    for (i = 0; i < n; i++) {
        xabs = fabs(x[i]);
        if (xabs > rdwarf && xabs < agiant) {
            s2 += xabs * xabs;
        } else if (xabs > rdwarf) {
            if (xabs > x1max) { temp = x1max / xabs; s1 = 1 + s1 * temp * temp; x1max = xabs; }
            else { temp = xabs / x1max; s1 += temp * temp; }
        } else {
            if (xabs > x3max) { temp = x3max / xabs; s3 = 1 + s3 * temp * temp; x3max = xabs; }
            else if (xabs != 0.) { temp = xabs / x3max; s3 += temp * temp; }
        }
    }
    if (s1 != 0) return x1max * sqrt(s1 + (s2 / x1max) / x1max);
    if (s2 != 0) {
        if (s2 >= x3max) return sqrt(s2 * (1 + (x3max / s2) * (x3max * s3)));
        return sqrt(x3max * ((s2 / x3max) + (x3max * s3)));
    }
    return x3max * sqrt(s3);
}

/* ---- ORC_LM_TREE: every m_dat-long sum as the LM kernel's fixed blocked tree ----
   (csrc/fm3d_lm2.hip, TREE).  Entry e (its absolute neighbourhood-entry index) belongs
   to lane l = e % 64 of chunk e / 64.  acc[l] is the sequential sum, from +0, of the lane's terms in
   chunk order; then the xor butterfly p[l] = p[l] + p[l ^ o] for o = 32, 16, ..., 1.  IEEE addition
   is commutative, so every lane ends with the same value: the sum. */
#define ORC_TL 64
typedef struct {
    double acc[ORC_TL];
} orc_tree;
static void orc_tree_init(orc_tree *t) { memset(t, 0, sizeof *t); }
static inline void orc_tree_add(orc_tree *t, int e, double v) { t->acc[e % ORC_TL] += v; }
static double orc_tree_finish(const orc_tree *t)
{
    double p[ORC_TL], q[ORC_TL];
    int l, o;
    memcpy(p, t->acc, sizeof p);
    for (o = ORC_TL / 2; o > 0; o >>= 1) {
        for (l = 0; l < ORC_TL; l++) q[l] = p[l] + p[l ^ o];
        memcpy(p, q, sizeof p);
    }
    return p[0];
}
/* the enorm of x[j0..n) (entries at their absolute positions): sqrt of the tree sum of squares when
   every component lies in MINPACK's intermediate range or is zero (enorm's own result there is
   sqrt(s2)); otherwise MINPACK's sequential enorm (a chunk with a value outside that range: the
   kernel's rare serial path) */
/* tree-mode path counters (tests/test_gpu_lm_tree.py, tools/full_parity.py): [0] Jacobians whose QR
   took the Gram form, [1] the Householder form (ill conditioned, a slow column or non-finite sums),
   [2] sums of squares that took the sequential enorm, [3] the Householder form for a zero Jacobian */
ORC_API long long orc_tree_stats[4];
static void orc_tree_count(int k)
{
#ifdef _OPENMP
#pragma omp atomic
#endif
    orc_tree_stats[k]++;
}
static int orc_enorm_slow(int j0, int n, const double *x)
{
    const double rdwarf = orc_lmv_enorm ? sqrt(DBL_MIN) : 3.834e-20, rgiant = orc_lmv_enorm ? sqrt(DBL_MAX) : 1.304e19;
    const double agiant = rgiant / (double)(n - j0);
    int i;
    for (i = j0; i < n; i++) {
        double xa = fabs(x[i]);
        if (!(xa < agiant) || (xa <= rdwarf && xa != 0.)) return 1;
    }
    return 0;
}
static double orc_enorm_tree(int j0, int n, const double *x)
{
    orc_tree t;
    int i;
    if (orc_enorm_slow(j0, n, x)) {
        orc_tree_count(2);
        return orc_enorm(n - j0, x + j0);
    }
    orc_tree_init(&t);
    for (i = j0; i < n; i++) orc_tree_add(&t, i, x[i] * x[i]);
    return sqrt(orc_tree_finish(&t));
}
static double orc_dot_tree(int j0, int n, const double *a, const double *b)
{
    orc_tree t;
    int i;
    orc_tree_init(&t);
    for (i = j0; i < n; i++) orc_tree_add(&t, i, a[i] * b[i]);
    return orc_tree_finish(&t);
}

/* qrsolv (MINPACK), r column-major with leading dimension ldr */
static void orc_qrsolv(int n, double *r, int ldr, const int *ipvt, const double *diag, const double *qtb,
                       double *x, double *sdiag, double *wa)
{
    int i, j, k, l, nsing;
    double qtbpj, sum, temp, sn, cs, tn, ct;
#define R_(i, j) r[(j) * ldr + (i)]
    for (j = 0; j < n; j++) {
        for (i = j; i < n; i++) R_(i, j) = R_(j, i);
        x[j] = R_(j, j);
        wa[j] = qtb[j];
    }
    for (j = 0; j < n; j++) {
        l = ipvt[j];
        if (diag[l] != 0.) {
            for (k = j; k < n; k++) sdiag[k] = 0.;
            sdiag[j] = diag[l];
            qtbpj = 0.;
            for (k = j; k < n; k++) {
                if (sdiag[k] == 0.) continue;
                if (fabs(R_(k, k)) < fabs(sdiag[k])) {
                    ct = R_(k, k) / sdiag[k];
                    sn = 0.5 / sqrt(0.25 + 0.25 * ct * ct);
                    cs = sn * ct;
                } else {
                    tn = sdiag[k] / R_(k, k);
                    cs = 0.5 / sqrt(0.25 + 0.25 * tn * tn);
                    sn = cs * tn;
                }
                R_(k, k) = cs * R_(k, k) + sn * sdiag[k];
                temp = cs * wa[k] + sn * qtbpj;
                qtbpj = -sn * wa[k] + cs * qtbpj;
                wa[k] = temp;
                for (i = k + 1; i < n; i++) {
                    temp = cs * R_(i, k) + sn * sdiag[i];
                    sdiag[i] = -sn * R_(i, k) + cs * sdiag[i];
                    R_(i, k) = temp;
                }
            }
        }
        sdiag[j] = R_(j, j);
        R_(j, j) = x[j];
    }
    nsing = n;
    for (j = 0; j < n; j++) {
        if (sdiag[j] == 0. && nsing == n) nsing = j;
        if (nsing < n) wa[j] = 0.;
    }
    for (k = 0; k < nsing; k++) {
        j = nsing - k - 1;
        sum = 0.;
        for (i = j + 1; i < nsing; i++) sum += R_(i, j) * wa[i];
        wa[j] = (wa[j] - sum) / sdiag[j];
    }
    for (j = 0; j < n; j++) x[ipvt[j]] = wa[j];
#undef R_
}

/* lmpar (MINPACK) */
static void orc_lmpar(int n, double *r, int ldr, const int *ipvt, const double *diag, const double *qtb,
                      double delta, double *par, double *x, double *sdiag, double *wa1, double *wa2)
{
    const double p1 = 0.1, p001 = 0.001;
    int i, iter, j, l, nsing;
    double dxnorm, fp, gnorm, parc, parl, paru, sum, temp;
#define R_(i, j) r[(j) * ldr + (i)]
    nsing = n;
    for (j = 0; j < n; j++) {
        wa1[j] = qtb[j];
        if (R_(j, j) == 0. && nsing == n) nsing = j;
        if (nsing < n) wa1[j] = 0.;
    }
    for (i = 0; i < nsing; i++) {
        j = nsing - i - 1;
        wa1[j] = wa1[j] / R_(j, j);
        temp = wa1[j];
        for (l = 0; l < j; l++) wa1[l] -= R_(l, j) * temp;
    }
    for (j = 0; j < n; j++) x[ipvt[j]] = wa1[j];
    iter = 0;
    for (j = 0; j < n; j++) wa2[j] = diag[j] * x[j];
    dxnorm = orc_enorm(n, wa2);
    fp = dxnorm - delta;
    if (fp <= p1 * delta) goto done;
    parl = 0.;
    if (nsing >= n) {
        for (j = 0; j < n; j++) { l = ipvt[j]; wa1[j] = diag[l] * (wa2[l] / dxnorm); }
        for (j = 0; j < n; j++) {
            sum = 0.;
            for (i = 0; i < j; i++) sum += R_(i, j) * wa1[i];
            wa1[j] = (wa1[j] - sum) / R_(j, j);
        }
        temp = orc_enorm(n, wa1);
        parl = ((fp / delta) / temp) / temp;
    }
    for (j = 0; j < n; j++) {
        sum = 0.;
        for (i = 0; i <= j; i++) sum += R_(i, j) * qtb[i];
        l = ipvt[j];
        wa1[j] = sum / diag[l];
    }
    gnorm = orc_enorm(n, wa1);
    paru = gnorm / delta;
    if (paru == 0.) paru = LM_DWARF / (delta < p1 ? delta : p1);
    *par = *par > parl ? *par : parl;
    *par = *par < paru ? *par : paru;
    if (*par == 0.) *par = gnorm / dxnorm;
    for (;;) {
        iter++;
        if (*par == 0.) *par = (LM_DWARF > p001 * paru) ? LM_DWARF : p001 * paru;
        temp = sqrt(*par);
        for (j = 0; j < n; j++) wa1[j] = temp * diag[j];
        orc_qrsolv(n, r, ldr, ipvt, wa1, qtb, x, sdiag, wa2);
        for (j = 0; j < n; j++) wa2[j] = diag[j] * x[j];
        dxnorm = orc_enorm(n, wa2);
        temp = fp;
        fp = dxnorm - delta;
        if (fabs(fp) <= p1 * delta || (parl == 0. && fp <= temp && temp < 0.) || iter == 10) break;
        for (j = 0; j < n; j++) { l = ipvt[j]; wa1[j] = diag[l] * (wa2[l] / dxnorm); }
        for (j = 0; j < n; j++) {
            wa1[j] = wa1[j] / sdiag[j];
            temp = wa1[j];
            for (i = j + 1; i < n; i++) wa1[i] -= R_(i, j) * temp;
        }
        temp = orc_enorm(n, wa1);
        parc = ((fp / delta) / temp) / temp;
        if (fp > 0.) parl = parl > *par ? parl : *par;
        if (fp < 0.) paru = paru < *par ? paru : *par;
        *par = parl > *par + parc ? parl : *par + parc;
    }
done:
    if (iter == 0) *par = 0.;
#undef R_
}

/* qrfac with column pivoting + lmdif's qtf for n = 2 with the tree sums (ORC_LM_TREE).  The same
   steps as orc_jac_qr's Householder form, every m-long sum an orc_tree over absolute entry positions.
   With ORC_LM_GRAM the Householder quantities come from the tree sums of the Jacobian sweep, by
   exact identities of the reflections (H0 = I - v v^T / v0, v = a_p / s0 + e0, s0 = +-||a_p||):
     r00 = -s0,  r01 = (H0 a_q)_0 = -(a_p.a_q) / s0,  qtf0 = (H0 f)_0 = -(a_p.f) / s0,
     ||(H0 a_q)_{1..}||^2 = S_qq - r01^2,  s1 = +-sqrt(that) with the sign of (H0 a_q)_1,
     r11 = -s1,  qtf1 = -((a_q.f) - r01 qtf0) / s1
   where (H0 a_q)_1 = a_q1 - t v1, t = ((a_p.a_q) / s0 + a_q0) / v0.  Used when every column value is
   in enorm's intermediate range (or zero), s0 != 0, the sums are finite and S_qq - r01^2 >
   ORC_GRAM_C * S_qq; otherwise the Householder form. */
static void orc_qr_tree(int mode, int m, double *fjac, const double *fvec, double *wa4, double r[4], double qtf[2],
                        double acnorm[2], int ipvt[2])
{
    double rdiag[2], ajnorm, sum, temp;
    int i, j, k, pc;
    for (j = 0; j < 2; j++) acnorm[j] = orc_enorm_tree(0, m, &fjac[j * m]);
    pc = acnorm[1] > acnorm[0] ? 1 : 0;
    ipvt[0] = pc;
    ipvt[1] = 1 - pc;
    if (pc) {
        for (i = 0; i < m; i++) { temp = fjac[i]; fjac[i] = fjac[m + i]; fjac[m + i] = temp; }
    }
    if ((mode & ORC_LM_GRAM) && !orc_enorm_slow(0, m, fjac) && !orc_enorm_slow(0, m, fjac + m) && acnorm[pc] != 0.) {
        const double *ap = fjac, *aq = fjac + m;
        double Spq = orc_dot_tree(0, m, ap, aq), Spf = orc_dot_tree(0, m, ap, fvec), Sqf = orc_dot_tree(0, m, aq, fvec);
        double Sqq = orc_dot_tree(0, m, aq, aq);
        double s0 = ap[0] < 0. ? -acnorm[pc] : acnorm[pc];
        double r01 = -(Spq / s0), qtf0 = -(Spf / s0), d = Sqq - r01 * r01;
        if (isfinite(Spq) && isfinite(Spf) && isfinite(Sqf) && isfinite(Sqq) && d > ORC_GRAM_C * Sqq) {
            double v0 = ap[0] / s0 + 1., v1 = ap[1] / s0, t = (Spq / s0 + aq[0]) / v0, a1 = aq[1] - t * v1;
            double s1 = sqrt(d);
            if (a1 < 0.) s1 = -s1;
            r[0] = -s0; r[1] = 0.; r[2] = r01; r[3] = -s1;
            qtf[0] = qtf0;
            qtf[1] = -((Sqf - r01 * qtf0) / s1);
            orc_tree_count(0);
            return;
        }
    }
    /* the Householder form (MINPACK qrfac, n = 2; the rdiag update of column 1 after step 0 does not
       reach the result for n = 2) */
    orc_tree_count(acnorm[pc] == 0. ? 3 : 1);
    for (j = 0; j < 2; j++) {
        ajnorm = j == 0 ? acnorm[pc] : orc_enorm_tree(1, m, &fjac[m]);
        if (ajnorm == 0.) { rdiag[j] = 0.; continue; }
        if (fjac[j * m + j] < 0.) ajnorm = -ajnorm;
        for (i = j; i < m; i++) fjac[j * m + i] /= ajnorm;
        fjac[j * m + j] += 1.;
        for (k = j + 1; k < 2; k++) {
            sum = orc_dot_tree(j, m, &fjac[j * m], &fjac[k * m]);
            temp = sum / fjac[j * m + j];
            for (i = j; i < m; i++) fjac[k * m + i] -= temp * fjac[j * m + i];
        }
        rdiag[j] = -ajnorm;
    }
    for (i = 0; i < m; i++) wa4[i] = fvec[i];
    for (j = 0; j < 2; j++) {
        if (fjac[j * m + j] != 0.) {
            sum = orc_dot_tree(j, m, &fjac[j * m], wa4);
            temp = -sum / fjac[j * m + j];
            for (i = j; i < m; i++) wa4[i] += fjac[j * m + i] * temp;
        }
        fjac[j * m + j] = rdiag[j];
        qtf[j] = wa4[j];
    }
    r[0] = fjac[0]; r[1] = 0.; r[2] = fjac[m + 0]; r[3] = fjac[m + 1];
}

/* Jacobian + QR.  Output: r (2x2 column-major upper triangle), qtf, acnorm,
   ipvt.  Returns 0 or a failure status of one of the two evaluations. */
static int orc_jac_qr(orc_lmdata *D, double *x, const double *fvec, double eps,
                      double *fjac, double *wa4, double *tmp, double r[4], double qtf[2],
                      double acnorm[2], int ipvt[2])
{
    int m = D->m, i, j, st;
    double h[2];
    /* fdjac2 (MINPACK): forward differences, h = eps*|x_j| (eps if 0) */
    for (j = 0; j < 2; j++) {
        double temp = x[j];
        h[j] = eps * fabs(temp);
        if (D->mode & ORC_LMV_FDFLOOR) {
            if (h[j] < eps * eps) h[j] = eps * eps;  /* lmfit: step = MAX(eps*eps, eps*fabs(x)) */
        } else if (h[j] == 0.) h[j] = eps;
        x[j] = temp + h[j];
        st = orc_eval(D, x, wa4);
        x[j] = temp;
        if (st) return st;
        for (i = 0; i < m; i++) fjac[j * m + i] = (wa4[i] - fvec[i]) / h[j];
    }
    if (D->mode & ORC_LM_TREE) {
        orc_qr_tree(D->mode, m, fjac, fvec, wa4, r, qtf, acnorm, ipvt);
        return 0;
    }
    {
        /* qrfac with column pivoting (MINPACK), n = 2 */
        double rdiag[2], wa[2], ajnorm, sum, temp;
        int k, kmax;
        for (j = 0; j < 2; j++) {
            acnorm[j] = orc_enorm(m, &fjac[j * m]);
            rdiag[j] = acnorm[j];
            wa[j] = rdiag[j];
            ipvt[j] = j;
        }
        for (j = 0; j < 2; j++) {
            kmax = j;
            for (k = j + 1; k < 2; k++)
                if (rdiag[k] > rdiag[kmax]) kmax = k;
            if (kmax != j) {
                for (i = 0; i < m; i++) { temp = fjac[j * m + i]; fjac[j * m + i] = fjac[kmax * m + i]; fjac[kmax * m + i] = temp; }
                rdiag[kmax] = rdiag[j];
                wa[kmax] = wa[j];
                k = ipvt[j]; ipvt[j] = ipvt[kmax]; ipvt[kmax] = k;
            }
            ajnorm = orc_enorm(m - j, &fjac[j * m + j]);
            if (ajnorm == 0.) { rdiag[j] = 0.; continue; }
            if (fjac[j * m + j] < 0.) ajnorm = -ajnorm;
            for (i = j; i < m; i++) fjac[j * m + i] /= ajnorm;
            fjac[j * m + j] += 1.;
            for (k = j + 1; k < 2; k++) {
                sum = 0.;
                for (i = j; i < m; i++) sum += fjac[j * m + i] * fjac[k * m + i];
                temp = sum / fjac[j * m + j];
                for (i = j; i < m; i++) fjac[k * m + i] -= temp * fjac[j * m + i];
                if (rdiag[k] != 0.) {
                    temp = fjac[k * m + j] / rdiag[k];
                    temp = 1. - temp * temp;
                    rdiag[k] *= sqrt(temp > 0. ? temp : 0.);
                    temp = rdiag[k] / wa[k];
                    if (0.05 * temp * temp <= LM_EPSMCH) {
                        rdiag[k] = orc_enorm(m - j - 1, &fjac[k * m + j + 1]);
                        wa[k] = rdiag[k];
                    }
                }
            }
            rdiag[j] = -ajnorm;
        }
        /* lmdif: form (q transpose)*fvec, keep the first n components */
        for (i = 0; i < m; i++) wa4[i] = fvec[i];
        for (j = 0; j < 2; j++) {
            if (fjac[j * m + j] != 0.) {
                sum = 0.;
                for (i = j; i < m; i++) sum += fjac[j * m + i] * wa4[i];
                temp = -sum / fjac[j * m + j];
                for (i = j; i < m; i++) wa4[i] += fjac[j * m + i] * temp;
            }
            fjac[j * m + j] = rdiag[j];
            qtf[j] = wa4[j];
        }
        r[0] = fjac[0]; r[1] = 0.; r[2] = fjac[m + 0]; r[3] = fjac[m + 1];
    }
    return 0;
}

/* lmdif (MINPACK) with lmfit's lmmin control (lm_control_double:
   ftol=xtol=gtol=30*DBL_EPSILON, stepbound(factor)=100, patience=100 ->
   maxfev = 300, scale_diag = 1 -> mode 1).  Returns the lmdif info (1..8) or,
   for a user break (evaluateNormal *info = -1, lmmin status.info = 11), the
   negated failure status. */
static int orc_lmdif(orc_lmdata *D, double *x, double epsfcn, double *fvec, double *fjac, double *wa4,
                     double *tmp, int *nfev_out)
{
    const int n = 2, maxfev = 100 * (2 + 1);
    const double tol = (D->mode & ORC_LMV_TOL1E14) ? 1e-14 : 30 * LM_EPSMCH;
    const double ftol = tol, xtol = tol, gtol = tol, factor = 100.;
    const double p1 = 0.1, p5 = 0.5, p25 = 0.25, p75 = 0.75, p0001 = 1.0e-4;
    double eps = sqrt(epsfcn > LM_EPSMCH ? epsfcn : LM_EPSMCH);
    double diag[2], r[4], qtf[2], acnorm[2], wa1[2], wa2[2], wa3[2], sdiag[2], lw[2];
    double par = 0., delta = 0., xnorm = 0., fnorm, fnorm1, gnorm, pnorm, actred, prered, dirder, ratio, temp, temp1, temp2, sum;
    int ipvt[2], iter = 1, info = 0, st, i, j, l;
    D->nfev = 0;
    /* lmdif input check: m < n is "improper input parameters" (info 0), no evaluation */
    if (D->m < n) { *nfev_out = 0; return 0; }
    st = orc_eval(D, x, fvec);
    if (st) { *nfev_out = (int)D->nfev; return -st; }
    fnorm = (D->mode & ORC_LM_TREE) ? orc_enorm_tree(0, D->m, fvec) : orc_enorm(D->m, fvec);
    if ((D->mode & ORC_LMV_DWARFEXIT) && fnorm <= LM_DWARF) { *nfev_out = (int)D->nfev; return 0; }
    for (;;) {
        st = orc_jac_qr(D, x, fvec, eps, fjac, wa4, tmp, r, qtf, acnorm, ipvt);
        if (st) { *nfev_out = (int)D->nfev; return -st; }
        if (iter == 1) {
            for (j = 0; j < n; j++) {
                diag[j] = acnorm[j];
                if (acnorm[j] == 0.) diag[j] = 1.;
            }
            for (j = 0; j < n; j++) wa3[j] = diag[j] * x[j];
            xnorm = orc_enorm(n, wa3);
            delta = factor * xnorm;
            if (delta == 0.) delta = factor;
        }
        gnorm = 0.;
        if (fnorm != 0.) {
            for (j = 0; j < n; j++) {
                l = ipvt[j];
                if (acnorm[l] == 0.) continue;
                sum = 0.;
                for (i = 0; i <= j; i++) sum += r[j * 2 + i] * (qtf[i] / fnorm);
                temp = fabs(sum / acnorm[l]);
                gnorm = gnorm > temp ? gnorm : temp;
            }
        }
        if (gnorm <= gtol) info = 4;
        if (info != 0) break;
        for (j = 0; j < n; j++) diag[j] = diag[j] > acnorm[j] ? diag[j] : acnorm[j];
        do {
            double rr[4];
            for (j = 0; j < 4; j++) rr[j] = r[j];
            orc_lmpar(n, rr, 2, ipvt, diag, qtf, delta, &par, wa1, sdiag, lw, wa3);
            /* the R upper triangle is restored by qrsolv; keep the original */
            for (j = 0; j < n; j++) {
                wa1[j] = -wa1[j];
                wa2[j] = x[j] + wa1[j];
                wa3[j] = diag[j] * wa1[j];
            }
            pnorm = orc_enorm(n, wa3);
            if (iter == 1) delta = delta < pnorm ? delta : pnorm;
            st = orc_eval(D, wa2, wa4);
            if (st) { *nfev_out = (int)D->nfev; return -st; }
            fnorm1 = (D->mode & ORC_LM_TREE) ? orc_enorm_tree(0, D->m, wa4) : orc_enorm(D->m, wa4);
            actred = -1.;
            if (p1 * fnorm1 < fnorm) actred = 1. - (fnorm1 / fnorm) * (fnorm1 / fnorm);
            for (j = 0; j < n; j++) {
                wa3[j] = 0.;
                l = ipvt[j];
                temp = wa1[l];
                for (i = 0; i <= j; i++) wa3[i] += r[j * 2 + i] * temp;
            }
            temp1 = orc_enorm(n, wa3) / fnorm;
            temp2 = (sqrt(par) * pnorm) / fnorm;
            prered = temp1 * temp1 + temp2 * temp2 / p5;
            dirder = -(temp1 * temp1 + temp2 * temp2);
            ratio = 0.;
            if (prered != 0.) ratio = actred / prered;
            if (ratio <= p25) {
                if (actred >= 0.) temp = p5;
                else temp = p5 * dirder / (dirder + p5 * actred);
                if (p1 * fnorm1 >= fnorm || temp < p1) temp = p1;
                delta = temp * (delta < pnorm / p1 ? delta : pnorm / p1);
                par = par / temp;
            } else if (par == 0. || ratio >= p75) {
                delta = pnorm / p5;
                par = p5 * par;
            }
            if (ratio >= p0001) {
                for (j = 0; j < n; j++) {
                    x[j] = wa2[j];
                    wa2[j] = diag[j] * x[j];
                }
                for (i = 0; i < D->m; i++) fvec[i] = wa4[i];
                xnorm = orc_enorm(n, wa2);
                fnorm = fnorm1;
                iter++;
            }
            if (fabs(actred) <= ftol && prered <= ftol && p5 * ratio <= 1.) info = 1;
            if (delta <= xtol * xnorm) info = 2;
            if (fabs(actred) <= ftol && prered <= ftol && p5 * ratio <= 1. && info == 2) info = 3;
            if (info != 0) goto out;
            if (D->nfev >= maxfev) info = 5;
            if (fabs(actred) <= LM_EPSMCH && prered <= LM_EPSMCH && p5 * ratio <= 1.) info = 6;
            if (delta <= LM_EPSMCH * xnorm) info = 7;
            if (gnorm <= LM_EPSMCH) info = 8;
            if (info != 0) goto out;
        } while (ratio < p0001);
    }
out:
    *nfev_out = (int)D->nfev;
    return info;
}

/* Standalone LM driver for tests: minimises the evaluateNormal residual of one
   point at one pyramid level starting from par.  Returns info. */

/* One point: computeOptimizedNormals body (:335-449) with optimize_pyramid
   (:223-245) and optimize (:247-292).  Returns the status; normal in n_out;
   per-level lmdif info and evaluation counts (index = level). */
static int orc_point(const orc_camera *cam, const double R2[9], const double t2[3], const orc_pyramid *pyr,
                     int levels, const double X[3], int ray, int boundW, int boundH, double epsfcn, int cmax,
                     int mode, double n_out[3], int *info_out, int *nfev_out, int *mdat_out)
{
    int side = 2 * ray + 1, cap = side * side, m, L, i, status = ORC_ST_OK;
    double *pix, *rays, *fvec, *fjac, *wa4, *tmp, nrm, norm[3], inv;
    float *I1;
    float img_scale;
    orc_lmdata D;
    for (L = 0; L <= levels; L++) { info_out[L] = 0; nfev_out[L] = 0; }
    pix = (double *)malloc(sizeof(double) * 2 * cap);
    m = orc_neighborhood(cam, X, ray, boundW, boundH, pix, cap);
    *mdat_out = m;
    if (m <= 0) { free(pix); return ORC_ST_NO_PIXELS; }
    rays = (double *)malloc(sizeof(double) * 2 * m);
    fvec = (double *)malloc(sizeof(double) * m);
    fjac = (double *)malloc(sizeof(double) * 2 * m);
    wa4 = (double *)malloc(sizeof(double) * m);
    tmp = (double *)malloc(sizeof(double) * m);
    I1 = (float *)malloc(sizeof(float) * m);
    for (i = 0; i < m; i++) orc_undistort1(cam, pix[2 * i], pix[2 * i + 1], &rays[2 * i], &rays[2 * i + 1]);
    /* initial guess: viewing ray, Vec3d / norm == multiply by 1/norm (:342-343) */
    nrm = sqrt(X[0] * X[0] + X[1] * X[1] + X[2] * X[2]);
    inv = 1. / nrm;
    norm[0] = X[0] * inv; norm[1] = X[1] * inv; norm[2] = X[2] * inv;
    memset(&D, 0, sizeof(D));
    D.cam = cam; D.R2 = R2; D.t2 = t2; D.pyr = pyr;
    D.X[0] = X[0]; D.X[1] = X[1]; D.X[2] = X[2];
    D.cmax = cmax; D.m = m; D.ray = rays; D.pix = pix; D.I1 = I1; D.mode = mode;
    img_scale = (float)pow(2.0, (double)levels);
    for (L = levels; L >= 0; L--) {
        double par[2];
        int info, nfev;
        D.level = L;
        D.scale = 1.0 / img_scale;
        orc_update_I1(&D);
        orc_car2sph(mode, norm, &par[0], &par[1]);
        info = orc_lmdif(&D, par, epsfcn, fvec, fjac, wa4, tmp, &nfev);
        info_out[L] = info;
        nfev_out[L] = nfev;
        if (info < 0) { status = -info; break; }
        orc_sph2car(mode, par[0], par[1], norm);
        img_scale /= 2.0f;
    }
    n_out[0] = norm[0]; n_out[1] = norm[1]; n_out[2] = norm[2];
    free(pix); free(rays); free(fvec); free(fjac); free(wa4); free(tmp); free(I1);
    return status;
}

/* pyramid storage owned by the caller: levels+1 images of each frame */
static void orc_build_pyramid(const uint8_t *img1, const uint8_t *img2, int w, int h, int levels,
                              orc_pyramid *pyr, uint8_t **bufs)
{
    int L, f;
    pyr->w[0] = w; pyr->h[0] = h;
    pyr->img[0][0] = img1; pyr->img[1][0] = img2;
    for (L = 1; L <= levels; L++) {
        pyr->w[L] = (pyr->w[L - 1] + 1) / 2;
        pyr->h[L] = (pyr->h[L - 1] + 1) / 2;
        for (f = 0; f < 2; f++) {
            uint8_t *b = (uint8_t *)malloc((size_t)pyr->w[L] * pyr->h[L]);
            orc_pyrdown(pyr->img[f][L - 1], pyr->w[L - 1], pyr->h[L - 1], b);
            pyr->img[f][L] = b;
            bufs[2 * L + f] = b;
        }
    }
}

/* NormalOptimizer::computeOptimizedNormals over P points.  Per point: normal,
   status (0 = kept; the reference erases every other point from points3D in
   place, preserving order), per-level info and nfev (8 slots per point, index
   = pyramid level), m_dat.  Returns the number of kept points. */
ORC_API int orc_optimize_normals(const orc_camera *cam, const double R2[9], const double t2[3],
                                 const uint8_t *img1, const uint8_t *img2, int w, int h, int levels,
                                 const double *points, int P, int ray, int boundW, int boundH, double epsfcn,
                                 double zmax, int mode, double *normals, int *status, int *info,
                                 int *nfev, int *mdat, int nthreads)
{
    orc_pyramid pyr;
    uint8_t *bufs[16] = {0};
    int i, kept = 0, cmax = (int)(2 * zmax);
    if (levels > 7) return -1;
    orc_lmv_enorm = (mode & ORC_LMV_ENORM) != 0;
    orc_build_pyramid(img1, img2, w, h, levels, &pyr, bufs);
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : kept)
#endif
    for (i = 0; i < P; i++) {
        status[i] = orc_point(cam, R2, t2, &pyr, levels, &points[3 * i], ray, boundW, boundH, epsfcn, cmax, mode,
                              &normals[3 * i], &info[8 * i], &nfev[8 * i], &mdat[i]);
        if (status[i] == ORC_ST_OK) kept++;
    }
    for (i = 0; i < 16; i++) free(bufs[i]);
    return kept;
}

/* NCC scoring of candidate normals (fm3d_ncc_hypotheses; BASELINE.json's "patch NCC over 16 / 32
   normal hypotheses" -- the reference has none, SURVEY.md D2, so this restates the extension on the
   reference's own geometry: extractPixelsContour :341-397, evaluateNormal :65-149 with the
   deterministic transcendentals).  Per point: normals sph2car(phi0 + dphi, theta0 + dtheta) on an
   Hphi x Htheta grid of half width span around car2sph(X/|X|); per normal the level-0 samples
   I1 (image 1 at the pixel) and I2 (image 2 through the plane); score = NCC or -2 (a failing
   pixel, a flat patch).  Round 5: the plane point P = (mm / nn) r of the ray r = (ux, uy, 1) is
   tested against the bounding box and projected without the quotient (camera 2 sees it at
   (mm R2 r + nn t2) / nn, so x = (mm q0 + nn t0) / (mm q2 + nn t2), q = R2 r), and every
   product-and-sum from nn to the pixel coordinates is one fma (orc_ncc_project).  The five sums are accumulated per lane l = offset index mod 64 in offset
   order and combined by the xor tree over 64 lanes -- the GPU's order, so the scores are bit-equal.
   scores: P x H, normals: P x 3 (best, lowest h on ties; X/|X| if none), best: P (-1 if none). */
ORC_API void orc_ncc_hypotheses(const orc_camera *cam, const double R2[9], const double t2[3], const uint8_t *img1,
                                const uint8_t *img2, int w, int h, const double *points, int P, int ray, int boundW,
                                int boundH, double zmax, int Hphi, int Htheta, double span, double *scores,
                                double *normals, int *best)
{
    static const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    static const double Z[3] = {0, 0, 0};
    const int H = Hphi * Htheta, cmax = (int)(2 * zmax);
    const double cm = (double)cmax;
    int p;
    #pragma omp parallel for schedule(dynamic, 1)
    for (p = 0; p < P; p++) {
        const double *X = points + 3 * (size_t)p;
        double ccx, ccy, g[3], phi0, theta0, inv;
        int hh, e, l, bestH = -1, i, j;
        double bs = -2.;
        orc_project1(cam, I, Z, X[0], X[1], X[2], &ccx, &ccy);
        inv = 1. / sqrt(X[0] * X[0] + X[1] * X[1] + X[2] * X[2]);
        g[0] = X[0] * inv; g[1] = X[1] * inv; g[2] = X[2] * inv;
        orc_car2sph(ORC_LM_DETMATH | ORC_DET_1ULP, g, &phi0, &theta0);
        for (hh = 0; hh < H; hh++) {
            const int ip = hh / Htheta, it = hh - ip * Htheta;
            const double dphi = span * (double)(2 * ip + 1 - Hphi) / Hphi;
            const double dtheta = span * (double)(2 * it + 1 - Htheta) / Htheta;
            double n[3], mm, S[5][64], T[5], sc = -2.;
            int m = 0, fail = 0, o;
            orc_sph2car(ORC_LM_DETMATH | ORC_DET_1ULP, phi0 + dphi, theta0 + dtheta, n);
            mm = n[0] * X[0] + n[1] * X[1] + n[2] * X[2];
            memset(S, 0, sizeof(S));
            e = 0;
            for (i = -ray; i <= ray; i++)
                for (j = -ray; j <= ray; j++) {
                    double px, py, ux, uy, nn, lim, q0, q1, q2, u, v, a, b;
                    if (i * i + j * j > ray * ray) continue;
                    l = e++ & 63;  /* the offset index's lane */
                    px = ccx + i;
                    py = ccy + j;
                    if (px < 0 || py < 0 || px >= boundW || py >= boundH) continue;
                    m++;
                    if (fail) continue;
                    if (!orc_pixel_good(px, py, 1.0, w, h)) { fail = 1; continue; }
                    a = (double)orc_bilinear(img1, w, h, (float)px, (float)py);
                    orc_undistort1(cam, px, py, &ux, &uy);
                    nn = fma(n[1], uy, fma(n[0], ux, n[2]));
                    /* the plane point P = (mm / nn) r without the division: |P0|, |P1| < cm and
                       0 < P2 < cm as |mm ux|, |mm uy|, |mm| < cm |nn| with mm, nn of one sign */
                    lim = cm * fabs(nn);
                    if (!(fabs(mm * ux) < lim && fabs(mm * uy) < lim && fabs(mm) < lim &&
                          ((mm > 0. && nn > 0.) || (mm < 0. && nn < 0.)))) { fail = 1; continue; }
                    /* camera 2 sees P at (mm q + nn t2) / nn, q = R2 r (the GPU stages q once per
                       entry): the normalised coordinates need one reciprocal */
                    q0 = R2[0] * ux + R2[1] * uy + R2[2];
                    q1 = R2[3] * ux + R2[4] * uy + R2[5];
                    q2 = R2[6] * ux + R2[7] * uy + R2[8];
                    orc_ncc_project(cam, fma(nn, t2[0], mm * q0), fma(nn, t2[1], mm * q1), fma(nn, t2[2], mm * q2),
                                    &u, &v);
                    if (!orc_pixel_good(u, v, 1.0, w, h)) { fail = 1; continue; }
                    b = (double)orc_bilinear(img2, w, h, (float)u, (float)v);
                    S[0][l] += a; S[1][l] += b; S[2][l] += a * a; S[3][l] += b * b; S[4][l] += a * b;
                }
            for (o = 0; o < 5; o++) {
                double v[64], t[64];
                int s2;
                memcpy(v, S[o], sizeof(v));
                for (s2 = 32; s2 > 0; s2 >>= 1) {
                    for (l = 0; l < 64; l++) t[l] = v[l] + v[l ^ s2];
                    memcpy(v, t, sizeof(v));
                }
                T[o] = v[0];
            }
            if (!fail && m > 0) {
                const double cov = T[4] - T[0] * T[1] / m, va = T[2] - T[0] * T[0] / m, vb = T[3] - T[1] * T[1] / m;
                if (va > 0 && vb > 0) sc = cov / sqrt(va * vb);
            }
            scores[(size_t)p * H + hh] = sc;
            if (sc > bs) { bs = sc; bestH = hh; }
        }
        best[p] = bestH;
        if (bestH >= 0) {
            const int ip = bestH / Htheta, it = bestH - ip * Htheta;
            orc_sph2car(ORC_LM_DETMATH | ORC_DET_1ULP, phi0 + span * (double)(2 * ip + 1 - Hphi) / Hphi,
                        theta0 + span * (double)(2 * it + 1 - Htheta) / Htheta, normals + 3 * (size_t)p);
        } else {
            normals[3 * p] = g[0]; normals[3 * p + 1] = g[1]; normals[3 * p + 2] = g[2];
        }
    }
}

/* Single-level LM on one point from a given starting (phi, theta): used by the
   tests that pin lmdif against scipy.optimize.leastsq on the same residual. */
ORC_API int orc_lm_single_level(const orc_camera *cam, const double R2[9], const double t2[3],
                                const uint8_t *img1, const uint8_t *img2, int w, int h, const double X[3],
                                const double *pix, int m, double epsfcn, double zmax, int mode,
                                double par[2], int *nfev_out)
{
    orc_pyramid pyr;
    orc_lmdata D;
    double *rays = (double *)malloc(sizeof(double) * 2 * m), *fvec = (double *)malloc(sizeof(double) * m);
    double *fjac = (double *)malloc(sizeof(double) * 2 * m), *wa4 = (double *)malloc(sizeof(double) * m);
    double *tmp = (double *)malloc(sizeof(double) * m);
    float *I1 = (float *)malloc(sizeof(float) * m);
    int i, info;
    pyr.img[0][0] = img1; pyr.img[1][0] = img2; pyr.w[0] = w; pyr.h[0] = h;
    for (i = 0; i < m; i++) orc_undistort1(cam, pix[2 * i], pix[2 * i + 1], &rays[2 * i], &rays[2 * i + 1]);
    memset(&D, 0, sizeof(D));
    D.cam = cam; D.R2 = R2; D.t2 = t2; D.pyr = &pyr; D.level = 0; D.scale = 1.0;
    D.X[0] = X[0]; D.X[1] = X[1]; D.X[2] = X[2];
    D.cmax = (int)(2 * zmax); D.m = m; D.ray = rays; D.pix = pix; D.I1 = I1; D.mode = mode;
    orc_update_I1(&D);
    info = orc_lmdif(&D, par, epsfcn, fvec, fjac, wa4, tmp, nfev_out);
    free(rays); free(fvec); free(fjac); free(wa4); free(tmp); free(I1);
    return info;
}

/* Residual vector of evaluateNormal at (phi, theta), level 0 (tests). */
ORC_API int orc_eval_residual(const orc_camera *cam, const double R2[9], const double t2[3],
                              const uint8_t *img1, const uint8_t *img2, int w, int h, const double X[3],
                              const double *pix, int m, double zmax, int mode, const double par[2], double *fvec)
{
    orc_pyramid pyr;
    orc_lmdata D;
    double *rays = (double *)malloc(sizeof(double) * 2 * m);
    float *I1 = (float *)malloc(sizeof(float) * m);
    int i, st;
    pyr.img[0][0] = img1; pyr.img[1][0] = img2; pyr.w[0] = w; pyr.h[0] = h;
    for (i = 0; i < m; i++) orc_undistort1(cam, pix[2 * i], pix[2 * i + 1], &rays[2 * i], &rays[2 * i + 1]);
    memset(&D, 0, sizeof(D));
    D.cam = cam; D.R2 = R2; D.t2 = t2; D.pyr = &pyr; D.level = 0; D.scale = 1.0;
    D.X[0] = X[0]; D.X[1] = X[1]; D.X[2] = X[2];
    D.cmax = (int)(2 * zmax); D.m = m; D.ray = rays; D.pix = pix; D.I1 = I1; D.mode = mode;
    orc_update_I1(&D);
    st = orc_eval(&D, par, fvec);
    free(rays); free(I1);
    return st;
}


/* ------------------------------------------------------------------ */
/* Feature frames + patch export              */
/* ------------------------------------------------------------------ */
/* NormalOptimizer ctor (normaloptimizer.cpp:160-178): gravity = Rodrigues(rodriguesIC).inv() *
   (0,0,-1), with OpenCV 2.4's closed-form 3x3 Matx inverse (Matx_FastInvOp<_Tp,3>, determinant by
   cofactors of the first row) and Matx * Vec accumulating from 0 in index order. */
ORC_API void orc_gravity(const double rIC[3], double g[3])
{
    double a[9], b[9], d;
    const double v[3] = {0, 0, -1};
    int i, k;
    orc_rodrigues_v2m(rIC, a);
#define A(i, j) a[(i)*3 + (j)]
    d = A(0, 0) * (A(1, 1) * A(2, 2) - A(2, 1) * A(1, 2)) - A(0, 1) * (A(1, 0) * A(2, 2) - A(2, 0) * A(1, 2)) +
        A(0, 2) * (A(1, 0) * A(2, 1) - A(2, 0) * A(1, 1));
    d = 1 / d;
    b[0] = (A(1, 1) * A(2, 2) - A(1, 2) * A(2, 1)) * d;
    b[1] = (A(0, 2) * A(2, 1) - A(0, 1) * A(2, 2)) * d;
    b[2] = (A(0, 1) * A(1, 2) - A(0, 2) * A(1, 1)) * d;
    b[3] = (A(1, 2) * A(2, 0) - A(1, 0) * A(2, 2)) * d;
    b[4] = (A(0, 0) * A(2, 2) - A(0, 2) * A(2, 0)) * d;
    b[5] = (A(0, 2) * A(1, 0) - A(0, 0) * A(1, 2)) * d;
    b[6] = (A(1, 0) * A(2, 1) - A(1, 1) * A(2, 0)) * d;
    b[7] = (A(0, 1) * A(2, 0) - A(0, 0) * A(2, 1)) * d;
    b[8] = (A(0, 0) * A(1, 1) - A(0, 1) * A(1, 0)) * d;
#undef A
    for (i = 0; i < 3; i++) {
        double s = 0;
        for (k = 0; k < 3; k++) s += b[i * 3 + k] * v[k];
        g[i] = s;
    }
}

/* cv::normalize(v, v) of a Vec3d: scale = 1/||v|| (sum of squares from 0 in index order),
   0 if ||v|| <= DBL_EPSILON; then v*scale + 0 (convertTo with scale and shift 0). */
static void orc_normalize3(double v[3])
{
    double s = 0, scale;
    int i;
    for (i = 0; i < 3; i++) s += v[i] * v[i];
    s = sqrt(s);
    scale = s > DBL_EPSILON ? 1 / s : 0.;
    for (i = 0; i < 3; i++) v[i] = v[i] * scale + 0.;
}

/* computeFeaturesFrames (normaloptimizer.cpp:454-504): z = n, x = g x z, y = z x x (before
   normalisation), normalise x and y, columns (e.x, e.y, e.z) with Vec::dot accumulating from 0,
   translation = the point.  frames: 16 doubles per point, row major. */
ORC_API void orc_features_frames(const double *pts, const double *nrm, int P, const double g[3], double *frames)
{
    int p, r;
    for (p = 0; p < P; p++) {
        const double *z = nrm + 3 * p;
        double x[3], y[3], *F = frames + 16 * p;
        x[0] = g[1] * z[2] - g[2] * z[1];
        x[1] = g[2] * z[0] - g[0] * z[2];
        x[2] = g[0] * z[1] - g[1] * z[0];
        y[0] = z[1] * x[2] - z[2] * x[1];
        y[1] = z[2] * x[0] - z[0] * x[2];
        y[2] = z[0] * x[1] - z[1] * x[0];
        orc_normalize3(x);
        orc_normalize3(y);
        for (r = 0; r < 3; r++) {
            const double e[3] = {r == 0, r == 1, r == 2};
            F[4 * r + 0] = ((0 + e[0] * x[0]) + e[1] * x[1]) + e[2] * x[2];
            F[4 * r + 1] = ((0 + e[0] * y[0]) + e[1] * y[1]) + e[2] * y[2];
            F[4 * r + 2] = ((0 + e[0] * z[0]) + e[1] * z[1]) + e[2] * z[2];
            F[4 * r + 3] = pts[3 * p + r];
        }
        F[12] = 0; F[13] = 0; F[14] = 0; F[15] = 1;
    }
}

/* numberOfPointsPerEdge of getReferenceSquaredNeighborhood (neighborhoodsgenerator.cpp:136-137) */
ORC_API int orc_patch_size(double eps, double cmpp)
{
    return 2 * ((int)floor(eps / (0.01 * cmpp)));
}

/* computeSquareNeighborhoodsByNormals (neighborhoodsgenerator.cpp:76-90) ->
   computeSquareNeighborhoodByNormal (:92-132) for every frame: point (i, j), i outer, =
   featureFrame * (-eps + inc*i, -eps + inc*j, 0, 1) with Matx44d * Vec4d's sum order
   (s = 0; s += m(r,k) * v(k), k = 0..3); when the w component != 1 the point is scaled by 1/w
   (OpenCV Vec / double), then (x, y, z) kept.  out: P*size*size*3, point order i*size + j. */
ORC_API int orc_square_neighborhoods(const double *frames, int P, double eps, double cmpp, double *out)
{
    const int size = orc_patch_size(eps, cmpp);
    const double inc = cmpp * 0.01;
    int p;
    if (size <= 0) return 0;
    #pragma omp parallel for schedule(static)
    for (p = 0; p < P; p++) {
        const double *F = frames + (size_t)16 * p;
        int i, j, r;
        for (i = 0; i < size; i++)
            for (j = 0; j < size; j++) {
                const double v[4] = {-eps + inc * i, -eps + inc * j, 0, 1};
                double h[4];
                double *o = out + ((size_t)p * size * size + (size_t)i * size + j) * 3;
                for (r = 0; r < 4; r++)
                    h[r] = (((0 + F[4 * r] * v[0]) + F[4 * r + 1] * v[1]) + F[4 * r + 2] * v[2]) + F[4 * r + 3] * v[3];
                if (h[3] != 1) {
                    const double a = 1. / h[3];
                    h[0] = h[0] * a; h[1] = h[1] * a; h[2] = h[2] * a;
                }
                o[0] = h[0]; o[1] = h[1]; o[2] = h[2];
            }
    }
    return size;
}

/* NeighborhoodsGenerator circular method.  The constructor's lookup table
   (neighborhoodsgenerator.cpp:50-64): for ray i = 1..rays (outer), angle j = 0..thetas-1 (inner):
   r = i * (eps/rays), t = j * (2*pi/thetas), st = sin(t), st2 = 2*sin(t/2)*sin(t/2) (libm).
   computeCircularNeighborhoodsByNormals (:160-224): normals NULL -> n = X * (1/norm(X)) (the
   empty-normals branch, Vec / double); spanner = (0, 1, -n1/n2) * (1/norm) * eps; W = skew(n)
   (tools.cpp:122-127); sample = X + r * ((spanner + (W*spanner)*st) + ((st2*W)*W)*spanner), every
   Matx product summed from 0 in k order (Matx_MatMulOp), norms as normL2Sqr from 0.
   points / normals: P*3; out: P*thetas*rays*3, sample order ray outer, angle inner. */
ORC_API int orc_circular_neighborhoods(const double *points, const double *normals, int P, double eps, int thetas,
                                       int rays, double *out)
{
    const int S = thetas * rays;
    const double rayIncrement = eps / rays, thetaIncrement = 2 * M_PI / thetas;
    double *lut;
    int p, i, j;
    if (thetas <= 0 || rays <= 0) return -1;
    lut = (double *)malloc(sizeof(double) * 3 * (size_t)S);
    for (i = 1; i <= rays; i++)
        for (j = 0; j < thetas; j++) {
            const double t = j * thetaIncrement;
            double *e = lut + 3 * ((size_t)(i - 1) * thetas + j);
            e[0] = (double)i * rayIncrement;
            e[1] = sin(t);
            e[2] = 2 * (sin(t / 2)) * (sin(t / 2));
        }
    #pragma omp parallel for schedule(static)
    for (p = 0; p < P; p++) {
        const double *X = points + 3 * (size_t)p;
        double n[3], sp[3], W[9], Ws[3], sW[9], M[9], B[3], q, inv;
        int k, a, b, c;
        if (normals) {
            n[0] = normals[3 * (size_t)p]; n[1] = normals[3 * (size_t)p + 1]; n[2] = normals[3 * (size_t)p + 2];
        } else {
            q = 0;
            for (a = 0; a < 3; a++) q += X[a] * X[a];
            inv = 1. / sqrt(q);
            for (a = 0; a < 3; a++) n[a] = X[a] * inv;
        }
        sp[0] = 0.; sp[1] = 1.; sp[2] = -n[1] / n[2];
        q = 0;
        for (a = 0; a < 3; a++) q += sp[a] * sp[a];
        inv = 1. / sqrt(q);
        for (a = 0; a < 3; a++) sp[a] = sp[a] * inv * eps;
        W[0] = 0;     W[1] = -n[2]; W[2] = n[1];
        W[3] = n[2];  W[4] = 0;     W[5] = -n[0];
        W[6] = -n[1]; W[7] = n[0];  W[8] = 0;
        for (a = 0; a < 3; a++) {
            double s = 0;
            for (c = 0; c < 3; c++) s += W[3 * a + c] * sp[c];
            Ws[a] = s;
        }
        for (k = 0; k < S; k++) {
            const double r = lut[3 * k], st = lut[3 * k + 1], st2 = lut[3 * k + 2];
            double *o = out + ((size_t)p * S + k) * 3;
            for (a = 0; a < 9; a++) sW[a] = W[a] * st2;
            for (a = 0; a < 3; a++)
                for (b = 0; b < 3; b++) {
                    double s = 0;
                    for (c = 0; c < 3; c++) s += sW[3 * a + c] * W[3 * c + b];
                    M[3 * a + b] = s;
                }
            for (a = 0; a < 3; a++) {
                double s = 0;
                for (c = 0; c < 3; c++) s += M[3 * a + c] * sp[c];
                B[a] = s;
            }
            for (a = 0; a < 3; a++) o[a] = X[a] + ((sp[a] + Ws[a] * st) + B[a]) * r;
        }
    }
    free(lut);
    return S;
}

/* cvRodrigues2 round trip of decomposeTransformation + cvProjectPoints2, with libm (mode 0) or
   the deterministic transcendentals (mode ORC_LM_DETMATH; acos(c) = atan2(sqrt((1-c)(1+c)), c)).
   Both orthonormalise R by OpenCV's SVD (orc_cv_polar3). */
static void orc_frame_camera(const double F[16], int mode, double R2[9], double t2[3])
{
    double R[9], r[3], rx, ry, rz, theta;
    int k;
    R[0] = F[0]; R[1] = F[1]; R[2] = F[2];
    R[3] = F[4]; R[4] = F[5]; R[5] = F[6];
    R[6] = F[8]; R[7] = F[9]; R[8] = F[10];
    t2[0] = F[3]; t2[1] = F[7]; t2[2] = F[11];
    if (!(mode & ORC_LM_DETMATH)) {
        orc_rodrigues_m2v(R, r);
        orc_rodrigues_v2m(r, R2);
        return;
    }
    orc_rodrigues_m2v_acos(R, r, 1);
    rx = r[0]; ry = r[1]; rz = r[2];
    /* orc_rodrigues_v2m with fm3d_cos / fm3d_sin */
    theta = sqrt(rx * rx + ry * ry + rz * rz);
    if (theta < DBL_EPSILON) {
        for (k = 0; k < 9; k++) R2[k] = (k % 4 == 0) ? 1. : 0.;
        return;
    }
    {
        const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        double cc = fm3d_cos(theta), ss = fm3d_sin(theta), c1 = 1. - cc;
        double itheta = theta ? 1. / theta : 0.;
        double rrt[9], rxm[9];
        rx *= itheta; ry *= itheta; rz *= itheta;
        rrt[0] = rx * rx; rrt[1] = rx * ry; rrt[2] = rx * rz;
        rrt[3] = rx * ry; rrt[4] = ry * ry; rrt[5] = ry * rz;
        rrt[6] = rx * rz; rrt[7] = ry * rz; rrt[8] = rz * rz;
        rxm[0] = 0; rxm[1] = -rz; rxm[2] = ry;
        rxm[3] = rz; rxm[4] = 0; rxm[5] = -rx;
        rxm[6] = -ry; rxm[7] = rx; rxm[8] = 0;
        for (k = 0; k < 9; k++) R2[k] = cc * I[k] + c1 * rrt[k] + ss * rxm[k];
    }
}

/* getReferenceSquaredNeighborhood (neighborhoodsgenerator.cpp:134-158) projected with every frame
   (projectReferencePointsToImageWithFrame, singlecameratriangulator.cpp:805-849): point (i, j) =
   (-eps + inc*i, -eps + inc*j, 0), inc = cmPerPixel*0.01; pixel outside isPixelGood(p, 1.0) of
   image 1 (or NaN) -> 0, else (uchar) of the bilinear sample; written to patch row j, column i
   (the reference's patch.at<uchar>(col, row)).  patches: P*size*size; imagePoints (may be NULL):
   P*size*size*2 in point order i*size + j. */
ORC_API int orc_export_patches(const orc_camera *cam, const uint8_t *img, int w, int h, const double *frames,
                               int P, double eps, double cmpp, int mode, uint8_t *patches, double *imagePoints)
{
    const int size = orc_patch_size(eps, cmpp);
    const double inc = cmpp * 0.01;
    int p;
    if (size <= 0) return 0;
#pragma omp parallel for schedule(dynamic, 4)
    for (p = 0; p < P; p++) {
        double R2[9], t2[3];
        int i, j;
        orc_frame_camera(frames + 16 * (size_t)p, mode, R2, t2);
        for (i = 0; i < size; i++)
            for (j = 0; j < size; j++) {
                double u, v;
                uint8_t val = 0;
                orc_project1(cam, R2, t2, -eps + inc * i, -eps + inc * j, 0, &u, &v);
                if (imagePoints) {
                    imagePoints[((size_t)p * size * size + (size_t)i * size + j) * 2] = u;
                    imagePoints[((size_t)p * size * size + (size_t)i * size + j) * 2 + 1] = v;
                }
                if (orc_pixel_good(u, v, 1.0, w, h)) val = (uint8_t)orc_bilinear(img, w, h, (float)u, (float)v);
                patches[(size_t)p * size * size + (size_t)j * size + i] = val;
            }
    }
    return size;
}
