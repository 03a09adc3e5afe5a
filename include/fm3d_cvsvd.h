/*
 * fm3d_cvsvd.h -- OpenCV 2.4's SVD where the reference's hot path calls it (host and device).
 *
 * The reference calls cvSVD twice on the path (both through cv::SVD::compute -> _SVDcompute ->
 * JacobiSVD(double) = JacobiSVDImpl_<double>(At, ..., minval = DBL_MIN, eps = 10 DBL_EPSILON),
 * OpenCV 2.4.9 core/src/lapack.cpp):
 *
 *   - cv::triangulatePoints (Triangulator/singlecameratriangulator.cpp:186) -> cvTriangulatePoints:
 *     per point a 6 x 4 matrA (three rows per view: x P.row2 - P.row0, y P.row2 - P.row1,
 *     x P.row1 - y P.row0), cvSVD(matrA, matrW, 0, matrV, CV_SVD_V_T), X = matrV's row 3;
 *   - cv::Rodrigues(R, r) in decomposeTransformation (tools.cpp:110) -> cvRodrigues2: R replaced by
 *     U V^T of cvSVD(R, W, U, V, CV_SVD_MODIFY_A + CV_SVD_U_T + CV_SVD_V_T) and cvGEMM(.., CV_GEMM_A_T).
 *
 * JacobiSVDImpl_ is a one-sided Jacobi over the rows of At = A^T (the columns of A): cyclic i < j
 * sweeps (at most max(m, 30)), each pair skipped when |p| <= eps sqrt(W_i W_j) (p their dot product,
 * W the tracked squared norms), else rotated by the hypot-based (c, s) of its beta < 0 / >= 0
 * branches, the rotated rows' squared norms becoming the new W; then W = sqrt(row norms), a selection
 * sort into descending order swapping At and Vt rows, and the first n1 rows of At normalised by
 * 1/W (a zero singular value takes a cv::RNG vector orthogonalised against the earlier rows).
 * x86 builds vectorise only the Vt rotation (VBLAS<double>::givens, two SSE2 lanes), which gives
 * the scalar loop's bits (no FMA; -(s Vi) + c Vj is c Vj - s Vi exactly), so the scalar order below
 * IS the x86 order.  The oracle restates the same function independently and generically
 * (oracle/fm3d_oracle.c orc_cv_jacobi_svd, strided loops, physical row swaps); this header is the
 * product's fixed-size form (compile-time loops, so a GPU thread keeps every array in registers, and
 * the sort on an index permutation).  Both are compiled without FMA contraction; hypot is the
 * correctly rounded fm3d_hypot_cr (fm3d_crmath.h) on both sides.
 */
#ifndef FM3D_CVSVD_H
#define FM3D_CVSVD_H

#include <float.h>
#include <stdint.h>

#include "fm3d_crmath.h"

#if defined(__HIPCC__)
#define FM3D_CVSVD_HD __host__ __device__ inline
#else
#define FM3D_CVSVD_HD inline
#endif

namespace fm3d_cv {

// one pair (i, j) of JacobiSVDImpl_'s sweep: the skip test, the rotation of the At and Vt rows and
// the new squared norms; true when it rotated
template <int M, int N>
FM3D_CVSVD_HD bool jacobi_rotate(double (&Ai)[M], double (&Aj)[M], double& Wi, double& Wj, double (&Vi)[N],
                                 double (&Vj)[N]) {
    const double eps = DBL_EPSILON * 10;
    double a = Wi, b = Wj, p = 0;
#pragma unroll
    for (int k = 0; k < M; k++) p += Ai[k] * Aj[k];
    if (fabs(p) <= eps * sqrt(a * b)) return false;
    p *= 2;
    const double beta = a - b, gamma = fm3d_hypot_cr(p, beta);
    double c, s;
    if (beta < 0) {
        const double delta = (gamma - beta) * 0.5;
        s = sqrt(delta / gamma);
        c = p / (gamma * s * 2);
    } else {
        c = sqrt((gamma + beta) / (gamma * 2));
        s = p / (gamma * c * 2);
    }
    a = b = 0;
#pragma unroll
    for (int k = 0; k < M; k++) {
        const double t0 = c * Ai[k] + s * Aj[k];
        const double t1 = -s * Ai[k] + c * Aj[k];
        Ai[k] = t0;
        Aj[k] = t1;
        a += t0 * t0;
        b += t1 * t1;
    }
    Wi = a;
    Wj = b;
#pragma unroll
    for (int k = 0; k < N; k++) {
        const double t0 = c * Vi[k] + s * Vj[k];
        const double t1 = -s * Vi[k] + c * Vj[k];
        Vi[k] = t0;
        Vj[k] = t1;
    }
    return true;
}

// JacobiSVDImpl_'s sweeps, final norms and descending selection sort.  At: the N columns of A as rows
// of M (rotated in place, unsorted); on return W[i] is the i-th largest singular value (OpenCV's
// sorted W) and perm[i] the At / Vt row that the sort moves to position i.
template <int M, int N>
FM3D_CVSVD_HD void jacobi_svd(double (&At)[N][M], double (&W)[N], double (&Vt)[N][N], int (&perm)[N]) {
#pragma unroll
    for (int i = 0; i < N; i++) {
        double sd = 0;
#pragma unroll
        for (int k = 0; k < M; k++) sd += At[i][k] * At[i][k];
        W[i] = sd;
#pragma unroll
        for (int k = 0; k < N; k++) Vt[i][k] = i == k ? 1. : 0.;
    }
    const int maxIter = M > 30 ? M : 30;
    for (int iter = 0; iter < maxIter; iter++) {
        bool changed = false;
#pragma unroll
        for (int i = 0; i < N - 1; i++)
#pragma unroll
            for (int j = i + 1; j < N; j++) changed |= jacobi_rotate<M, N>(At[i], At[j], W[i], W[j], Vt[i], Vt[j]);
        if (!changed) break;
    }
#pragma unroll
    for (int i = 0; i < N; i++) {
        double sd = 0;
#pragma unroll
        for (int k = 0; k < M; k++) sd += At[i][k] * At[i][k];
        W[i] = sqrt(sd);
        perm[i] = i;
    }
    // for i: j = i; for k > i: if (W[j] < W[k]) j = k; if (i != j) swap rows i, j
#pragma unroll
    for (int i = 0; i < N - 1; i++) {
        int j = i;
        double wj = W[i];
#pragma unroll
        for (int k = i + 1; k < N; k++)
            if (wj < W[k]) {
                j = k;
                wj = W[k];
            }
        const double wi = W[i];
        const int pi = perm[i];
        int pj = pi;
#pragma unroll
        for (int k = i + 1; k < N; k++)
            if (k == j) pj = perm[k];
#pragma unroll
        for (int k = i + 1; k < N; k++)
            if (k == j) {
                W[k] = wi;
                perm[k] = pi;
            }
        W[i] = wj;
        perm[i] = pj;
    }
}

// row r (a runtime index < N) of a register array
template <int N, int L>
FM3D_CVSVD_HD void pick_row(const double (&A)[N][L], int r, double (&out)[L]) {
#pragma unroll
    for (int k = 0; k < L; k++) out[k] = A[0][k];
#pragma unroll
    for (int i = 1; i < N; i++)
#pragma unroll
        for (int k = 0; k < L; k++) out[k] = r == i ? A[i][k] : out[k];
}

// cvTriangulatePoints (OpenCV 2.4 calib3d/src/triangulate.cpp) for one point: P1 = [I|0], P2 = the
// first three rows of g12 (row-major 4 x 4), (u1x, u1y) / (u2x, u2y) the undistorted points of the two
// views; X = the homogeneous point (matrV's row 3)
FM3D_CVSVD_HD void triangulate_point(const double* g12, double u1x, double u1y, double u2x, double u2y,
                                     double X[4]) {
    const double P1[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    double At[4][6], W[4], Vt[4][4];
    int perm[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {  // At = matrA^T
        At[k][0] = u1x * P1[8 + k] - P1[0 + k];
        At[k][1] = u1y * P1[8 + k] - P1[4 + k];
        At[k][2] = u1x * P1[4 + k] - u1y * P1[0 + k];
        At[k][3] = u2x * g12[8 + k] - g12[0 + k];
        At[k][4] = u2y * g12[8 + k] - g12[4 + k];
        At[k][5] = u2x * g12[4 + k] - u2y * g12[0 + k];
    }
    jacobi_svd<6, 4>(At, W, Vt, perm);
    double v[4];
    pick_row<4, 4>(Vt, perm[3], v);
#pragma unroll
    for (int k = 0; k < 4; k++) X[k] = v[k];
}

// cv::RNG::next (core.hpp)
FM3D_CVSVD_HD unsigned rng_next(uint64_t& state) {
    state = (uint64_t)(unsigned)state * 4164903690U + (unsigned)(state >> 32);
    return (unsigned)state;
}

// cvRodrigues2's orthonormalisation of a row-major 3 x 3 R (OpenCV 2.4 calib3d/src/calibration.cpp):
// cvSVD(R, W, U, V, CV_SVD_MODIFY_A + CV_SVD_U_T + CV_SVD_V_T) -- _SVDcompute's temp_a = R^T,
// JacobiSVD(m = n = n1 = 3) -- then cvGEMM(U, V, 1, 0, 0, R, CV_GEMM_A_T): flags != 0, so
// GEMMSingleMul's generic loop, s = 0; s += U(i,k) Vt(k,j) for k = 0..2; R(i,j) = s * alpha
FM3D_CVSVD_HD void polar3(const double R[9], double Rp[9]) {
    double At[3][3], W[3], Vt[3][3];
    int perm[3];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int k = 0; k < 3; k++) At[i][k] = R[k * 3 + i];
    jacobi_svd<3, 3>(At, W, Vt, perm);
    double U[3][3], V[3][3];  // rows in sorted order
#pragma unroll
    for (int i = 0; i < 3; i++) {
        pick_row<3, 3>(At, perm[i], U[i]);
        pick_row<3, 3>(Vt, perm[i], V[i]);
    }
    uint64_t rng = 0x12345678;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        double sd = W[i];
        while (sd <= DBL_MIN) {  // a zero singular value (JacobiSVDImpl_'s random left vector)
            const double val0 = 1. / 3;
#pragma unroll
            for (int k = 0; k < 3; k++) U[i][k] = (rng_next(rng) & 256) != 0 ? val0 : -val0;
            for (int it = 0; it < 2; it++)
#pragma unroll
                for (int j = 0; j < i; j++) {
                    double asum = 0;
                    sd = 0;
#pragma unroll
                    for (int k = 0; k < 3; k++) sd += U[i][k] * U[j][k];
#pragma unroll
                    for (int k = 0; k < 3; k++) {
                        const double t = U[i][k] - sd * U[j][k];
                        U[i][k] = t;
                        asum += fabs(t);
                    }
                    asum = asum ? 1 / asum : 0;
#pragma unroll
                    for (int k = 0; k < 3; k++) U[i][k] *= asum;
                }
            sd = 0;
#pragma unroll
            for (int k = 0; k < 3; k++) sd += U[i][k] * U[i][k];
            sd = sqrt(sd);
        }
        const double s = 1 / sd;
#pragma unroll
        for (int k = 0; k < 3; k++) U[i][k] *= s;
    }
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) {
            double s = 0;
#pragma unroll
            for (int k = 0; k < 3; k++) s += U[k][i] * V[k][j];
            Rp[i * 3 + j] = s * 1.;
        }
}

}  // namespace fm3d_cv

#endif /* FM3D_CVSVD_H */
