// Host build of include/fm3d_cvsvd.h (the product's restatement of OpenCV 2.4's JacobiSVD, which the
// triangulation kernel, the LM's R2 and the patch frames run) for tests/test_cvsvd.py: compared bit for
// bit with the oracle's independent restatement (oracle/fm3d_oracle.c orc_cv_jacobi_svd).
// Test infrastructure: g++ -O2 -ffp-contract=off -shared -fPIC -I include.
#include "fm3d_cvsvd.h"

extern "C" {

// n systems: g12 (16 doubles, shared), u (n x 4: u1x, u1y, u2x, u2y) -> X (n x 4)
void shim_triangulate(const double* g12, const double* u, int n, double* X) {
    for (int i = 0; i < n; i++)
        fm3d_cv::triangulate_point(g12, u[4 * i], u[4 * i + 1], u[4 * i + 2], u[4 * i + 3], X + 4 * i);
}

// n row-major 3 x 3 matrices -> their polar factors
void shim_polar3(const double* R, int n, double* Rp) {
    for (int i = 0; i < n; i++) fm3d_cv::polar3(R + 9 * i, Rp + 9 * i);
}

// the 6 x 4 / 3 x 3 SVD pieces: W (sorted), perm
void shim_svd64(const double* A, double* W, double* Vt, int* perm) {
    double At[4][6], w[4], vt[4][4];
    int p[4];
    for (int k = 0; k < 4; k++)
        for (int r = 0; r < 6; r++) At[k][r] = A[r * 4 + k];
    fm3d_cv::jacobi_svd<6, 4>(At, w, vt, p);
    for (int i = 0; i < 4; i++) {
        W[i] = w[i];
        perm[i] = p[i];
        for (int k = 0; k < 4; k++) Vt[i * 4 + k] = vt[p[i]][k];
    }
}

}  // extern "C"
