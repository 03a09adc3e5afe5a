// fm3d_patch.hip -- feature frames and normal-rectified patch export.
//
// Reference: NormalOptimizer::computeFeaturesFrames (Triangulator/normaloptimizer.cpp:454-504),
// NeighborhoodsGenerator::getReferenceSquaredNeighborhood (neighborhoodsgenerator.cpp:134-158) and
// SingleCameraTriangulator::projectReferencePointsToImageWithFrame(s)
// (singlecameratriangulator.cpp:769-849).  main.cpp:157-180 runs them after the normals.
//
// Four kernels, all bit-exact against oracle/fm3d_oracle.c (deterministic-math mode):
//   frames_kernel        one thread per point: z = n, x = g x z, y = z x x, cv::normalize(x), (y),
//                        columns through Vec::dot, translation = the point;
//   frame_camera_kernel  one thread per frame: decomposeTransformation + the cvRodrigues2 round trip
//                        cvProjectPoints2 applies (matrix -> vector -> matrix);
//   patch_kernel         one thread per (reference point, frame): projectPoints, isPixelGood(p, 1.0)
//                        of image 1, (uchar) bilinear sample, written transposed (patch.at(col, row));
//   square_neighborhoods_kernel  NeighborhoodsGenerator::computeSquareNeighborhoodsByNormals
//                        (neighborhoodsgenerator.cpp:76-132, main.cpp:187): the square grid through
//                        every frame, 24 B written per point (HBM-bound, 5.3 TB/s);
//   circular_neighborhoods_kernel  NeighborhoodsGenerator::computeCircularNeighborhoodsByNormals
//                        (neighborhoodsgenerator.cpp:160-224): one thread per (point, sample).
// Every output byte depends on one projected sample; the patch kernel is a projection + gather
// bound by the fp64 VALU (≈60 fp64 ops per sample) -- there is no reduction and no data reuse
// beyond the image in L2.
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include "fm3d_device.h"
#include "fm3d_kernels.h"

namespace fm3d {

namespace {

// cv::normalize(v, v) of a Vec3d: 1/||v|| (squares summed from 0 in index order; 0 if the norm is
// <= DBL_EPSILON), then v*scale + 0 (convertTo with scale, shift 0)
__device__ inline void normalize3(double v[3]) {
    double s = 0;
    for (int i = 0; i < 3; i++) s += v[i] * v[i];
    s = sqrt(s);
    const double scale = s > DBL_EPSILON ? 1 / s : 0.;
    for (int i = 0; i < 3; i++) v[i] = v[i] * scale + 0.;
}

__global__ void frames_kernel(const double* __restrict__ pts, const double* __restrict__ nrm, int P, double g0,
                              double g1, double g2, double* __restrict__ frames) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    const double z[3] = {nrm[3 * p], nrm[3 * p + 1], nrm[3 * p + 2]};
    // x = gravity.cross(z), y = z.cross(x) (cv::Vec3d::cross), normalised afterwards (:476-481)
    double x[3] = {g1 * z[2] - g2 * z[1], g2 * z[0] - g0 * z[2], g0 * z[1] - g1 * z[0]};
    double y[3] = {z[1] * x[2] - z[2] * x[1], z[2] * x[0] - z[0] * x[2], z[0] * x[1] - z[1] * x[0]};
    normalize3(x);
    normalize3(y);
    double* F = frames + 16 * (size_t)p;
    for (int r = 0; r < 3; r++) {
        // actualFrame(r, c) = e_r.dot(c-th basis vector) (:484-486)
        const double e[3] = {(double)(r == 0), (double)(r == 1), (double)(r == 2)};
        F[4 * r + 0] = ((0 + e[0] * x[0]) + e[1] * x[1]) + e[2] * x[2];
        F[4 * r + 1] = ((0 + e[0] * y[0]) + e[1] * y[1]) + e[2] * y[2];
        F[4 * r + 2] = ((0 + e[0] * z[0]) + e[1] * z[1]) + e[2] * z[2];
        F[4 * r + 3] = pts[3 * p + r];
    }
    F[12] = 0;
    F[13] = 0;
    F[14] = 0;
    F[15] = 1;
}

// decomposeTransformation (tools.cpp:101-114) then cvProjectPoints2's Rodrigues: the R, t that
// projectReferencePointsToImageWithFrame projects with.  cvRodrigues2 (matrix -> vector) first
// replaces R by its nearest orthonormal matrix, U V^T of OpenCV 2.4's SVD (include/fm3d_cvsvd.h).
__global__ void frame_camera_kernel(const double* __restrict__ frames, int P, double* __restrict__ RT) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    const double* F = frames + 16 * (size_t)p;
    const double Rin[9] = {F[0], F[1], F[2], F[4], F[5], F[6], F[8], F[9], F[10]};
    double R[9];
    fm3d_cv::polar3(Rin, R);
    double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
    const double s = sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    double c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    double theta = fm3d_acos(c);
    if (s < 1e-5) {
        if (c > 0) {
            rx = ry = rz = 0;
        } else {
            double t = (R[0] + 1) * 0.5;
            rx = sqrt(t > 0. ? t : 0.);
            t = (R[4] + 1) * 0.5;
            ry = sqrt(t > 0. ? t : 0.) * (R[1] < 0 ? -1. : 1.);
            t = (R[8] + 1) * 0.5;
            rz = sqrt(t > 0. ? t : 0.) * (R[2] < 0 ? -1. : 1.);
            if (fabs(rx) < fabs(ry) && fabs(rx) < fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
            theta /= sqrt(rx * rx + ry * ry + rz * rz);
            rx *= theta;
            ry *= theta;
            rz *= theta;
        }
    } else {
        double vth = 1 / (2 * s);
        vth *= theta;
        rx *= vth;
        ry *= vth;
        rz *= vth;
    }
    // vector -> matrix
    double* out = RT + 12 * (size_t)p;
    theta = sqrt(rx * rx + ry * ry + rz * rz);
    if (theta < DBL_EPSILON) {
        for (int k = 0; k < 9; k++) out[k] = (k % 4 == 0) ? 1. : 0.;
    } else {
        const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        const double cc = fm3d_cos(theta), ss = fm3d_sin(theta), c1 = 1. - cc;
        const double itheta = theta ? 1. / theta : 0.;
        rx *= itheta;
        ry *= itheta;
        rz *= itheta;
        const double rrt[9] = {rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz};
        const double rxm[9] = {0, -rz, ry, rz, 0, -rx, -ry, rx, 0};
        for (int k = 0; k < 9; k++) out[k] = cc * I[k] + c1 * rrt[k] + ss * rxm[k];
    }
    out[9] = F[3];
    out[10] = F[7];
    out[11] = F[11];
}

__global__ __launch_bounds__(256) void patch_kernel(const double* __restrict__ RT, int P, int size, double eps,
                                                    double inc, Camera cam, const uint8_t* __restrict__ img, int w,
                                                    int h, uint8_t* __restrict__ patches,
                                                    double* __restrict__ imagePoints) {
    const int p = blockIdx.y;
    // threads run over the patch bytes (row j, column i), so a wave's byte stores are contiguous;
    // the reference point is i*size + j
    const int o = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P || o >= size * size) return;
    const int j = o / size, i = o - j * size;
    const int k = i * size + j;
    const double* rt = RT + 12 * (size_t)p;
    const double R[9] = {rt[0], rt[1], rt[2], rt[3], rt[4], rt[5], rt[6], rt[7], rt[8]};
    const double t[3] = {rt[9], rt[10], rt[11]};
    double u, v;
    project1(cam, R, t, -eps + inc * i, -eps + inc * j, 0, u, v);
    const size_t base = (size_t)p * size * size;
    if (imagePoints) {
        imagePoints[(base + k) * 2] = u;
        imagePoints[(base + k) * 2 + 1] = v;
    }
    uint8_t val = 0;
    if (pixel_good(u, v, 1.0, w, h)) val = (uint8_t)bilinear(img, w, (float)u, (float)v);
    patches[base + o] = val;  // o = j*size + i: patch.at<uchar>(col, row), :842-846
}

// computeSquareNeighborhoodByNormal (neighborhoodsgenerator.cpp:92-132) of every frame: point
// (i, j) = frame * (-eps + inc*i, -eps + inc*j, 0, 1) in Matx44d * Vec4d's order (s = 0, then
// += m(r,k) v(k) for k = 0..3), scaled by 1/w when w != 1.  One thread per output point, a block =
// 256 consecutive points; the 24-byte records go through LDS and leave as coalesced 16-byte
// nontemporal stores (the kernel is bound by the HBM writes, 24 B per point).
constexpr int kSqThreads = 256;
typedef double f64x2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(kSqThreads) void square_neighborhoods_kernel(const double* __restrict__ frames,
                                                                           long long total, int size, double eps,
                                                                           double inc, double* __restrict__ out) {
    __shared__ double rec[kSqThreads * 3];
    const long long base = (long long)blockIdx.x * kSqThreads;
    const long long idx = base + threadIdx.x;
    const long long per = (long long)size * size;
    auto point = [&](const double* F, long long f) {
        const int ij = (int)(idx - f * per);
        const int i = ij / size, j = ij - (ij / size) * size;
        const double v0 = -eps + inc * i, v1 = -eps + inc * j, v2 = 0, v3 = 1;
        double h[4];
#pragma unroll
        for (int r = 0; r < 4; r++)
            h[r] = (((0 + F[4 * r] * v0) + F[4 * r + 1] * v1) + F[4 * r + 2] * v2) + F[4 * r + 3] * v3;
        if (h[3] != 1) {
            const double a = 1. / h[3];
            h[0] = h[0] * a;
            h[1] = h[1] * a;
            h[2] = h[2] * a;
        }
        rec[3 * threadIdx.x] = h[0];
        rec[3 * threadIdx.x + 1] = h[1];
        rec[3 * threadIdx.x + 2] = h[2];
    };
    if (per % kSqThreads == 0) {
        // the block lies inside one frame: its index is uniform, the 16 values come through scalar loads
        const long long f = base / per;
        if (idx < total) point(frames + 16 * f, f);
    } else if (idx < total) {
        const long long f = idx / per;
        point(frames + 16 * f, f);
    }
    __syncthreads();
    const long long n = total - base < kSqThreads ? total - base : kSqThreads;  // points of this block
    const int nd = (int)(3 * n);                                                  // doubles (even unless n odd)
    double* o = out + 3 * base;
    for (int k = threadIdx.x; 2 * k < nd; k += kSqThreads) {
        if (2 * k + 1 < nd)
            __builtin_nontemporal_store(*(const f64x2*)&rec[2 * k], (f64x2*)(o + 2 * k));
        else
            __builtin_nontemporal_store(rec[2 * k], o + 2 * k);
    }
}

// ---------------- circular neighbourhoods (neighborhoodsgenerator.cpp:160-277)
// Matx33d * Vec3d / Matx33d * Matx33d as OpenCV's Matx_MatMulOp: s = 0; s += a(i,k)*b(k,j) in k order
__device__ inline void matvec3(const double A[9], const double v[3], double o[3]) {
    for (int i = 0; i < 3; i++) {
        double s = 0;
        for (int k = 0; k < 3; k++) s += A[3 * i + k] * v[k];
        o[i] = s;
    }
}

// one thread per (point, sample): the spanner, W = skew(n) (tools.cpp:122-127) and the sample
// X + r*((s + (W*s)*st) + ((st2*W)*W)*s), each operation in the reference's Matx / Vec order.  lut:
// (r, sin t, 2 sin^2(t/2)) per sample, built on the host by the constructor's formulas (:50-64).
__global__ __launch_bounds__(256) void circular_neighborhoods_kernel(const double* __restrict__ pts,
                                                                     const double* __restrict__ nrm, long long total,
                                                                     int S, const double* __restrict__ lut, double eps,
                                                                     double* __restrict__ out) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= total) return;
    const long long p = t / S;
    const int k = (int)(t - p * S);
    const double X[3] = {pts[3 * p], pts[3 * p + 1], pts[3 * p + 2]};
    double n[3];
    if (nrm) {
        n[0] = nrm[3 * p];
        n[1] = nrm[3 * p + 1];
        n[2] = nrm[3 * p + 2];
    } else {
        // normal = point / cv::norm(point): Vec / double multiplies by the reciprocal
        double q = 0;
        for (int i = 0; i < 3; i++) q += X[i] * X[i];
        const double inv = 1. / sqrt(q);
        for (int i = 0; i < 3; i++) n[i] = X[i] * inv;
    }
    // spanner(0, 1, -n1/n2); spanner / cv::norm(spanner) * epsilon
    double sp[3] = {0., 1., -n[1] / n[2]};
    double q = 0;
    for (int i = 0; i < 3; i++) q += sp[i] * sp[i];
    const double inv = 1. / sqrt(q);
    for (int i = 0; i < 3; i++) sp[i] = sp[i] * inv * eps;
    const double W[9] = {0, -n[2], n[1], n[2], 0, -n[0], -n[1], n[0], 0};
    const double r = lut[3 * k], st = lut[3 * k + 1], st2 = lut[3 * k + 2];
    double Ws[3], sW[9], M[9], B[3];
    matvec3(W, sp, Ws);
    for (int i = 0; i < 9; i++) sW[i] = W[i] * st2;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double s = 0;
            for (int l = 0; l < 3; l++) s += sW[3 * i + l] * W[3 * l + j];
            M[3 * i + j] = s;
        }
    matvec3(M, sp, B);
    double* o = out + 3 * t;
    for (int i = 0; i < 3; i++) {
        const double v = (sp[i] + Ws[i] * st) + B[i];
        o[i] = X[i] + v * r;
    }
}

}  // namespace

void launch_circular_neighborhoods(const double* pts, const double* nrm, int P, int S, const double* lut, double eps,
                                   double* out, hipStream_t s) {
    const long long total = (long long)P * S;
    if (total <= 0) return;
    circular_neighborhoods_kernel<<<(unsigned)((total + 255) / 256), 256, 0, s>>>(pts, nrm, total, S, lut, eps, out);
}

void launch_square_neighborhoods(const double* frames, int P, int size, double eps, double inc, double* out,
                                 hipStream_t s) {
    const long long total = (long long)P * size * size;
    if (total <= 0) return;
    square_neighborhoods_kernel<<<(unsigned)((total + kSqThreads - 1) / kSqThreads), kSqThreads, 0, s>>>(
        frames, total, size, eps, inc, out);
}

void launch_features_frames(const double* pts, const double* nrm, int P, const double g[3], double* frames,
                            hipStream_t s) {
    if (P <= 0) return;
    hipLaunchKernelGGL(frames_kernel, dim3((P + 255) / 256), dim3(256), 0, s, pts, nrm, P, g[0], g[1], g[2], frames);
}

void launch_export_patches(const double* frames, int P, int size, double eps, double inc, const Camera& cam,
                           const uint8_t* img, int w, int h, double* RT, uint8_t* patches, double* imagePoints,
                           hipStream_t s) {
    if (P <= 0 || size <= 0) return;
    hipLaunchKernelGGL(frame_camera_kernel, dim3((P + 255) / 256), dim3(256), 0, s, frames, P, RT);
    const size_t per = (size_t)size * size;
    for (int p0 = 0; p0 < P; p0 += 65535) {  // grid.y limit
        const int n = P - p0 < 65535 ? P - p0 : 65535;
        dim3 grid((unsigned)((per + 255) / 256), (unsigned)n);
        hipLaunchKernelGGL(patch_kernel, grid, dim3(256), 0, s, RT + 12 * (size_t)p0, n, size, eps, inc, cam, img, w,
                           h, patches + per * p0, imagePoints ? imagePoints + 2 * per * p0 : nullptr);
    }
}

}  // namespace fm3d
