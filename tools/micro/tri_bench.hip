// tri_bench.hip -- the DLT null-vector chain of triangulate_kernel (csrc/fm3d_misc.hip) timed alone on
// C2-like 4x4 systems (two views, small baseline): V0 the cyclic pair order with runtime column
// indices (round 4's kernel), V2 the same order with compile-time indices (must equal V0 bit for
// bit), V4 the round-robin order of round 5's kernel (other bits: a different, equally valid order).
// Round 5 (MI355X): V0 11.3 us, V2 11.2 us -- the chain of divisions and square roots bounds it,
// not the indexing; a guarded fast division / sqrt sequence (no v_div_scale / fixup) did not help
// either (12.2 us), so round 5 halves the chain instead (V4: two independent rotations per step).
//
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I3dfeaturematcher_amd/csrc \
//         tools/micro/tri_bench.hip -o tools/micro/_bin/tri_bench && tools/micro/_bin/tri_bench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "fm3d_fastdiv.h"

using namespace fm3d;

__device__ inline uint64_t mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
__device__ inline double unit(uint64_t r) { return (double)(r >> 11) * 0x1p-53; }

template <bool FAST>
__device__ inline double DIV(double a, double d) { return a / d; }
template <bool FAST>
__device__ inline double SQRT(double x) { return sqrt(x); }

// one Jacobi rotation of columns (p, q) of A (and V), if the pair is not yet orthogonal
template <bool FAST>
__device__ __forceinline__ bool jacobi_pair(double* A, double* V, int p, int q) {
    double alpha = 0, beta = 0, gamma = 0;
    for (int i = 0; i < 4; i++) {
        double ap = A[i * 4 + p], aq = A[i * 4 + q];
        alpha += ap * ap;
        beta += aq * aq;
        gamma += ap * aq;
    }
    if (gamma != 0. && fabs(gamma) > 1e-15 * SQRT<FAST>(alpha * beta)) {
        double zeta = DIV<FAST>(beta - alpha, 2. * gamma);
        double t = DIV<FAST>(zeta >= 0. ? 1. : -1., fabs(zeta) + SQRT<FAST>(1. + zeta * zeta));
        double cs = DIV<FAST>(1., SQRT<FAST>(1. + t * t));
        double sn = cs * t;
        for (int i = 0; i < 4; i++) {
            double ap = A[i * 4 + p], aq = A[i * 4 + q];
            A[i * 4 + p] = cs * ap - sn * aq;
            A[i * 4 + q] = sn * ap + cs * aq;
            ap = V[i * 4 + p];
            aq = V[i * 4 + q];
            V[i * 4 + p] = cs * ap - sn * aq;
            V[i * 4 + q] = sn * ap + cs * aq;
        }
        return true;
    }
    return false;
}

template <bool FAST, bool UNROLL>
__device__ inline int dlt_nullvec(double* A, double* v) {
    double V[16];
    int rots = 0;
    for (int i = 0; i < 16; i++) V[i] = (i % 5 == 0) ? 1. : 0.;
    for (int sweep = 0; sweep < 30; sweep++) {
        bool rotated = false;
        if constexpr (FAST) {
            // the round-robin order (0,1)+(2,3), (0,2)+(1,3), (0,3)+(1,2) (fm3d_misc.hip)
            const bool r0 = jacobi_pair<false>(A, V, 0, 1);
            const bool r1 = jacobi_pair<false>(A, V, 2, 3);
            const bool r2 = jacobi_pair<false>(A, V, 0, 2);
            const bool r3 = jacobi_pair<false>(A, V, 1, 3);
            const bool r4 = jacobi_pair<false>(A, V, 0, 3);
            const bool r5 = jacobi_pair<false>(A, V, 1, 2);
            const int n = r0 + r1 + r2 + r3 + r4 + r5;
            rots += n;
            rotated = n > 0;
        } else if constexpr (UNROLL) {
            // the cyclic pair order with compile-time column indices (registers, no indexed moves)
            const bool r0 = jacobi_pair<FAST>(A, V, 0, 1);
            const bool r1 = jacobi_pair<FAST>(A, V, 0, 2);
            const bool r2 = jacobi_pair<FAST>(A, V, 0, 3);
            const bool r3 = jacobi_pair<FAST>(A, V, 1, 2);
            const bool r4 = jacobi_pair<FAST>(A, V, 1, 3);
            const bool r5 = jacobi_pair<FAST>(A, V, 2, 3);
            const int n = r0 + r1 + r2 + r3 + r4 + r5;
            rots += n;
            rotated = n > 0;
        } else {
            for (int p = 0; p < 3; p++)
                for (int q = p + 1; q < 4; q++)
                    if (jacobi_pair<FAST>(A, V, p, q)) {
                        rotated = true;
                        rots++;
                    }
        }
        if (!rotated) break;
    }
    double nrm[4];
    for (int p = 0; p < 4; p++) {
        double s = 0;
        for (int i = 0; i < 4; i++) s += A[i * 4 + p] * A[i * 4 + p];
        nrm[p] = s;
    }
    int best = 0;
    for (int p = 1; p < 4; p++)
        if (nrm[p] < nrm[best]) best = p;
    for (int i = 0; i < 4; i++) v[i] = V[i * 4 + best];
    return rots;
}

// C2-like systems: a point at depth 1.6-2.3 m seen by P1 = [I|0] and P2 = [R|t] (a small rotation
// about y, t = (0.1, 0, 0)), normalised image coordinates with ~1e-3 noise
__device__ void make_A(int i, double* A) {
    const uint64_t r = mix(i * 7919ull + 1);
    const double X = unit(mix(r)) - 0.5, Y = unit(mix(r + 1)) * 0.8 - 0.4, Z = 1.6 + 0.7 * unit(mix(r + 2));
    const double c = cos(0.05), s = sin(0.05);
    const double P2[12] = {c, 0, s, 0.1, 0, 1, 0, 0., -s, 0, c, 0.01};
    const double x1 = X / Z + 1e-3 * (unit(mix(r + 3)) - 0.5), y1 = Y / Z + 1e-3 * (unit(mix(r + 4)) - 0.5);
    const double Xc = P2[0] * X + P2[1] * Y + P2[2] * Z + P2[3], Yc = P2[4] * X + P2[5] * Y + P2[6] * Z + P2[7],
                 Zc = P2[8] * X + P2[9] * Y + P2[10] * Z + P2[11];
    const double x2 = Xc / Zc + 1e-3 * (unit(mix(r + 5)) - 0.5), y2 = Yc / Zc + 1e-3 * (unit(mix(r + 6)) - 0.5);
    const double P1[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    for (int k = 0; k < 4; k++) {
        A[0 * 4 + k] = x1 * P1[8 + k] - P1[0 + k];
        A[1 * 4 + k] = y1 * P1[8 + k] - P1[4 + k];
        A[2 * 4 + k] = x2 * P2[8 + k] - P2[0 + k];
        A[3 * 4 + k] = y2 * P2[8 + k] - P2[4 + k];
    }
}

template <bool FAST, bool UNROLL = false>
__global__ __launch_bounds__(64) void tri_kernel(int n, double* out, int* rots) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double A[16], v[4];
    make_A(i, A);
    rots[i] = dlt_nullvec<FAST, UNROLL>(A, v);
    for (int k = 0; k < 4; k++) out[4 * i + k] = v[k];
}

int main() {
    const int n = 9000;
    double *o0, *o1;
    int *r0, *r1;
    hipMalloc(&o0, n * 32);
    hipMalloc(&o1, n * 32);
    hipMalloc(&r0, n * 4);
    hipMalloc(&r1, n * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int grid = (n + 63) / 64;
    auto launch = [&](int v) {
        if (v == 2) hipLaunchKernelGGL((tri_kernel<false, true>), grid, 64, 0, 0, n, o1, r1);
        else if (v == 4) hipLaunchKernelGGL((tri_kernel<true, false>), grid, 64, 0, 0, n, o1, r1);
        else hipLaunchKernelGGL(tri_kernel<false>, grid, 64, 0, 0, n, o0, r0);
    };
    int diffs[5] = {0, 0, 0, 0, 0};
    double *h0 = new double[4 * n], *h1 = new double[4 * n];
    for (int v : {0, 2, 4}) {
        for (int rep = 0; rep < 3; rep++) launch(v);  // warm up
        hipEventRecord(a);
        const int reps = 50;
        for (int rep = 0; rep < reps; rep++) launch(v);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        printf("V%d: %.2f us per launch (%d systems)\n", v, 1e3 * ms / reps, n);
        hipMemcpy(h0, o0, n * 32, hipMemcpyDeviceToHost);
        hipMemcpy(h1, o1, n * 32, hipMemcpyDeviceToHost);
        for (int i = 0; v && i < 4 * n; i++) diffs[v] += memcmp(&h0[i], &h1[i], 8) != 0;
    }
    printf("null vectors differing from V0: V2 (unrolled) %d, V4 (round robin, another order) %d\n", diffs[2], diffs[4]);
    int* hr = new int[n];
    hipMemcpy(h0, o0, n * 32, hipMemcpyDeviceToHost);
    hipMemcpy(h1, o1, n * 32, hipMemcpyDeviceToHost);
    hipMemcpy(hr, r0, n * 4, hipMemcpyDeviceToHost);
    int diff = 0, mx = 0;
    double mean = 0;
    for (int i = 0; i < 4 * n; i++) diff += memcmp(&h0[i], &h1[i], 8) != 0;
    for (int i = 0; i < n; i++) {
        mx = hr[i] > mx ? hr[i] : mx;
        mean += hr[i];
    }
    printf("null vectors differing V0 vs V1: %d of %d; rotations mean %.1f max %d\n", diff, 4 * n, mean / n, mx);
    return (diff || diffs[2]) ? 1 : 0;
}
