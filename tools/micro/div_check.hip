// div_check.hip -- the fast divisions of csrc/fm3d_fastdiv.h against the division operator,
// bit for bit, on random operands (log-uniform exponents across and beyond the guarded
// ranges, both signs, plus zeros, denormals, infinities and NaNs).
//
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I3dfeaturematcher_amd/csrc \
//         tools/micro/div_check.hip -o tools/micro/div_check && tools/micro/div_check
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
// +-m * 2^e, e uniform in [lo, hi]; 1 in 64 draws a special value
__device__ inline double draw(uint64_t r, int lo, int hi) {
    if ((r & 63) == 0) {
        const double sp[8] = {0., -0., 4.9e-324, -2.2e-310, __builtin_inf(), -__builtin_inf(), __builtin_nan(""), 1.};
        return sp[(r >> 6) & 7];
    }
    const int e = lo + (int)((r >> 8) % (uint64_t)(hi - lo + 1));
    const double m = 1. + (double)(r >> 12 & ((1ull << 52) - 1)) * 0x1p-52;
    return ((r >> 7) & 1 ? -m : m) * __builtin_ldexp(1., e);
}
__device__ inline bool same(double a, double b) {
    if (a != a && b != b) return true;
    return __double_as_longlong(a) == __double_as_longlong(b);
}

__device__ double g_fail[64][3];  // first failing mdiv operands: a, d, fast result
__device__ double g_fail2[8][3];  // first failing div_nn operands: mm, nn, fast result
__device__ unsigned long long bad_[2];

__global__ void check(uint64_t seed, int iters, unsigned long long* bad, unsigned long long* fast) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    unsigned long long nb[3] = {0, 0, 0}, nf[3] = {0, 0, 0};
    for (int i = 0; i < iters; i++) {
        const uint64_t r0 = mix(seed ^ (t * 0x100000001B3ull + i)), r1 = mix(r0), r2 = mix(r1);
        // recip_z; recip_z_lo where |z| <= 2^700
        {
            const double z = draw(r0, -1100, 760);
            const double ref = z ? 1. / z : 1.;
            nb[0] += !same(recip_z(z), ref);
            if (!(fabs(z) > 0x1p700)) nb[0] += !same(recip_z_lo(z), ref);
            nf[0] += fabs(z) >= 0x1p-700 && fabs(z) <= 0x1p700;
        }
        // div_nn (the numerator is pass-uniform in the kernel; any value here; |nn| <= 2^60):
        // the IEEE quotient where that is below 2^100, NaN or >= 2^100 where it is not
        {
            const double mm = draw(r1, -640, 80);
            double nn = draw(r2, -1100, 60);
            if (__builtin_isinf(nn)) nn = 0x1p60;  // outside the precondition
            const bool ok = div_nn_ok(mm);
            const double f = div_nn(mm, nn, ok), x = mm / nn;
            const bool bad = fabs(x) < 0x1p100 ? !same(f, x) : !(f != f || !(fabs(f) < 0x1p100));
            nb[1] += bad;
            nf[1] += ok;
            if (bad) {
                const unsigned long long slot = atomicAdd(&bad_[1], 1ull);
                if (slot < 8) {
                    g_fail2[slot][0] = mm;
                    g_fail2[slot][1] = nn;
                    g_fail2[slot][2] = f;
                }
            }
        }
        // mdiv on its operand domain: |a| = 0 or in [2^-200, 2^370], any d
        {
            const double d = draw(r2 >> 3, -700, 700);
            double a = draw(r1 >> 5, -200, 370);
            // the passes never divide -0 (numerators are differences, +0 when equal): -0 / d > 0
            // gives +0 here, -0 in IEEE
            if (a != a || __builtin_isinf(a) || (a != 0. && fabs(a) < 0x1p-200) || a == 0.) a = 0.;
            const double y = 1. / d;
            const bool ok = mdiv_ok(d);
            const double q = mdiv(a, d, y, ok);
            if (!same(q, a / d)) {
                nb[2]++;
                const unsigned long long slot = atomicAdd(&bad[3], 1ull);
                if (slot < 64) {
                    g_fail[slot][0] = a;
                    g_fail[slot][1] = d;
                    g_fail[slot][2] = q;
                }
            }
            nf[2] += ok && fabs(a) < 1e100;
        }
    }
    for (int k = 0; k < 3; k++) {
        atomicAdd(&bad[k], nb[k]);
        atomicAdd(&fast[k], nf[k]);
    }
}

int main(int argc, char** argv) {
    const int blocks = 1024, threads = 256, iters = argc > 1 ? atoi(argv[1]) : 400;
    unsigned long long *bad, *fast, hb[3], hf[3];
    if (hipMalloc(&bad, 32) != hipSuccess || hipMalloc(&fast, 24) != hipSuccess) return 2;
    (void)hipMemset(bad, 0, 32);
    (void)hipMemset(fast, 0, 24);
    hipLaunchKernelGGL(check, dim3(blocks), dim3(threads), 0, 0, 0x5eedull, iters, bad, fast);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    (void)hipMemcpy(hb, bad, 24, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hf, fast, 24, hipMemcpyDeviceToHost);
    const char* names[3] = {"recip_z", "div_nn", "mdiv"};
    const unsigned long long n = (unsigned long long)blocks * threads * iters;
    double hfail2[8][3];
    (void)hipMemcpyFromSymbol(hfail2, HIP_SYMBOL(g_fail2), sizeof(hfail2));
    for (int i = 0; i < (hb[1] < 8 ? (int)hb[1] : 8); i++)
        printf("div_nn mismatch: mm=%a nn=%a fast=%a ieee=%a\n", hfail2[i][0], hfail2[i][1], hfail2[i][2],
               hfail2[i][0] / hfail2[i][1]);
    double hfail[64][3];
    (void)hipMemcpyFromSymbol(hfail, HIP_SYMBOL(g_fail), sizeof(hfail));
    for (int i = 0; i < (hb[2] < 8 ? (int)hb[2] : 8); i++)
        printf("mdiv mismatch: a=%a d=%a fast=%a ieee=%a\n", hfail[i][0], hfail[i][1], hfail[i][2],
               hfail[i][0] / hfail[i][1]);
    int rc = 0;
    for (int k = 0; k < 3; k++) {
        printf("%-8s samples %llu  fast path %llu  mismatches %llu\n", names[k], n, hf[k], hb[k]);
        if (hb[k]) rc = 1;
    }
    return rc;
}
