// Microbenchmark: cost of a dependent fp64 add chain fed from LDS (the LM chain lane),
// alone and next to fp64-busy waves on the same CU, with and without s_setprio.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int kN = 4096;

__device__ inline double chain_sum(double sum, const double* t, int n) {
    const double2* t2 = reinterpret_cast<const double2*>(t);
    double2 cur[8], nxt[8];
#pragma unroll
    for (int i = 0; i < 8; i++) cur[i] = t2[i];
    for (int q = 16; q < n; q += 16) {
#pragma unroll
        for (int i = 0; i < 8; i++) nxt[i] = t2[q / 2 + i];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            sum += cur[i].x;
            sum += cur[i].y;
        }
#pragma unroll
        for (int i = 0; i < 8; i++) cur[i] = nxt[i];
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
        sum += cur[i].x;
        sum += cur[i].y;
    }
    return sum;
}

template <int B>  // B doubles per batch (B/2 ds_read_b128), one batch of lookahead
__device__ inline double chain_sum_b(double sum, const double* t, int n) {
    const double2* t2 = reinterpret_cast<const double2*>(t);
    double2 cur[B / 2], nxt[B / 2];
#pragma unroll
    for (int i = 0; i < B / 2; i++) cur[i] = t2[i];
    for (int q = B; q < n; q += B) {
#pragma unroll
        for (int i = 0; i < B / 2; i++) nxt[i] = t2[q / 2 + i];
#pragma unroll
        for (int i = 0; i < B / 2; i++) {
            sum += cur[i].x;
            sum += cur[i].y;
        }
#pragma unroll
        for (int i = 0; i < B / 2; i++) cur[i] = nxt[i];
    }
#pragma unroll
    for (int i = 0; i < B / 2; i++) {
        sum += cur[i].x;
        sum += cur[i].y;
    }
    return sum;
}
// two batches of 16 in flight
__device__ inline double chain_sum_d2(double sum, const double* t, int n) {
    const double2* t2 = reinterpret_cast<const double2*>(t);
    double2 a[8], b[8], c[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = t2[i];
#pragma unroll
    for (int i = 0; i < 8; i++) b[i] = t2[8 + i];
    for (int q = 32; q < n; q += 16) {
#pragma unroll
        for (int i = 0; i < 8; i++) c[i] = t2[q / 2 + i];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            sum += a[i].x;
            sum += a[i].y;
        }
#pragma unroll
        for (int i = 0; i < 8; i++) {
            a[i] = b[i];
            b[i] = c[i];
        }
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
        sum += a[i].x;
        sum += a[i].y;
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
        sum += b[i].x;
        sum += b[i].y;
    }
    return sum;
}

// mode 0: registers only dependent adds; 1: chain_sum from LDS
// busyWaves: other waves in the block doing independent fp64 FMAs; prio: chain wave priority
__global__ void bench(int mode, int reps, int prio, double* out, long long* cyc) {
    __shared__ double t[kN];
    for (int i = threadIdx.x; i < kN; i += blockDim.x) t[i] = 1e-3 * (i % 97);
    __syncthreads();
    const int wave = threadIdx.x >> 6;
    if (wave == 0) {
        if (prio) __builtin_amdgcn_s_setprio(3);
        double s = threadIdx.x;
        long long c0 = clock64();
        if (threadIdx.x < 8) {
            for (int r = 0; r < reps; r++) {
                if (mode == 0) {
                    double a = t[r & 1023], b = t[(r + 7) & 1023];
#pragma unroll 64
                    for (int i = 0; i < 1024; i++) s += (i & 1) ? a : b;
                } else if (mode == 1) {
                    s = chain_sum(s, t + (r & 1) * 1024, 1024);
                } else if (mode == 2) {
                    s = chain_sum_b<32>(s, t + (r & 1) * 1024, 1024);
                } else if (mode == 3) {
                    s = chain_sum_b<64>(s, t + (r & 1) * 1024, 1024);
                } else {
                    s = chain_sum_d2(s, t + (r & 1) * 1024, 1024);
                }
            }
        }
        long long c1 = clock64();
        if (threadIdx.x == 0) cyc[blockIdx.x] = c1 - c0;
        out[threadIdx.x] = s;
    } else {
        double a = threadIdx.x, b = 1.0000001, c = 0.9999999, d = 0.5;
        for (int r = 0; r < reps * 64; r++) {
#pragma unroll 16
            for (int i = 0; i < 16; i++) {
                a = a * b + c;
                d = d * c + b;
            }
        }
        out[threadIdx.x] = a + d;
    }
}

int main() {
    double* out;
    long long* cyc;
    hipMalloc(&out, 4096 * sizeof(double));
    hipMalloc(&cyc, 4096 * sizeof(long long));
    const int reps = 200;
    const char* names[] = {"reg", "lds16", "lds32", "lds64", "lds16x2"};
    for (int mode = 0; mode < 5; mode++)
        for (int waves = 1; waves <= 16; waves *= 4)
            for (int prio = 0; prio < 1; prio++) {
                hipLaunchKernelGGL(bench, dim3(1), dim3(64 * waves), 0, 0, mode, reps, prio, out, cyc);
                hipDeviceSynchronize();
                long long c;
                hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
                printf("mode %s waves %2d prio %d: %.2f cycles per dependent add\n", names[mode],
                       waves, prio, (double)c / (reps * 1024.0));
            }
    return 0;
}
