// Microbenchmark (round 3): the LM chain lane's 64-term chunk sums fed from LDS, by how the terms
// reach the registers.  Prints cycles per dependent fp64 add for each variant, one wave alone and
// next to 3 / 15 fp64-busy waves.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kN = 4096;

// the kernel's chain_sum64: four rotating sets of 8 values (ds_read_b128), sched barriers
__device__ __forceinline__ double sum64_rot4(double sum, const double* row) {
    const double2* R = reinterpret_cast<const double2*>(row);
    double2 v0[4], v1[4], v2[4], v3[4];
    auto ld = [&](double2 (&v)[4], int k) {
#pragma unroll
        for (int i = 0; i < 4; i++) v[i] = R[4 * k + i];
        __asm__ __volatile__("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };
    auto add = [&](const double2 (&v)[4]) {
#pragma unroll
        for (int i = 0; i < 4; i++) { sum += v[i].x; sum += v[i].y; }
        __asm__ __volatile__("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };
    ld(v0, 0); ld(v1, 1); ld(v2, 2); ld(v3, 3);
    add(v0); ld(v0, 4); add(v1); ld(v1, 5); add(v2); ld(v2, 6); add(v3); ld(v3, 7);
    add(v0); add(v1); add(v2); add(v3);
    return sum;
}
// all 64 terms into registers first (32 ds_read_b128), then 64 adds
__device__ __forceinline__ double sum64_all(double sum, const double* row) {
    const double2* R = reinterpret_cast<const double2*>(row);
    double2 v[32];
#pragma unroll
    for (int i = 0; i < 32; i++) v[i] = R[i];
#pragma unroll
    for (int i = 0; i < 32; i++) { sum += v[i].x; sum += v[i].y; }
    return sum;
}
// two halves of 32 terms
__device__ __forceinline__ double sum64_half(double sum, const double* row) {
    const double2* R = reinterpret_cast<const double2*>(row);
    double2 a[16], b[16];
#pragma unroll
    for (int i = 0; i < 16; i++) a[i] = R[i];
#pragma unroll
    for (int i = 0; i < 16; i++) b[i] = R[16 + i];
#pragma unroll
    for (int i = 0; i < 16; i++) { sum += a[i].x; sum += a[i].y; }
#pragma unroll
    for (int i = 0; i < 16; i++) { sum += b[i].x; sum += b[i].y; }
    return sum;
}
// terms as ds_read_b64 (one double per read), 16 in flight
__device__ __forceinline__ double sum64_b64(double sum, const double* row) {
    double v[64];
#pragma unroll
    for (int i = 0; i < 64; i++) v[i] = row[i];
#pragma unroll
    for (int i = 0; i < 64; i++) sum += v[i];
    return sum;
}
// two independent sums interleaved in one lane (two rows), 32-term halves
__device__ __forceinline__ void sum64_two(double& s0, double& s1, const double* r0, const double* r1) {
    const double2* A = reinterpret_cast<const double2*>(r0);
    const double2* B = reinterpret_cast<const double2*>(r1);
#pragma unroll
    for (int h = 0; h < 2; h++) {
        double2 a[16], b[16];
#pragma unroll
        for (int i = 0; i < 16; i++) { a[i] = A[16 * h + i]; b[i] = B[16 * h + i]; }
#pragma unroll
        for (int i = 0; i < 16; i++) { s0 += a[i].x; s1 += b[i].x; s0 += a[i].y; s1 += b[i].y; }
    }
}

__global__ void bench(int mode, int reps, int active, double* out, long long* cyc) {
    __shared__ double t[kN];
    for (int i = threadIdx.x; i < kN; i += blockDim.x) t[i] = 1e-3 * (i % 97);
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (wave == 0) {
        __builtin_amdgcn_s_setprio(3);
        double s = threadIdx.x, s1 = 0.5;
        // each lane its own row of 64 (lane-strided rows, 528-byte pitch like the kernel's ring)
        const double* row = t + (lane % 30) * 66;
        long long c0 = clock64();
        if (lane < active) for (int r = 0; r < reps; r++) {
            const double* rr = row + (r & 1) * 2;
            if (mode == 0) s = sum64_rot4(s, rr);
            else if (mode == 1) s = sum64_all(s, rr);
            else if (mode == 2) s = sum64_half(s, rr);
            else if (mode == 3) s = sum64_b64(s, rr);
            else { sum64_two(s, s1, rr, rr + 30 * 66 > t + kN - 64 ? rr : rr + 2); }
        }
        long long c1 = clock64();
        if (threadIdx.x == 0) cyc[blockIdx.x] = c1 - c0;
        out[threadIdx.x] = s + s1;
    } else {
        double a = threadIdx.x, b = 1.0000001, c = 0.9999999, d = 0.5;
        for (int r = 0; r < reps * 4; r++) {
#pragma unroll 16
            for (int i = 0; i < 16; i++) { a = a * b + c; d = d * c + b; }
        }
        out[threadIdx.x] = a + d;
    }
}

int main() {
    double* out;
    long long* cyc;
    hipMalloc(&out, 4096 * sizeof(double));
    hipMalloc(&cyc, 4096 * sizeof(long long));
    const int reps = 400;
    const char* names[] = {"rot4 (kernel)", "all64", "half32", "b64", "two sums"};
    for (int mode = 0; mode < 5; mode++)
        for (int active : {64, 32, 16})
        for (int waves : {1, 16}) {
            hipLaunchKernelGGL(bench, dim3(1), dim3(64 * waves), 0, 0, mode, reps, active, out, cyc);
            hipDeviceSynchronize();
            long long c;
            hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
            const double adds = reps * 64.0 * (mode == 4 ? 2 : 1);
            printf("%-14s lanes %2d waves %2d: %.2f cycles per add (%.1f per 64-term chunk and sum)\n", names[mode], active, waves,
                   (double)c / adds, (double)c / (reps * (mode == 4 ? 2.0 : 1.0)));
        }
    return 0;
}
