// fetch_calib.hip -- calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths
// of the LM kernel's slab streams (MI355X_MICROARCH.md: FETCH_SIZE reads half the bytes of 16-B
// per-lane streaming loads; other widths uncalibrated).  Each kernel streams a known byte count
// once (buffer >> Infinity Cache); run under `rocprofv3 --pmc FETCH_SIZE` and
// `--pmc WRITE_SIZE` and compare the counter with the bytes printed here.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __attribute__((address_space(1))) const double gd;
typedef __attribute__((address_space(1))) const float gf;

__global__ void rd_f64_nt(const double* p, size_t n, double* out) {
    double acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc += __builtin_nontemporal_load((gd*)p + i);
    if (acc == 12345.678) out[0] = acc;
}
__global__ void rd_f32_nt(const float* p, size_t n, double* out) {
    float acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc += __builtin_nontemporal_load((gf*)p + i);
    if (acc == 12345.678f) out[0] = acc;
}
__global__ void rd_f32x4(const float4* p, size_t n, double* out) {
    float acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        float4 v = p[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 12345.678f) out[0] = acc;
}
__global__ void wr_f32(float* p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = (float)i;
}

int main() {
    const size_t bytes = (size_t)2 << 30;
    void* buf;
    double* out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    hipMemset(buf, 0, bytes);
    const dim3 g(4096), b(256);
    for (int rep = 0; rep < 2; rep++) {
        rd_f64_nt<<<g, b>>>((const double*)buf, bytes / 8, out);
        rd_f32_nt<<<g, b>>>((const float*)buf, bytes / 4, out);
        rd_f32x4<<<g, b>>>((const float4*)buf, bytes / 16, out);
        wr_f32<<<g, b>>>((float*)buf, bytes / 4);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("fetch_calib: every kernel moves %zu bytes (%.1f KiB) per launch\n", bytes, bytes / 1024.0);
    hipFree(buf);
    hipFree(out);
    return 0;
}
