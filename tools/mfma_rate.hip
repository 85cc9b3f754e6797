// Microbenchmark: sustained MFMA rate under a full-chip load (register-only loops), and
// the streaming store rate, to calibrate the Ozaki GEMM / residue kernels.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mfma_rate tools/mfma_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef double v4d __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256, 1) void k_i8(int iters, int *out) {
    v16i acc[16];
    for (int i = 0; i < 16; ++i) for (int r = 0; r < 16; ++r) acc[i][r] = 0;
    v4i a = (v4i){(int)threadIdx.x, 3, 5, 7}, b = (v4i){11, (int)blockIdx.x, 13, 17};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[i], 0, 0, 0);
        a.x += 1;
    }
    int s = 0;
    for (int i = 0; i < 16; ++i) for (int r = 0; r < 16; ++r) s += acc[i][r];
    if (s == 0x7fffffff) out[0] = s;
}

__global__ __launch_bounds__(256, 1) void k_f64(int iters, double *out) {
    v4d acc[16];
    for (int i = 0; i < 16; ++i) acc[i] = (v4d){0, 0, 0, 0};
    double a = threadIdx.x * 1e-3, b = blockIdx.x * 1e-3;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
        a += 1e-9;
    }
    double s = 0;
    for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    if (s == 12345.0) out[0] = s;
}

__global__ __launch_bounds__(256) void k_store(v4i *dst, size_t n16) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * 256;
    for (; i < n16; i += stride) dst[i] = (v4i){(int)i, 1, 2, 3};
}

__global__ __launch_bounds__(256) void k_copy(const double *src, v4i *dst, size_t nd, size_t n16) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * 256;
    double s = 0;
    for (size_t j = i; j < nd; j += stride) s += src[j];
    for (; i < n16; i += stride) dst[i] = (v4i){(int)s, 1, 2, 3};
}

int main() {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int *oi;
    double *od;
    hipMalloc(&oi, 64);
    hipMalloc(&od, 64);
    for (int rep = 0; rep < 2; ++rep) {
        const int grid = 256 * 9, iters = 392;  // the C3 Ozaki GEMM: 9 rounds, 6272 MFMA/wave
        hipEventRecord(e0);
        k_i8<<<grid, 256>>>(iters, oi);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        double ops = (double)grid * 4 * iters * 16 * 32 * 32 * 32 * 2;
        printf("i8 32x32x32: %.3f ms  %.0f TOP/s  (%.1f cycles/MFMA at 2.4 GHz)\n", ms,
               ops / ms / 1e9, ms * 1e-3 * 2.4e9 / (9.0 * iters * 16));
        hipEventRecord(e0);
        k_f64<<<256 * 4, 256>>>(400, od);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        ops = (double)256 * 4 * 4 * 400 * 16 * 16 * 16 * 4 * 2;
        printf("f64 16x16x4: %.3f ms  %.1f TFLOP/s\n", ms, ops / ms / 1e9);
    }
    const size_t bytes = (size_t)1640 << 20;
    v4i *dst;
    double *src;
    hipMalloc(&dst, bytes);
    hipMalloc(&src, (size_t)822 << 20);
    for (int rep = 0; rep < 3; ++rep) {
        float ms;
        hipEventRecord(e0);
        k_store<<<256 * 16, 256>>>(dst, bytes / 16);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        printf("store 1.64 GB: %.3f ms  %.2f TB/s\n", ms, bytes / ms / 1e9);
        hipEventRecord(e0);
        k_copy<<<256 * 16, 256>>>(src, dst, ((size_t)822 << 20) / 8, bytes / 16);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        printf("read 0.82 GB + store 1.64 GB: %.3f ms  %.2f TB/s\n", ms,
               (bytes + ((size_t)822 << 20)) / ms / 1e9);
    }
    return 0;
}
