// Counter calibration for LDS-DMA streaming reads (global_load_lds_dwordx4, the Ozaki GEMM's
// operand path): every byte of a 1 GiB buffer is read exactly once, 1 KB per wave
// instruction, into an LDS ring; the same buffer is then read once more with plain
// global_load_dwordx4 for comparison.  Profile with rocprofv3 --pmc FETCH_SIZE (one pass) and
// --pmc TCC_HIT_sum TCC_MISS_sum (another pass); the bytes per dispatch are printed here.
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ __launch_bounds__(256) void k_dma(const int8_t *src, size_t bytes, int *sink) {
    __shared__ __attribute__((aligned(1024))) int8_t lds[4][4096];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const size_t per_wave = 1024, stride = (size_t)gridDim.x * 4 * per_wave;
    int it = 0;
    for (size_t off = ((size_t)blockIdx.x * 4 + wid) * per_wave; off + per_wave <= bytes;
         off += stride, ++it) {
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void *)(src + off + lane * 16),
            (__attribute__((address_space(3))) void *)&lds[it & 3][wid * 1024], 16, 0, 0);
        if ((it & 3) == 3) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0 && lds[0][0] == 123 && lds[1][5] == 45) atomicAdd(sink, 1);
}

__global__ __launch_bounds__(256) void k_plain(const int4 *src, size_t n16, int *sink) {
    int acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const int4 v = src[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678) atomicAdd(sink, 1);
}

int main() {
    const size_t bytes = (size_t)1 << 30;
    int8_t *buf;
    int *sink;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, bytes);
    (void)hipMemset(sink, 0, 4);
    for (int r = 0; r < 2; ++r) {
        k_dma<<<2048, 256>>>(buf, bytes, sink);
        k_plain<<<2048, 256>>>((const int4 *)buf, bytes / 16, sink);
    }
    (void)hipDeviceSynchronize();
    printf("bytes per dispatch: %zu\n", bytes);
    return 0;
}
