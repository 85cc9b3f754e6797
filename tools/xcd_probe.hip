// Microbenchmark (not product code): which XCD does workgroup b of a one-workgroup-per-CU
// grid run on?  Each workgroup (256 threads, 128 KB of LDS, like k_oz_gemm16u) records
// HW_REG_XCC_ID; the histogram of (b % 8, xcc) shows whether b % 8 is the XCD.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/xcd_probe tools/xcd_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256, 1) void k_probe(int *xcc, int spin) {
    __shared__ int big[32768];  // 128 KB: one workgroup per CU
    big[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (threadIdx.x == 0) {
        // HW_REG_XCC_ID = 20, bits [3:0]
        xcc[blockIdx.x] = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11)) + big[5] - 5;
    }
    // keep the CU busy for a while so later blocks go to other CUs
    long long t0 = clock64();
    while (clock64() - t0 < spin) {
    }
}

int main() {
    for (int grid : {256, 512, 2048}) {
        int *d;
        (void)hipMalloc(&d, grid * sizeof(int));
        for (int rep = 0; rep < 2; ++rep) k_probe<<<grid, 256>>>(d, 200000);
        (void)hipDeviceSynchronize();
        std::vector<int> h(grid);
        (void)hipMemcpy(h.data(), d, grid * sizeof(int), hipMemcpyDeviceToHost);
        int hist[8][8] = {};
        for (int b = 0; b < grid; ++b) hist[b % 8][h[b] & 7]++;
        printf("grid %d: rows = b %% 8, cols = xcc\n", grid);
        for (int i = 0; i < 8; ++i) {
            printf("  ");
            for (int j = 0; j < 8; ++j) printf("%5d", hist[i][j]);
            printf("\n");
        }
        printf("  first 32 blocks' xcc:");
        for (int b = 0; b < 32; ++b) printf(" %d", h[b]);
        printf("\n");
        (void)hipFree(d);
    }
    return 0;
}
