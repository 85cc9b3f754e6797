// Divergent-lane check of gamma1: every lane draws Ga(shape_l, 1) at its own counter, once
// with all lanes active and once one lane at a time; prints mismatches.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "bb_sampler.h"

__global__ void k_all(double *o, uint32_t *err) {
    const int l = threadIdx.x;
    const double shape = (l % 3 == 0) ? 22.0 : (l % 3 == 1 ? 221.0 : 0.0);
    if (l % 3 != 2) o[l] = bb::gamma1(shape, bb::Key{11, 22}, 1 + l / 3, 3 + (l % 3), err);
    else o[l] = bb::normal_at(bb::Key{11, 22}, 1 + l / 3, 5, l);
}
__global__ void k_one(double *o, uint32_t *err) {
    for (int q = 0; q < 64; ++q) {
        const int l = threadIdx.x;
        if (l != q) continue;
        const double shape = (l % 3 == 0) ? 22.0 : (l % 3 == 1 ? 221.0 : 0.0);
        if (l % 3 != 2) o[l] = bb::gamma1(shape, bb::Key{11, 22}, 1 + l / 3, 3 + (l % 3), err);
        else o[l] = bb::normal_at(bb::Key{11, 22}, 1 + l / 3, 5, l);
    }
}
int main() {
    double *a, *b;
    uint32_t *err;
    hipMalloc(&a, 64 * 8);
    hipMalloc(&b, 64 * 8);
    hipMalloc(&err, 4);
    hipMemset(err, 0, 4);
    k_one<<<1, 64>>>(b, err);
    hipDeviceSynchronize();
    printf("one-lane done\n");
    fflush(stdout);
    k_all<<<1, 64>>>(a, err);
    hipDeviceSynchronize();
    double ha[64], hb[64];
    hipMemcpy(ha, a, sizeof(ha), hipMemcpyDeviceToHost);
    hipMemcpy(hb, b, sizeof(hb), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        if (ha[l] != hb[l]) {
            ++bad;
            printf("lane %d: all %.17g one %.17g\n", l, ha[l], hb[l]);
        }
    printf("mismatches %d\n", bad);
    return 0;
}
