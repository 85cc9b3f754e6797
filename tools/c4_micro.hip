// Microbenchmark (not product code): the building blocks of chain v4 (bb_chol4.h) on one CU.
//   leaf      : the 16-pivot [D | I] leaf of one wave (v_fmac_f64 row_newbcast), cycles per leaf
//   leaf+mfma : the same while the CU's other 7 waves issue fp64 MFMA back to back
//   mfma dep  : dependent v_mfma_f64_16x16x4f64 on one accumulator, cycles per MFMA
//   mfma ind  : 4 independent accumulators, cycles per MFMA (one wave; and 8 waves per CU)
//   fma ind   : independent v_fma_f64 (one wave), cycles per instruction
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/c4_micro tools/c4_micro.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double v4d __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double fast_rcp(double p) {
    const double r = __builtin_amdgcn_rcp(p);
    return __builtin_fma(r, __builtin_fma(-p, r, 1.0), r);
}
template <int C>
__device__ __forceinline__ void fmac_bc(double &acc, double src, double mul) {
    asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc) : "v"(src), "v"(mul), "n"(C));
}
template <int C>
__device__ __forceinline__ void fmac_bc_self(double &acc, double mul) {
    asm volatile("v_fmac_f64_dpp %0, %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc) : "v"(mul), "n"(C));
}
template <int C>
__device__ __forceinline__ void pivot(double (&a)[16], double (&e)[16], double (&pv)[16]) {
    double p;
    asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf"
                 : "=v"(p) : "v"(a[C]), "n"(C));
    pv[C] = p;
    if constexpr (C < 15) {
        const double inv = fast_rcp(p);
        const double na = -a[C] * inv, ne = -e[C] * inv;
#pragma unroll
        for (int i = C + 1; i < 16; ++i) {
            fmac_bc<C>(e[i], a[i], ne);
            fmac_bc_self<C>(a[i], na);
        }
    }
}
template <int C>
__device__ __forceinline__ void pivots(double (&a)[16], double (&e)[16], double (&pv)[16]) {
    pivot<C>(a, e, pv);
    if constexpr (C < 15) pivots<C + 1>(a, e, pv);
}

// MODE 0: leaf on wave 0 alone; 1: leaf on wave 0, MFMA on waves 1-7; 2: mfma dep (wave 0);
// 3: mfma independent (wave 0); 4: mfma independent on all 8 waves; 5: fma independent
template <int MODE>
__global__ void k_micro(double *out, unsigned long long *cyc, int reps, volatile int *stop) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, x = lane & 15;
    __shared__ int done;
    if (threadIdx.x == 0) done = 0;
    __syncthreads();
    unsigned long long t0 = 0, t1 = 0;
    double sink = 0.0;
    if ((MODE == 0 || MODE == 1) && wid == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < reps; ++r) {
            double a[16], e[16], pv[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                a[i] = (i == x ? 20.0 : 0.5 / (1 + i + x)) + 1e-9 * r;
                e[i] = i == x ? 1.0 : 0.0;
            }
            pivots<0>(a, e, pv);
#pragma unroll
            for (int i = 0; i < 16; ++i) sink += e[i] + pv[i];
        }
        t1 = __builtin_amdgcn_s_memtime();
        if (MODE == 1 && lane == 0) *(volatile int *)&done = 1;
    } else if (MODE == 1) {
        v4d acc[4] = {};
        double av = 1.0 + 1e-3 * lane, bv = 0.5;
        while (!*(volatile int *)&done) {
#pragma unroll
            for (int q = 0; q < 16; ++q)
                acc[q & 3] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[q & 3], 0, 0, 0);
        }
        sink = acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3];
    } else if ((MODE == 2 || MODE == 3 || MODE == 5) && wid == 0) {
        v4d acc[4] = {};
        double av = 1.0 + 1e-3 * lane, bv = 0.5, f[8];
        for (int q = 0; q < 8; ++q) f[q] = av + q;
        t0 = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < reps; ++r) {
            if (MODE == 2) {
#pragma unroll
                for (int q = 0; q < 16; ++q)
                    acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[0], 0, 0, 0);
            } else if (MODE == 3) {
#pragma unroll
                for (int q = 0; q < 16; ++q)
                    acc[q & 3] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[q & 3], 0, 0, 0);
            } else {
#pragma unroll
                for (int q = 0; q < 16; ++q) f[q & 7] = __builtin_fma(f[q & 7], bv, av);
            }
        }
        t1 = __builtin_amdgcn_s_memtime();
        sink = acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3] + f[0] + f[7];
    } else if (MODE == 4) {
        v4d acc[4] = {};
        double av = 1.0 + 1e-3 * lane, bv = 0.5;
        t0 = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < reps; ++r) {
#pragma unroll
            for (int q = 0; q < 16; ++q)
                acc[q & 3] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[q & 3], 0, 0, 0);
        }
        t1 = __builtin_amdgcn_s_memtime();
        sink = acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3];
    }
    out[threadIdx.x] = sink;
    if (lane == 0) cyc[wid] = t1 - t0;
}

int main() {
    double *out;
    unsigned long long *cyc, h[8];
    int *stop;
    hipMalloc(&out, 512 * sizeof(double));
    hipMalloc(&cyc, 8 * sizeof(unsigned long long));
    hipMalloc(&stop, sizeof(int));
    const int reps = 2000;
#define RUN(M, NT, PER, NAME)                                                              \
    for (int w = 0; w < 2; ++w) k_micro<M><<<1, NT>>>(out, cyc, reps, stop);                 \
    hipDeviceSynchronize();                                                                \
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);                                   \
    printf("%-34s %8.1f cycles per %s\n", NAME, (double)h[0] / reps / (PER), M == 0 || M == 1 ? "leaf" : "instr");
    RUN(0, 64, 1, "leaf (1 wave)")
    RUN(1, 512, 1, "leaf + 7 MFMA waves")
    RUN(2, 64, 16, "mfma f64 dependent")
    RUN(3, 64, 16, "mfma f64 4 independent")
    RUN(4, 512, 16, "mfma f64 4 indep, 8 waves/CU")
    RUN(5, 64, 16, "fma f64 8 independent")
    return 0;
}
