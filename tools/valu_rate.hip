// Microbenchmark (not product code): VALU issue cost per wave64 instruction on gfx950, for the
// instructions the tilted-stable sampler compiles to, grouped by the classes rocprofv3 counts
// (SQ_INSTS_VALU_{FMA,MUL,ADD,TRANS}_{F32,F64}, _INT32, _INT64, _CVT; an instruction in none of
// them is "other").  bench.py prices the lambda launch's per-class instruction counts with these
// costs.  Each wave runs 8 independent chains of one instruction (inline asm:
// exactly that instruction), W waves per SIMD on every CU.  Every wave stamps s_memtime (shader
// clock) before and after its loop; a workgroup's span (last end - first start over its 4 W
// waves, all on one CU) over the W instructions per chain slot each SIMD issued gives cycles per
// wave-instruction per SIMD.  Run under `rocprofv3 --pmc SQ_INSTS_VALU_<class>` (one counter per
// pass) the per-kernel counts show which class each instruction falls in (kernel k_rate<op>).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/valu_rate tools/valu_rate.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define OPS(X)                                                                                \
    X(0, "v_fma_f64", F64, BIN, "v_fma_f64 %0, %0, %1, %2")                                    \
    X(1, "v_mul_f64", F64, BIN, "v_mul_f64 %0, %0, %1 ; %2")                                   \
    X(2, "v_add_f64", F64, BIN, "v_add_f64 %0, %0, %1 ; %2")                                   \
    X(3, "v_rcp_f64", F64, UN, "v_rcp_f64 %0, %0")                                             \
    X(4, "v_sqrt_f64", F64, UN, "v_sqrt_f64 %0, %0")                                           \
    X(5, "v_ldexp_f64", F64, UN, "v_ldexp_f64 %0, %0, 1")                                      \
    X(6, "v_fract_f64", F64, UN, "v_fract_f64 %0, %0")                                         \
    X(7, "v_frexp_mant_f64", F64, UN, "v_frexp_mant_f64 %0, %0")                               \
    X(8, "v_div_fixup_f64", F64, BIN, "v_div_fixup_f64 %0, %0, %1, %2")                        \
    X(9, "v_cmp_gt_f64", F64, CMP, "v_cmp_gt_f64 vcc, %0, %1")                                 \
    X(10, "v_fma_f32", F32, BIN, "v_fma_f32 %0, %0, %1, %2")                                   \
    X(11, "v_exp_f32", F32, UN, "v_exp_f32 %0, %0")                                            \
    X(12, "v_log_f32", F32, UN, "v_log_f32 %0, %0")                                            \
    X(13, "v_add_u32", U32, BIN, "v_add_u32 %0, %0, %1 ; %2")                                  \
    X(14, "v_mul_lo_u32", U32, BIN, "v_mul_lo_u32 %0, %0, %1 ; %2")                            \
    X(15, "v_and_b32", U32, BIN, "v_and_b32 %0, %0, %1 ; %2")                                  \
    X(16, "v_cndmask_b32", U32, BINV, "v_cndmask_b32 %0, %0, %1, vcc ; %2")                    \
    X(17, "v_bfe_u32", U32, BIN, "v_bfe_u32 %0, %0, %1, %2")                                   \
    X(18, "v_mov_b32", U32, UN, "v_mov_b32 %0, %0")                                            \
    X(19, "v_mad_u64_u32", U64, BINV, "v_mad_u64_u32 %0, vcc, %1, %2, %0")                   \
    X(20, "v_lshlrev_b64", U64, UN, "v_lshlrev_b64 %0, 1, %0")                                 \
    X(21, "v_cvt_f64_u32", U32, CVT, "v_cvt_f64_u32 %0, %1")

#define DESC(i, nm, T, S, ins) nm,
static const char *kNames[] = {OPS(DESC)};
constexpr int kNops = sizeof(kNames) / sizeof(kNames[0]);

// chain-variable initialisations per operand type
#define INIT_F64                                                                              \
    double a0 = threadIdx.x * 1e-3 + 1.5, a1 = a0 + 0.1, a2 = a0 + 0.2, a3 = a0 + 0.3,          \
           a4 = a0 + 0.4, a5 = a0 + 0.5, a6 = a0 + 0.6, a7 = a0 + 0.7, b = 0.999, c = 1e-3;
#define INIT_F32                                                                              \
    float a0 = threadIdx.x * 1e-3f + 0.5f, a1 = a0 + 0.1f, a2 = a0 + 0.2f, a3 = a0 + 0.3f,      \
          a4 = a0 + 0.4f, a5 = a0 + 0.5f, a6 = a0 + 0.6f, a7 = a0 + 0.7f, b = 0.999f, c = 1e-3f;
#define INIT_U32                                                                              \
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, \
             a6 = a0 + 6, a7 = a0 + 7, b = 2654435761u, c = 7;
#define INIT_U64                                                                              \
    unsigned long long a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,    \
                       a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                 \
    unsigned b = 3, c = 5;
// one statement of the chain slot a, instruction string I
#define S_BIN(a, I) asm volatile(I : "+v"(a) : "v"(b), "v"(c));
#define S_BINV(a, I) asm volatile(I : "+v"(a) : "v"(b), "v"(c) : "vcc");
#define S_UN(a, I) asm volatile(I : "+v"(a));
#define S_UNV(a, I) asm volatile(I : "+v"(a) : : "vcc");
#define S_CMP(a, I) asm volatile(I : : "v"(a), "v"(b) : "vcc");
#define S_CVT(a, I)                                                                           \
    {                                                                                         \
        double d;                                                                             \
        asm volatile(I : "=v"(d) : "v"(a));                                                   \
        asm volatile("" : "+v"(a) : "v"(d));                                                  \
    }
#define R8(S, I) S(a0, I) S(a1, I) S(a2, I) S(a3, I) S(a4, I) S(a5, I) S(a6, I) S(a7, I)

template <int OP>
__global__ void k_rate(unsigned long long *stamp, double *sink, int iters);

#define KERNEL(i, nm, T, S, ins)                                                               \
    template <>                                                                                \
    __global__ void k_rate<i>(unsigned long long *stamp, double *sink, int iters) {            \
        INIT_##T(void) b;                                                                      \
        (void)c;                                                                               \
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();                           \
        for (int it = 0; it < iters; ++it) { R8(S_##S, ins) }                                  \
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();                            \
        sink[blockIdx.x * blockDim.x + threadIdx.x] =                                          \
            (double)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);                                   \
        if ((threadIdx.x & 63) == 0) {                                                         \
            const int w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;                   \
            stamp[2 * w] = t0;                                                                 \
            stamp[2 * w + 1] = t1;                                                             \
        }                                                                                      \
    }
OPS(KERNEL)

template <int OP>
static void run(int waves_per_simd, int iters) {
    const int cus = 256, threads = 256 * waves_per_simd;  // 4 SIMDs x waves_per_simd waves
    const int wpb = threads / 64, nw = cus * wpb;
    unsigned long long *st;
    double *sink;
    (void)hipMalloc(&st, 2 * nw * sizeof(unsigned long long));
    (void)hipMalloc(&sink, (size_t)cus * threads * sizeof(double));
    k_rate<OP><<<cus, threads>>>(st, sink, 16);  // warm
    k_rate<OP><<<cus, threads>>>(st, sink, iters);
    (void)hipDeviceSynchronize();
    unsigned long long *h = new unsigned long long[2 * nw];
    (void)hipMemcpy(h, st, 2 * nw * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    double span_sum = 0.0, span_max = 0.0;
    for (int b = 0; b < cus; ++b) {
        unsigned long long lo = ~0ull, hi = 0;
        for (int w = 0; w < wpb; ++w) {
            lo = h[2 * (b * wpb + w)] < lo ? h[2 * (b * wpb + w)] : lo;
            hi = h[2 * (b * wpb + w) + 1] > hi ? h[2 * (b * wpb + w) + 1] : hi;
        }
        span_sum += (double)(hi - lo);
        span_max = (double)(hi - lo) > span_max ? (double)(hi - lo) : span_max;
    }
    const double inst = 8.0 * iters * waves_per_simd;  // wave-instructions per SIMD
    printf("%-18s W=%d  %.2f cyc per wave-instruction per SIMD (mean CU span; max %.2f)\n",
           kNames[OP], waves_per_simd, span_sum / cus / inst, span_max / inst);
    delete[] h;
    (void)hipFree(st);
    (void)hipFree(sink);
}

template <int OP>
static void run_all(int iters) {
    for (int w : {1, 2, 4}) run<OP>(w, iters);
    if constexpr (OP + 1 < kNops) run_all<OP + 1>(iters);
}

int main(int argc, char **argv) {
    run_all<0>(argc > 1 ? atoi(argv[1]) : 2048);
    return 0;
}
