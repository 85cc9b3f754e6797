// Microbenchmark (not product code): latency of the Cholesky pivot recurrence
// p' = d - x^2 / p on one wave, in several fp64 formulations, plus single-op latencies.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/chain_lat tools/chain_lat.hip
#include <hip/hip_runtime.h>

#include <cstdio>

__device__ __forceinline__ double rl5(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, 5);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), 5);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// DPP row_newbcast:5 (gfx90a+ encoding 0x150 + lane): lane 5 of each 16-lane row to the row
__device__ __forceinline__ double dpp_bcast5(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x155, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x155, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

template <int V>
__global__ void k_chain(double *out, unsigned long long *t, int n) {
    double p = 3.0 + out[threadIdx.x], d = 3.0, tt = 1.0 + 1e-3 * out[threadIdx.x + 64];
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
        if (V == 0) {  // rcp + 2 Newton fma + mul + fma (product scheme)
            const double r = __builtin_amdgcn_rcp(p);
            const double inv = __builtin_fma(r, __builtin_fma(-p, r, 1.0), r);
            const double l = tt * inv;
            p = __builtin_fma(-l, tt, d);
        } else if (V == 1) {  // rcp -> (u, v) -> fma
            const double r = __builtin_amdgcn_rcp(p);
            const double u = __builtin_fma(-p, r, 2.0);
            const double v = (tt * tt) * r;
            p = __builtin_fma(-v, u, d);
        } else if (V == 2) {  // dependent fma only
            p = __builtin_fma(p, 0.999, 1e-3);
        } else if (V == 3) {  // dependent rcp only
            p = __builtin_amdgcn_rcp(p);
        } else if (V == 4) {  // dependent mul
            p = p * 1.0000001;
        } else if (V == 5) {  // readlane round trip + fma
            const long long b = __double_as_longlong(p);
            const int lo = __builtin_amdgcn_readlane((int)b, 5);
            const int hi = __builtin_amdgcn_readlane((int)(b >> 32), 5);
            p = __builtin_fma(__longlong_as_double(((long long)hi << 32) | (unsigned)lo), 0.999, 1e-3);
        } else if (V == 6) {  // f32 fma
            float q = (float)p;
            for (int k = 0; k < 8; ++k) q = __builtin_fmaf(q, 0.999f, 1e-3f);
            p = (double)q;
        } else if (V == 7) {  // v_div_scale-free division p' = d - t/p via IEEE divide
            p = d - tt / p;
        } else if (V == 8) {  // DPP row_newbcast (lane 5 of each 16-lane row) + fma
            p = __builtin_fma(dpp_bcast5(p), 0.999, 1e-3);
        } else if (V == 9) {  // ds_bpermute (__shfl from lane 5) + fma
            p = __builtin_fma(__shfl(p, 5, 64), 0.999, 1e-3);
        } else if (V == 10) {  // one pivot of the product's in-wave step, readlane broadcasts:
            // pivot -> rcp -> 2 Newton fmas -> multiplier (broadcast a_ci * inv) -> the next
            // pivot's entry updated
            const double pv = rl5(p);
            const double r = __builtin_amdgcn_rcp(pv);
            const double inv = __builtin_fma(r, __builtin_fma(-pv, r, 1.0), r);
            const double l = rl5(tt * p) * inv;
            p = __builtin_fma(-l, tt, d);
        } else if (V == 11) {  // the same pivot with DPP broadcasts
            const double pv = dpp_bcast5(p);
            const double r = __builtin_amdgcn_rcp(pv);
            const double inv = __builtin_fma(r, __builtin_fma(-pv, r, 1.0), r);
            const double l = dpp_bcast5(tt * p) * inv;
            p = __builtin_fma(-l, tt, d);
        } else if (V == 12) {  // two pivots per step (2x2 Schur): p1 broadcast, p2 formed
            // from uniform values, both reciprocals, the next pair's entry updated (one
            // broadcast per two pivots); cycles per iteration = two pivots
            const double p1 = rl5(p);
            const double r1 = __builtin_amdgcn_rcp(p1);
            const double i1 = __builtin_fma(r1, __builtin_fma(-p1, r1, 1.0), r1);
            const double p2 = __builtin_fma(-(tt * tt), i1, d);
            const double r2 = __builtin_amdgcn_rcp(p2);
            const double i2 = __builtin_fma(r2, __builtin_fma(-p2, r2, 1.0), r2);
            p = __builtin_fma(-(tt * i1), tt, __builtin_fma(-(tt * i2), tt, d));
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = p;
    if (threadIdx.x == 0) t[0] = t1 - t0;
}

int main() {
    double *out;
    unsigned long long *t, h;
    hipMalloc(&out, 256 * sizeof(double));
    hipMemset(out, 0, 256 * sizeof(double));
    hipMalloc(&t, 8);
    const int n = 20000;
    const char *names[] = {"rcp+newton+mul+fma (current)", "rcp->(u,v)->fma", "dep fma",
                           "dep rcp", "dep mul", "readlane+fma", "8 dep f32 fma + 2 cvt",
                           "d - t/p (IEEE div)", "dpp row_newbcast+fma", "ds_bpermute+fma",
                           "pivot step, readlane (product)", "pivot step, dpp",
                           "2 pivots (2x2 Schur), 1 readlane"};
#define RUN(V)                                                    \
    for (int rep = 0; rep < 2; ++rep) k_chain<V><<<1, 64>>>(out, t, n); \
    hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);                     \
    printf("%-34s %7.1f cycles/iter\n", names[V], (double)h / n);
    RUN(0) RUN(1) RUN(2) RUN(3) RUN(4) RUN(5) RUN(6) RUN(7) RUN(8) RUN(9) RUN(10) RUN(11) RUN(12)
    // the effective shader clock for the ns conversion
    k_chain<2><<<1, 64>>>(out, t, n);
    hipDeviceSynchronize();
    return 0;
}
