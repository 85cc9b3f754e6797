// Diagnostic microbenchmarks (not part of the product): effective shader clock, dependent
// fp64 FMA latency, s_barrier cost at several workgroup sizes, LDS write->barrier->read
// round trip -- the primitives that bound the Cholesky diagonal chain.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_fma_chain(double *out, unsigned long long *t, int n) {
    double a = out[threadIdx.x], b = 1.0000001, c = 1e-9;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < n; ++i) a = __builtin_fma(a, b, c);
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) { t[0] = t1 - t0; t[1] = r1 - r0; }
}

template <int NT>
__global__ __launch_bounds__(NT) void k_barrier(double *out, unsigned long long *t, int n) {
    __shared__ double buf[2][128];
    double a = out[threadIdx.x];
    if (threadIdx.x < 128) buf[0][threadIdx.x] = a;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
        a += buf[i & 1][(threadIdx.x + i) & 127];  // LDS read of the previous step's write
        if (threadIdx.x == (i & 63)) buf[(i + 1) & 1][i & 127] = a;
        __syncthreads();
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) t[0] = t1 - t0;
}

template <int NT>
__global__ __launch_bounds__(NT) void k_barrier_only(unsigned long long *t, int n) {
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) __syncthreads();
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) t[0] = t1 - t0;
}

typedef double v4d __attribute__((ext_vector_type(4)));
// NACC independent accumulators per wave; all waves of the block issue MFMAs.
template <int NACC>
__global__ void k_mfma_rate(double *out, unsigned long long *t, int n) {
    v4d acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = (v4d){0, 0, 0, 0};
    double a = out[threadIdx.x & 63] + 1.0, b = 0.5;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int q = 0; q < NACC; ++q) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[q], 0, 0, 0);
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) t[0] = t1 - t0;
}

// The Cholesky diagonal elimination loop of bb_kernels.hip (k_chol_step), isolated.
// VAR bits: 1 = skip reciprocal (use lr), 2 = plain fma (no select), 4 = rows from regs
template <int VAR, int NT>
__global__ __launch_bounds__(NT) void k_elim(double *out, unsigned long long *t) {
    constexpr int CPT = 128 / (NT / 64);
    __shared__ __attribute__((aligned(16))) double buf[2][128];
    const int tid = threadIdx.x, r = tid & 63, cg = tid >> 6;
    const int mstart = r - cg * CPT;
    double a[CPT];
    for (int m = 0; m < CPT; ++m) a[m] = 1.0 + 0.001 * (r + m) + (r == cg * CPT + m ? 64.0 : 0.0);
    if (r == 0) for (int m = 0; m < CPT; ++m) buf[0][cg * CPT + m] = a[m];
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int c = 0; c < 64; ++c) {
        const double *bc = buf[c & 1];
        double rv[CPT];
        if (VAR & 4) {
            for (int m = 0; m < CPT; ++m) rv[m] = a[m] * 0.5;
        } else {
#pragma unroll
            for (int m = 0; m < CPT; m += 2) {
                const double2 t2 = *(const double2 *)&bc[cg * CPT + m];
                rv[m] = t2.x;
                rv[m + 1] = t2.y;
            }
        }
        const double lr = (r > c) ? bc[r] : 0.0;
        double l;
        if (VAR & 1) l = lr * 0.01;
        else {
            double p = bc[c];
            double q = __builtin_amdgcn_rcp(p);
            q = q * (2.0 - p * q);
            l = lr * q;
        }
#pragma unroll
        for (int m = 0; m < CPT; ++m) {
            const double nv = __builtin_fma(-l, rv[m], a[m]);
            if (VAR & 2) a[m] = nv;
            else a[m] = (m >= mstart) ? nv : a[m];
        }
        if (r == c + 1) {
            double *bn = buf[(c + 1) & 1];
#pragma unroll
            for (int m = 0; m < CPT; m += 2)
                *(double2 *)&bn[cg * CPT + m] = make_double2(a[m], a[m + 1]);
        }
        __syncthreads();
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
    for (int m = 0; m < CPT; ++m) s += a[m];
    out[tid] = s;
    if (tid == 0) t[0] = t1 - t0;
}

// Full-chip fp64 MFMA throughput: grid of blocks, NACC accumulators per wave.
template <int NACC>
__global__ __launch_bounds__(256) void k_mfma_chip(double *out, int n) {
    v4d acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = (v4d){0, 0, 0, 0};
    double a = out[threadIdx.x & 63] + 1.0, b = 0.5;
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int q = 0; q < NACC; ++q) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[q], 0, 0, 0);
    }
    double s = 0;
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    if (s == 12345.0 && blockIdx.x < 1024) out[blockIdx.x] = s;
}

// The row-blocked elimination loop of k_chol_step (wave = 8 rows, lane = 2 columns).
__global__ __launch_bounds__(512) void k_elim_rows(double *out, unsigned long long *t) {
    __shared__ __attribute__((aligned(16))) double buf[2][128];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int r0 = wid * 8, c0 = lane * 2;
    double a[8][2];
    for (int i = 0; i < 8; ++i)
        for (int q = 0; q < 2; ++q) a[i][q] = 1.0 + 0.001 * (i + q + lane) + ((r0 + i == c0 + q) ? 64.0 : 0.0);
    if (wid == 0) *(double2 *)&buf[0][c0] = make_double2(a[0][0], a[0][1]);
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int c = 0; c < 64; ++c) {
        const double *bc = buf[c & 1];
        const double2 rv = *(const double2 *)&bc[c0];
        double lr[8];
#pragma unroll
        for (int i = 0; i < 8; i += 2) {
            const double2 t2 = *(const double2 *)&bc[r0 + i];
            lr[i] = t2.x;
            lr[i + 1] = t2.y;
        }
        double p = bc[c];
        double inv = __builtin_amdgcn_rcp(p);
        inv = inv * (2.0 - p * inv);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int row = r0 + i;
            const double li = (row > c) ? lr[i] * inv : 0.0;
            const double n0 = __builtin_fma(-li, rv.x, a[i][0]);
            const double n1 = __builtin_fma(-li, rv.y, a[i][1]);
            a[i][0] = (c0 >= 64 || c0 >= row) ? n0 : a[i][0];
            a[i][1] = (c0 + 1 >= 64 || c0 + 1 >= row) ? n1 : a[i][1];
        }
        const int nr = c + 1;
        if (nr < 64 && (nr >> 3) == wid) {
            double v0 = 0.0, v1 = 0.0;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                v0 = (i == (nr & 7)) ? a[i][0] : v0;
                v1 = (i == (nr & 7)) ? a[i][1] : v1;
            }
            *(double2 *)&buf[nr & 1][c0] = make_double2(v0, v1);
        }
        __syncthreads();
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
    for (int i = 0; i < 8; ++i) s += a[i][0] + a[i][1];
    out[tid] = s;
    if (tid == 0) t[0] = t1 - t0;
}

int main() {
    double *out;
    unsigned long long *t, h[2];
    hipMalloc(&out, 1024 * sizeof(double));
    hipMemset(out, 0, 1024 * sizeof(double));
    hipMalloc(&t, 2 * sizeof(unsigned long long));
    const int n = 100000;
    for (int rep = 0; rep < 2; ++rep) {
        k_fma_chain<<<1, 64>>>(out, t, n);
        hipMemcpy(h, t, sizeof(h), hipMemcpyDeviceToHost);
    }
    double clk = (double)h[0] / ((double)h[1] / 100e6);
    printf("dependent v_fma_f64 chain, 1 wave: %.2f cycles/FMA; shader clock %.0f MHz\n",
           (double)h[0] / n, clk / 1e6);
    const int nb = 20000;
#define BAR(NT)                                                                          \
    k_barrier_only<NT><<<1, NT>>>(t, nb);                                                \
    hipMemcpy(h, t, 8, hipMemcpyDeviceToHost);                                           \
    printf("s_barrier only, %4d threads: %.1f cycles/barrier\n", NT, (double)h[0] / nb); \
    k_barrier<NT><<<1, NT>>>(out, t, nb);                                                \
    hipMemcpy(h, t, 8, hipMemcpyDeviceToHost);                                           \
    printf("LDS read + write + barrier, %4d threads: %.1f cycles/step\n", NT, (double)h[0] / nb);
    BAR(64) BAR(128) BAR(256) BAR(512) BAR(1024)
    const int nm = 4000;
#define MF(NACC, NT)                                                                      \
    k_mfma_rate<NACC><<<1, NT>>>(out, t, nm);                                             \
    hipMemcpy(h, t, 8, hipMemcpyDeviceToHost);                                            \
    printf("mfma_f64_16x16x4: %2d acc, %4d threads: %.1f cycles per MFMA per wave "       \
           "(%.1f flop/clk/SIMD if %d waves/SIMD)\n", NACC, NT,                           \
           (double)h[0] / (nm * NACC), 2048.0 * nm * NACC * ((NT / 64 + 3) / 4) / h[0], (NT / 64 + 3) / 4);
#define EL(VAR, NT)                                                                       \
    k_elim<VAR, NT><<<1, NT>>>(out, t);                                                   \
    hipMemcpy(h, t, 8, hipMemcpyDeviceToHost);                                            \
    printf("elimination VAR=%d threads=%4d: %.0f cycles / pivot\n", VAR, NT, (double)h[0] / 64);
    k_elim_rows<<<1, 512>>>(out, t);
    hipMemcpy(h, t, 8, hipMemcpyDeviceToHost);
    printf("row-blocked elimination (512 threads): %.0f cycles / pivot\n", (double)h[0] / 64);
    EL(0, 512) EL(1, 512) EL(2, 512) EL(3, 512) EL(4, 512) EL(7, 512) EL(0, 256) EL(0, 1024)
    MF(1, 64) MF(4, 64) MF(8, 64) MF(4, 256) MF(8, 256) MF(4, 512) MF(8, 512)
    {
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        const int n = 2000;
        for (int bpc : {1, 2, 3, 4, 8}) {
            int blocks = 256 * bpc;
            k_mfma_chip<4><<<blocks, 256>>>(out, 10);
            hipEventRecord(e0);
            k_mfma_chip<4><<<blocks, 256>>>(out, n);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            double flops = 2048.0 * 4 * n * 4 /*waves*/ * blocks;
            printf("chip fp64 MFMA: %d blocks/CU of 256 thr (%d waves/SIMD): %.1f TFLOP/s\n", bpc,
                   bpc, flops / (ms * 1e-3) / 1e12);
        }
    }
    hipDeviceSynchronize();
    return 0;
}
