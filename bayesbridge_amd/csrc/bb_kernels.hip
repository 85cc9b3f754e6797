// bb_kernels.hip -- gfx950 (MI355X, CDNA4) kernels of the BayesBridge stable Gibbs sweep.
//
// Reference call sites replaced (Code/C/...):
//   retstable.cpp:94-271 / BridgeRegression.cpp:506-510   -> k_retstable_batch, k_lambda
//   BridgeRegression.cpp:436-465 (sig2, tau)               -> k_pre, k_scalars
//   BridgeRegression.cpp:552-575 (beta, p x p Cholesky)    -> k_form_a, chol_*, k_chol_rhs,
//                                                             k_beta_chol
//   beta | rest for p > n (Woodbury form of the same law)  -> k_gram, k_xv, k_slab_sum,
//                                                             k_form_m, chol_*, k_beta_wb
//   BridgeRegression.cpp:514-521 (ortho)                   -> k_beta_ortho
//   BridgeRegression.cpp:469-503 (alpha MH)                -> k_alpha_mh
//   BridgeRegression.cpp:24-25 (X'X, X'y setup)            -> k_transpose + k_gram, k_coldot
//
// Layout: X is column-major n_pad x p_pad (n_pad multiple of 128, zero padded rows and
// columns).  Symmetric matrices keep their UPPER triangle in column-major storage, the
// reference's chol(U, VInv, 'U') convention (A = U'U).
#include <hip/hip_runtime.h>

#include <atomic>

#include <mutex>
#include <stdexcept>
#include <unordered_map>

#include <algorithm>
#include <cstring>

#include "bb_kernels.h"
#include "bb_pg.h"
#include "bb_sampler.h"

namespace bb {

typedef double v4d __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// reductions (deterministic: fixed tree per launch geometry)
// ---------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    return v;  // lane 0
}

__device__ __forceinline__ double wave_allsum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <int NT>
__device__ __forceinline__ double block_sum(double v, double *sh) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) sh[w] = v;
    __syncthreads();
    double r = 0.0;
    if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 0; i < NT / 64; ++i) r += sh[i];
    }
    __syncthreads();
    return r;  // thread 0
}

// ---------------------------------------------------------------------------
// tilted stable draws
// ---------------------------------------------------------------------------
// Lanes per coefficient (inner-attempt speculation).  Measured on MI355X with the C3
// h-distribution (tools/bench_lambda.py): p=50000 best at G=4..8, p=6250 at G=16;
// tiny p (C1) wants the widest group for latency.
// Large batches are throughput-bound: the sampler in non-inlined calls (111 VGPRs, 4 waves
// per SIMD) with G = 8 beats the inlined one (248 VGPRs, 1 wave per SIMD); small batches are
// bound by the slowest draw, where the inlined body wins (tools/bench_lambda_steady.py:
// p = 50000 187 vs 226 us, 25000 129 vs 142 us, 12500 98 vs 98 us, 6250 88 vs 67 us).
bool stable_noinline_for(long count) { return count >= 20000; }

int stable_group_for(long count) {
    if (stable_noinline_for(count)) return 8;
    if (count <= 1024) return 64;
    long g = 1;
    // measured at a steady-state C3 chain (tools/bench_lambda_steady.py): p = 50000 -> 4,
    // p = 6250 (8-way shard) -> 8
    while (g < 16 && count * g * 2 <= 50000) g *= 2;
    return (int)(g < 4 ? 4 : g);
}

template <int G>
__global__ __launch_bounds__(256) void k_retstable_batch(double *x, const double *alpha,
                                                         const double *V0, const double *h,
                                                         int num, Key key, uint64_t t,
                                                         uint32_t *err) {
    const long gid = (long)blockIdx.x * 256 + threadIdx.x;
    const long i = gid / G;
    const bool active = i < num;
    const double hh = active ? h[i] : 0.0;
    const double aa = active ? alpha[i] : 0.5;
    const double vv = active ? V0[i] : 1.0;
    double r = stable_group_draw<G>(active, hh, aa, vv, key, t, (uint64_t)i, err);
    if (active && (threadIdx.x & (G - 1)) == 0) x[i] = r;
}

void launch_retstable_batch(hipStream_t s, double *x, const double *alpha, const double *V0,
                            const double *h, int num, uint64_t k0, uint64_t k1, uint64_t t,
                            int group, uint32_t *err) {
    if (num <= 0) return;
    Key key{k0, k1};
    long threads = (long)num * group;
    int blocks = (int)((threads + 255) / 256);
    switch (group) {
#define BB_CASE(G)                                                                           \
    case G:                                                                                  \
        k_retstable_batch<G><<<blocks, 256, 0, s>>>(x, alpha, V0, h, num, key, t, err);     \
        break;
        BB_CASE(1) BB_CASE(2) BB_CASE(4) BB_CASE(8) BB_CASE(16) BB_CASE(32) BB_CASE(64)
#undef BB_CASE
        default:
            k_retstable_batch<1><<<(num + 255) / 256, 256, 0, s>>>(x, alpha, V0, h, num, key, t,
                                                                   err);
    }
}

// lambda_j = 2 retstable(beta_j^2 / tau^2, alpha / 2, 1)   (BridgeRegression.cpp:506-510);
// Woodbury mode also forms D_j = tau^2 / lambda_j and u_j = sqrt(D_j) z_j.
template <int G, bool NI = (BB_STABLE_NOINLINE != 0)>
__global__ __launch_bounds__(256) void k_lambda(const double *beta, int p_loc, int p_pad,
                                                uint64_t j0, const DevScalars *sc, Key key,
                                                uint64_t t, int mode, double *lam, double *D,
                                                double *u, double *lam_trace, uint32_t *err) {
    const long gid = (long)blockIdx.x * 256 + threadIdx.x;
    const long i = gid / G;
    const bool active = i < p_loc;
    const double tau = sc->tau;
    const double alpha = sc->alpha;
    const double b = active ? beta[i] : 0.0;
    const double h = b * b / (tau * tau);
    double x = stable_group_draw<G, NI, true>(active, h, 0.5 * alpha, 1.0, key, t, j0 + (uint64_t)i,
                                        err);
    if ((threadIdx.x & (G - 1)) == 0 && i < p_pad) {
        if (active) {
            const double l = 2 * x;
            lam[i] = l;
            if (lam_trace) lam_trace[i] = l;
            if (mode == LAMBDA_WOODBURY) {
                const double d = (tau * tau) / l;
                D[i] = d;
                u[i] = sqrt(d) * normal_at(key, t, KIND_BETA_Z, j0 + (uint64_t)i);
            }
        } else {
            lam[i] = 1.0;
            if (mode == LAMBDA_WOODBURY) {
                D[i] = 0.0;
                u[i] = 0.0;
            }
        }
    }
}

// p_loc <= kLamSpecMax: L lanes per coefficient with outer-attempt speculation
// (stable_spec_draw<L, 8>: L/8 outer attempts of 8 inner attempts per round, the sequential
// loop's draw) instead of inner-only speculation (k_lambda: G lanes on G inner attempts of
// one outer attempt).  A launch is as long as its slowest draw, and the outer segments cut
// the slowest draw's rounds.  Measured lambda phase (bench, alpha = 0.5):
//   p = 1000 (C4):   L = 64  40 us, L = 32 43, L = 16 47, k_lambda G = 64 49 us;
//   p = 5000 (C2):   L = 16  58 us, L = 32 60, L = 64 75, k_lambda G = 8 74 us;
//   p = 6250 / 12500 / 25000 / 50000:  L = 16  58 / 76 / 111 / 202 us against
//                    k_lambda(_cb) 76 / 101 / 141 / 216 us;
//   p = 200000 (C5, alpha = 0.3):      L = 16 0.61 ms against k_lambda_cb 0.42 ms.
constexpr int kLamSpecWide = 1024;  // L = 64 up to here, L = 16 above
// ... and L = 8 above kLamSpecNarrow (round 3, tools/lambda_lanes_ab.py, two alternations from
// a steady state: C3 p = 50000 L = 8 0.192-0.197 ms, 16 0.205-0.206, 32 0.298-0.300; C2
// p = 5000 L = 8 0.074-0.079, 16 0.056-0.058, 32 0.057)
constexpr int kLamSpecNarrow = 40000;
constexpr int kLamSpecMax = 50000;

// PgTail: the logistic sweep's omega ~ PG(1, psi) draws (independent of lambda: psi = X beta
// is known before tau) ride in the same launch as trailing workgroups -- 10 000 draws are
// only 157 waves, which alone leave most of the chip idle for the draw's latency.
struct PgTail {
    const double *psi = nullptr;
    int n = 0, n_pad = 0;
    double *omega = nullptr;
};

template <int L, int I>
__device__ __forceinline__ void lambda_spec_body(const double *beta, int p_loc, int p_pad,
                                                 uint64_t j0, const DevScalars *sc, Key key,
                                                 uint64_t t, int mode, double *lam, double *D,
                                                 double *u, double *lam_trace, uint32_t *err,
                                                 int lam_blocks, const PgTail &pgt) {
    if ((int)blockIdx.x >= lam_blocks) {
        pg_draw_at(((int)blockIdx.x - lam_blocks) * 256 + (int)threadIdx.x, pgt.psi, pgt.n,
                   pgt.n_pad, key, t, pgt.omega, err);
        return;
    }
    const int i = blockIdx.x * (256 / L) + (threadIdx.x / L);  // group-uniform
    const bool active = i < p_loc;
    const double tau = sc->tau;
    const double b = active ? beta[i] : 0.0;
    const double x = stable_spec_draw<L, I>(active, b * b / (tau * tau), 0.5 * sc->alpha, 1.0,
                                            key, t, j0 + (uint64_t)i, err);
    if ((threadIdx.x % L) != 0 || i >= p_pad) return;
    if (active) {
        const double l = 2 * x;
        lam[i] = l;
        if (lam_trace) lam_trace[i] = l;
        if (mode == LAMBDA_WOODBURY) {
            const double d = (tau * tau) / l;
            D[i] = d;
            u[i] = sqrt(d) * normal_at(key, t, KIND_BETA_Z, j0 + (uint64_t)i);
        }
    } else {
        lam[i] = 1.0;
        if (mode == LAMBDA_WOODBURY) {
            D[i] = 0.0;
            u[i] = 0.0;
        }
    }
}

// The sampler needs 157 VGPRs inlined (3 waves per SIMD); the O4 instance is capped at 128
// (4 waves per SIMD, a few spills to scratch) -- bb_set_tuning key 4 selects it for A/B.
#define BB_LAMBDA_SPEC_ARGS                                                                  \
    const double *beta, int p_loc, int p_pad, uint64_t j0, const DevScalars *sc, Key key,    \
        uint64_t t, int mode, double *lam, double *D, double *u, double *lam_trace,          \
        uint32_t *err, int lam_blocks, PgTail pgt
template <int L, int I = 8>
__global__ __launch_bounds__(256) void k_lambda_spec(BB_LAMBDA_SPEC_ARGS) {
    lambda_spec_body<L, I>(beta, p_loc, p_pad, j0, sc, key, t, mode, lam, D, u, lam_trace, err,
                        lam_blocks, pgt);
}
template <int L, int I = 8>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) void
k_lambda_spec_o4(BB_LAMBDA_SPEC_ARGS) {
    lambda_spec_body<L, I>(beta, p_loc, p_pad, j0, sc, key, t, mode, lam, D, u, lam_trace, err,
                        lam_blocks, pgt);
}
#undef BB_LAMBDA_SPEC_ARGS
// bb_set_tuning key 4: bit 0 = k_lambda_spec at 4 waves per SIMD, bit 1 = k_lambda_cb at 4,
// bit 2 = k_lambda_cb with the sampler bodies inlined (3 waves; overrides bit 1).  Measured
// (round 3, tools/lambda_occ_ab.py, three alternations): C3 k_lambda_spec<16> 0.200-0.208 ms
// at either occupancy; C5 k_lambda_cb<8> 0.418-0.428 -> 0.402-0.407 ms at 4 waves; round 4
// (gpurun_out/r04k_*, two alternations at the driver's settings): C5 inlined 1933-1939
// sweeps/s against 1824-1831 out of line at 4 waves (lambda 0.334-0.341 against 0.351-0.356
// ms); the fused k_lambda_xu and k_lambda_spec at 4 waves (bit 0, 128 VGPRs with 92-124 B of
// spills) are slower: C3 1791-1794 against 1944-1948 sweeps/s, C2 6097-6114 against 6312-6423
// (gpurun_out/r04n_*).  Bit 3: the inlined continuous-batching launch also for
// 40000 < p <= 50000 (the separate launch of C3's fitted-regime sweeps): lambda 0.157-0.161
// against 0.169-0.174 ms for k_lambda_spec<8> (gpurun_out/r04s_*).  Default 12.
int g_lam_occ = 12;

// Large batches (p_loc >= 20000): continuous batching.  A launch of stable_group_draw is
// as long as its slowest wave, and a wave is as long as the slowest of its G-lane groups'
// draws; here each workgroup owns a contiguous range of coefficients and a group that has
// finished its draw takes the next coefficient of the range from an LDS counter, so lanes
// stay busy until the range is exhausted and only the last draws of a range form the
// tail.  Every draw runs the sequential loop of stable_group_draw on its own counters, so
// the values are the same.  Measured (bench phases): C5 (200 000 draws) 0.54 -> 0.44 ms, C3
// (50 000) unchanged at 0.21 ms; one lane per draw (no redundant outer tests, but divergent
// inner/outer paths) 0.54 / 0.84 ms and four lanes 0.27 / 0.42 ms, so eight lanes stay.
constexpr int kLamCbWG = 256;  // threads per workgroup (4 waves)

static int device_cus_lam() {
    static int n = [] {
        int dev = 0, v = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            v <= 0)
            v = 256;
        return v;
    }();
    return n;
}

// chunk: the workgroup's range is [chunk per_wg, chunk per_wg + per_wg); us (LDS, or null):
// u_j of the range, for the fused X u pass (k_lambda_xu); NI: the sampler bodies out of line
template <int G, bool NI = true, bool LEND = false>
__device__ __forceinline__ void lambda_cb_body(const double *beta, int p_loc, int p_pad,
                                               int per_wg, uint64_t j0, const DevScalars *sc,
                                               Key key, uint64_t t, int mode, double *lam,
                                               double *D, double *u, double *lam_trace,
                                               uint32_t *err, int &s_next, int chunk,
                                               double *us = nullptr) {
    const int lane = threadIdx.x & 63;
    const int g = lane & (G - 1), gbase = lane & ~(G - 1);
    const uint64_t gmask = (G == 64) ? ~0ull : ((1ull << (G & 63)) - 1ull);
    const int jbeg = chunk * per_wg;
    const int jend = min(p_pad, jbeg + per_wg);
    if (threadIdx.x == 0) s_next = jbeg + kLamCbWG / G;
    __syncthreads();
    const double tau = sc->tau;
    const double alpha = sc->alpha;
    const double a2 = 0.5 * alpha;
    StableParams sp;
    int j = jbeg + (int)threadIdx.x / G;
    bool have = j < jend;  // this group holds coefficient j
    bool draw = false;     // ... and it needs the rejection sampler
    uint64_t o = 0, ib = 0;
    auto start = [&]() {
        o = 0;
        ib = 0;
        draw = j < p_loc && a2 != 1.0;  // retstable.cpp:104-110: alpha = 1 returns V0
        if (draw) {
            const double b = beta[j];
            const double h = b * b / (tau * tau);
            if (h < 0 || a2 < 0 || a2 > 1) atomicOr(err, 4u);  // :112-115
            sp = stable_params<true>(h, a2, 1.0);
        }
    };
    auto finish = [&](double x) {  // x: the tilted-stable draw of coefficient j
        if (g == 0) {
            double uv = 0.0;
            if (j < p_loc) {
                const double l = 2 * x;
                lam[j] = l;
                if (lam_trace) lam_trace[j] = l;
                if (mode == LAMBDA_WOODBURY) {
                    const double d = (tau * tau) / l;
                    D[j] = d;
                    uv = sqrt(d) * normal_at(key, t, KIND_BETA_Z, j0 + (uint64_t)j);
                    u[j] = uv;
                }
            } else {
                lam[j] = 1.0;
                if (mode == LAMBDA_WOODBURY) {
                    D[j] = 0.0;
                    u[j] = 0.0;
                }
            }
            if (us) us[j - jbeg] = uv;
        }
    };
    if (have) start();
    for (long iter = 0; iter < (1l << 26); ++iter) {
        bool acc = false;
        double U = 0.0, z = 0.0, Z = 0.0, B = 1.0;
        if (have && draw)
            acc = stable_inner<NI>(sp, key, t, j0 + (uint64_t)j, o, ib + (uint64_t)g, U, z, Z, B);
        const uint64_t m = (__ballot(acc) >> gbase) & gmask;
        const int win = m ? (__ffsll((unsigned long long)m) - 1) : 0;
        const double Uw = __shfl(U, gbase + win, 64);
        const double zw = __shfl(z, gbase + win, 64);
        const double Zw = __shfl(Z, gbase + win, 64);
        const double Bw = __shfl(B, gbase + win, 64);
        bool fin = false;
        if (have) {
            if (!draw) {
                finish(1.0);  // V0
                fin = true;
            } else if (!m) {
                ib += G;
            } else {
                double X;
                if (stable_outer<NI>(sp, key, t, j0 + (uint64_t)j, o, Uw, zw, Zw, Bw, X)) {
                    finish(stable_finish(sp, X));
                    fin = true;
                } else {
                    ++o;
                    ib = 0;
                }
            }
        }
        if (fin) {
            int jn = 0;
            if (g == 0) jn = atomicAdd(&s_next, 1);
            jn = __shfl(jn, gbase, 64);
            j = jn;
            have = j < jend;
            if (have) start();
        }
        if (__all(!have)) break;
        if constexpr (LEND) {
            // A group without a coefficient means the range is used up: the wave's remaining
            // draws continue from their state with the idle groups' lanes dealt to them
            // (wave_draw_rounds, as the fused launch's stable_wave_draw) -- the same attempts
            // in the same order, so the same draws.
            static_assert(G == 8 && !NI, "lending deals 8-lane home groups, sampler inlined");
            if (__any(!have)) {
                if (have && !draw) {
                    finish(1.0);  // V0
                    have = false;
                }
                // the wave-uniform constants must be valid on every lane that may serve
                if (!have) sp = stable_params<true>(1.0, a2, 1.0);
                unsigned um = 0;
                const unsigned long long hb = __ballot(have && g == 0);
#pragma unroll
                for (int c = 0; c < 8; ++c) um |= (unsigned)((hb >> (8 * c)) & 1ull) << c;
                uint64_t o0 = o, ibv = ib, jc = j0 + (uint64_t)j;
                double res = 0.0;
                const unsigned left = wave_draw_rounds(sp, o0, ibv, jc, um, res, key, t);
                if (have) {
                    if ((left >> (lane >> 3)) & 1u) atomicOr(err, 2u);
                    else finish(res);
                }
                have = false;
                break;
            }
        }
    }
    if (have) atomicOr(err, 2u);  // bounded: a draw that never finished is flagged
}

#define BB_LAMBDA_CB_ARGS                                                                    \
    const double *beta, int p_loc, int p_pad, int per_wg, uint64_t j0, const DevScalars *sc, \
        Key key, uint64_t t, int mode, double *lam, double *D, double *u, double *lam_trace,  \
        uint32_t *err
template <int G>
__global__ __launch_bounds__(kLamCbWG) void k_lambda_cb(BB_LAMBDA_CB_ARGS) {
    __shared__ int s_next;
    lambda_cb_body<G>(beta, p_loc, p_pad, per_wg, j0, sc, key, t, mode, lam, D, u, lam_trace,
                      err, s_next, blockIdx.x);
}
template <int G>
__global__ __launch_bounds__(kLamCbWG) __attribute__((amdgpu_waves_per_eu(4, 8))) void
k_lambda_cb_o4(BB_LAMBDA_CB_ARGS) {
    __shared__ int s_next;
    lambda_cb_body<G>(beta, p_loc, p_pad, per_wg, j0, sc, key, t, mode, lam, D, u, lam_trace,
                      err, s_next, blockIdx.x);
}
// the sampler bodies inlined (bb_set_tuning key 4 bit 2; 3 waves per SIMD)
template <int G>
__global__ __launch_bounds__(kLamCbWG) void k_lambda_cb_in(BB_LAMBDA_CB_ARGS) {
    __shared__ int s_next;
    lambda_cb_body<G, false>(beta, p_loc, p_pad, per_wg, j0, sc, key, t, mode, lam, D, u,
                             lam_trace, err, s_next, blockIdx.x);
}
// ... and the tail's lanes lent to the unfinished draws (bb_set_tuning key 15)
template <int G>
__global__ __launch_bounds__(kLamCbWG) __attribute__((amdgpu_waves_per_eu(3, 8))) void
k_lambda_cl(BB_LAMBDA_CB_ARGS) {
    __shared__ int s_next;
    lambda_cb_body<G, false, true>(beta, p_loc, p_pad, per_wg, j0, sc, key, t, mode, lam, D, u,
                                   lam_trace, err, s_next, blockIdx.x);
}
int g_lam_lend = 1;
#undef BB_LAMBDA_CB_ARGS

// One speculative lambda launch with L lanes per coefficient (the draws do not depend on L);
// pgb trailing workgroups draw the logistic omegas.  g_lam_lanes (bb_set_tuning key 5)
// overrides the default L for A/B measurements.
int g_lam_lanes = 0;
static int spec_lanes(int p_loc) {
    return p_loc <= kLamSpecWide ? 64 : p_loc <= kLamSpecNarrow ? 16 : 8;
}
static void launch_spec(hipStream_t s, int L, int pgb, const double *beta, int p_loc, int p_pad,
                        uint64_t j0, const DevScalars *sc, Key key, uint64_t t, int mode,
                        double *lam, double *D, double *u, double *lam_trace, uint32_t *err,
                        const PgTail &pgt) {
    if (g_lam_lanes) L = g_lam_lanes;
    const int per = 256 / L;
    const int lb = (p_pad + per - 1) / per;
    const bool o4 = (g_lam_occ & 1) != 0;
    switch (L) {
#define BB_SPEC_CASE(LL)                                                                      \
    case LL:                                                                                  \
        note_launch(KF_LAMBDA, (const void *)(o4 ? k_lambda_spec_o4<LL> : k_lambda_spec<LL>)); \
        (o4 ? k_lambda_spec_o4<LL> : k_lambda_spec<LL>)<<<lb + pgb, 256, 0, s>>>(             \
            beta, p_loc, p_pad, j0, sc, key, t, mode, lam, D, u, lam_trace, err, lb, pgt);    \
        break;
        case 4:  // one outer attempt of 4 inner attempts per round (A/B only)
            (o4 ? k_lambda_spec_o4<4, 4> : k_lambda_spec<4, 4>)<<<lb + pgb, 256, 0, s>>>(
                beta, p_loc, p_pad, j0, sc, key, t, mode, lam, D, u, lam_trace, err, lb, pgt);
            break;
        BB_SPEC_CASE(8)
        BB_SPEC_CASE(32)
        BB_SPEC_CASE(64)
        default: BB_SPEC_CASE(16)
#undef BB_SPEC_CASE
    }
}

// lambda fused with the X u pass of the near-identity solve (dense Woodbury, DESIGN.md
// s6.5): the draws are VALU-bound and X u is HBM-bound, and u_j is known as soon as the
// draw of column j is, so a workgroup draws the C = 256 / L coefficients of a column chunk,
// then streams those C columns of X into its X u partial (rows t + 256 m of the chunk held
// by thread t, accumulated in LDS across chunks), while the other workgroups on the CU are
// drawing.  Chunks g, g + G, ... per workgroup (G <= 3 per CU, the sampler's occupancy);
// each workgroup writes one partial n-vector, summed in workgroup order by k_cheb_init, so
// the result is bitwise reproducible.  The draws are those of k_lambda_spec<L>.
// bb_set_tuning key 7: 0 = separate lambda and X u launches; 1, 2: below.  Measured at the
// driver's settings (round 4, gpurun_out/r04i_*): C3 mode 2 1899 / 1902 sweeps/s against mode 1
// 1871 / 1871 (the lambda phase 0.202 against 0.220 ms); C2 6109 / 5931 against 6088 / 6023.
// (A batched mode -- chunks of two coefficients per lane group drawn by lambda_cb_body with
// continuous batching -- measured slower, C3 1895 against 1937-1948, C2 5532-5557 against
// 6322-6372, gpurun_out/r04k_*, and was removed.)
int g_lam_xu = 3;
// bb_set_tuning key 13: the fused launch at 8 lanes per coefficient draws with the
// wave-adaptive sampler (stable_wave_draw; 1) or with fixed 8-lane groups (0); the same draws
int g_lam_wave = 1;
template <int L, int NR, bool WAVE = false>
__device__ __forceinline__ void lambda_xu_body(const double *beta, int p_loc, int p_pad,
                                                   uint64_t j0, const DevScalars *sc, Key key,
                                                   uint64_t t, double *lam, double *D,
                                                   double *u, double *lam_trace, uint32_t *err,
                                                   const double *__restrict__ X, int ldx,
                                                   int n_pad, int nchunk,
                                                   double *__restrict__ xu_part) {
    constexpr int C = 256 / L;
    constexpr int CQ = NR >= 16 ? 1 : 16 / NR;  // columns in flight: 16 loads per thread
    __shared__ double us[C];
    __shared__ double accs[NR * 256];
    const int tid = threadIdx.x;
#pragma unroll
    for (int m = 0; m < NR; ++m) accs[m * 256 + tid] = 0.0;
    const double tau = sc->tau;
    for (int ch = blockIdx.x; ch < nchunk; ch += gridDim.x) {
        const int i = ch * C + tid / L;  // group-uniform
        const bool active = i < p_loc;
        const double b = active ? beta[i] : 0.0;
        double x;
        if constexpr (WAVE) {
            static_assert(L == 8, "the wave-adaptive draw deals 8-lane home groups");
            x = stable_wave_draw(active, b * b / (tau * tau), 0.5 * sc->alpha, 1.0, key, t,
                                 j0 + (uint64_t)i, err);
        } else {
            x = stable_spec_draw<L, 8>(active, b * b / (tau * tau), 0.5 * sc->alpha, 1.0, key, t,
                                       j0 + (uint64_t)i, err);
        }
        if ((tid % L) == 0) {
            double uv = 0.0;
            if (active) {
                const double l = 2 * x;
                lam[i] = l;
                if (lam_trace) lam_trace[i] = l;
                const double d = (tau * tau) / l;
                D[i] = d;
                uv = sqrt(d) * normal_at(key, t, KIND_BETA_Z, j0 + (uint64_t)i);
                u[i] = uv;
            } else if (i < p_pad) {
                lam[i] = 1.0;
                D[i] = 0.0;
                u[i] = 0.0;
            }
            us[tid / L] = uv;
        }
        __syncthreads();  // the chunk's u
        double a[NR];
#pragma unroll
        for (int m = 0; m < NR; ++m) a[m] = accs[m * 256 + tid];
#pragma unroll 1
        for (int c = 0; c < C; c += CQ) {
            double xv[CQ][NR];
#pragma unroll
            for (int q = 0; q < CQ; ++q) {
                const int col = ch * C + c + q;
                const bool ok = col < p_loc;
                const double *xc = X + (size_t)col * ldx;
#pragma unroll
                for (int m = 0; m < NR; ++m) {
                    const int row = tid + 256 * m;
                    xv[q][m] = (ok && row < n_pad) ? __builtin_nontemporal_load(xc + row) : 0.0;
                }
            }
#pragma unroll
            for (int q = 0; q < CQ; ++q) {
                const double f = us[c + q];
#pragma unroll
                for (int m = 0; m < NR; ++m) a[m] = __builtin_fma(xv[q][m], f, a[m]);
            }
        }
#pragma unroll
        for (int m = 0; m < NR; ++m) accs[m * 256 + tid] = a[m];
        __syncthreads();  // us is rewritten by the next chunk
    }
#pragma unroll
    for (int m = 0; m < NR; ++m) {
        const int row = tid + 256 * m;
        if (row < n_pad) xu_part[(size_t)blockIdx.x * n_pad + row] = accs[m * 256 + tid];
    }
}

// partial n-vectors of the fused launch for this shape, 0 if the shape does not take it
#define BB_LXU_ARGS                                                                          \
    const double *beta, int p_loc, int p_pad, uint64_t j0, const DevScalars *sc, Key key,    \
        uint64_t t, double *lam, double *D, double *u, double *lam_trace, uint32_t *err,     \
        const double *__restrict__ X, int ldx, int n_pad, int nchunk, double *__restrict__ xu_part
template <int L, int NR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 8))) void
k_lambda_xu(BB_LXU_ARGS) {
    lambda_xu_body<L, NR>(beta, p_loc, p_pad, j0, sc, key, t, lam, D, u, lam_trace, err, X, ldx,
                          n_pad, nchunk, xu_part);
}
// capped at 128 VGPRs for 4 waves per SIMD (bb_set_tuning key 4 bit 0, as k_lambda_spec_o4)
template <int L, int NR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) void
k_lambda_xu_o4(BB_LXU_ARGS) {
    lambda_xu_body<L, NR>(beta, p_loc, p_pad, j0, sc, key, t, lam, D, u, lam_trace, err, X, ldx,
                          n_pad, nchunk, xu_part);
}
// the wave-adaptive draw (stable_wave_draw, 8 lanes per coefficient): bb_set_tuning key 13
template <int NR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 8))) void
k_lambda_xw(BB_LXU_ARGS) {
    lambda_xu_body<8, NR, true>(beta, p_loc, p_pad, j0, sc, key, t, lam, D, u, lam_trace, err, X,
                                ldx, n_pad, nchunk, xu_part);
}

#undef BB_LXU_ARGS

// (mode 1: G = min(chunks, 3 per CU), each workgroup loops over its chunks; mode 2: one
// chunk per workgroup, the hardware scheduling them -- more partials, no static tail, and the
// workgroups' draw and stream phases drift apart; bb_set_tuning key 7 picks the mode)
static int lambda_xu_groups(int p_loc, int p_pad, int n_pad, int mode) {
    if (!mode || p_loc > kLamSpecMax || n_pad > 4096) return 0;
    const int L = spec_lanes(p_loc);
    if (L != 8 && L != 16) return 0;
    const int nchunk = (p_pad + 256 / L - 1) / (256 / L);
    if (mode == 3) return L == 8 ? std::min(nchunk, device_cus_lam()) : 0;  // stream workgroups
    return mode == 1 ? std::min(nchunk, 3 * device_cus_lam()) : nchunk;
}
int lambda_xu_parts(int p_loc, int p_pad, int n_pad) {
    return lambda_xu_groups(p_loc, p_pad, n_pad, 2);  // the most any mode writes
}

int launch_lambda_xu(hipStream_t s, const double *beta, int p_loc, int p_pad, uint64_t j0,
                     const DevScalars *sc, uint64_t k0, uint64_t k1, uint64_t t, double *lam,
                     double *D, double *u, double *lam_trace, uint32_t *err, const double *X,
                     int ldx, int n_pad, double *xu_part, unsigned int *sync, unsigned int ep,
                     const NidFold *fold, int *folded) {
    const int nr = (n_pad + 255) / 256;
    int mode = g_lam_xu;
    if (mode == 3 && (!sync || !g_lam_wave || (g_lam_occ & 1) || lambda_xs_resident(nr) < 3))
        mode = 2;
    if (folded) *folded = 0;
    int G = g_lam_lanes ? 0 : lambda_xu_groups(p_loc, p_pad, n_pad, mode);
    if (!G && mode == 3) {
        // the split launch takes 8 lanes per coefficient only: 16-lane shapes (p_loc <= 40000,
        // e.g. a C3 rank at N = 8) fall back to one chunk per workgroup (mode 2)
        mode = 2;
        G = g_lam_lanes ? 0 : lambda_xu_groups(p_loc, p_pad, n_pad, mode);
    }
    const Key key{k0, k1};
    const int L = spec_lanes(p_loc);
    const int nchunk = (p_pad + 256 / L - 1) / (256 / L);
    const bool o4 = (g_lam_occ & 1) != 0;
    if (mode == 3 && G) {
        const int f = launch_lambda_xs(s, beta, p_loc, p_pad, j0, sc, k0, k1, t, lam, D, u,
                                       lam_trace, err, X, ldx, n_pad, nchunk, xu_part, sync, ep,
                                       2 * G, G, fold);
        if (folded) *folded = f;
        return G;
    }
    if (!G) return 0;
#define BB_LXU(LL, NN)                                                                        \
    do {                                                                                      \
        auto *kk = o4 ? k_lambda_xu_o4<LL, NN> : k_lambda_xu<LL, NN>;                         \
        note_launch(KF_LAMBDA, (const void *)kk);                                             \
        kk<<<G, 256, 0, s>>>(beta, p_loc, p_pad, j0, sc, key, t, lam, D, u, lam_trace, err, X, \
                             ldx, n_pad, nchunk, xu_part);                                    \
    } while (0)
    if (L == 8 && g_lam_wave && !o4) {
        auto *kk = nr <= 4 ? k_lambda_xw<4> : nr <= 8 ? k_lambda_xw<8> : k_lambda_xw<16>;
        note_launch(KF_LAMBDA, (const void *)kk);
        kk<<<G, 256, 0, s>>>(beta, p_loc, p_pad, j0, sc, key, t, lam, D, u, lam_trace, err, X, ldx,
                             n_pad, nchunk, xu_part);
    } else if (L == 8) {
        if (nr <= 4) BB_LXU(8, 4); else if (nr <= 8) BB_LXU(8, 8); else BB_LXU(8, 16);
    } else {
        if (nr <= 4) BB_LXU(16, 4); else if (nr <= 8) BB_LXU(16, 8); else BB_LXU(16, 16);
    }
#undef BB_LXU
    return G;
}

bool launch_lambda_pg(hipStream_t s, const double *beta, int p_loc, int p_pad, uint64_t j0,
                      const DevScalars *sc, uint64_t k0, uint64_t k1, uint64_t t, int group,
                      double *lam, double *lam_trace, const double *psi, int n, int n_pad,
                      double *omega, uint32_t *err) {
    if (p_loc > kLamSpecMax) return false;  // the caller launches k_pg itself
    const Key key{k0, k1};
    const PgTail pgt{psi, n, n_pad, omega};
    const int pgb = (n_pad + 255) / 256;
    (void)group;
    launch_spec(s, spec_lanes(p_loc), pgb, beta, p_loc, p_pad, j0, sc, key, t,
                LAMBDA_ONLY, lam, nullptr, nullptr, lam_trace, err, pgt);
    return true;
}

void launch_lambda(hipStream_t s, const double *beta, int p_loc, int p_pad, uint64_t j0,
                   const DevScalars *sc, uint64_t k0, uint64_t k1, uint64_t t, int mode,
                   int group, double *lam, double *D, double *u, double *lam_trace,
                   uint32_t *err) {
    Key key{k0, k1};
    long threads = (long)p_pad * group;
    int blocks = (int)((threads + 255) / 256);
    const bool ni = stable_noinline_for(p_loc);
    // bb_set_tuning key 4 bit 3 (default on): the continuous-batching launch also for p in
    // (kLamSpecNarrow, kLamSpecMax]; a lane count forced through key 5 takes the speculative
    // launch
    const bool force_cb = (g_lam_occ & 8) && p_loc > kLamSpecNarrow && !g_lam_lanes;
    if (p_loc <= kLamSpecMax && !force_cb) {
        launch_spec(s, spec_lanes(p_loc), 0, beta, p_loc, p_pad, j0, sc, key, t,
                    mode, lam, D, u, lam_trace, err, PgTail{});
        return;
    }
    if ((ni && group == 8) || force_cb) {
        // 4 workgroups of 4 waves per CU (the out-of-line sampler's occupancy; 3 inlined)
        const bool inl = (g_lam_occ & 4) != 0;
        const int nwg = std::max(1, std::min((inl ? 3 : 4) * device_cus_lam(), (p_pad + 31) / 32));
        const int per = (p_pad + nwg - 1) / nwg;
        auto *kern = inl ? (g_lam_lend ? k_lambda_cl<8> : k_lambda_cb_in<8>)
                         : (g_lam_occ & 2) ? k_lambda_cb_o4<8> : k_lambda_cb<8>;
        note_launch(KF_LAMBDA, (const void *)kern);
        kern<<<(p_pad + per - 1) / per, kLamCbWG, 0, s>>>(beta, p_loc, p_pad, per, j0, sc, key,
                                                          t, mode, lam, D, u, lam_trace, err);
        return;
    }
    switch (group) {
#define BB_CASE(G)                                                                            \
    case G:                                                                                   \
        if (ni)                                                                               \
            k_lambda<G, true><<<blocks, 256, 0, s>>>(beta, p_loc, p_pad, j0, sc, key, t, mode, \
                                                     lam, D, u, lam_trace, err);              \
        else                                                                                  \
            k_lambda<G, false><<<blocks, 256, 0, s>>>(beta, p_loc, p_pad, j0, sc, key, t,      \
                                                      mode, lam, D, u, lam_trace, err);       \
        break;
        BB_CASE(1) BB_CASE(2) BB_CASE(4) BB_CASE(8) BB_CASE(16) BB_CASE(32) BB_CASE(64)
#undef BB_CASE
        default:
            k_lambda<1><<<(p_pad + 255) / 256, 256, 0, s>>>(beta, p_loc, p_pad, j0, sc, key, t,
                                                            mode, lam, D, u, lam_trace, err);
    }
}

// Microbenchmark: launch k_lambda with an explicit group size and inlining variant.
void launch_lambda_variant(hipStream_t s, const double *beta, int p, const DevScalars *sc,
                           uint64_t k0, uint64_t k1, uint64_t t, int group, int noinline,
                           double *lam, uint32_t *err) {
    Key key{k0, k1};
    long threads = (long)p * group;
    int blocks = (int)((threads + 255) / 256);
#define BB_V(G)                                                                               \
    case G:                                                                                   \
        if (noinline == 1)                                                                    \
            k_lambda<G, true><<<blocks, 256, 0, s>>>(beta, p, p, 0, sc, key, t, LAMBDA_ONLY,   \
                                                     lam, nullptr, nullptr, nullptr, err);    \
        else                                                                                  \
            k_lambda<G, false><<<blocks, 256, 0, s>>>(beta, p, p, 0, sc, key, t, LAMBDA_ONLY,  \
                                                      lam, nullptr, nullptr, nullptr, err);   \
        break;
    switch (group) {
        BB_V(1) BB_V(2) BB_V(4) BB_V(8) BB_V(16) BB_V(32) BB_V(64)
        default:
            break;
    }
#undef BB_V
}

// ---------------------------------------------------------------------------
// Gram: slabs[s] = Y[:, Ks] diag(w[Ks]) Y[:, Ks]'  with v_mfma_f64_16x16x4_f64.
// Block = one 128x128 lower tile (I >= J) x one K split; 4 waves in 2x2, each wave
// 64x64 = 4x4 MFMA tiles.  Y tiles staged through LDS as [k][row] (row contiguous,
// ld 144 so that the two 16-lane halves of a ds_read_b64 group hit disjoint banks);
// w is applied while staging the B operand.  Output tile D[i][j] is stored transposed
// at (J*128+j, I*128+i) -> upper triangle of a column-major matrix, coalesced.
// Split s = blockIdx % S so that all blocks of one split share an XCD (and its L2).
// ---------------------------------------------------------------------------
constexpr int kGLD = 144;

__global__ __launch_bounds__(256, 2) void k_gram(const double *__restrict__ Y, int ldy,
                                                 const double *__restrict__ w, int K, int S,
                                                 double *__restrict__ out, int ldo,
                                                 size_t slab_stride, const int *gate) {
    if (gated(gate)) return;
    __shared__ double As[kGramBK * kGLD];
    __shared__ double Bs[kGramBK * kGLD];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int s = blockIdx.x % S;
    const int tile = blockIdx.x / S;
    int I = (int)((sqrt(8.0 * tile + 1.0) - 1.0) * 0.5);
    while ((I + 1) * (I + 2) / 2 <= tile) ++I;
    while (I * (I + 1) / 2 > tile) --I;
    const int J = tile - I * (I + 1) / 2;
    const int kchunk = K / S;
    const int kb = s * kchunk, ke = kb + kchunk;
    const double *Ya = Y + (size_t)I * kGramTile;
    const double *Yb = Y + (size_t)J * kGramTile;
    const int lr = (tid & 63) * 2;
    const int lk = tid >> 6;
    double2 ra[4], rb[4];
    double wk[4];
    v4d acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = (v4d){0.0, 0.0, 0.0, 0.0};
    const int wr = wid >> 1, wc = wid & 1;

    auto gload = [&](int k0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int k = k0 + lk + 4 * q;
            ra[q] = *(const double2 *)(Ya + lr + (size_t)k * ldy);
            rb[q] = *(const double2 *)(Yb + lr + (size_t)k * ldy);
            wk[q] = w[k];
        }
    };
    auto sstore = [&]() {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int kk = lk + 4 * q;
            *(double2 *)(As + kk * kGLD + lr) = ra[q];
            double2 b = rb[q];
            b.x *= wk[q];
            b.y *= wk[q];
            *(double2 *)(Bs + kk * kGLD + lr) = b;
        }
    };

    if (kb < ke) {
        gload(kb);
        sstore();
        __syncthreads();
        for (int k0 = kb; k0 < ke; k0 += kGramBK) {
            const bool more = (k0 + kGramBK) < ke;
            if (more) gload(k0 + kGramBK);
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                const int krow = kk * 4 + (lane >> 4);
                double a[4], b[4];
#pragma unroll
                for (int m = 0; m < 4; ++m) a[m] = As[krow * kGLD + wr * 64 + m * 16 + (lane & 15)];
#pragma unroll
                for (int m = 0; m < 4; ++m) b[m] = Bs[krow * kGLD + wc * 64 + m * 16 + (lane & 15)];
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int nj = 0; nj < 4; ++nj)
                        acc[mi][nj] =
                            __builtin_amdgcn_mfma_f64_16x16x4f64(a[mi], b[nj], acc[mi][nj], 0, 0, 0);
            }
            __syncthreads();
            if (more) {
                sstore();
                __syncthreads();
            }
        }
    }
    double *o = out + (size_t)s * slab_stride;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int nj = 0; nj < 4; ++nj)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = wr * 64 + mi * 16 + (lane >> 4) + 4 * r;
                const int j = wc * 64 + nj * 16 + (lane & 15);
                o[(size_t)(J * kGramTile + j) + (size_t)(I * kGramTile + i) * ldo] = acc[mi][nj][r];
            }
}

int gram_splits_for(int n_pad, int K) {
    const int nt = n_pad / kGramTile;
    const int tiles = nt * (nt + 1) / 2;
    int S = 1;
    // aim for >= 4 blocks per CU, keep >= 8 K-steps per split, K % (16 S) == 0
    while (S < 64 && tiles * S < 1024 && (K % (kGramBK * S * 2)) == 0 &&
           K / (S * 2) >= 8 * kGramBK)
        S *= 2;
    return S;
}

void launch_gram(hipStream_t s, const double *Y, int ldy, const double *w, int n_pad, int K,
                 int S, double *slabs, int ldo, size_t slab_stride, const int *gate) {
    const int nt = n_pad / kGramTile;
    const int tiles = nt * (nt + 1) / 2;
    note_launch(KF_GRAM, (const void *)k_gram);
    k_gram<<<tiles * S, 256, 0, s>>>(Y, ldy, w, K, S, slabs, ldo, slab_stride, gate);
}

// ---------------------------------------------------------------------------
// X.v partial sums: part[cb][r] = sum_{j in chunk cb} X[r, j] v[j] (column order).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_xv(const double *__restrict__ X, int ldx,
                                            const double *__restrict__ v, int ncols, int n_pad,
                                            int cols, double *__restrict__ part, const int *gate) {
    if (gated(gate)) return;
    __shared__ double vs[kXvCols];
    const int cb = blockIdx.x, rb = blockIdx.y;
    const int c0 = cb * cols;
    const int nc = min(cols, ncols - c0);
    for (int i = threadIdx.x; i < kXvCols; i += 256) vs[i] = (i < nc) ? v[c0 + i] : 0.0;
    __syncthreads();
    const int r = rb * kXvRows + 2 * threadIdx.x;
    if (r >= n_pad) return;
    const double *xp = X + (size_t)c0 * ldx + r;
    double ax = 0.0, ay = 0.0;
    int j = 0;
    for (; j + 4 <= nc; j += 4) {
        double2 x0 = *(const double2 *)(xp + (size_t)(j + 0) * ldx);
        double2 x1 = *(const double2 *)(xp + (size_t)(j + 1) * ldx);
        double2 x2 = *(const double2 *)(xp + (size_t)(j + 2) * ldx);
        double2 x3 = *(const double2 *)(xp + (size_t)(j + 3) * ldx);
        ax += x0.x * vs[j];
        ay += x0.y * vs[j];
        ax += x1.x * vs[j + 1];
        ay += x1.y * vs[j + 1];
        ax += x2.x * vs[j + 2];
        ay += x2.y * vs[j + 2];
        ax += x3.x * vs[j + 3];
        ay += x3.y * vs[j + 3];
    }
    for (; j < nc; ++j) {
        double2 x0 = *(const double2 *)(xp + (size_t)j * ldx);
        ax += x0.x * vs[j];
        ay += x0.y * vs[j];
    }
    *(double2 *)(part + (size_t)cb * n_pad + r) = make_double2(ax, ay);
}

// Columns per partial: kXvCols, halved (down to 32) until the launch has >= 1024 workgroups
// -- at C4 (n = 10 000, p = 1000) 256 columns gave 80 workgroups and 2.2 TB/s
static int xv_cols(int ncols, int n_pad) {
    const long rb = (n_pad + kXvRows - 1) / kXvRows;
    int c = kXvCols;
    while (c > kXvMinCols && (long)((ncols + c - 1) / c) * rb < 1024) c >>= 1;
    return c;
}

int xv_chunks(int ncols, int n_pad) {
    const int c = xv_cols(ncols, n_pad);
    return (ncols + c - 1) / c;
}

int xv_chunks_max(int ncols) { return (ncols + kXvMinCols - 1) / kXvMinCols; }

void launch_xv(hipStream_t s, const double *X, int ldx, const double *v, int ncols, int n_pad,
               double *part, const int *gate) {
    const int cols = xv_cols(ncols, n_pad);
    dim3 grid((ncols + cols - 1) / cols, (n_pad + kXvRows - 1) / kXvRows);
    k_xv<<<grid, 256, 0, s>>>(X, ldx, v, ncols, n_pad, cols, part, gate);
}

// ---------------------------------------------------------------------------
// pre-scalar reductions: S_alpha partials and X beta (sum of X.v partials).
// ---------------------------------------------------------------------------
int pre_blocks_s(int p_loc) {
    int b = (p_loc + 2047) / 2048;
    return b < 1 ? 1 : (b > 128 ? 128 : b);
}

__global__ __launch_bounds__(256) void k_pre(const double *part, int nparts, int n_pad,
                                             const double *beta, int p_loc,
                                             const DevScalars *sc, double *red1, int nbS) {
    __shared__ double sh[4];
    if ((int)blockIdx.x < nbS) {
        const double alpha = sc->alpha;
        const int per = (p_loc + nbS - 1) / nbS;
        const int j0 = blockIdx.x * per, j1 = min(p_loc, j0 + per);
        double v = 0.0;
        for (int j = j0 + threadIdx.x; j < j1; j += 256) v += exp(alpha * log(fabs(beta[j])));
        v = block_sum<256>(v, sh);
        if (threadIdx.x == 0) red1[blockIdx.x] = v;
    } else {
        // 16 rows per workgroup, 16 threads per row each summing every 16th partial, then
        // the 16 segment sums in segment order (fixed tree; 16x the loads in flight of a
        // one-thread-per-row loop over up to 256 partials)
        __shared__ double seg_sum[16][17];
        const int rl = threadIdx.x & 15, seg = threadIdx.x >> 4;
        const int r = (blockIdx.x - nbS) * 16 + rl;
        double v = 0.0;
        if (r < n_pad)
            for (int q = seg; q < nparts; q += 16) v += part[(size_t)q * n_pad + r];
        seg_sum[seg][rl] = v;
        __syncthreads();
        if (threadIdx.x < 16 && r < n_pad) {
            double t = 0.0;
#pragma unroll
            for (int g = 0; g < 16; ++g) t += seg_sum[g][rl];
            red1[nbS + r] = t;
        }
    }
}

void launch_pre(hipStream_t s, const double *part, int nparts, int n_pad, const double *beta,
                int p_loc, const DevScalars *sc, double *red1, int nbS) {
    k_pre<<<nbS + (n_pad + 15) / 16, 256, 0, s>>>(part, nparts, n_pad, beta, p_loc, sc, red1,
                                                   nbS);
}

// tau | beta (BridgeRegression.cpp:453-465) and sig2 | beta (:436-450).
__global__ __launch_bounds__(256) void k_scalars(const double *red1, int nbS, const double *y,
                                                 int n, int p, DevScalars *sc, Hyper hy,
                                                 Key key, uint64_t t, double *tau_tr,
                                                 double *sig2_tr, double *alpha_tr, int tau_only,
                                                 uint32_t *err) {
    __shared__ double sh[5];
    const double *xb = red1 + nbS;
    double v = 0.0;
    // the residual sum of squares (sig2 only: the logistic sweep skips it), eight loads of
    // y and X.beta per thread in flight at a time -- a one-load-pair loop paid the memory
    // latency once per iteration (21 us at n = 10 000)
    for (int i0 = tau_only ? n : (int)threadIdx.x; i0 < n; i0 += 256 * 8) {
        double yv[8], xv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = i0 + u * 256;
            yv[u] = i < n ? y[i] : 0.0;
            xv[u] = i < n ? xb[i] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const double r = yv[u] - xv[u];
            v += r * r;
        }
    }
    const double rss0 = block_sum<256>(v, sh);
    if (threadIdx.x == 0) sh[4] = rss0;
    __syncthreads();
    const double rss = sh[4];
    // S_alpha: the nbS workgroup partials summed by all threads (strided, then the fixed
    // tree of block_sum) -- one thread adding them in turn paid a load latency per partial
    // (nbS = 782 at p = 200 000)
    double sv = 0.0;
    for (int q = threadIdx.x; q < nbS; q += 256) sv += red1[q];
    const double S0 = block_sum<256>(sv, sh);
    // tau (wave 0) and sig2 (wave 1) are independent draws on their own counters: one lane
    // of each wave, concurrently
    if (threadIdx.x == 0) {
        const double S = S0;
        const double alpha = sc->alpha;
        if (!hy.know_tau) {
            const double shape = hy.nu_shape + ((double)p) / alpha;
            const double rate = hy.nu_rate + S;
            const double nu = gamma1(shape, key, t, KIND_TAU, err) / rate;
            sc->tau = exp(-1.0 * log(nu) / alpha);
        }
        sc->s_abs_pow = S;
        sc->rss = rss;
        if (tau_tr) *tau_tr = sc->tau;
        if (alpha_tr) *alpha_tr = alpha;
    } else if (threadIdx.x == 64) {
        if (!tau_only && !hy.know_sig2) {
            const double shape = hy.sig2_shape + 0.5 * (double)n;
            const double scale = hy.sig2_scale + 0.5 * rss;
            sc->sig2 = scale / gamma1(shape, key, t, KIND_SIG2, err);
        }
        if (sig2_tr) *sig2_tr = sc->sig2;
    }
}

void launch_scalars(hipStream_t s, const double *red1, int nbS, const double *y, int n,
                    int p, DevScalars *sc, Hyper hy, uint64_t k0, uint64_t k1, uint64_t t,
                    double *tau_tr, double *sig2_tr, double *alpha_tr, int tau_only,
                    uint32_t *err) {
    k_scalars<<<1, 256, 0, s>>>(red1, nbS, y, n, p, sc, hy, Key{k0, k1}, t, tau_tr, sig2_tr,
                                alpha_tr, tau_only, err);
}

// ---------------------------------------------------------------------------
// Woodbury system assembly.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_slab_sum(const double *slabs, int S, size_t stride,
                                                  int n_pad, const double *xu_part, int nxu,
                                                  double *red2, int packed, const int *gate) {
    if (gated(gate)) return;
    const size_t nn = (size_t)n_pad * n_pad;
    const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (idx < nn) {
        const int r = (int)(idx % n_pad), c = (int)(idx / n_pad);
        if (r <= c) {
            double v = 0.0;
            for (int q = 0; q < S; ++q) v += slabs[(size_t)q * stride + idx];
            red2[packed ? tri_index(r, c) : idx] = v;
        } else if (!packed) {
            red2[idx] = 0.0;
        }
    } else if (idx < nn + (size_t)n_pad) {
        const int r = (int)(idx - nn);
        double v = 0.0;
        for (int q = 0; q < nxu; ++q) v += xu_part[(size_t)q * n_pad + r];
        red2[(packed ? tri_count(n_pad) : nn) + r] = v;
    }
}

void launch_slab_sum(hipStream_t s, const double *slabs, int S, size_t slab_stride, int n_pad,
                     const double *xu_part, int nxu, double *red2, int packed, const int *gate) {
    const size_t tot = (size_t)n_pad * n_pad + n_pad;
    k_slab_sum<<<(unsigned)((tot + 255) / 256), 256, 0, s>>>(slabs, S, slab_stride, n_pad,
                                                             xu_part, nxu, red2, packed, gate);
}

// One thread per upper-triangle entry (packed index e -> (r, c): consecutive threads walk a
// column, so the red2 reads and the M writes are both contiguous), then one per entry of the
// right-hand-side block columns.  (The first version ran a thread per entry of the full
// n_pad x (n_pad + 64) matrix, half of them idle: C3 13.3 -> 11.6 us, C5 57 -> 45 us.)
__global__ __launch_bounds__(256) void k_form_m(const double *red2, int n, int n_pad,
                                                const double *y, const DevScalars *sc, Key key,
                                                uint64_t t, double *M, int ldm, int rhs_col, const int *gate) {
    if (gated(gate)) return;
    const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t ntri = tri_count(n_pad);
    const double sig2 = sc->sig2;
    if (idx < ntri) {
        // c = floor((sqrt(8 e + 1) - 1) / 2), corrected by one either way
        int c = (int)((sqrt(8.0 * (double)idx + 1.0) - 1.0) * 0.5);
        while ((size_t)c * (c + 1) / 2 > idx) --c;
        while ((size_t)(c + 1) * (c + 2) / 2 <= idx) ++c;
        const int r = (int)(idx - (size_t)c * (c + 1) / 2);
        M[(size_t)r + (size_t)c * ldm] = red2[idx] / sig2 + (r == c ? 1.0 : 0.0);
        return;
    }
    const size_t e = idx - ntri;
    if (e >= (size_t)n_pad * kNB) return;
    const int r = (int)(e % n_pad), c = n_pad + (int)(e / n_pad);
    double *dst = M + (size_t)r + (size_t)c * ldm;
    if (c == rhs_col) {
        double v = 0.0;
        if (r < n) {
            const double sig = sqrt(sig2);
            const double delta = normal_at(key, t, KIND_DELTA, (uint64_t)r);
            const double xu = red2[ntri + r];
            v = y[r] / sig - (xu / sig + delta);
        }
        *dst = v;
    } else {
        *dst = 0.0;
    }
}

void launch_form_m(hipStream_t s, const double *red2, int n, int n_pad, const double *y,
                   const DevScalars *sc, uint64_t k0, uint64_t k1, uint64_t t, double *M,
                   int ldm, int rhs_col, const int *gate) {
    const size_t tot = tri_count(n_pad) + (size_t)n_pad * kNB;
    k_form_m<<<(unsigned)((tot + 255) / 256), 256, 0, s>>>(red2, n, n_pad, y, sc, Key{k0, k1}, t,
                                                           M, ldm, rhs_col, gate);
}

__global__ __launch_bounds__(256) void k_form_a(const double *G, int ldg, const double *lam,
                                                const DevScalars *sc, const double *cvec, int p,
                                                int p_pad, double *A, int lda, int rhs_col,
                                                int packed) {
    const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t tot = (size_t)p_pad * (p_pad + kNB);
    if (idx >= tot) return;
    const int r = (int)(idx % p_pad), c = (int)(idx / p_pad);
    double *dst = A + (size_t)r + (size_t)c * lda;
    if (c < p_pad) {
        if (r <= c) {
            double v = G[packed ? tri_index(r, c) : (size_t)r + (size_t)c * ldg];
            if (r == c) {
                if (r < p) {
                    if (lam) {
                        const double tau = sc->tau;
                        v += lam[r] * sc->sig2 / (tau * tau);
                    }
                } else {
                    v = 1.0;
                }
            }
            *dst = v;
        }
    } else if (c == rhs_col) {
        *dst = (r < p) ? cvec[r] : 0.0;
    } else {
        *dst = 0.0;
    }
}

// ---------------------------------------------------------------------------
// Bridge EM (BridgeRegression.cpp:600-708): the maximisation step's system for the
// active coordinates, A = XX_active + c2 diag(lam_active), b_active, laid out over the
// full p_pad index space with every dropped (mask 0) or padding coordinate as an identity
// row/column and a zero right-hand side -- the active block's elimination is then exactly
// the one of the compacted system, and the dropped unknowns solve to 0.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_em_form(const double *G, int ldg, const double *dlam,
                                                 const int *mask, const double *b, int p,
                                                 int p_pad, double *A, int lda, int rhs_col) {
    const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t tot = (size_t)p_pad * (p_pad + kNB);
    if (idx >= tot) return;
    const int r = (int)(idx % p_pad), c = (int)(idx / p_pad);
    double *dst = A + (size_t)r + (size_t)c * lda;
    const bool ar = r < p && mask[r];
    if (c < p_pad) {
        if (r <= c) {
            const bool ac = c < p && mask[c];
            double v;
            if (ar && ac)
                v = G[(size_t)r + (size_t)c * ldg] + (r == c && dlam ? dlam[r] : 0.0);
            else
                v = (r == c) ? 1.0 : 0.0;
            *dst = v;
        }
    } else if (c == rhs_col) {
        *dst = ar ? b[r] : 0.0;
    } else {
        *dst = 0.0;
    }
}

void launch_em_form(hipStream_t s, const double *G, int ldg, const double *dlam, const int *mask,
                    const double *b, int p, int p_pad, double *A, int lda, int rhs_col) {
    const size_t tot = (size_t)p_pad * (p_pad + kNB);
    k_em_form<<<(unsigned)((tot + 255) / 256), 256, 0, s>>>(G, ldg, dlam, mask, b, p, p_pad, A,
                                                            lda, rhs_col);
}

// Conjugate gradients on the masked system (upper triangle of A, column-major), one
// workgroup: r = b - A x, d = r; while it < max_it and |r| > tol: a = r.r / d.Ad,
// x += a d, r -= a Ad, d = r + (r'.r' / r.r) d.  Dot products are fixed-order block trees,
// so the iteration count and the result are deterministic.  out_it = iterations taken.
constexpr int kEmCgThreads = 1024;

__device__ double em_block_dot(const double *u, const double *v, int n, double *sh) {
    double a = 0.0;
    for (int i = threadIdx.x; i < n; i += kEmCgThreads) a += u[i] * v[i];
    a = wave_allsum(a);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) sh[w] = a;
    __syncthreads();
    double r = 0.0;
#pragma unroll
    for (int i = 0; i < kEmCgThreads / 64; ++i) r += sh[i];
    return r;  // every thread
}

__device__ void em_matvec(const double *A, int lda, int n, const double *v, double *out) {
    for (int r = threadIdx.x; r < n; r += kEmCgThreads) {
        double a = 0.0;
        for (int c = 0; c < n; ++c) {
            const double m = c >= r ? A[(size_t)r + (size_t)c * lda] : A[(size_t)c + (size_t)r * lda];
            a += m * v[c];
        }
        out[r] = a;
    }
}

__global__ __launch_bounds__(kEmCgThreads) void k_em_cg(const double *A, int lda, int n,
                                                        const double *b, double *x, double tol,
                                                        int max_it, double *work, int *out_it) {
    __shared__ double sh[kEmCgThreads / 64];
    double *r = work, *d = work + n, *ad = work + 2 * (size_t)n;
    em_matvec(A, lda, n, x, ad);
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += kEmCgThreads) {
        r[i] = b[i] - ad[i];
        d[i] = r[i];
    }
    __syncthreads();
    double rr = em_block_dot(r, r, n, sh);
    int it = 0;
    while (it < max_it && sqrt(rr) > tol) {
        em_matvec(A, lda, n, d, ad);
        __syncthreads();
        const double dad = em_block_dot(d, ad, n, sh);
        const double a = rr / dad;
        for (int i = threadIdx.x; i < n; i += kEmCgThreads) {
            x[i] += a * d[i];
            r[i] -= a * ad[i];
        }
        __syncthreads();
        const double rn = em_block_dot(r, r, n, sh);
        const double bt = rn / rr;
        for (int i = threadIdx.x; i < n; i += kEmCgThreads) d[i] = r[i] + bt * d[i];
        __syncthreads();
        rr = rn;
        ++it;
    }
    if (threadIdx.x == 0) *out_it = it;
}

void launch_em_cg(hipStream_t s, const double *A, int lda, int n, const double *b, double *x,
                  double tol, int max_it, double *work, int *out_it) {
    k_em_cg<<<1, kEmCgThreads, 0, s>>>(A, lda, n, b, x, tol, max_it, work, out_it);
}

// Batched bridge EM over a ratio grid (trace.beta, Code/R/bridge-trace.R): one workgroup
// per ratio runs the whole EM of BR::EM (BridgeRegression.cpp:600-708, direct solves) with
// the system in LDS -- thread i owns row i (MAXP = 64: one wave for p <= 64; MAXP = 128: two
// waves and a 129 KB system for p <= 128); right-looking Cholesky, forward and backward
// substitution; dropped coordinates are identity rows with a zero right-hand side, as in
// k_em_form.  No host round trip per iteration.
template <int MAXP>
__device__ bool em_lds_solve(double (*A)[MAXP + 1], double *y, int p) {
    const int lane = threadIdx.x;
    bool ok = true;
    for (int k = 0; k < p; ++k) {
        __syncthreads();
        const double akk = A[k][k];
        if (!(akk > 0.0)) ok = false;
        const double d = sqrt(akk);
        __syncthreads();
        if (lane > k && lane < p) A[lane][k] /= d;
        if (lane == k) A[k][k] = d;
        __syncthreads();
        if (lane > k && lane < p) {
            const double lik = A[lane][k];
            for (int j = k + 1; j <= lane; ++j) A[lane][j] -= lik * A[j][k];
        }
    }
    for (int k = 0; k < p; ++k) {  // L y' = y
        __syncthreads();
        const double yk = y[k] / A[k][k];
        __syncthreads();
        if (lane == k) y[k] = yk;
        if (lane > k && lane < p) y[lane] -= A[lane][k] * yk;
    }
    for (int k = p - 1; k >= 0; --k) {  // L' x = y'
        __syncthreads();
        const double xk = y[k] / A[k][k];
        __syncthreads();
        if (lane == k) y[k] = xk;
        if (lane < k) y[lane] -= A[k][lane] * xk;
    }
    __syncthreads();
    return ok;
}

template <int MAXP>
__global__ __launch_bounds__(MAXP) void k_em_batch(const double *G, int ldg, const double *bvec,
                                                   int p, const double *ratios,
                                                   const double *lambda_max, double alpha,
                                                   double tol, int max_iter, double *beta_out,
                                                   int *solves_out) {
    constexpr int NW = MAXP / 64;
    __shared__ double A[MAXP][MAXP + 1];
    __shared__ double x[MAXP], old[MAXP], lam[MAXP];
    __shared__ int mask[MAXP];
    __shared__ double red[MAXP];
    __shared__ int wcount[NW];
    const int lane = threadIdx.x, r = blockIdx.x;
    const double tau = ratios[r], sig = 1.0, lmax = lambda_max[r];
    const double c1 = alpha * exp((2 - alpha) * (log(tau) - log(sig)));
    const double c2 = exp(-2 * (log(tau) - log(sig)));
    double *out = beta_out + (size_t)r * p;
    mask[lane] = lane < p;
    lam[lane] = 0.0;
    auto form = [&](bool with_lam) {
        __syncthreads();
        if (lane < p) {
            const bool ai = mask[lane];
            for (int j = 0; j < p; ++j) {
                const int lo = lane < j ? lane : j, hi = lane < j ? j : lane;
                double v;
                if (ai && mask[j])
                    v = G[(size_t)lo + (size_t)hi * ldg] + (with_lam && j == lane ? c2 * lam[lane] : 0.0);
                else
                    v = (j == lane) ? 1.0 : 0.0;
                A[lane][j] = v;
            }
            x[lane] = ai ? bvec[lane] : 0.0;
        }
        __syncthreads();
    };
    form(false);
    if (!em_lds_solve<MAXP>(A, x, p)) {
        if (lane < p) out[lane] = 0.0;
        if (lane == 0) solves_out[r] = -1;
        return;
    }
    long total = p;
    double dist = tol + 1.0;
    int it = 0, pa = p;
    while (dist > tol && it < max_iter) {
        // expectation step: lambda_j, the active set (all lanes evaluate, lane j owns j)
        int keep = 0;
        if (lane < p && mask[lane]) {
            const double l = c1 * exp((alpha - 2) * log(fabs(x[lane])));
            if (l < lmax) {
                lam[lane] = l;
                old[lane] = x[lane];
                keep = 1;
            } else {
                mask[lane] = 0;
            }
        }
        const int wc = __popcll(__ballot(keep));
        if ((lane & 63) == 0) wcount[lane >> 6] = wc;
        __syncthreads();
        int num = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) num += wcount[w];
        if (num == 0) {
            if (lane < p) out[lane] = 0.0;
            if (lane == 0) solves_out[r] = it;
            return;
        }
        pa = num;
        form(true);
        if (!em_lds_solve<MAXP>(A, x, p)) {
            if (lane < p) out[lane] = 0.0;
            if (lane == 0) solves_out[r] = -1;
            return;
        }
        total += pa;
        // distance over the active set, summed in coordinate order (as the host loop)
        const double dv = (lane < p && mask[lane]) ? (x[lane] - old[lane]) : 0.0;
        red[lane] = dv * dv;
        __syncthreads();
        double d2 = 0.0;
        for (int j = 0; j < p; ++j) d2 += red[j];
        dist = sqrt(d2);
        ++it;
        __syncthreads();
    }
    if (lane < p) out[lane] = mask[lane] ? x[lane] : 0.0;
    if (lane == 0) solves_out[r] = (int)total;
}

void launch_em_batch(hipStream_t s, const double *G, int ldg, const double *b, int p,
                     const double *ratios, const double *lambda_max, int count, double alpha,
                     double tol, int max_iter, double *beta_out, int *solves_out) {
    if (p <= 64)
        k_em_batch<64><<<count, 64, 0, s>>>(G, ldg, b, p, ratios, lambda_max, alpha, tol,
                                            max_iter, beta_out, solves_out);
    else
        k_em_batch<128><<<count, 128, 0, s>>>(G, ldg, b, p, ratios, lambda_max, alpha, tol,
                                              max_iter, beta_out, solves_out);
}

// Batched bridge EM for p > 128 (trace.beta at any p): the EM loop of k_em_batch, one
// workgroup per ratio, with the ratio's p_pad x p_pad system (lower triangle, column-major)
// in a global scratch slice instead of LDS.  Tiled right-looking Cholesky over 64 x 64 tiles
// staged in LDS: the diagonal tile factored in place (two barriers per pivot), its
// triangular inverse formed by one wave (a lane per column), the panel tiles multiplied by
// it, the trailing tiles updated by 64^3 products (4 x 4 outputs per thread, in m order);
// substitution tile by tile, the off-diagonal part as matvecs over LDS tiles (four fixed
// partial sums per row) and the diagonal part on one wave with shuffles.  Every sum has a
// fixed order, so a ratio's result does not depend on the batch it runs in.
constexpr int kEmTile = 64, kEmLd = kEmTile + 1;

namespace {

// t[m * kEmLd + r] = A(r0 + r, c0 + m): a tile column is a contiguous LDS row
__device__ __forceinline__ void em_tile_load(const double *A, int lda, int r0, int c0,
                                             double *t) {
    for (int e = threadIdx.x; e < kEmTile * kEmTile; e += 256) {
        const int r = e & (kEmTile - 1), m = e / kEmTile;
        t[m * kEmLd + r] = A[(size_t)(r0 + r) + (size_t)(c0 + m) * lda];
    }
}

// tile (r0, c0) of A = [A -] sum_m a[m][r] b[m][c]; thread owns rows (tid & 15) + 16 ii
// and columns (tid >> 4) + 16 jj (a wave stores 4 columns x 128 contiguous bytes)
template <bool SUB>
__device__ __forceinline__ void em_tile_mm(const double *a, const double *b, double *A, int lda,
                                           int r0, int c0) {
    const int tr = threadIdx.x & 15, tc = threadIdx.x >> 4;
    double acc[4][4] = {};
    for (int m = 0; m < kEmTile; ++m) {
        double av[4], bv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) av[i] = a[m * kEmLd + tr + 16 * i];
#pragma unroll
        for (int j = 0; j < 4; ++j) bv[j] = b[m * kEmLd + tc + 16 * j];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = fma(av[i], bv[j], acc[i][j]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            double *cp = A + (size_t)(r0 + tr + 16 * i) + (size_t)(c0 + tc + 16 * j) * lda;
            *cp = SUB ? *cp - acc[i][j] : acc[i][j];
        }
}

// In-place lower Cholesky of the p_pad x p_pad matrix (T tiles a side).  false (uniformly
// across the workgroup) on a pivot that is not > 0.
__device__ bool em_chol_tiled(double *A, int lda, int T, double *ta, double *tb) {
    const int tid = threadIdx.x;
    for (int k = 0; k < T; ++k) {
        const int k0 = k * kEmTile;
        __syncthreads();
        em_tile_load(A, lda, k0, k0, ta);
        for (int c = 0; c < kEmTile; ++c) {
            __syncthreads();
            const double piv = ta[c * kEmLd + c];
            if (!(piv > 0.0)) return false;
            const double d = sqrt(piv);
            __syncthreads();
            if (tid < kEmTile) {
                if (tid > c) ta[c * kEmLd + tid] /= d;
                else if (tid == c) ta[c * kEmLd + c] = d;
            }
            __syncthreads();
            const int w = kEmTile - 1 - c;  // columns j = c + 1 .. 63, rows r >= j
            for (int e = tid; e < w * kEmTile; e += 256) {
                const int j = c + 1 + e / kEmTile, r = e & (kEmTile - 1);
                if (r >= j) ta[j * kEmLd + r] -= ta[c * kEmLd + r] * ta[c * kEmLd + j];
            }
        }
        __syncthreads();
        for (int e = tid; e < kEmTile * kEmTile; e += 256) {
            const int r = e & (kEmTile - 1), m = e / kEmTile;
            if (r >= m) A[(size_t)(k0 + r) + (size_t)(k0 + m) * lda] = ta[m * kEmLd + r];
        }
        if (k + 1 == T) break;
        // Linv = L_kk^-1 (lower), stored tb[m][c] = Linv(c, m): lane cc forms column cc
        if (tid < kEmTile) {
            const int cc = tid;
            for (int r = 0; r < kEmTile; ++r) {
                double s = (r == cc) ? 1.0 : 0.0;
                for (int m = cc; m < r; ++m) s -= ta[m * kEmLd + r] * tb[cc * kEmLd + m];
                tb[cc * kEmLd + r] = (r >= cc) ? s / ta[r * kEmLd + r] : 0.0;
            }
        }
        // panel: L_ik = A_ik L_kk^-T
        for (int i = k + 1; i < T; ++i) {
            __syncthreads();
            em_tile_load(A, lda, i * kEmTile, k0, ta);
            __syncthreads();
            em_tile_mm<false>(ta, tb, A, lda, i * kEmTile, k0);
        }
        // trailing: A_ij -= L_ik L_jk^T, j <= i
        for (int j = k + 1; j < T; ++j) {
            __syncthreads();
            em_tile_load(A, lda, j * kEmTile, k0, tb);
            for (int i = j; i < T; ++i) {
                __syncthreads();
                em_tile_load(A, lda, i * kEmTile, k0, ta);
                __syncthreads();
                em_tile_mm<true>(ta, tb, A, lda, i * kEmTile, j * kEmTile);
            }
        }
    }
    __syncthreads();
    return true;
}

// v <- L^-T L^-1 v with the factor em_chol_tiled left in A
__device__ void em_solve_tiled(const double *A, int lda, int T, double *v, double *ta,
                               double *red) {
    const int tid = threadIdx.x, i = tid & (kEmTile - 1), q = tid / kEmTile;
    for (int k = 0; k < T; ++k) {  // L y = v
        const int k0 = k * kEmTile;
        double s = 0.0;
        __syncthreads();
        for (int j = 0; j < k; ++j) {
            __syncthreads();
            em_tile_load(A, lda, k0, j * kEmTile, ta);
            __syncthreads();
            for (int m = q * 16; m < q * 16 + 16; ++m) s += ta[m * kEmLd + i] * v[j * kEmTile + m];
        }
        red[tid] = s;
        __syncthreads();
        em_tile_load(A, lda, k0, k0, ta);
        __syncthreads();
        if (tid < kEmTile) {
            double val = v[k0 + i] - (((red[i] + red[64 + i]) + red[128 + i]) + red[192 + i]);
            for (int c = 0; c < kEmTile; ++c) {
                const double yc = __shfl(val, c, 64) / ta[c * kEmLd + c];
                if (i > c) val -= ta[c * kEmLd + i] * yc;
                else if (i == c) val = yc;
            }
            v[k0 + i] = val;
        }
    }
    for (int k = T - 1; k >= 0; --k) {  // L' x = y
        const int k0 = k * kEmTile;
        double s = 0.0;
        __syncthreads();
        for (int j = k + 1; j < T; ++j) {
            __syncthreads();
            em_tile_load(A, lda, j * kEmTile, k0, ta);  // ta[m][r] = L(j0 + r, k0 + m)
            __syncthreads();
            for (int r = q * 16; r < q * 16 + 16; ++r) s += ta[i * kEmLd + r] * v[j * kEmTile + r];
        }
        red[tid] = s;
        __syncthreads();
        em_tile_load(A, lda, k0, k0, ta);
        __syncthreads();
        if (tid < kEmTile) {
            double val = v[k0 + i] - (((red[i] + red[64 + i]) + red[128 + i]) + red[192 + i]);
            for (int c = kEmTile - 1; c >= 0; --c) {
                const double zc = __shfl(val, c, 64) / ta[c * kEmLd + c];
                if (i < c) val -= ta[i * kEmLd + c] * zc;
                else if (i == c) val = zc;
            }
            v[k0 + i] = val;
        }
    }
    __syncthreads();
}

}  // namespace

__global__ __launch_bounds__(256) void k_em_batch_tiled(
    const double *__restrict__ G, int ldg, const double *__restrict__ bvec, int p, int p_pad,
    const double *__restrict__ ratios, const double *__restrict__ lambda_max, int r0,
    double alpha, double tol, int max_iter, double *__restrict__ scratch,
    double *__restrict__ vecs, int *__restrict__ masks, double *__restrict__ beta_out,
    int *__restrict__ solves_out) {
    __shared__ double ta[kEmTile * kEmLd], tb[kEmTile * kEmLd];
    __shared__ double red[256];
    __shared__ int cnt[4];
    __shared__ double dsh;
    const int tid = threadIdx.x, T = p_pad / kEmTile, r = r0 + (int)blockIdx.x;
    double *A = scratch + (size_t)blockIdx.x * p_pad * p_pad;
    double *x = vecs + (size_t)blockIdx.x * 3 * p_pad, *old = x + p_pad, *lam = old + p_pad;
    int *mask = masks + (size_t)blockIdx.x * p_pad;
    const double tau = ratios[r], sig = 1.0, lmax = lambda_max[r];
    const double c1 = alpha * exp((2 - alpha) * (log(tau) - log(sig)));
    const double c2 = exp(-2 * (log(tau) - log(sig)));
    double *out = beta_out + (size_t)r * p;
    for (int i = tid; i < p_pad; i += 256) {
        mask[i] = i < p;
        lam[i] = 0.0;
    }
    auto form = [&](bool with_lam) {
        __syncthreads();
        for (int j = tid / 64; j < p_pad; j += 4)
            for (int i = j + (tid & 63); i < p_pad; i += 64) {
                double v;
                if (i < p && mask[i] && mask[j])  // j <= i < p
                    v = G[(size_t)j + (size_t)i * ldg] + (with_lam && i == j ? c2 * lam[i] : 0.0);
                else
                    v = (i == j) ? 1.0 : 0.0;
                A[(size_t)i + (size_t)j * p_pad] = v;
            }
        for (int i = tid; i < p_pad; i += 256) x[i] = (i < p && mask[i]) ? bvec[i] : 0.0;
        __syncthreads();
    };
    auto fail = [&]() {
        for (int i = tid; i < p; i += 256) out[i] = 0.0;
        if (tid == 0) solves_out[r] = -1;
    };
    form(false);
    if (!em_chol_tiled(A, p_pad, T, ta, tb)) return fail();
    em_solve_tiled(A, p_pad, T, x, ta, red);
    long total = p;
    double dist = tol + 1.0;
    int it = 0;
    while (dist > tol && it < max_iter) {
        // expectation step: lambda_j and the active set, coordinate j on thread j % 256
        int keep = 0;
        for (int i = tid; i < p; i += 256) {
            if (!mask[i]) continue;
            const double l = c1 * exp((alpha - 2) * log(fabs(x[i])));
            if (l < lmax) {
                lam[i] = l;
                old[i] = x[i];
                ++keep;
            } else {
                mask[i] = 0;
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) keep += __shfl_xor(keep, o, 64);
        if ((tid & 63) == 0) cnt[tid >> 6] = keep;
        __syncthreads();
        const int num = ((cnt[0] + cnt[1]) + cnt[2]) + cnt[3];
        if (num == 0) {
            for (int i = tid; i < p; i += 256) out[i] = 0.0;
            if (tid == 0) solves_out[r] = it;
            return;
        }
        form(true);
        if (!em_chol_tiled(A, p_pad, T, ta, tb)) return fail();
        em_solve_tiled(A, p_pad, T, x, ta, red);
        total += num;
        // distance over the active set, summed in coordinate order (as the host loop)
        if (tid == 0) {
            double d2 = 0.0;
            for (int j = 0; j < p; ++j)
                if (mask[j]) d2 += (x[j] - old[j]) * (x[j] - old[j]);
            dsh = d2;
        }
        __syncthreads();
        dist = sqrt(dsh);
        ++it;
        __syncthreads();
    }
    for (int i = tid; i < p; i += 256) out[i] = mask[i] ? x[i] : 0.0;
    if (tid == 0) solves_out[r] = (int)total;
}

void launch_em_batch_tiled(hipStream_t s, const double *G, int ldg, const double *b, int p,
                           int p_pad, const double *ratios, const double *lambda_max, int r0,
                           int count, double alpha, double tol, int max_iter, double *scratch,
                           double *vecs, int *masks, double *beta_out, int *solves_out) {
    k_em_batch_tiled<<<count, 256, 0, s>>>(G, ldg, b, p, p_pad, ratios, lambda_max, r0, alpha,
                                           tol, max_iter, scratch, vecs, masks, beta_out,
                                           solves_out);
}

int em_tile() { return kEmTile; }

void launch_form_a(hipStream_t s, const double *G, int ldg, const double *lam,
                   const DevScalars *sc, const double *c, int p, int p_pad, double *A, int lda,
                   int rhs_col, int packed) {
    const size_t tot = (size_t)p_pad * (p_pad + kNB);
    k_form_a<<<(unsigned)((tot + 255) / 256), 256, 0, s>>>(G, ldg, lam, sc, c, p, p_pad, A, lda,
                                                           rhs_col, packed);
}

// ---------------------------------------------------------------------------
// Blocked Cholesky A = U'U (upper, column-major, NB = 64) with the forward solve folded into
// trailing right-hand-side column blocks: k_chol_persistent below.
// Pivot chain (tools/diag_latency.hip: a dependent fp64 op ~48 cycles, an LDS
// write/barrier/read round trip ~270): the wave owning rows 8b..8b+7 factors them with
// v_readlane broadcasts (no barrier) and publishes each pivot row as soon as it is final;
// the other waves apply it -- valid because a symmetric elimination's multipliers depend
// only on the final pivot rows.  U_kk itself is never stored: the backward solve uses W_k.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double fast_rcp(double p) {
    // v_rcp_f64 (~2^-26 accurate) + one Newton step in FMA form: ~1 ulp for the normal
    // positive pivots, two dependent FMAs after the reciprocal
    const double r = __builtin_amdgcn_rcp(p);
    return __builtin_fma(r, __builtin_fma(-p, r, 1.0), r);
}

__device__ __forceinline__ double readlane_d(double v, int lane) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, lane);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// ---------------------------------------------------------------------------
// Persistent dataflow Cholesky: ONE launch factors the whole matrix.
//   workgroup 0 (the chain) owns the critical path: for k = 0 .. nblk-1 it eliminates the
//     diagonal block D_k (held in LDS, all updates applied) -> W_k = U_kk^-T, publishes W_k,
//     then takes the hand-off tiles A_{k,k+1}, A_{k+1,k+1} (updated by their owners through
//     step k-1), forms U_{k,k+1} = W_k A_{k,k+1} (published: it feeds the updates of step k)
//     and D_{k+1} = A_{k+1,k+1} - U_{k,k+1}' U_{k,k+1} locally -- no launch boundary and no
//     flag round trip between two consecutive eliminations;
//   workgroups 1.. own the other tiles (i <= j, RHS block columns included), taken in
//     row-major order, round-robin: a tile is loaded into LDS, receives its updates
//     A_ij -= U_ki' U_kj (k < i; MFMA) as the panels U_k* are published, then either becomes
//     U_ij = W_i A_ij (published) or, for the hand-off tiles (i,i) / (i,i+1), is written
//     back and handed to the chain.
// Every dependency points to an earlier tile row or to the chain at a step <= the tile's
// row, and each owner takes its tiles in row-major order, so the schedule cannot deadlock
// with every workgroup resident (grid <= CUs, one 512-thread workgroup per CU).
// Flags: fW[k], fP[k][j] (U_kj published), fR[k][0/1] (tile (k,k) / (k,k+1) handed over);
// a flag is set by storing the factorisation's epoch (1, 2, ... per flag buffer), so the
// buffer is never re-zeroed; agent-scope release/acquire, spins bounded (error bit 16).
// ---------------------------------------------------------------------------
struct CholFlags {
    unsigned int *W, *P, *R;
    unsigned int *H;  // H[i]: tile (i, i+2) updated through step i-1 and stored (i >= 1)
    int ncb;
    unsigned int ep;  // this factorisation's epoch
};

// Cross-workgroup hand-offs inside the persistent kernel follow the write-through recipe of
// cdna_hip_programming.md Guideline 16 (R1, "every load sc1"): every handed-off double is
// stored with an agent-scope relaxed atomic (global_store ... sc1, written through the XCD's
// L2) and every load of handed-off data is an agent-scope relaxed atomic load (sc1, bypasses
// the CU's L1), so neither side needs an L2 write-back (buffer_wbl2, ~2-6 us) or an L1
// invalidate (buffer_inv, ~1.7 us) per hop.  Release = every storing wave drains its stores,
// barrier, one lane stores the flag (relaxed, agent).
__device__ __forceinline__ double ld_sc1(const double *p) {
    return __hip_atomic_load(const_cast<double *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(double *p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Bounded cross-workgroup waits.  A wait gives up (error bit 16) after kSpinTicks of the
// 100 MHz s_memrealtime clock -- 2 s, three orders of magnitude beyond any hand-off of a
// factorisation that takes milliseconds -- or as soon as any other wait of the launch gave
// up (bit 16 already set), so a launch that cannot make progress (a workgroup of its grid
// never became resident, a broken hand-off) ends within seconds with the error flag, which
// the .C driver reports as "Aborting Gibbs sampler.", instead of timing out wait after wait.
constexpr uint64_t kSpinTicks = 200000000ull;
struct SpinGuard {
    uint64_t t0;
    unsigned n = 0;
    __device__ SpinGuard() : t0(__builtin_amdgcn_s_memrealtime()) {}
    // call once per unsuccessful poll, by every lane of the waiting wave (the answer is
    // wave-uniform); true: stop waiting (bit 16 set in *err)
    __device__ bool expired(uint32_t *err) {
        if ((++n & 255u) != 0) return false;
        if (err && (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 16u))
            return true;
        if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) {
            if (err && (threadIdx.x & 63) == 0) atomicOr(err, 16u);
            return true;
        }
        return false;
    }
};

__device__ __forceinline__ void flag_release(unsigned int *f, unsigned int ep) {
    // caller: every wave's sc1 stores issued; each wave drains them before the barrier
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(f, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void flag_acquire2(const unsigned int *f1, const unsigned int *f2,
                                              unsigned int ep, uint32_t *err) {
    if (threadIdx.x == 0) {
        SpinGuard sg;
        while (__hip_atomic_load(f1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != ep ||
               (f2 && __hip_atomic_load(f2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != ep)) {
            __builtin_amdgcn_s_sleep(2);
            if (sg.expired(err)) break;
        }
    }
    // the payload is read with sc1 loads only: no L1 invalidate, just keep the compiler
    // from hoisting them above the poll
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __syncthreads();
}

// Load tile (row block i, col block j) of column-major A into L[y][x] (all 8 sc1 loads of
// a thread in flight before the first LDS write).
__device__ __forceinline__ void tile_load(double (*L)[65], const double *A, int lda, int i, int j,
                                          bool upper_only) {
    double v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int e = threadIdx.x + q * 512, y = e & 63, x = e >> 6;
        v[q] = ld_sc1(&A[(size_t)(i * kNB + y) + (size_t)(j * kNB + x) * lda]);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int e = threadIdx.x + q * 512, y = e & 63, x = e >> 6;
        L[y][x] = (!upper_only || y <= x) ? v[q] : 0.0;
    }
}

__device__ __forceinline__ void tile_store(const double (*L)[65], double *A, int lda, int i,
                                           int j) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int e = threadIdx.x + q * 512, y = e & 63, x = e >> 6;
        st_sc1(&A[(size_t)(i * kNB + y) + (size_t)(j * kNB + x) * lda], L[y][x]);
    }
}

// C[y][x] = sum_s P[s][y] Q[s][x] over 64 s (P'Q), 8 waves x 2 blocks of 16x16 (fp64 MFMA);
// the lane's results are acc[h][r] at y = by*16 + (lane>>4) + 4r, x = bx*16 + (lane&15).
// ACC: add to acc instead of overwriting it.
template <bool ACC = false>
__device__ __forceinline__ void mm_tn(const double (*P)[65], const double (*Q)[65], v4d acc[2]) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int b0 = wid * 2, b1 = wid * 2 + 1;
    const int bx0 = b0 >> 2, by0 = b0 & 3, bx1 = b1 >> 2, by1 = b1 & 3;
    if (!ACC) acc[0] = acc[1] = (v4d){0.0, 0.0, 0.0, 0.0};
    // the two blocks' accumulation chains interleaved: consecutive MFMAs are independent
#pragma unroll 4
    for (int kk = 0; kk < 16; ++kk) {
        const int sr = kk * 4 + (lane >> 4);
        acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(P[sr][by0 * 16 + (lane & 15)],
                                                     Q[sr][bx0 * 16 + (lane & 15)], acc[0], 0, 0,
                                                     0);
        acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(P[sr][by1 * 16 + (lane & 15)],
                                                     Q[sr][bx1 * 16 + (lane & 15)], acc[1], 0, 0,
                                                     0);
    }
}

// C = Wl * B for a lower-triangular 64 x 64 Wl (K steps 0 .. 4 by + 3 of block row by):
// wave w takes column block w >> 1 and the block-row pair {0, 3} (w even) or {1, 2} (w odd),
// 20 MFMAs per wave with compile-time trip counts; the two chains interleaved and the longer
// one split even / odd.  lo = block row 0 / 1, hi = block row 3 / 2.  wl_put stores them.
__device__ __forceinline__ void wl_times(const double (*Wl)[65], const double (*B)[65], v4d &lo,
                                         v4d &hi) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, ubx = wid >> 1;
    auto wop = [&](int by, int kk) { return Wl[by * 16 + (lane & 15)][kk * 4 + (lane >> 4)]; };
    auto bop = [&](int kk) { return B[kk * 4 + (lane >> 4)][ubx * 16 + (lane & 15)]; };
    v4d a0 = {0.0, 0.0, 0.0, 0.0}, a1 = a0, b0 = a0, b1 = a0;
    if (!(wid & 1)) {  // by = 0 (4 steps) and by = 3 (16 steps)
#pragma unroll
        for (int kk = 0; kk < 16; kk += 2) {
            const double s0 = bop(kk), s1 = bop(kk + 1);
            b0 = __builtin_amdgcn_mfma_f64_16x16x4f64(wop(3, kk), s0, b0, 0, 0, 0);
            if (kk < 4) a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(wop(0, kk), s0, a0, 0, 0, 0);
            b1 = __builtin_amdgcn_mfma_f64_16x16x4f64(wop(3, kk + 1), s1, b1, 0, 0, 0);
            if (kk < 4) a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(wop(0, kk + 1), s1, a1, 0, 0, 0);
        }
    } else {  // by = 1 (8 steps) and by = 2 (12 steps)
#pragma unroll
        for (int kk = 0; kk < 12; kk += 2) {
            const double s0 = bop(kk), s1 = bop(kk + 1);
            b0 = __builtin_amdgcn_mfma_f64_16x16x4f64(wop(2, kk), s0, b0, 0, 0, 0);
            if (kk < 8) a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(wop(1, kk), s0, a0, 0, 0, 0);
            b1 = __builtin_amdgcn_mfma_f64_16x16x4f64(wop(2, kk + 1), s1, b1, 0, 0, 0);
            if (kk < 8) a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(wop(1, kk + 1), s1, a1, 0, 0, 0);
        }
    }
    lo = a0 + a1;
    hi = b0 + b1;
}

__device__ __forceinline__ void wl_put(double (*L)[65], const v4d &lo, const v4d &hi) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, ubx = wid >> 1;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int by = (wid & 1) ? (h ? 2 : 1) : (h ? 3 : 0);
        const v4d &v = h ? hi : lo;
#pragma unroll
        for (int r = 0; r < 4; ++r)
            L[by * 16 + (lane >> 4) + 4 * r][ubx * 16 + (lane & 15)] = v[r];
    }
}

#define MM_FOR(h, r, y, x)                                                                  \
    for (int h = 0; h < 2; ++h)                                                             \
        for (int r = 0; r < 4; ++r)                                                         \
            if (const int blk_ = (threadIdx.x >> 6) * 2 + h, y = (blk_ & 3) * 16 +           \
                                                             ((threadIdx.x & 63) >> 4) + 4 * r, \
                      x = (blk_ >> 2) * 16 + (threadIdx.x & 15); true)

// Eliminate the SPD diagonal block held in T (upper triangle used; the lower part may hold
// anything finite); on return T[y][x] holds W = U^-T (lower triangular) and piv[] the pivots.
// Wave w owns rows 8w .. 8w+7 of [A | I] (lane = columns 2l, 2l+1).  Pipelined groups
// (tools/elim_bench.hip, V6: 9.3 us vs 13.7 us for the barrier-per-group scheme):
//   the producing wave w factors its 8 rows in-wave (readlane broadcasts with compile-time
//   lane indices, priority 3) and publishes every pivot row the moment it is final: the
//   scaled row [A | I] / p into ROWS and the unscaled A part (the multipliers) into MUL, then
//   bumps an LDS counter;
//   every later wave applies each published row to its own rows as soon as the counter
//   passes it (no workgroup barrier between groups), so the next producer starts one
//   rank-1 update after the previous group's last pivot.
// The multipliers of a symmetric elimination come from the pivot row's upper part, and the
// I part of pivot row c is zero beyond column c, so no entry needs masking.
// ROWS (64 x 128) may alias any LDS except T/MUL; MUL (64 x 64) aliases T (T is read into
// registers first; W is written back after a barrier).  cnt: an LDS int.
template <int W>
__device__ __forceinline__ void elim_produce(double (&a)[8][2], double (*ROWS)[128],
                                            double (*MUL)[64], double *piv,
                                            volatile __attribute__((address_space(3))) int *vc) {
    const int lane = threadIdx.x & 63, c0 = lane * 2;
#pragma unroll
    for (int ci = 0; ci < 8; ++ci) {
        const int c = 8 * W + ci;
        const double pv = readlane_d(a[ci][ci & 1], 4 * W + (ci >> 1));
        const double inv = fast_rcp(pv);
        const double rs0 = a[ci][0] * inv, rs1 = a[ci][1] * inv;
#pragma unroll
        for (int i = ci + 1; i < 8; ++i) {
            const double m = readlane_d(a[ci][i & 1], 4 * W + (i >> 1));
            a[i][0] = __builtin_fma(-m, rs0, a[i][0]);
            a[i][1] = __builtin_fma(-m, rs1, a[i][1]);
        }
        if (W < 7) {
            *(double2 *)&ROWS[c][c0] = make_double2(rs0, rs1);
            if (lane < 32) *(double2 *)&MUL[c][c0] = make_double2(a[ci][0], a[ci][1]);
            asm volatile("" ::: "memory");
            if (lane == 0) *vc = c + 1;
        }
        if (lane == 0) piv[c] = pv;
    }
}

// The chain's next hand-off tiles (k, k+1) -> S and (k+1, k+1) -> Q, fetched by waves 0..3
// once their pivot groups are done (they are idle for the rest of the elimination): each
// polls the two flags and has its sc1 loads in flight before the post-elimination barrier,
// so the tiles land in LDS without a separate acquire + load phase.
struct HandoffPrefetch {
    const unsigned int *f1, *f2;  // nullptr: no prefetch (last step)
    unsigned int ep;
    const double *t1, *t2;        // tile origins in the column-major matrix
    int lda;
    double (*S)[65], (*Q)[65];
};

__device__ __forceinline__ void diag_eliminate(double (*T)[65], double (*ROWS)[128], double *piv,
                                               int *cnt, uint32_t *err,
                                               unsigned long long *gts = nullptr,
                                               const HandoffPrefetch *pf = nullptr) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int r0 = wid * 8, c0 = lane * 2;
    double(*MUL)[64] = (double(*)[64]) & T[0][0];
    double a[8][2];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int row = r0 + i, col = c0 + q;
            a[i][q] = (col < 64) ? T[row][col] : ((col - 64 == row) ? 1.0 : 0.0);
        }
    if (tid == 0) *cnt = 0;
    __syncthreads();  // T is in registers: MUL may overwrite it
    volatile __attribute__((address_space(3))) int *vc =
        (volatile __attribute__((address_space(3))) int *)cnt;
    // ---- apply the pivot rows of the earlier groups as they are published ----
    // (the counter is read only when the rows already seen are used up, so a wave that
    // lags applies its backlog without LDS round trips)
    int avail = 0;
    for (int c = 0; c < r0; ++c) {
        if (c >= avail) {
            for (unsigned spins = 0; (avail = *vc) <= c;) {
                if (++spins > (1u << 22)) {  // bounded: a broken hand-off flags, never hangs
                    if (lane == 0 && err) atomicOr(err, 16u);
                    avail = r0;
                    break;
                }
            }
            asm volatile("" ::: "memory");
        }
        const double2 v = *(const double2 *)&ROWS[c][c0];
#pragma unroll
        for (int i = 0; i < 8; i += 2) {
            const double2 mm = *(const double2 *)&MUL[c][r0 + i];
            a[i][0] = __builtin_fma(-mm.x, v.x, a[i][0]);
            a[i][1] = __builtin_fma(-mm.x, v.y, a[i][1]);
            a[i + 1][0] = __builtin_fma(-mm.y, v.x, a[i + 1][0]);
            a[i + 1][1] = __builtin_fma(-mm.y, v.y, a[i + 1][1]);
        }
    }
    // ---- my group: 8 pivots in-wave (compile-time lane indices) ----
    if (gts && lane == 0) gts[wid] = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_setprio(3);
    switch (wid) {
        case 0: elim_produce<0>(a, ROWS, MUL, piv, vc); break;
        case 1: elim_produce<1>(a, ROWS, MUL, piv, vc); break;
        case 2: elim_produce<2>(a, ROWS, MUL, piv, vc); break;
        case 3: elim_produce<3>(a, ROWS, MUL, piv, vc); break;
        case 4: elim_produce<4>(a, ROWS, MUL, piv, vc); break;
        case 5: elim_produce<5>(a, ROWS, MUL, piv, vc); break;
        case 6: elim_produce<6>(a, ROWS, MUL, piv, vc); break;
        default: elim_produce<7>(a, ROWS, MUL, piv, vc); break;
    }
    __builtin_amdgcn_s_setprio(0);
    if (gts && lane == 0) gts[8 + wid] = __builtin_amdgcn_s_memrealtime();
    const bool fetch = pf && pf->f1 && wid < 4;
    double h1[16], h2[16];
    if (fetch) {
        for (SpinGuard sg;;) {
            const unsigned int v1 = __hip_atomic_load(pf->f1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned int v2 = __hip_atomic_load(pf->f2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__builtin_amdgcn_readfirstlane((int)(v1 == pf->ep && v2 == pf->ep))) break;
            __builtin_amdgcn_s_sleep(2);
            if (sg.expired(err)) break;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int e = tid + q * 256, y = e & 63, x = e >> 6;
            h1[q] = ld_sc1(&pf->t1[(size_t)y + (size_t)x * pf->lda]);
            h2[q] = ld_sc1(&pf->t2[(size_t)y + (size_t)x * pf->lda]);
        }
    }
    __syncthreads();  // every wave is done with MUL (= T) and ROWS (= S, Q)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const double pv = piv[r0 + i];
        if (lane == 0 && err && !(pv > 0.0)) atomicOr(err, 8u);
        // 1/sqrt(p): v_rsq_f64 + two Newton steps (full fp64 accuracy, no IEEE sequences)
        double r = __builtin_amdgcn_rsq(pv);
        r = r * __builtin_fma(-0.5 * pv * r, r, 1.5);
        r = r * __builtin_fma(-0.5 * pv * r, r, 1.5);
#pragma unroll
        for (int q = 0; q < 2; ++q)
            if (c0 + q >= 64) T[r0 + i][c0 + q - 64] = a[i][q] * r;
    }
    if (fetch) {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int e = tid + q * 256, y = e & 63, x = e >> 6;
            pf->S[y][x] = h1[q];
            pf->Q[y][x] = h2[q];
        }
    }
    __syncthreads();
}

// ---------------------------------------------------------------------------
// Chain v2 (round 3): the post-elimination products leave the critical path.
// v1 runs, per 64-block step, elimination (10.9 us at m = 2048) -> W pass -> U_{k,k+1} =
// W_k A_{k,k+1} (1.8 us) -> D_{k+1} = A_{k+1,k+1} - U'U (2.0 us) -> publish: ~17 us.  Here:
//   - the pivot rows are published without the separate multiplier array (consumers take the
//     multiplier from the scaled row and rescale the row by p_c), which frees the LDS for the
//     hand-off tile S = A_{k,k+1} and the U rows during the elimination;
//   - W_k rows go to global memory from the producing wave's registers as soon as its group
//     is done; W_k is published when the last wave's stores have drained;
//   - once S has arrived (the hand-off lands ~7.5 us after W_{k-1}) and row blocks 0-2 are
//     eliminated, waves 0-5 form U rows 0..47 (U = W_k S = sqrt(p) ROWS_I S, fp64 MFMA) and
//     the partial D_{k+1} = A_{k+1,k+1} - sum_{s < 48} U_s' U_s of the 10 upper 16x16 blocks,
//     while waves 6-7 are still pivoting;
//   - after the last pivot only U row block 3 (waves 4-7, 16 MFMAs each) and the last four
//     K steps of D_{k+1} remain: the next elimination starts ~0.5 us after the last pivot.
// Same flags, tiles and owners as v1; U_{k,k+1} is published by the last of its storing waves.
// ---------------------------------------------------------------------------
// pivot-row stride: 128 + 2 doubles, so the 16 rows an MFMA A-operand read touches (rows
// 16 by + (lane & 15), one column) fall in distinct LDS banks (a 128-double stride put them
// all in one bank: 16-way conflicts on every U operand); 16-byte aligned for the double2
// row stores
constexpr int kRowsLd = 130;

__device__ __forceinline__ void lds_wait_ge(const volatile __attribute__((address_space(3))) int *p,
                                            int v, uint32_t *err) {
    for (unsigned spins = 0; *p < v;) {
        __builtin_amdgcn_s_sleep(1);  // a waiting wave leaves the LDS and issue slots to the
                                      // producers it waits for
        if (++spins > (1u << 22)) {  // bounded: a broken hand-off flags, never hangs
            if ((threadIdx.x & 63) == 0 && err) atomicOr(err, 16u);
            break;
        }
    }
    asm volatile("" ::: "memory");
}

// lane 0 adds 1 to an LDS counter; returns the value before (uniform across the wave)
__device__ __forceinline__ int lds_bump(int *p) {
    int old = 0;
    asm volatile("" ::: "memory");
    if ((threadIdx.x & 63) == 0)  // release: this wave's earlier LDS / drained stores first
        old = __hip_atomic_fetch_add(p, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    return __builtin_amdgcn_readfirstlane(old);
}

template <int W>
__device__ __forceinline__ void elim_produce2(double (&a)[8][2], double (*ROWS)[kRowsLd], double *piv,
                                             volatile __attribute__((address_space(3))) int *vc) {
    const int lane = threadIdx.x & 63, c0 = lane * 2;
#pragma unroll
    for (int ci = 0; ci < 8; ++ci) {
        const int c = 8 * W + ci;
        const double pv = readlane_d(a[ci][ci & 1], 4 * W + (ci >> 1));
        const double inv = fast_rcp(pv);
        const double rs0 = a[ci][0] * inv, rs1 = a[ci][1] * inv;
#pragma unroll
        for (int i = ci + 1; i < 8; ++i) {
            const double m = readlane_d(a[ci][i & 1], 4 * W + (i >> 1));
            a[i][0] = __builtin_fma(-m, rs0, a[i][0]);
            a[i][1] = __builtin_fma(-m, rs1, a[i][1]);
        }
        *(double2 *)&ROWS[c][c0] = make_double2(rs0, rs1);
        if (lane == 0) piv[c] = pv;
        asm volatile("" ::: "memory");
        if (lane == 0) *vc = c + 1;
    }
}

// U block (by, bx) of U = W S, W = diag(sqrt p) ROWS_I (lower triangular: K steps < 4 by + 4)
__device__ __forceinline__ v4d u_block2(const double (*ROWS)[kRowsLd], const double (*S)[65],
                                        const double *piv, int by, int bx) {
    const int lane = threadIdx.x & 63, ry = by * 16 + (lane & 15), cx = bx * 16 + (lane & 15);
    v4d a0 = {0.0, 0.0, 0.0, 0.0}, a1 = a0;
    const int nk = 4 * by + 4;
    for (int kk = 0; kk < nk; kk += 2) {
        const int s0 = 4 * kk + (lane >> 4);
        a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(ROWS[ry][64 + s0], S[s0][cx], a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(ROWS[ry][68 + s0], S[s0 + 4][cx], a1, 0, 0, 0);
    }
    v4d u = a0 + a1;
#pragma unroll
    for (int r = 0; r < 4; ++r) u[r] *= sqrt(piv[by * 16 + (lane >> 4) + 4 * r]);
    return u;
}

// U block -> LDS rows (T) and the (k, k+1) tile of A (write-through, for the owners)
__device__ __forceinline__ void u_put2(double (*T)[65], double *A, int lda, int k, int by, int bx,
                                       const v4d &u) {
    const int lane = threadIdx.x & 63, x = bx * 16 + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int y = by * 16 + (lane >> 4) + 4 * r;
        T[y][x] = u[r];
        st_sc1(&A[(size_t)(k * kNB + y) + (size_t)((k + 1) * kNB + x) * lda], u[r]);
    }
}

// acc += sum_{s in [4 k0, 4 k1)} U[s][16 by + .]' U[s][16 bx + .]
__device__ __forceinline__ void dprime_acc2(const double (*T)[65], int by, int bx, int k0, int k1,
                                            v4d &acc) {
    const int lane = threadIdx.x & 63, cy = by * 16 + (lane & 15), cx = bx * 16 + (lane & 15);
    for (int kk = k0; kk < k1; ++kk) {
        const int s0 = 4 * kk + (lane >> 4);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(T[s0][cy], T[s0][cx], acc, 0, 0, 0);
    }
}

// Phase a on waves 0-5, U row block 3 on waves 4-7.  V = 2 drains stores and releases W_k /
// U_{k,k+1} through LDS counters as they complete; V = 3 forms the partial next diagonal
// block before polling the (k+1, k+1) hand-off and drains every store once, before the
// step's closing barrier, releasing both flags after it (v1's release).
template <int V>
__device__ void chol_chain_v2(double *A, int lda, int nblk, int ncb, double *Wd,
                              const CholFlags &F, uint32_t *err, unsigned long long *trace,
                              double *L) {
    double(*T)[65] = (double(*)[65])L;                 // U_{k,k+1} rows
    double(*S)[65] = (double(*)[65])(L + 4160);        // hand-off A_{k,k+1}
    double(*ROWS)[kRowsLd] = (double(*)[kRowsLd])(L + 8320);  // pivot rows [A | I] / p
    double(*Dn)[65] = (double(*)[65])(L + 8320);       // next diagonal block (aliases ROWS)
    __shared__ double piv[64];
    __shared__ int cnt, s_ready, ua_cnt, w_drain, u_drain;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int r0 = wid * 8, c0 = lane * 2;
    volatile __attribute__((address_space(3))) int *vc =
        (volatile __attribute__((address_space(3))) int *)&cnt;
    auto vlds = [](int *p) {
        return (volatile __attribute__((address_space(3))) int *)p;
    };
    // D_{k+1} blocks of this wave (waves 0-5; upper blocks in order (0,0) (0,1) (1,1) (0,2)
    // (1,2) (2,2) (0,3) (1,3) (2,3) (3,3)): waves 0-3 take blocks w and w + 4, waves 4-5
    // blocks 8 and 9
    auto bxy = [](int blk, int &by, int &bx) {
        bx = blk < 1 ? 0 : blk < 3 ? 1 : blk < 6 ? 2 : 3;
        by = blk - bx * (bx + 1) / 2;
    };
    const bool pa = wid < 6;  // a phase-a wave
    int nd = wid < 4 ? 2 : wid < 6 ? 1 : 0;
    int dby[3] = {0, 0, 0}, dbx[3] = {0, 0, 0};
    if (wid < 4) {
        bxy(wid, dby[0], dbx[0]);
        bxy(wid + 4, dby[1], dbx[1]);
    } else if (wid < 6) {
        bxy(wid + 4, dby[0], dbx[0]);
    }
#define CHAIN2_TS(slot)                                                                 \
    do {                                                                                \
        if (trace && lane == 0) trace[k * 32 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
    tile_load(Dn, A, lda, 0, 0, true);
    for (int k = 0; k < nblk; ++k) {
        if (V != 3 || k == 0) __syncthreads();  // Dn (the diagonal block) complete
        double a[8][2];
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int row = r0 + i, col = c0 + q;
                a[i][q] = (col < 64) ? Dn[row][col] : ((col - 64 == row) ? 1.0 : 0.0);
            }
        if (tid == 0) cnt = s_ready = ua_cnt = w_drain = u_drain = 0;
        __syncthreads();  // a[][] in registers: ROWS (= Dn) may be overwritten
        if (wid == 0) CHAIN2_TS(0);
        // ---- apply the earlier groups' pivot rows as they are published ----
        int avail = 0;
        for (int c = 0; c < r0; ++c) {
            if (c >= avail) {
                for (unsigned spins = 0; (avail = *vc) <= c;) {
                    if (++spins > (1u << 22)) {
                        if (lane == 0) atomicOr(err, 16u);
                        avail = r0;
                        break;
                    }
                }
                asm volatile("" ::: "memory");
            }
            const double2 v = *(const double2 *)&ROWS[c][c0];
            const double pc = piv[c];
            const double vx = v.x * pc, vy = v.y * pc;  // the unscaled pivot row
#pragma unroll
            for (int i = 0; i < 8; i += 2) {
                const double2 mm = *(const double2 *)&ROWS[c][r0 + i];  // multipliers / p_c
                a[i][0] = __builtin_fma(-mm.x, vx, a[i][0]);
                a[i][1] = __builtin_fma(-mm.x, vy, a[i][1]);
                a[i + 1][0] = __builtin_fma(-mm.y, vx, a[i + 1][0]);
                a[i + 1][1] = __builtin_fma(-mm.y, vy, a[i + 1][1]);
            }
        }
        // ---- my group: 8 pivots in-wave ----
        __builtin_amdgcn_s_setprio(3);
        switch (wid) {
            case 0: elim_produce2<0>(a, ROWS, piv, vc); break;
            case 1: elim_produce2<1>(a, ROWS, piv, vc); break;
            case 2: elim_produce2<2>(a, ROWS, piv, vc); break;
            case 3: elim_produce2<3>(a, ROWS, piv, vc); break;
            case 4: elim_produce2<4>(a, ROWS, piv, vc); break;
            case 5: elim_produce2<5>(a, ROWS, piv, vc); break;
            case 6: elim_produce2<6>(a, ROWS, piv, vc); break;
            default: elim_produce2<7>(a, ROWS, piv, vc); break;
        }
        __builtin_amdgcn_s_setprio(0);
        if (wid == 7) CHAIN2_TS(1);
        // ---- my rows of W_k = U_kk^-T (the I part / sqrt p) to global memory ----
        double *Wk = Wd + (size_t)k * kNB * kNB;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const double pv = piv[r0 + i];
            if (lane == 0 && !(pv > 0.0)) atomicOr(err, 8u);
            double r = __builtin_amdgcn_rsq(pv);
            r = r * __builtin_fma(-0.5 * pv * r, r, 1.5);
            r = r * __builtin_fma(-0.5 * pv * r, r, 1.5);
            if (lane >= 32) {
#pragma unroll
                for (int q = 0; q < 2; ++q)
                    st_sc1(&Wk[(size_t)(c0 + q - 64) * kNB + r0 + i], a[i][q] * r);
            }
        }
        if (wid == 7) CHAIN2_TS(2);
        if (k + 1 == nblk) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lds_bump(&w_drain) == 7 && lane == 0)
                __hip_atomic_store(&F.W[k], F.ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
        // (the W stores drain behind this wave's U work; W_k is released before the barrier)
        // ---- the hand-off tile S = A_{k,k+1} (updated by its owner through step k-1) ----
        if (wid < 4) {
            const unsigned int *f1 = &F.R[2 * k + 1];
            for (SpinGuard sg;;) {
                const unsigned int v1 = __hip_atomic_load(f1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (__builtin_amdgcn_readfirstlane((int)(v1 == F.ep))) break;
                __builtin_amdgcn_s_sleep(2);
                if (sg.expired(err)) break;
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const double *t1 = A + (size_t)k * kNB + (size_t)(k + 1) * kNB * lda;
            double h[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int e = tid + q * 256, y = e & 63, x = e >> 6;
                h[q] = ld_sc1(&t1[(size_t)y + (size_t)x * lda]);
            }
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int e = tid + q * 256, y = e & 63, x = e >> 6;
                S[y][x] = h[q];
            }
            asm volatile("" ::: "memory");
            lds_bump(&s_ready);
        }
        v4d dacc[3] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};
        double qv[3][4] = {};
        if (pa) {
            // ---- phase a: U rows 0..47 and the partial next diagonal block ----
            lds_wait_ge(vc, 48, err);
            lds_wait_ge(vlds(&s_ready), 4, err);
            if (wid < 4) {
                const v4d u2 = u_block2(ROWS, S, piv, 2, wid);
                u_put2(T, A, lda, k, 2, wid, u2);
                const v4d u0 = u_block2(ROWS, S, piv, 0, wid);
                u_put2(T, A, lda, k, 0, wid, u0);
            } else {
                const int b0 = 2 * (wid - 4);
                const v4d ua = u_block2(ROWS, S, piv, 1, b0);
                u_put2(T, A, lda, k, 1, b0, ua);
                const v4d ub = u_block2(ROWS, S, piv, 1, b0 + 1);
                u_put2(T, A, lda, k, 1, b0 + 1, ub);
            }
            lds_bump(&ua_cnt);  // this wave's U rows are in T (LDS, in order)
            if (V == 2) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // W rows and U blocks
                lds_bump(&u_drain);
                if (lds_bump(&w_drain) == 7 && lane == 0)
                    __hip_atomic_store(&F.W[k], F.ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                // V = 3: the partial next diagonal block needs only U rows 0..47, not the
                // (k+1, k+1) hand-off (subtracted at the end)
                lds_wait_ge(vlds(&ua_cnt), 6, err);
                for (int d = 0; d < nd; ++d) dprime_acc2(T, dby[d], dbx[d], 0, 12, dacc[d]);
            }
            // the (k+1, k+1) hand-off: this wave's D blocks of A_{k+1,k+1}
            const unsigned int *f2 = &F.R[2 * (k + 1)];
            for (SpinGuard sg;;) {
                const unsigned int v2 = __hip_atomic_load(f2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (__builtin_amdgcn_readfirstlane((int)(v2 == F.ep))) break;
                __builtin_amdgcn_s_sleep(2);
                if (sg.expired(err)) break;
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const double *t2 = A + (size_t)(k + 1) * kNB + (size_t)(k + 1) * kNB * lda;
            for (int d = 0; d < nd; ++d)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int y = dby[d] * 16 + (lane >> 4) + 4 * r, x = dbx[d] * 16 + (lane & 15);
                    qv[d][r] = ld_sc1(&t2[(size_t)y + (size_t)x * lda]);
                }
            if (wid == 0) CHAIN2_TS(6);
            if (wid == 4) CHAIN2_TS(4);
            if (V == 2) {
                lds_wait_ge(vlds(&ua_cnt), 6, err);
                for (int d = 0; d < nd; ++d) dprime_acc2(T, dby[d], dbx[d], 0, 12, dacc[d]);
            }
        }
        const bool pb = wid >= 4;  // a U-row-block-3 wave
        if (pb) {
            // ---- phase b: U row block 3, once every pivot is published ----
            lds_wait_ge(vc, 64, err);
            lds_wait_ge(vlds(&s_ready), 4, err);
            const int bx = wid - 4;
            const v4d u3 = u_block2(ROWS, S, piv, 3, bx);
            u_put2(T, A, lda, k, 3, bx, u3);
            if (wid == 7) CHAIN2_TS(3);
            if (V == 2 && wid >= 6) {  // waves 6-7 have not released their W rows yet
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (lds_bump(&w_drain) == 7 && lane == 0)
                    __hip_atomic_store(&F.W[k], F.ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();  // U complete in T; every read of ROWS and S done
        if (wid == 0) CHAIN2_TS(5);
        for (int d = 0; d < nd; ++d) {
            dprime_acc2(T, dby[d], dbx[d], 12, 16, dacc[d]);
            const int by = dby[d], bx = dbx[d];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int y = by * 16 + (lane >> 4) + 4 * r, x = bx * 16 + (lane & 15);
                Dn[y][x] = (y <= x) ? qv[d][r] - dacc[d][r] : 0.0;
                if (by != bx) Dn[x][y] = 0.0;  // the mirrored lower block
            }
        }
        if (V == 2) {
            if (wid >= 4) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (lds_bump(&u_drain) == 9 && lane == 0)
                    __hip_atomic_store(&F.P[k * F.ncb + k + 1], F.ep, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            }
        } else {
            // V = 3: every wave drains its own W-row and U-block stores (long issued for all
            // but the last producers) before the step's closing barrier; W_k and U_{k,k+1} are
            // then released together by one thread after it (as v1 releases them)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) {
                __hip_atomic_store(&F.W[k], F.ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&F.P[k * F.ncb + k + 1], F.ep, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (wid == 0) CHAIN2_TS(7);
    }
#undef CHAIN2_TS
}

#include "bb_chol4.h"

template <int V>
__global__ __launch_bounds__(512) void k_chol_persistent(double *A, int lda, int nblk, int ncb,
                                                         double *Wd, CholFlags F,
                                                         uint32_t *err,
                                                         unsigned long long *trace, const int *gate) {
    if (gated(gate)) return;
    // T: tile being updated / the chain's diagonal block -> W; S: staging U_ki / the chain's
    // A_{k,k+1} -> U_{k,k+1}; Q: staging U_kj / W_i / the chain's next diagonal block.
    // During the v1 chain's elimination S and Q together hold the published pivot rows; the
    // v2 chain (chol_chain_v2) lays out U rows, S and the pivot rows side by side.
    constexpr bool kV2 = V == 2 || V == 3;  // the pipelined chains
    constexpr bool kV4 = V == 4;            // the 16-column leaf pipeline (bb_chol4.h)
    __shared__ __attribute__((aligned(16))) double Lraw[kV4 ? 4 * 64 * kC4Ld
                                                        : kV2 ? 8320 + 64 * 130 : 3 * 64 * 65];
    double(*Lb)[64][65] = (double(*)[64][65])Lraw;
    __shared__ double piv[64];
    __shared__ int cnt;
    __shared__ int pre_ready;  // owner: the next update's panels are published
    double(*T)[65] = Lb[0];
    double(*S)[65] = Lb[1];
    double(*Q)[65] = Lb[2];
    const int tid = threadIdx.x;
    v4d acc[2];
    if (blockIdx.x == 0) {
        // ------------------------------ the chain ------------------------------
        if constexpr (kV4) {
            chol_chain_v4(A, lda, nblk, ncb, Wd, F, err, trace, Lraw);
            return;
        } else if constexpr (kV2) {
            chol_chain_v2<V>(A, lda, nblk, ncb, Wd, F, err, trace, Lraw);
            return;
        }
        const int lane = tid & 63, wid = tid >> 6;
        double(*ROWS)[128] = (double(*)[128]) & Lb[1][0][0];
        tile_load(T, A, lda, 0, 0, true);
        __syncthreads();
#define CHAIN_TS(slot)                                                                  \
    do {                                                                                \
        if (trace && tid == 0) {                                                        \
            trace[k * 32 + (slot)] = __builtin_amdgcn_s_memrealtime();                    \
            trace[k * 32 + 8 + (slot)] = __builtin_amdgcn_s_memtime();                    \
        }                                                                               \
    } while (0)
        for (int k = 0; k < nblk; ++k) {
            CHAIN_TS(0);
            // hand-off tiles (k, k+1) -> S, (k+1, k+1) -> Q (updated by their owners through
            // step k-1) are fetched during the elimination by the waves done pivoting
            HandoffPrefetch pf{nullptr, nullptr, F.ep, nullptr, nullptr, lda, S, Q};
            if (k + 1 < nblk) {
                pf.f1 = &F.R[2 * k + 1];
                pf.f2 = &F.R[2 * (k + 1)];
                pf.t1 = A + (size_t)k * kNB + (size_t)(k + 1) * kNB * lda;
                pf.t2 = A + (size_t)(k + 1) * kNB + (size_t)(k + 1) * kNB * lda;
            }
            diag_eliminate(T, ROWS, piv, &cnt, err, trace ? trace + k * 32 + 16 : nullptr, &pf);
            CHAIN_TS(1);
            double *W = Wd + (size_t)k * kNB * kNB;
            for (int e = tid; e < 64 * 64; e += 512) {  // stores drain behind the next work
                const int y = e & 63, x = e >> 6;
                st_sc1(&W[(size_t)x * kNB + y], T[y][x]);  // W[y][x], column-major
            }
            CHAIN_TS(2);
            if (k + 1 < nblk) {
                CHAIN_TS(3);
                CHAIN_TS(4);
                // U_{k,k+1}[r][x] = sum_{s <= r} W[r][s] S[s][x]  (W = T lower triangular):
                // block row by needs K steps 0 .. 4 by + 3 only; wave w takes column block
                // w >> 1 and the row-block pair {0, 3} or {1, 2} (20 MFMAs per wave), the
                // two blocks' chains interleaved and the longer one split even / odd
                // U_{k,k+1} = W_k A_{k,k+1}  (W = T lower triangular)
                wl_times(T, S, acc[0], acc[1]);
                __syncthreads();  // all reads of S (and of W in T) done
                wl_put(S, acc[0], acc[1]);  // U_{k,k+1}
                __syncthreads();
                tile_store(S, A, lda, k, k + 1);  // coalesced; drains behind D_{k+1}
                CHAIN_TS(5);
                // D_{k+1} = A_{k+1,k+1} - U' U on the 10 upper 16x16 blocks (waves 0, 1 take
                // two, all chains interleaved and split even / odd); the strictly lower
                // blocks of T are zeroed
                {
                    // upper blocks in order (0,0) (0,1) (1,1) (0,2) (1,2) (2,2) (0,3) ...
                    auto bxy = [](int blk, int &by, int &bx) {
                        bx = blk < 1 ? 0 : blk < 3 ? 1 : blk < 6 ? 2 : 3;
                        by = blk - bx * (bx + 1) / 2;
                    };
                    int by0, bx0, by1, bx1;
                    bxy(wid, by0, bx0);
                    bxy(8 + (wid & 1), by1, bx1);
                    auto sop = [&](int kk, int b) {
                        return S[kk * 4 + (lane >> 4)][b * 16 + (lane & 15)];
                    };
                    v4d d0 = {0.0, 0.0, 0.0, 0.0}, d1 = d0, e0 = d0, e1 = d0;
                    if (wid < 2) {
#pragma unroll
                        for (int kk = 0; kk < 16; kk += 2) {
                            d0 = __builtin_amdgcn_mfma_f64_16x16x4f64(sop(kk, by0), sop(kk, bx0), d0, 0, 0, 0);
                            e0 = __builtin_amdgcn_mfma_f64_16x16x4f64(sop(kk, by1), sop(kk, bx1), e0, 0, 0, 0);
                            d1 = __builtin_amdgcn_mfma_f64_16x16x4f64(sop(kk + 1, by0), sop(kk + 1, bx0), d1, 0, 0, 0);
                            e1 = __builtin_amdgcn_mfma_f64_16x16x4f64(sop(kk + 1, by1), sop(kk + 1, bx1), e1, 0, 0, 0);
                        }
                    } else {
#pragma unroll
                        for (int kk = 0; kk < 16; kk += 2) {
                            d0 = __builtin_amdgcn_mfma_f64_16x16x4f64(sop(kk, by0), sop(kk, bx0), d0, 0, 0, 0);
                            d1 = __builtin_amdgcn_mfma_f64_16x16x4f64(sop(kk + 1, by0), sop(kk + 1, bx0), d1, 0, 0, 0);
                        }
                    }
                    const v4d dd = d0 + d1, ee = e0 + e1;
                    auto put = [&](int by, int bx, const v4d &d) {
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int y = by * 16 + (lane >> 4) + 4 * r, x = bx * 16 + (lane & 15);
                            T[y][x] = (y <= x) ? Q[y][x] - d[r] : 0.0;
                            if (by != bx) T[x][y] = 0.0;  // the mirrored lower block
                        }
                    };
                    put(by0, bx0, dd);
                    if (wid < 2) put(by1, bx1, ee);
                }
                CHAIN_TS(6);
                // publish W_k and U_{k,k+1} together (their sc1 stores have drained meanwhile)
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (tid == 0) {
                    __hip_atomic_store(&F.W[k], F.ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(&F.P[k * F.ncb + k + 1], F.ep, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                }
            } else {
                flag_release(&F.W[k], F.ep);
            }
            CHAIN_TS(7);
        }
#undef CHAIN_TS
        return;
    }
    // ------------------------------ tile owners ------------------------------
    double *Hs = Wd + (size_t)nblk * kNB * kNB;  // scratch tiles behind the W_k blocks
    const int nowner = gridDim.x - 1;
    int n = blockIdx.x - 1;
    int ti = 0, tj = 0, base = 0;  // tile (ti, tj) = the n-th tile in row-major order
    for (;; n += nowner) {
        while (ti < nblk && n - base >= ncb - ti) {
            base += ncb - ti;
            ++ti;
        }
        if (ti >= nblk) break;
        tj = ti + (n - base);
        const int i = ti, j = tj;
        if (i == 0 && j == 0) continue;  // the chain starts from A_00 itself
        const bool diag = (j == i);
        const bool handoff = diag || (j == i + 1 && j < nblk);
        // (i, i+2): only updated and stored; the owner of (i+1, i+2) forms U_{i,i+2} itself
        // (one flag hop less on the path that feeds the chain).  (0, 2) is read raw.
        // (i, i+2): updated through step i-1 and stored into the scratch tile Hs[i] (raw for
        // i = 0) for the owners of (i+1, i+2) and (i+2, i+2), which form U_{i,i+2} from it;
        // the published U_{i,i+2} must not alias it (those two read it at different times)
        const bool hstore = (j == i + 2 && j < nblk);
        // (i, i+1), i >= 1, and (i, i), i >= 2: the last owner update k (k = i-1 resp. i-2)
        // needs U_{k,j} with j = k+2, which the owner forms itself from W_k and the stored
        // tile (k, k+2): the hand-offs are one flag hop behind W_k
        const bool merge = (j == i + 1 && j < nblk && i >= 1);
        const bool dmerge = diag && i >= 2;
        const int nupd = diag ? i - 1 : i;  // (i,i): updates 0..i-2, the chain applies i-1
        const int nstd = (merge || dmerge) ? nupd - 1 : nupd;
        bool pub = false;  // merge: U_{k,j} (in Q) is published with the hand-off
        // owner trace (bb_bench_chol): hop B = hand-off tile (kt, kt+1), hop A = (kt-1, kt+1),
        // D = the diagonal hand-off (kt+1, kt+1)
        const int kt = nblk >= 48 ? nblk / 2 : 6;  // the middle step for large m
        unsigned long long *otr = nullptr;
        if (trace && nblk > kt + 1) {
            if (i == kt && j == kt + 1) otr = trace + (size_t)nblk * 32 + 8;
            if (i == kt - 1 && j == kt + 1) otr = trace + (size_t)nblk * 32;
            if (i == kt + 1 && j == kt + 1) otr = trace + (size_t)nblk * 32 + 16;
        }
#define OWN_TS(slot)                                                                \
    do {                                                                            \
        if (otr && tid == 0) otr[slot] = __builtin_amdgcn_s_memrealtime();          \
    } while (0)
        tile_load(T, A, lda, i, j, diag);
        OWN_TS(6);  // traced hand-off tiles: when the owner started the tile
        __syncthreads();
        // An owner that lags the chain finds the next panels already published: their loads
        // (into registers) are issued before this update's MFMAs and land in S / Q after
        // them, so a lagging owner's update costs max(load, MFMA) instead of their sum
        // (at m = 5120 the owners, not the chain, set the pace through the middle third).
        // The updates sum in the MFMA accumulators, T -= sum once at the end: no LDS
        // read-modify-write of T and one barrier fewer per update.
        // Round 3: a catching-up owner checked the next panel's flags once per update (one
        // serial L2 round trip per update, issued by thread 0 before the barrier); now wave 0
        // checks up to eight upcoming panels at once and the owner remembers how far they are
        // published (ready_to), so most updates of a catch-up skip the check.
        bool have = false;  // S (and Q) already hold panel k
        int ready_to = -1;  // panels <= ready_to are known to be published (uniform)
        acc[0] = acc[1] = (v4d){0.0, 0.0, 0.0, 0.0};
        for (int k = 0; k < nstd; ++k) {
            if (k == nupd - 1) OWN_TS(0);
            if (!have) {
                flag_acquire2(&F.P[k * F.ncb + i], diag ? nullptr : &F.P[k * F.ncb + j], F.ep,
                              err);
                if (k == nupd - 1) OWN_TS(1);
                tile_load(S, A, lda, k, i, false);
                if (!diag) tile_load(Q, A, lda, k, j, false);
                if (ready_to < k) ready_to = k;
            }
            if (k + 1 < nstd && k + 1 > ready_to) {
                if (tid < 64) {
                    const int kk = k + 1 + (int)tid;
                    bool ok = false;
                    if (tid < 8 && kk < nstd)
                        ok = __hip_atomic_load(&F.P[kk * F.ncb + i], __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT) == F.ep &&
                             (diag || __hip_atomic_load(&F.P[kk * F.ncb + j], __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT) == F.ep);
                    // the published prefix k+1 .. k+n (lanes >= 8 count as unpublished)
                    const unsigned long long bad = __ballot(!ok);
                    if (tid == 0) pre_ready = k + (int)__builtin_ctzll(bad);
                }
            } else if (tid == 0) {
                pre_ready = ready_to;
            }
            __syncthreads();
            ready_to = pre_ready;
            const bool pre = k + 1 < nstd && k + 1 <= ready_to;
            if (k == nupd - 1) OWN_TS(2);
            double vs[8], vq[8];
            if (pre) {
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int e = tid + q * 512, y = e & 63, x = e >> 6;
                    vs[q] = ld_sc1(&A[(size_t)((k + 1) * kNB + y) + (size_t)(i * kNB + x) * lda]);
                    vq[q] = diag ? 0.0
                                 : ld_sc1(&A[(size_t)((k + 1) * kNB + y) +
                                             (size_t)(j * kNB + x) * lda]);
                }
            }
            mm_tn<true>(S, diag ? S : Q, acc);
            __syncthreads();  // every wave has read S and Q
            if (pre) {
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int e = tid + q * 512, y = e & 63, x = e >> 6;
                    S[y][x] = vs[q];
                    if (!diag) Q[y][x] = vq[q];
                }
            }
            have = pre;
            if (k == nupd - 1) OWN_TS(3);
        }
        if (merge || dmerge) {
            // U_{k,j} = W_k A_{k,j} (A_{k,j} stored by its owner through step k-1, raw for
            // k = 0); merge: A_{i,i+1} -= U_{k,i}' U_{k,j}, dmerge: A_{i,i} -= U_{k,i}' U_{k,i}
            const int k = merge ? i - 1 : i - 2;
            OWN_TS(0);
            flag_acquire2(&F.W[k], &F.H[k], F.ep, err);
            OWN_TS(1);
            const double *Wk = Wd + (size_t)k * kNB * kNB;
            double vw[8], va[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int e = tid + q * 512, y = e & 63, x = e >> 6;
                vw[q] = ld_sc1(&Wk[(size_t)x * kNB + y]);
                va[q] = ld_sc1(&Hs[(size_t)k * kNB * kNB + (size_t)y + (size_t)x * kNB]);
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int e = tid + q * 512, y = e & 63, x = e >> 6;
                Q[y][x] = vw[q];  // Q[r][s] = W_k[r][s]
                S[y][x] = va[q];
            }
            __syncthreads();
            v4d u2[2];
            wl_times(Q, S, u2[0], u2[1]);  // U_{k,j} = W_k A_{k,j}
            OWN_TS(2);
            __syncthreads();  // every wave has read W_k and A_{k,j}
            wl_put(Q, u2[0], u2[1]);
            if (merge) {
                // U_{k,j} is stored now (released with the hand-off below), so the hand-off's
                // drain waits only for T.  Merge also reads the chain's U_{k,i} (i = k + 1).
                // The v2 and v4 chains publish W_k before U_{k,k+1} (v1 releases both
                // together), so U_{k,j} is formed above while the chain finishes U_{k,k+1}.
                __syncthreads();
                tile_store(Q, A, lda, k, j);
                pub = true;
                flag_acquire2(&F.P[k * F.ncb + i], nullptr, F.ep, err);
                double vu[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int e = tid + q * 512, y = e & 63, x = e >> 6;
                    vu[q] = ld_sc1(&A[(size_t)(k * kNB + y) + (size_t)(i * kNB + x) * lda]);
                }
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int e = tid + q * 512, y = e & 63, x = e >> 6;
                    S[y][x] = vu[q];
                }
            }
            __syncthreads();
            if (merge) mm_tn<true>(S, Q, acc);
            else mm_tn<true>(Q, Q, acc);
            OWN_TS(3);
        }
        if (nupd > 0) {
            MM_FOR(h, r, y, x) {
                if (!diag || y <= x) T[y][x] -= acc[h][r];
            }
            __syncthreads();
        }
        if (hstore) {
            tile_store(T, Hs + (size_t)i * kNB * kNB, kNB, 0, 0);
            flag_release(&F.H[i], F.ep);
            OWN_TS(4);
            continue;
        }
        if (handoff) {
            tile_store(T, A, lda, i, j);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) {
                __hip_atomic_store(&F.R[2 * i + (diag ? 0 : 1)], F.ep, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                if (pub)
                    __hip_atomic_store(&F.P[(i - 1) * F.ncb + j], F.ep, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            }
            OWN_TS(4);
            continue;
        }
        // U_ij = W_i A_ij
        OWN_TS(4);
        flag_acquire2(&F.W[i], nullptr, F.ep, err);
        OWN_TS(5);
        {
            const double *W = Wd + (size_t)i * kNB * kNB;
            double v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int e = tid + q * 512, y = e & 63, x = e >> 6;
                v[q] = ld_sc1(&W[(size_t)x * kNB + y]);
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int e = tid + q * 512, y = e & 63, x = e >> 6;
                Q[y][x] = v[q];  // Q[r][s] = W[r][s]
            }
        }
        __syncthreads();
        wl_times(Q, T, acc[0], acc[1]);  // U_ij = W_i A_ij
        OWN_TS(6);
        __syncthreads();  // every wave has read T
        wl_put(T, acc[0], acc[1]);
        __syncthreads();
        tile_store(T, A, lda, i, j);  // coalesced write-through stores
        flag_release(&F.P[i * F.ncb + j], F.ep);
        OWN_TS(7);
#undef OWN_TS
    }
}

// [W: nblk | P: nblk x ncb | R: 2 nblk | 4 pad | backward-solve: nblk]
static size_t bsolve_flag_offset(int m_pad, int nrhs_blocks) {
    const size_t nblk = (size_t)m_pad / kNB, ncb = nblk + nrhs_blocks;
    return nblk + nblk * ncb + 2 * nblk + 4;
}

// Wd: the nblk blocks W_k followed by nblk scratch tiles (chol_factor's Hs)
size_t chol_wd_words(int m_pad) { return 2 * (size_t)kNB * m_pad; }

// [... | backward-solve: nblk | H: nblk | pad to 8 bytes | the solve's LL hand-off words]
static size_t bsolve_ll_offset(int m_pad, int nrhs_blocks) {
    return (bsolve_flag_offset(m_pad, nrhs_blocks) + 2 * ((size_t)m_pad / kNB) + 1) & ~(size_t)1;
}
// per block: 2 right-hand sides x 64 elements x 2 tagged 64-bit words
constexpr size_t kBsLLWords = 2 * 64 * 2 * 2;
size_t chol_flag_words(int m_pad, int nrhs_blocks) {
    return bsolve_ll_offset(m_pad, nrhs_blocks) + kBsLLWords * ((size_t)m_pad / kNB);
}

// Host-side epoch per flag buffer: advance = true starts a new use (zeroing `words` flags
// when the buffer is first seen and on wrap); false returns the current epoch (0: none).
static unsigned int flag_epoch(unsigned int *flags, size_t words, hipStream_t s, bool advance) {
    static std::mutex mu;
    static std::unordered_map<const unsigned int *, unsigned int> epochs;
    std::lock_guard<std::mutex> lk(mu);
    unsigned int &e = epochs[flags];
    if (!advance) return e;
    if (e == 0u || e == 0xffffffffu) {
        (void)hipMemsetAsync(flags, 0, sizeof(unsigned int) * words, s);
        e = 0u;
    }
    return ++e;
}

static int device_cus() {
    static int n = [] {
        int dev = 0, v = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            v <= 0)
            v = 256;
        return v;
    }();
    return n;
}

// chain variant of k_chol_persistent (4: the default, the 16-column leaf pipeline of
// bb_chol4.h; 1: the round-2 chain; 2, 3: its pipelined variants, measured slower -- DESIGN.md
// §5.2); bb_set_chol_version switches it for A/B measurements
int g_chol_version = 4;

// Workgroups of k_chol_persistent<V> the device can hold at once (occupancy query x CUs),
// computed once per chain variant.
static int chol_max_resident(int version) {
    static int cache[5] = {-1, -1, -1, -1, -1};
    static std::mutex mu;
    std::lock_guard<std::mutex> lk(mu);
    int &c = cache[(version >= 1 && version <= 4) ? version : 1];
    if (c < 0) {
        int nb = 0;
        hipError_t e = version == 2
            ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_chol_persistent<2>, 512, 0)
            : version == 3
            ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_chol_persistent<3>, 512, 0)
            : version == 4
            ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_chol_persistent<4>, 512, 0)
            : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_chol_persistent<1>, 512, 0);
        c = (e == hipSuccess ? nb : 0) * device_cus();
    }
    return c;
}

void chol_factor(hipStream_t s, double *A, int lda, int m_pad, int nrhs_blocks, uint32_t *err,
                 double *Wd, unsigned int *flags, unsigned long long *trace, const int *gate) {
    const int nblk = m_pad / kNB;
    const int ncb = nblk + nrhs_blocks;
    const size_t words = chol_flag_words(m_pad, nrhs_blocks);
    const unsigned int ep = flag_epoch(flags, words, s, true);
    CholFlags F{flags, flags + nblk, flags + nblk + (size_t)nblk * ncb,
                flags + bsolve_flag_offset(m_pad, nrhs_blocks) + nblk, ncb, ep};
    const int ntiles = nblk * (nblk + 1) / 2 + nblk * nrhs_blocks;
    const int grid = std::min(device_cus(), 1 + ntiles);
    // every workgroup of the grid must be resident at once (the chain waits on tiles of every
    // owner): refuse a launch the device cannot hold rather than let it stall into the
    // bounded waits' error flag
    const int resident = chol_max_resident(g_chol_version);
    if (grid > resident) {
        char b[200];
        snprintf(b, sizeof(b),
                 "persistent Cholesky: %d workgroups exceed the %d the device holds at once",
                 grid, resident);
        throw std::runtime_error(b);
    }
    auto *kern = g_chol_version == 1 ? k_chol_persistent<1>
               : g_chol_version == 2 ? k_chol_persistent<2>
               : g_chol_version == 3 ? k_chol_persistent<3> : k_chol_persistent<4>;
    note_launch(KF_CHOL, (const void *)kern);
    kern<<<grid, 512, 0, s>>>(A, lda, nblk, ncb, Wd, F, err, trace, gate);
}


// Backward solve of kBsNB consecutive blocks per launch (kb, kb-1, .., kb-nb+1): every
// workgroup redundantly runs the short chain w_k = W_k' (y_k - sum_{k' in (k, kb]} U_kk' w_k')
// (from L2-resident tiles; no inter-workgroup hand-off), workgroup 0 stores the w's, and
// workgroup i < kb-nb+1 applies y_i -= sum_k U_ik w_k.  nblk/kBsNB launches instead of nblk.
constexpr int kBsNB = 4;

__global__ __launch_bounds__(256) void k_bsolve_multi(const double *A, int lda, int kb, int nb,
                                                      int m_pad, const double *__restrict__ Wd,
                                                      double *Y, double *Wout, int nrhs, const int *gate) {
    if (gated(gate)) return;
    __shared__ double yv[2][kBsNB][64];
    __shared__ double wv[2][kBsNB][64];
    __shared__ double part[4][2][64];
    const int tid = threadIdx.x, x = tid & 63, g = tid >> 6;  // g: 16-row slice
    for (int e = tid; e < 2 * kBsNB * 64; e += 256) {
        const int q = e / (kBsNB * 64), sb = (e / 64) % kBsNB;
        if (q < nrhs && sb < nb) yv[q][sb][e & 63] = Y[(size_t)q * m_pad + (kb - sb) * kNB + (e & 63)];
    }
    __syncthreads();
    for (int sb = 0; sb < nb; ++sb) {
        const int k = kb - sb;
        if (sb > 0) {
            // y_k -= sum_{s' < sb} U_{k, kb-s'} w_{s'}  (thread: row x, column slice g)
            for (int q = 0; q < nrhs; ++q) {
                double acc = 0.0;
                for (int s2 = 0; s2 < sb; ++s2) {
                    const double *col = A + (size_t)(k * kNB + x) + (size_t)((kb - s2) * kNB) * lda;
#pragma unroll
                    for (int cc = 0; cc < 16; ++cc) {
                        const int c = g * 16 + cc;
                        acc += col[(size_t)c * lda] * wv[q][s2][c];
                    }
                }
                part[g][q][x] = acc;
            }
            __syncthreads();
            if (tid < 64 * nrhs) {
                const int q = tid >> 6;
                yv[q][sb][x] -= ((part[0][q][x] + part[1][q][x]) + part[2][q][x]) + part[3][q][x];
            }
            __syncthreads();
        }
        // w[x] = sum_r W[r][x] y[r]; W column-major: column x contiguous in r
        const double *W = Wd + (size_t)k * kNB * kNB;
        for (int q = 0; q < nrhs; ++q) {
            double acc = 0.0;
            const double *col = W + (size_t)x * kNB + g * 16;
#pragma unroll
            for (int rr = 0; rr < 16; ++rr) acc += col[rr] * yv[q][sb][g * 16 + rr];
            part[g][q][x] = acc;
        }
        __syncthreads();
        if (tid < 64 * nrhs) {
            const int q = tid >> 6;
            wv[q][sb][x] = ((part[0][q][x] + part[1][q][x]) + part[2][q][x]) + part[3][q][x];
        }
        __syncthreads();
    }
    if (blockIdx.x == 0)
        for (int e = tid; e < 2 * kBsNB * 64; e += 256) {
            const int q = e / (kBsNB * 64), sb = (e / 64) % kBsNB;
            if (q < nrhs && sb < nb)
                Wout[(size_t)q * m_pad + (kb - sb) * kNB + (e & 63)] = wv[q][sb][e & 63];
        }
    const int nrow = kb - nb + 1;  // row blocks still to update
    if (nrow > 0) {
        const int ib = blockIdx.x * kNB;
        for (int q = 0; q < nrhs; ++q) {
            double acc = 0.0;
            for (int sb = 0; sb < nb; ++sb) {
                const double *col = A + (size_t)(ib + x) + (size_t)((kb - sb) * kNB) * lda;
#pragma unroll
                for (int cc = 0; cc < 16; ++cc) {
                    const int c = g * 16 + cc;
                    acc += col[(size_t)c * lda] * wv[q][sb][c];
                }
            }
            part[g][q][x] = acc;
        }
        __syncthreads();
        if (tid < 64 * nrhs) {
            const int q = tid >> 6;
            const double acc = ((part[0][q][x] + part[1][q][x]) + part[2][q][x]) + part[3][q][x];
            Y[(size_t)q * m_pad + ib + x] -= acc;
        }
    }
}

// Backward solve in ONE launch: workgroup b owns row block i = nblk-1-b.  It keeps y_i in
// LDS, and for j = nblk-1 .. i+1 prefetches its tile U_ij into registers, waits for w_j's
// flag (set-once, tagged with the factorisation's epoch), applies y_i -= U_ij w_j, then
// forms w_i = W_i' y_i, stores it write-through (sc1) and sets its flag.  The critical path
// is one hop + one 64 x 64 matvec per block instead of a launch per kBsNB blocks; every
// workgroup waits only on higher blocks, all are co-resident (nblk <= CUs).
//
// ll (bb_set_tuning key 20 = 1, the default): w_i travels as 64-bit words each holding 32 bits
// of it and the epoch in the other 32 (single-copy atomic stores), so the consumer polls the
// data itself -- one write-through round trip per hop instead of the flag's and then the
// data's -- and the producer needs no drain between data and flag.
__global__ __launch_bounds__(256) void k_bsolve_persist(const double *A, int lda, int nblk,
                                                        int m_pad, const double *__restrict__ Wd,
                                                        const double *Y, double *Wout, int nrhs,
                                                        unsigned int *fl, unsigned int ep,
                                                        uint32_t *err, const int *gate,
                                                        unsigned long long *ll) {
    if (gated(gate)) return;
    __shared__ double yv[2][64];
    __shared__ double wv[2][64];
    __shared__ double part[4][2][64];
    const int i = nblk - 1 - (int)blockIdx.x;
    const int tid = threadIdx.x, x = tid & 63, g = tid >> 6;  // g: 16-wide slice
    if (tid < 64 * nrhs) yv[tid >> 6][x] = Y[(size_t)(tid >> 6) * m_pad + i * kNB + x];
    // W_i column x, rows g*16 .. +15 (column-major: contiguous)
    double wreg[16];
    {
        const double *col = Wd + (size_t)i * kNB * kNB + (size_t)x * kNB + g * 16;
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) wreg[rr] = col[rr];
    }
    __syncthreads();
    for (int j = nblk - 1; j > i; --j) {
        // U_ij row x, columns g*16 .. +15 (loads in flight across the wait)
        double ureg[16];
        const double *row = A + (size_t)(i * kNB + x) + (size_t)(j * kNB + g * 16) * lda;
#pragma unroll
        for (int cc = 0; cc < 16; ++cc) ureg[cc] = row[(size_t)cc * lda];
        if (ll) {
            if (tid < 64 * nrhs) {  // whole waves: the readiness test is wave-uniform
                const unsigned long long *pw = ll + (((size_t)j * 2 + (tid >> 6)) * 64 + x) * 2;
                unsigned long long lo, hi;
                SpinGuard sg;
                for (;;) {
                    lo = __hip_atomic_load(pw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    hi = __hip_atomic_load(pw + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const bool ok = (unsigned)(lo >> 32) == ep && (unsigned)(hi >> 32) == ep;
                    if (__all(ok)) break;
                    __builtin_amdgcn_s_sleep(1);
                    if (sg.expired(err)) break;
                }
                wv[tid >> 6][x] = __longlong_as_double((long long)((hi << 32) | (lo & 0xffffffffull)));
            }
        } else {
            flag_acquire2(&fl[j], nullptr, ep, err);
            if (tid < 64 * nrhs)
                wv[tid >> 6][x] = ld_sc1(&Wout[(size_t)(tid >> 6) * m_pad + j * kNB + x]);
        }
        __syncthreads();
        for (int q = 0; q < nrhs; ++q) {
            double acc = 0.0;
#pragma unroll
            for (int cc = 0; cc < 16; ++cc) acc += ureg[cc] * wv[q][g * 16 + cc];
            part[g][q][x] = acc;
        }
        __syncthreads();
        if (tid < 64 * nrhs) {
            const int q = tid >> 6;
            yv[q][x] -= ((part[0][q][x] + part[1][q][x]) + part[2][q][x]) + part[3][q][x];
        }
        __syncthreads();
    }
    for (int q = 0; q < nrhs; ++q) {
        double acc = 0.0;
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) acc += wreg[rr] * yv[q][g * 16 + rr];
        part[g][q][x] = acc;
    }
    __syncthreads();
    if (tid < 64 * nrhs) {
        const int q = tid >> 6;
        const double w = ((part[0][q][x] + part[1][q][x]) + part[2][q][x]) + part[3][q][x];
        if (ll) {
            const unsigned long long b = (unsigned long long)__double_as_longlong(w);
            const unsigned long long tag = (unsigned long long)ep << 32;
            unsigned long long *pw = ll + (((size_t)i * 2 + q) * 64 + x) * 2;
            __hip_atomic_store(pw, (b & 0xffffffffull) | tag, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(pw + 1, (b >> 32) | tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            Wout[(size_t)q * m_pad + i * kNB + x] = w;  // the result (read after the launch)
        } else {
            st_sc1(&Wout[(size_t)q * m_pad + i * kNB + x], w);
        }
    }
    if (!ll) flag_release(&fl[i], ep);
}
int g_bsolve_ll = 1;

void chol_bsolve(hipStream_t s, const double *A, int lda, int m_pad, const double *Wd,
                 double *Y, double *W, int nrhs, unsigned int *flags, uint32_t *err, const int *gate) {
    const int nblk = m_pad / kNB;
    // one persistent launch (a workgroup per 64-row block, resident together) after the
    // factorisation that filled `flags`; otherwise one launch per kBsNB blocks
    if (flags && err && nblk <= device_cus()) {
        // the solve's flags have their own epoch sequence (one per solve)
        unsigned int *bf = flags + bsolve_flag_offset(m_pad, 1);
        unsigned int *llw = flags + bsolve_ll_offset(m_pad, 1);
        // (the LL words are zeroed with the flags on first use and on epoch wrap)
        const unsigned int ep =
            flag_epoch(bf, (size_t)(llw - bf) + kBsLLWords * (size_t)nblk, s, true);
        note_launch(KF_SOLVE, (const void *)k_bsolve_persist);
        k_bsolve_persist<<<nblk, 256, 0, s>>>(A, lda, nblk, m_pad, Wd, Y, W, nrhs, bf, ep, err, gate,
                                              (g_bsolve_ll && nrhs <= 2)
                                                  ? (unsigned long long *)llw
                                                  : nullptr);
        return;
    }
    for (int kb = nblk - 1; kb >= 0; kb -= kBsNB) {
        const int nb = std::min(kBsNB, kb + 1);
        const int nrow = kb - nb + 1;
        k_bsolve_multi<<<nrow > 0 ? nrow : 1, 256, 0, s>>>(A, lda, kb, nb, m_pad, Wd, Y, W, nrhs, gate);
    }
}

// ---------------------------------------------------------------------------
// beta updates
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_beta_wb(const double *__restrict__ X, int ldx,
                                                 int n_pad, const double *__restrict__ w,
                                                 const double *u, const double *D,
                                                 const DevScalars *sc, int p_loc, double *beta,
                                                 double *trace) {
    extern __shared__ double ws[];
    for (int i = threadIdx.x; i < n_pad; i += 256) ws[i] = w[i];
    __syncthreads();
    const double sig = sqrt(sc->sig2);
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int nw = gridDim.x * 4;
    for (int j = wave; j < p_loc; j += nw) {
        const double *col = X + (size_t)j * ldx;
        double s = 0.0;
        for (int r = 2 * lane; r < n_pad; r += 128) {
            const double2 x = *(const double2 *)(col + r);
            s += x.x * ws[r];
            s += x.y * ws[r + 1];
        }
        s = wave_allsum(s);
        if (lane == 0) {
            const double b = u[j] + D[j] * s / sig;
            beta[j] = b;
            if (trace) trace[j] = b;
        }
    }
}

void launch_beta_woodbury(hipStream_t s, const double *X, int ldx, int n_pad, const double *w,
                          const double *u, const double *D, const DevScalars *sc, int p_loc,
                          double *beta, double *beta_trace) {
    int blocks = (p_loc + 3) / 4;
    if (blocks > 2048) blocks = 2048;
    k_beta_wb<<<blocks, 256, n_pad * sizeof(double), s>>>(X, ldx, n_pad, w, u, D, sc, p_loc,
                                                          beta, beta_trace);
}

// Fused Woodbury beta update + X beta partials (one pass over X instead of two):
// wave = one column at a time: s = X_j . w (same per-lane order + wave tree as k_beta_wb),
// beta_j = u_j + D_j s / sig, then the lane's rows accumulate X_j beta_j in registers
// (rows 2 lane + 128 i, i < NR).  Four waves per workgroup (one per SIMD, so the wave has
// the whole 512-entry register file and nothing spills); each wave keeps the next TWO
// columns' loads in flight (three register buffers rotating), so the per-column memory
// latency is hidden behind two columns of work.  The workgroup's 4 wave accumulators are
// summed in wave order through LDS into part[blockIdx.x][row], which k_pre sums next
// sweep.  NR = n_pad / 128 <= 16.
constexpr int kBxbWaves = 4;

template <int NR, bool NTL>
__global__ __launch_bounds__(64 * kBxbWaves, 1) void k_beta_wb_xb(
    const double *__restrict__ X, int ldx, int n_pad, const double *__restrict__ w,
    const double *__restrict__ u, const double *__restrict__ D, const DevScalars *sc, int p_loc,
    double *__restrict__ beta, double *__restrict__ trace, double *__restrict__ part) {
    __shared__ double ws[NR * 128];
    for (int i = threadIdx.x; i < NR * 128; i += 64 * kBxbWaves) ws[i] = w[i];
    __syncthreads();
    const double sig = sqrt(sc->sig2);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int nw = gridDim.x * kBxbWaves;
    double2 acc[NR];
#pragma unroll
    for (int i = 0; i < NR; ++i) acc[i] = make_double2(0.0, 0.0);
    // a buffer holds column j and its (u_j, D_j): every load of a column is issued together,
    // so the counted waits for the oldest buffer never drain the two refills behind it
    // (past the end the last column is re-read: branch-free, so the waits stay counted)
    auto load = [&](int j, double2 (&xv)[NR], double2 &ud) {
        const int jj = min(j, p_loc - 1);
        const double *col = X + (size_t)jj * ldx + 2 * lane;
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            if constexpr (NTL) {
                typedef double v2d_ __attribute__((ext_vector_type(2)));
                const v2d_ t2 = __builtin_nontemporal_load((const v2d_ *)(col + 128 * i));
                xv[i] = make_double2(t2.x, t2.y);
            } else {
                xv[i] = *(const double2 *)(col + 128 * i);
            }
        }
        ud = make_double2(u[jj], D[jj]);
    };
    // consume column j from xc, then refill xc with column j + 3 nw
    auto step = [&](int j, double2 (&xc)[NR], double2 &ud) {
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            s += xc[i].x * ws[128 * i + 2 * lane];
            s += xc[i].y * ws[128 * i + 2 * lane + 1];
        }
        s = wave_allsum(s);
        const double bj = ud.x + ud.y * s / sig;
        if (lane == 0) {
            beta[j] = bj;
            if (trace) trace[j] = bj;
        }
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            acc[i].x = __builtin_fma(xc[i].x, bj, acc[i].x);
            acc[i].y = __builtin_fma(xc[i].y, bj, acc[i].y);
        }
        // keep the refill behind the last use of xc (else the scheduler hoists it and both
        // generations of the buffer are live at once)
        __builtin_amdgcn_sched_barrier(0);
        load(j + 3 * nw, xc, ud);
        __builtin_amdgcn_sched_barrier(0);
    };
    double2 xa[NR], xb[NR], xcol[NR], uda, udb, udc;
    int j = blockIdx.x * kBxbWaves + wid;
    load(j, xa, uda);
    load(j + nw, xb, udb);
    load(j + 2 * nw, xcol, udc);
    for (; j + 2 * nw < p_loc; j += 3 * nw) {
        step(j, xa, uda);
        step(j + nw, xb, udb);
        step(j + 2 * nw, xcol, udc);
    }
    if (j < p_loc) step(j, xa, uda);
    if (j + nw < p_loc) step(j + nw, xb, udb);
    // wave-ordered sum of the accumulators (ws is reused as the running sum)
    __syncthreads();
    for (int q = 0; q < kBxbWaves; ++q) {
        if (wid == q) {
#pragma unroll
            for (int i = 0; i < NR; ++i) {
                double2 *d = (double2 *)&ws[128 * i + 2 * lane];
                *d = q == 0 ? acc[i] : make_double2(d->x + acc[i].x, d->y + acc[i].y);
            }
        }
        __syncthreads();
    }
    for (int i = threadIdx.x; i < NR * 128; i += 64 * kBxbWaves)
        part[(size_t)blockIdx.x * n_pad + i] = ws[i];
}

int beta_xb_parts(int p_loc) {
    int g = (p_loc + 31) / 32;
    return g < 1 ? 1 : (g > 256 ? 256 : g);
}

static std::atomic<const void *> g_kinst[KF_COUNT];
void note_launch(KernelFamily f, const void *kernel) {
    g_kinst[f].store(kernel, std::memory_order_relaxed);
}
const void *launched_instance(int f) {
    return (f >= 0 && f < KF_COUNT) ? g_kinst[f].load(std::memory_order_relaxed) : nullptr;
}

bool beta_xb_supported(int n_pad) { return n_pad % 128 == 0 && n_pad <= 2048; }

// non-temporal X loads in the fused beta pass (X is streamed once per sweep, larger than
// every cache): C3 beta 0.151 -> 0.138 ms (tools/res_nt_ab.py); bb_set_tuning(2, v) for A/B
int g_bxb_nt = 1;

void launch_beta_woodbury_xb(hipStream_t s, const double *X, int ldx, int n_pad, const double *w,
                             const double *u, const double *D, const DevScalars *sc, int p_loc,
                             double *beta, double *beta_trace, double *part) {
    const int g = beta_xb_parts(p_loc);
    switch (n_pad / 128) {
#define BXB(NR)                                                                             \
    case NR:                                                                                \
        note_launch(KF_BETA, g_bxb_nt ? (const void *)k_beta_wb_xb<NR, true>                \
                                      : (const void *)k_beta_wb_xb<NR, false>);             \
        if (g_bxb_nt)                                                                       \
            k_beta_wb_xb<NR, true><<<g, 64 * kBxbWaves, 0, s>>>(X, ldx, n_pad, w, u, D, sc,     \
                                                               p_loc, beta, beta_trace, part); \
        else                                                                                \
            k_beta_wb_xb<NR, false><<<g, 64 * kBxbWaves, 0, s>>>(X, ldx, n_pad, w, u, D, sc,    \
                                                                p_loc, beta, beta_trace, part); \
        break;
        BXB(1) BXB(2) BXB(3) BXB(4) BXB(5) BXB(6) BXB(7) BXB(8)
        BXB(9) BXB(10) BXB(11) BXB(12) BXB(13) BXB(14) BXB(15) BXB(16)
#undef BXB
        default: break;
    }
}

__global__ __launch_bounds__(256) void k_chol_rhs(const double *A, int lda, int rhs_col, int p,
                                                  int p_pad, Key key, uint64_t t, double *Y2) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= p_pad) return;
    Y2[r] = A[(size_t)r + (size_t)rhs_col * lda];
    Y2[(size_t)p_pad + r] = (r < p) ? normal_at(key, t, KIND_BETA_Z, (uint64_t)r) : 0.0;
}

void launch_chol_rhs(hipStream_t s, const double *A, int lda, int rhs_col, int p, int p_pad,
                     uint64_t k0, uint64_t k1, uint64_t t, double *Y2) {
    k_chol_rhs<<<(p_pad + 255) / 256, 256, 0, s>>>(A, lda, rhs_col, p, p_pad, Key{k0, k1}, t, Y2);
}

__global__ __launch_bounds__(256) void k_beta_chol(const double *W2, int p_pad,
                                                   const DevScalars *sc, int p, double *beta,
                                                   double *trace) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= p) return;
    const double sig = sqrt(sc->sig2);
    const double b = W2[r] + sig * W2[(size_t)p_pad + r];
    beta[r] = b;
    if (trace) trace[r] = b;
}

void launch_beta_chol(hipStream_t s, const double *W2, int p_pad, const DevScalars *sc, int p,
                      double *beta, double *beta_trace) {
    k_beta_chol<<<(p + 255) / 256, 256, 0, s>>>(W2, p_pad, sc, p, beta, beta_trace);
}

__global__ __launch_bounds__(256) void k_beta_ortho(const double *gdiag, const double *cvec,
                                                    const double *lam, const DevScalars *sc,
                                                    int p, uint64_t j0, Key key, uint64_t t,
                                                    double *beta, double *trace) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= p) return;
    const double sig2 = sc->sig2, tau = sc->tau;
    const double uu = gdiag[i] + lam[i] * sig2 / (tau * tau);
    const double sd = sqrt(sig2 / uu);
    const double m = cvec[i] / uu;
    // z_j on the GLOBAL column index (j0 = a column shard's first column)
    const double b = m + sd * normal_at(key, t, KIND_BETA_Z, j0 + (uint64_t)i);
    beta[i] = b;
    if (trace) trace[i] = b;
}

void launch_beta_ortho(hipStream_t s, const double *gdiag, const double *c, const double *lam,
                       const DevScalars *sc, int p, uint64_t j0, uint64_t k0, uint64_t k1,
                       uint64_t t, double *beta, double *beta_trace) {
    k_beta_ortho<<<(p + 255) / 256, 256, 0, s>>>(gdiag, c, lam, sc, p, j0, Key{k0, k1}, t, beta,
                                                 beta_trace);
}

// alpha | beta, tau: BridgeRegression.cpp:469-503 (single workgroup).
__global__ __launch_bounds__(1024) void k_alpha_mh(const double *beta, int p, DevScalars *sc,
                                                   double pr_a, double pr_b, Key key,
                                                   uint64_t t, double *alpha_tr) {
    __shared__ double sh[16];
    const double tau = sc->tau;
    const double a_old = sc->alpha;
    const double ep = 0.1;
    U4 u = uniforms(key, t, KIND_ALPHA, 0, 0, 0);
    const double l_new = fmax(0.0, a_old - ep);
    const double r_new = fmin(1.0, a_old + ep);
    const double d_new = r_new - l_new;
    const double a_new = l_new + d_new * u.r[0];
    double sn = 0.0, so = 0.0;
    for (int i = threadIdx.x; i < p; i += 1024) {
        const double si = log(fabs(beta[i] / tau));
        sn += exp(a_new * si);
        so += exp(a_old * si);
    }
    const double Sn = block_sum<1024>(sn, sh);
    const double So = block_sum<1024>(so, sh);
    if (threadIdx.x == 0) {
        const double pp = (double)p;
        const double llh_new = pp * log(a_new) - pp * lgamma(1.0 / a_new) - Sn;
        const double llh_old = pp * log(a_old) - pp * lgamma(1.0 / a_old) - So;
        const double lbc = lgamma(pr_a) + lgamma(pr_b) - lgamma(pr_a + pr_b);
        const double ldb_new = (pr_a - 1.0) * log(a_new) + (pr_b - 1.0) * log(1.0 - a_new) - lbc;
        const double ldb_old = (pr_a - 1.0) * log(a_old) + (pr_b - 1.0) * log(1.0 - a_old) - lbc;
        const double l_old = fmax(0.0, a_new - ep);
        const double r_old = fmin(1.0, a_new + ep);
        const double d_old = r_old - l_old;
        const double log_accept = llh_new - llh_old + ldb_new - ldb_old + log(d_old) - log(d_new);
        double an = a_new;
        if (u.r[1] > exp(log_accept)) an = a_old;
        sc->alpha = an;
        if (alpha_tr) *alpha_tr = an;
    }
}

void launch_alpha_mh(hipStream_t s, const double *beta, int p, DevScalars *sc, double pr_a,
                     double pr_b, uint64_t k0, uint64_t k1, uint64_t t, double *alpha_tr) {
    k_alpha_mh<<<1, 1024, 0, s>>>(beta, p, sc, pr_a, pr_b, Key{k0, k1}, t, alpha_tr);
}

// The same MH step for a column-sharded chain, split around an exchange: k_alpha_sums writes
// this shard's [S(alpha_new), S(alpha_old)], S(a) = sum_j exp(a log|beta_j / tau|) (the
// proposal comes from the shared counter, so every shard proposes the same alpha_new); the
// caller sums the pairs over shards; k_alpha_decide evaluates llh_alpha_marg with the
// GLOBAL p and accepts or rejects (BridgeRegression.cpp:469-503).  One shard gives the bits
// of k_alpha_mh (same loop, tree and expressions).
__device__ __forceinline__ double alpha_proposal(double a_old, Key key, uint64_t t, double &u1) {
    const U4 u = uniforms(key, t, KIND_ALPHA, 0, 0, 0);
    u1 = u.r[1];
    const double ep = 0.1;
    const double l_new = fmax(0.0, a_old - ep);
    const double r_new = fmin(1.0, a_old + ep);
    return l_new + (r_new - l_new) * u.r[0];
}

__global__ __launch_bounds__(1024) void k_alpha_sums(const double *beta, int p_loc,
                                                     const DevScalars *sc, Key key, uint64_t t,
                                                     double *sums) {
    __shared__ double sh[16];
    const double tau = sc->tau, a_old = sc->alpha;
    double u1;
    const double a_new = alpha_proposal(a_old, key, t, u1);
    double sn = 0.0, so = 0.0;
    for (int i = threadIdx.x; i < p_loc; i += 1024) {
        const double si = log(fabs(beta[i] / tau));
        sn += exp(a_new * si);
        so += exp(a_old * si);
    }
    const double Sn = block_sum<1024>(sn, sh);
    const double So = block_sum<1024>(so, sh);
    if (threadIdx.x == 0) {
        sums[0] = Sn;
        sums[1] = So;
    }
}

__global__ void k_alpha_decide(const double *sums, int p, DevScalars *sc, double pr_a,
                               double pr_b, Key key, uint64_t t, double *alpha_tr) {
    if (threadIdx.x != 0) return;
    const double a_old = sc->alpha, ep = 0.1;
    double u1;
    const double a_new = alpha_proposal(a_old, key, t, u1);
    const double d_new = fmin(1.0, a_old + ep) - fmax(0.0, a_old - ep);
    const double pp = (double)p;
    const double llh_new = pp * log(a_new) - pp * lgamma(1.0 / a_new) - sums[0];
    const double llh_old = pp * log(a_old) - pp * lgamma(1.0 / a_old) - sums[1];
    const double lbc = lgamma(pr_a) + lgamma(pr_b) - lgamma(pr_a + pr_b);
    const double ldb_new = (pr_a - 1.0) * log(a_new) + (pr_b - 1.0) * log(1.0 - a_new) - lbc;
    const double ldb_old = (pr_a - 1.0) * log(a_old) + (pr_b - 1.0) * log(1.0 - a_old) - lbc;
    const double l_old = fmax(0.0, a_new - ep);
    const double r_old = fmin(1.0, a_new + ep);
    const double d_old = r_old - l_old;
    const double log_accept = llh_new - llh_old + ldb_new - ldb_old + log(d_old) - log(d_new);
    double an = a_new;
    if (u1 > exp(log_accept)) an = a_old;
    sc->alpha = an;
    if (alpha_tr) *alpha_tr = an;
}

void launch_alpha_sums(hipStream_t s, const double *beta, int p_loc, const DevScalars *sc,
                       uint64_t k0, uint64_t k1, uint64_t t, double *sums) {
    k_alpha_sums<<<1, 1024, 0, s>>>(beta, p_loc, sc, Key{k0, k1}, t, sums);
}

void launch_alpha_decide(hipStream_t s, const double *sums, int p, DevScalars *sc, double pr_a,
                         double pr_b, uint64_t k0, uint64_t k1, uint64_t t, double *alpha_tr) {
    k_alpha_decide<<<1, 64, 0, s>>>(sums, p, sc, pr_a, pr_b, Key{k0, k1}, t, alpha_tr);
}

__global__ void k_record_scalars(const DevScalars *sc, double *tau_tr, double *sig2_tr,
                                 double *alpha_tr) {
    if (threadIdx.x == 0) {
        if (tau_tr) *tau_tr = sc->tau;
        if (sig2_tr) *sig2_tr = sc->sig2;
        if (alpha_tr) *alpha_tr = sc->alpha;
    }
}

void launch_record_scalars(hipStream_t s, const DevScalars *sc, double *tau_tr,
                           double *sig2_tr, double *alpha_tr) {
    k_record_scalars<<<1, 64, 0, s>>>(sc, tau_tr, sig2_tr, alpha_tr);
}

// ---------------------------------------------------------------------------
// setup helpers
// ---------------------------------------------------------------------------
__global__ void k_copy_cols(const double *src, int lds, double *dst, int ldd, int rows,
                            int cols) {
    const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (size_t)rows * cols) return;
    const int r = (int)(idx % rows), c = (int)(idx / rows);
    dst[(size_t)r + (size_t)c * ldd] = src[(size_t)r + (size_t)c * lds];
}

void launch_copy_cols(hipStream_t s, const double *src, int lds, double *dst, int ldd, int rows,
                      int cols) {
    const size_t tot = (size_t)rows * cols;
    if (tot == 0) return;
    k_copy_cols<<<(unsigned)((tot + 255) / 256), 256, 0, s>>>(src, lds, dst, ldd, rows, cols);
}

__global__ void k_gdiag(const double *G, int ldg, int p, double *d) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < p) d[i] = G[(size_t)i + (size_t)i * ldg];
}

void launch_gdiag(hipStream_t s, const double *G, int ldg, int p, double *d) {
    k_gdiag<<<(p + 255) / 256, 256, 0, s>>>(G, ldg, p, d);
}

__global__ void k_sum_into(const double *a, double *b, size_t n) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) b[i] += a[i];
}

void launch_sum_into(hipStream_t s, const double *a, double *b, size_t n) {
    if (n == 0) return;
    k_sum_into<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(a, b, n);
}

// 32x32 LDS-tiled transpose: dst (cols x rows, ldd) = src' (rows x cols, lds).
__global__ __launch_bounds__(256) void k_transpose(const double *src, int lds, int rows,
                                                   int cols, double *dst, int ldd) {
    __shared__ double tile[32][33];
    const int bx = blockIdx.x * 32, by = blockIdx.y * 32;  // bx: rows of src, by: cols of src
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // ty 0..7
    for (int k = ty; k < 32; k += 8) {
        const int r = bx + tx, c = by + k;
        tile[k][tx] = (r < rows && c < cols) ? src[(size_t)r + (size_t)c * lds] : 0.0;
    }
    __syncthreads();
    for (int k = ty; k < 32; k += 8) {
        const int c = by + tx, r = bx + k;  // dst row = c, dst col = r
        if (c < cols && r < rows) dst[(size_t)c + (size_t)r * ldd] = tile[tx][k];
    }
}

void launch_transpose(hipStream_t s, const double *src, int lds, int rows, int cols, double *dst,
                      int ldd) {
    dim3 grid((rows + 31) / 32, (cols + 31) / 32);
    k_transpose<<<grid, 256, 0, s>>>(src, lds, rows, cols, dst, ldd);
}

// c_j = X_j . v for j < ncols (wave per column).
__global__ __launch_bounds__(256) void k_coldot(const double *__restrict__ X, int ldx,
                                                int n_pad, const double *__restrict__ v,
                                                int ncols, double *out) {
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int nw = gridDim.x * 4;
    for (int j = wave; j < ncols; j += nw) {
        const double *col = X + (size_t)j * ldx;
        double s = 0.0;
        for (int r = 2 * lane; r < n_pad; r += 128) {
            const double2 x = *(const double2 *)(col + r);
            s += x.x * v[r];
            s += x.y * v[r + 1];
        }
        s = wave_allsum(s);
        if (lane == 0) out[j] = s;
    }
}

void launch_coldot(hipStream_t s, const double *X, int ldx, int n_pad, const double *v, int ncols,
                   double *out) {
    int blocks = (ncols + 3) / 4;
    if (blocks > 2048) blocks = 2048;
    if (blocks < 1) blocks = 1;
    k_coldot<<<blocks, 256, 0, s>>>(X, ldx, n_pad, v, ncols, out);
}

// d_j = sum_r X[r, j]^2 (diagonal of X'X).
__global__ __launch_bounds__(256) void k_colnorm2(const double *__restrict__ X, int ldx,
                                                  int n_pad, int ncols, double *out) {
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int nw = gridDim.x * 4;
    for (int j = wave; j < ncols; j += nw) {
        const double *col = X + (size_t)j * ldx;
        double s = 0.0;
        for (int r = 2 * lane; r < n_pad; r += 128) {
            const double2 x = *(const double2 *)(col + r);
            s += x.x * x.x;
            s += x.y * x.y;
        }
        s = wave_allsum(s);
        if (lane == 0) out[j] = s;
    }
}

void launch_colnorm2(hipStream_t s, const double *X, int ldx, int n_pad, int ncols, double *out) {
    int blocks = (ncols + 3) / 4;
    if (blocks > 2048) blocks = 2048;
    if (blocks < 1) blocks = 1;
    k_colnorm2<<<blocks, 256, 0, s>>>(X, ldx, n_pad, ncols, out);
}

}  // namespace bb
