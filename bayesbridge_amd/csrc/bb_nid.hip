// bb_nid.hip -- the near-identity solve of the Woodbury system.
//
// The beta | rest draw for p > n (the reference's BridgeRegression.cpp:552-575 in its
// Woodbury form) needs w = M^-1 r with M = I + E, E = X diag(D) X' / sig2,
// r = y / sig - (X u / sig + delta).  E is symmetric positive semi-definite and
//   ||E||_2 <= tr(E) = eps = sum_j D_j |x_j|^2 / sig2,
// with the column norms |x_j|^2 computed once at setup.  So the spectrum of M lies in the
// certified interval [1, 1 + eps], and Chebyshev iteration on that interval converges with
// the guaranteed bound (Saad, Iterative Methods, Alg. 12.1 / Prop. 12.2; x_0 = 0)
//   |w - x_K| / |w| <= sqrt(1 + eps) / T_K(sigma1),  sigma1 = (1 + eps / 2) / (eps / 2),
// T_K the Chebyshev polynomial.  The engine takes this path for a sweep when K <= the
// iterations it launched and the bound is below 2^-56 (the solve is then more accurate
// than the dense Cholesky it replaces); otherwise the same sweep runs the Gram + Cholesky
// path.  The decision is made on the device (k_nid_sums, k_nid_reduce) every sweep; the kernels of the
// path not taken return at once (the gate word NidState::mode).
//
// x_K needs K - 1 products E d, each ONE pass over X: k_eapply forms X diag(D) (X' d)
// column chunk by column chunk with the chunk in registers (the dot products X_J' d and
// the update X_J (D_J s_J) read X_J once), writing one n-vector partial per workgroup;
// k_cheb_step sums the partials in a fixed order and advances the recurrence.  In the
// near-null regime a p > n chain starts in (beta0 = 0, BridgeRegression.cpp:85-89: tau and
// D tiny, eps ~ 1e-12 .. 1e-4 over the first hundreds of C3 sweeps) K is 2-4, so a sweep
// reads X 3-5 times instead of forming the n x n Gram and factoring it.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <mutex>

#include "bb_kernels.h"
#include "bb_sampler.h"

namespace bb {

namespace {

// rho_0 = 1 / sigma1, rho_{j} = 1 / (2 sigma1 - rho_{j-1})
__device__ inline double cheb_rho(double sigma1, int j) {
    double rho = 1.0 / sigma1;
    for (int i = 1; i <= j; ++i) rho = 1.0 / (2.0 * sigma1 - rho);
    return rho;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

}  // namespace

// ---------------------------------------------------------------------------------------
// Decision.  For any threshold T, E = sum_{D_j > T} D_j x_j x_j' / sig2 + (the rest) and the
// rest is <= (T / sig2) X X' in the semidefinite order, so
//   lambda_max(E) <= [ sum_{D_j > T} D_j |x_j|^2 + T Lambda ] / sig2
// with Lambda >= lambda_max(X X') certified at setup (nid_certify_lambda); T = 0 gives the
// trace.  The thresholds are fixed multiples of tau^2, T_k = tau^2 2^(40 - 2k), k < kNidTS
// (D_j = tau^2 / lambda_j: they span 1 / lambda_j from 2^40 down to 2^-22), so one pass over
// D gives every candidate, and column shards (world > 1), which hold disjoint columns, can
// add their sums:
//   red = [ S_0 .. S_{kNidTS-1}, trace, Lambda ],  S_k = sum_{D_j > T_k} D_j |x_j|^2,
// red[kNidTS + 1] = this engine's certified Lambda; after a shard exchange (sum) it is the sum
// of the shards' certificates, >= lambda_max(X X') (Weyl).  An engine without a certificate
// contributes +inf: the bound is the trace alone.  eps = least candidate / sig2 (x 1 + 1e-6).
//
// k_nid_sums: G workgroups, each writes its kNidTS + 1 partial sums; k_nid_reduce adds them
// in workgroup order (bitwise reproducible) and -- unsharded -- decides at once; a shard
// exchanges red first and decides in k_nid_decide_from (the same bits on every rank, so every
// rank takes the same path).  mode = K if the sweep takes the Chebyshev path (allow,
// K <= k_launched), else 0 (the Gram + Cholesky path).
// ---------------------------------------------------------------------------------------
constexpr int kNidSumWG = 256;

__device__ __forceinline__ double shard_threshold(double tau2, int k) {
    return ldexp(tau2, 40 - 2 * k);
}

// ---------------------------------------------------------------------------------------
// Mixed-precision plan (unsharded dense engines holding X32 = fl32(X)).
// E~ = X32 D X32' / sig2 is exactly PSD, and with |X - X32| <= u32 |X| entrywise (u32 = 2^-24)
//   |E - E~|_2 <= eta = 2 u32 sqrt(tr(E) eps) + u32^2 tr(E)
// (|(X - X32) D^1/2|_F <= u32 sig sqrt(tr E), |X D^1/2|_2 <= sig sqrt(eps)).  So M~ = I + E~ has
// its spectrum in [1, 1 + eps + eta] and |M^-1|, |M~^-1| <= 1.  The plan: x0 = K1 Chebyshev
// iterates on M~ (each product one pass over the fp32 copy: half the bytes), r = b - M x0 in
// fp64 (one pass over X), then K2 iterates on M~ from r, added to x0.  With t_K the Chebyshev
// bound on [1, 1 + eps + eta]:
//   |w - M^-1 b| / |M^-1 b| <= (eta + t_K2 (1 + eta)) (eta + t_K1 (1 + eta)),
// (x0's error is eta + t_K1 (1 + eta) of the solution, the correction's relative error
// eta + t_K2 (1 + eta)); the plan is taken when this is <= the tolerance and its cost -- in
// fp64 passes: 0.55 per fp32 pass, 1 for the residual pass, 0.05 per launch of a step -- is
// below the fp64 plan's and within the cap on the Chebyshev path's cost.
// ---------------------------------------------------------------------------------------
// The search runs on the 64 lanes of one wave: lane k - 1 holds t_k (T_k = cosh(k acosh
// sigma1), overflow giving t_k = 0; a 1e-12 relative margin covers the closed form's rounding),
// lane k1 - 1 finds its least k2 by a binary search (t_k2 by shuffle), then the cheapest
// (cost, k1) by a wave minimum: ~1 us, against ~40 us for the same search on one thread.
__device__ void nid_plan_mixed(double eps, double tr, int kcap, double cost_fp64,
                               const NidState *nid, int &K1, int &K2, double &eta, double &e2) {
    const int lane = threadIdx.x & 63;
    K1 = K2 = 0;
    eta = (2.0 * kU32 * sqrt(tr * eps) + kU32 * kU32 * tr) * (1.0 + 1e-6);
    e2 = eps + eta;
    if (!(e2 < 1e300) || kcap < 1) return;
    const ChebConst c = cheb_const(e2);
    const int kmax = kcap < 64 ? kcap : 64;
    const double ac = acosh(c.sigma1);
    const double tk = (lane + 1 <= kmax) ? sqrt(1.0 + e2) / cosh((lane + 1) * ac) * (1.0 + 1e-12)
                                         : HUGE_VAL;
    const double step32 = nid->c32 + nid->cstep, step64 = nid->c64 + nid->cstep;
    const double cap = fmin(cost_fp64, (kcap - 1) * step64);
    const int k1 = lane + 1;
    const double err1 = eta + tk * (1.0 + eta);
    const double need = kNidTol / err1;
    // least k2 in [1, kmax] with eta + t_k2 (1 + eta) <= need: t_k decreases in k, so the
    // predicate holds on [k2, kmax] -- a binary search, every lane shuffling each round
    int lo = 1, hi = kmax + 1;
#pragma unroll
    for (int it = 0; it < 7; ++it) {
        const int mid = (lo + hi) >> 1;
        const double t2 = __shfl(tk, (mid < kmax ? mid : kmax) - 1, 64);
        if (lo < hi) {
            if (eta + t2 * (1.0 + eta) <= need)
                hi = mid;
            else
                lo = mid + 1;
        }
    }
    const int k2 = lo <= kmax ? lo : 0;
    double cost = (k1 <= kmax && err1 < 1.0 && k2)
                      ? (k1 - 1) * step32 + step64 + (k2 - 1) * step32
                      : HUGE_VAL;
    if (!(cost < cap * (1.0 - 1e-9))) cost = HUGE_VAL;
    // wave minimum of (cost, k1): deterministic, ties to the smaller k1
    double bc = cost;
    int bk1 = k1, bk2 = k2;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double oc = __shfl_xor(bc, o, 64);
        const int ok1 = __shfl_xor(bk1, o, 64), ok2 = __shfl_xor(bk2, o, 64);
        if (oc < bc || (oc == bc && ok1 < bk1)) {
            bc = oc;
            bk1 = ok1;
            bk2 = ok2;
        }
    }
    if (bc < HUGE_VAL) {
        K1 = bk1;
        K2 = bk2;
    }
}

// bb_set_tuning key 16 (benchmarking only): a forced iteration count K > 0 replaces the
// certified one on the near-identity path (the solve is then no longer certified), so that the
// per-rank proxy of an N-GPU C3 job runs a C3 rank's product count
__device__ int g_dev_nid_force_k = 0;
int g_nid_force_k = 0;
void nid_set_force_k(int k) {
    g_nid_force_k = k;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_dev_nid_force_k), &k, sizeof(int));
}

// The bound and the trace are rounded UP to 12 significant bits (still bounds): the sums are
// added in another order by the split lambda launch (by column units) than by k_nid_sums (by
// strided threads), and the rounding makes the decision -- K, the Chebyshev interval, the mixed
// plan -- the same bits either way unless the two sums straddle a grid point (relative gap
// 2^-12 against a rounding difference ~1e-15: ~1e-12 of sweeps)
__device__ __forceinline__ double round_up_12(double x) {
    if (!(x > 0.0 && x < HUGE_VAL)) return x;
    constexpr unsigned long long m = (1ull << 40) - 1;
    unsigned long long b = (unsigned long long)__double_as_longlong(x);
    if (b & m) b = (b | m) + 1;
    return __longlong_as_double((long long)b);
}

// eps from the least bound, the iteration count K and the sweep's mode: called by the 64
// lanes of one wave (every lane computes the same values; lane 0 writes them)
__device__ void nid_finish(const double *red, const DevScalars *sc, int k_launched, int allow,
                           NidState *nid, double *eps_host, double *mode_host,
                           int allow_mixed = 0, double *k2_host = nullptr,
                           unsigned long long tag_seq = 0) {
    const double tau2 = sc->tau * sc->tau;
    const double lam = red[kNidTS + 1];
    double best = red[kNidTS];
    if (lam > 0.0 && lam < HUGE_VAL)
        for (int k = 0; k < kNidTS; ++k)
            best = fmin(best, red[k] + shard_threshold(tau2, k) * lam);
    // rounding of the sums: a relative margin far above its worst case (p u)
    const double eps = round_up_12(best / sc->sig2 * (1.0 + 1e-6));
    int K = cheb_iterations(eps, k_launched, kNidTol);
    if (g_dev_nid_force_k > 0) K = g_dev_nid_force_k < k_launched ? g_dev_nid_force_k : k_launched;
    int mode = (allow && K > 0) ? K : 0, k2 = 0;
    double ecb = eps, eta = 0.0;
    // a mixed plan costs at least one fp64 pass (k1 = k2 = 1): never below K <= 2's
    if (allow && allow_mixed && g_dev_nid_force_k == 0 && (K == 0 || K > 2)) {
        const double tr = round_up_12(red[kNidTS] / sc->sig2 * (1.0 + 1e-6));
        int k1m, k2m;
        double e2;
        nid_plan_mixed(eps, tr, k_launched, K > 0 ? (K - 1) * (nid->c64 + nid->cstep) : HUGE_VAL,
                       nid, k1m, k2m, eta, e2);
        if (k2m > 0) {
            mode = k1m;
            k2 = k2m;
            ecb = e2;
        } else {
            eta = 0.0;
        }
    }
    if ((threadIdx.x & 63) != 0) return;
    nid->eps = eps;
    nid->mode = mode;
    nid->k2 = k2;
    nid->eta = eta;
    const ChebConst c = cheb_const(ecb);
    nid->theta = c.theta;
    nid->delta = c.delta;
    nid->sigma1 = c.sigma1;
    if (mode && k2) {
        nid->n_cheb += 1;
        nid->n_mixed += 1;
        nid->n_products += 1ull;  // the fp64 residual pass
        nid->n_products32 += (unsigned long long)(mode - 1 + k2 - 1);
    } else if (mode) {
        nid->n_cheb += 1;
        nid->n_products += (unsigned long long)(mode - 1);
    } else {
        nid->n_chol += 1;
    }
    if (eps_host) *eps_host = eps;  // host-mapped: the launch hint / the shard's decision
    if (mode_host) *mode_host = (double)mode;
    if (k2_host) *k2_host = (double)k2;
    // the host's wake-up word (host2[3], coherent host memory): the decision's sequence number,
    // mode and k2 in one 64-bit store, so the host polls it instead of waiting on an event
    // (an event marker in the stream cost ~6 us of idle device per sweep)
    if (tag_seq && mode_host)
        __hip_atomic_store((unsigned long long *)(mode_host + 2),
                           (tag_seq << 16) | ((unsigned long long)mode << 8) | (unsigned)k2,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(kNidSumWG) void k_nid_sums(const double *__restrict__ D,
                                                        const double *__restrict__ cn, int p_loc,
                                                        const DevScalars *sc,
                                                        double *__restrict__ wg_part) {
    __shared__ double part[kNidSumWG / 64][kNidTS + 1];
    __shared__ double thr[kNidTS];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const double tau2 = sc->tau * sc->tau;
    if (threadIdx.x < kNidTS) thr[threadIdx.x] = shard_threshold(tau2, threadIdx.x);
    __syncthreads();
    double acc[kNidTS + 1];
#pragma unroll
    for (int k = 0; k <= kNidTS; ++k) acc[k] = 0.0;
    for (int j = blockIdx.x * kNidSumWG + threadIdx.x; j < p_loc; j += gridDim.x * kNidSumWG) {
        const double dj = D[j], v = dj * cn[j];
        acc[kNidTS] += v;
#pragma unroll
        for (int k = 0; k < kNidTS; ++k)
            if (dj > thr[k]) acc[k] += v;
    }
#pragma unroll
    for (int k = 0; k <= kNidTS; ++k) acc[k] = wave_sum(acc[k]);
    if (lane == 0)
#pragma unroll
        for (int k = 0; k <= kNidTS; ++k) part[wid][k] = acc[k];
    __syncthreads();
    if (threadIdx.x <= kNidTS) {
        double s = 0.0;
        for (int w = 0; w < kNidSumWG / 64; ++w) s += part[w][threadIdx.x];
        wg_part[(size_t)blockIdx.x * (kNidTS + 1) + threadIdx.x] = s;
    }
}

// red = the G workgroups' sums and Lambda (thread (k, q) adds workgroups q, q + 8, ... of
// sum k, then the eight in order: a fixed order); decide: the unsharded decision at once
constexpr int kNidRedQ = 8;
template <bool WT>
__device__ __forceinline__ void nid_reduce_body(const double *__restrict__ wg_part, int G,
                                                const DevScalars *sc, int k_launched, int allow,
                                                int decide, NidState *nid,
                                                double *__restrict__ red, double *eps_host,
                                                int allow_mixed, unsigned long long tag_seq) {
    __shared__ double pq[kNidRedQ][kNidTS + 1];
    __shared__ double r[kNidTS + 2];
    // WT: partials written through by other workgroups of the running launch
    auto ld = [&](size_t i) {
        return WT ? __hip_atomic_load(&wg_part[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                  : wg_part[i];
    };
    const int t = threadIdx.x;
    for (int tt = t; tt < kNidRedQ * (kNidTS + 1); tt += blockDim.x) {
        const int k = tt % (kNidTS + 1), q = tt / (kNidTS + 1);
        double a[4] = {0.0, 0.0, 0.0, 0.0};
        int b = q;
        for (; b + 3 * kNidRedQ < G; b += 4 * kNidRedQ)
#pragma unroll
            for (int u = 0; u < 4; ++u) a[u] += ld((size_t)(b + u * kNidRedQ) * (kNidTS + 1) + k);
        for (; b < G; b += kNidRedQ) a[0] += ld((size_t)b * (kNidTS + 1) + k);
        pq[q][k] = (a[0] + a[1]) + (a[2] + a[3]);
    }
    __syncthreads();
    if (t <= kNidTS) {
        double s = 0.0;
#pragma unroll
        for (int q = 0; q < kNidRedQ; ++q) s += pq[q][t];
        r[t] = s;
        red[t] = s;
    }
    if (t == kNidTS + 1) {
        const double lam = nid->lambda_x;
        const double v = lam > 0.0 ? lam : HUGE_VAL;
        r[t] = v;
        red[t] = v;
    }
    __syncthreads();
    // decide 1: eps into eps_host (the launch hint); 2: [eps, mode, k2] into eps_host[0..2]
    if (decide && t < 64)
        nid_finish(r, sc, k_launched, allow, nid, eps_host, decide == 2 ? eps_host + 1 : nullptr,
                   decide == 2 ? allow_mixed : 0, decide == 2 ? eps_host + 2 : nullptr,
                   decide == 2 ? tag_seq : 0ull);
}
__global__ __launch_bounds__(64 * 5) void k_nid_reduce(const double *__restrict__ wg_part, int G,
                                                       const DevScalars *sc, int k_launched,
                                                       int allow, int decide, NidState *nid,
                                                       double *__restrict__ red,
                                                       double *eps_host, int allow_mixed,
                                                       unsigned long long tag_seq) {
    nid_reduce_body<false>(wg_part, G, sc, k_launched, allow, decide, nid, red, eps_host,
                           allow_mixed, tag_seq);
}

__global__ __launch_bounds__(64) void k_nid_decide_from(const double *__restrict__ red,
                                                        const DevScalars *sc, int k_launched,
                                                        NidState *nid, double *host2,
                                                        unsigned long long tag_seq) {
    nid_finish(red, sc, k_launched, 1, nid, host2, host2 + 1, 0, host2 + 2, tag_seq);
}

// Row sums of the nparts partial n-vectors for rows [64 b, 64 b + 64): wave w adds partials
// w, w + 16, ... for its lane's row into eight independent accumulators (eight loads in
// flight per lane: the partials were written by every XCD, so each load is an L2 miss), the
// accumulators are added pairwise, then the sixteen wave sums in order (a fixed order:
// bitwise reproducible).  Returns the sum on wave 0 (lane = row offset).
constexpr int kRedWaves = 16;
__device__ __forceinline__ double part_rowsum(const double *__restrict__ part, int nparts,
                                              int n_pad, int row, double (*red)[64]) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    double a[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] = 0.0;
    if (row < n_pad) {
        int q = wid;
        for (; q + 7 * kRedWaves < nparts; q += 8 * kRedWaves)
#pragma unroll
            for (int u = 0; u < 8; ++u) a[u] += part[(size_t)(q + u * kRedWaves) * n_pad + row];
        for (; q < nparts; q += kRedWaves) a[0] += part[(size_t)q * n_pad + row];
    }
    red[wid][lane] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    __syncthreads();
    double s = 0.0;
    if (wid == 0)
#pragma unroll
        for (int w = 0; w < kRedWaves; ++w) s += red[w][lane];
    return s;
}

// Row sums of the nparts partial n-vectors for the RW rows [row0, row0 + RW) of a 1024-thread
// workgroup: thread (slot s, row r) adds partials s, s + S, ... (S = 1024 / RW slots, eight
// independent accumulators), then the S slot sums are added in a fixed two-level order (eight
// groups of S / 8 slots, then the eight groups): bitwise reproducible.  RW = 8 spreads the
// sum of many partials over n_pad / 8 workgroups -- at C3 the 1568 X u partials of the fused
// lambda launch (25.7 MB) took 15.7 us in 32 workgroups of 64 rows, each thread ~100 dependent
// loads deep; 10.9-11.0 us now, and the 512 E-apply partials 6.0 -> 5.0 us (round 4,
// gpurun_out/prof_v; non-temporal partial stores measured slower: 12.2 us).  Returns the row
// sum on threads [0, RW).
constexpr int kRsThreads = 1024;
template <int RW>
__device__ __forceinline__ double part_rowsum_rw(const double *__restrict__ part, int nparts,
                                                 int n_pad, int row0) {
    constexpr int S = kRsThreads / RW, G2 = S < 8 ? S : 8;
    __shared__ double red[S][RW];
    __shared__ double red2[G2][RW];
    const int r = threadIdx.x % RW, sl = threadIdx.x / RW;
    const int row = row0 + r;
    double a[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    if (row < n_pad) {
        int q = sl;
        for (; q + 7 * S < nparts; q += 8 * S)
#pragma unroll
            for (int u = 0; u < 8; ++u) a[u] += part[(size_t)(q + u * S) * n_pad + row];
        for (; q < nparts; q += S) a[0] += part[(size_t)q * n_pad + row];
    }
    red[sl][r] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    __syncthreads();
    if ((int)threadIdx.x < G2 * RW) {
        const int g = threadIdx.x / RW;
        double v = 0.0;
#pragma unroll
        for (int k = 0; k < S / G2; ++k) v += red[g * (S / G2) + k][r];
        red2[g][r] = v;
    }
    __syncthreads();
    double v = 0.0;
    if ((int)threadIdx.x < RW)
#pragma unroll
        for (int g = 0; g < G2; ++g) v += red2[g][r];
    return v;
}

// The row block of workgroup b: consecutive blocks on one XCD (dispatch deals workgroups to
// the 8 XCDs round-robin), so the two 64-byte halves of a partial's 128-byte line, read by
// blocks 2c and 2c + 1 at RW = 8, meet in the same L2.
__device__ __forceinline__ int rs_block(int xcd) {
    const int G = (int)gridDim.x, b = (int)blockIdx.x;
    if (!xcd || (G & 7)) return b;
    return (b & 7) * (G >> 3) + (b >> 3);
}

// rows per workgroup for nparts partials: 8 when there are many (more workgroups, fewer
// dependent loads per thread), else 64.  (4 rows -- 32-byte row segments -- for the 1568
// partials at C3 took 19.1 us against 11.0: gpurun_out/prof_ac.)
// bb_set_tuning key 12: the XCD-aware row blocks of the partial row sums (rs_block; 1, the
// default) or blocks in dispatch order (0).  C3 at the driver's settings 2010 against 1993
// sweeps/s (gpurun_out/ab_drv_p1_x*).
int g_rs_xcd = 1;
static int rowsum_rw(int nparts) { return nparts >= 128 ? 8 : 64; }

// r_0 = y / sig - (X u / sig + delta), x_1 = d_0 = r_0 / theta (x_0 = 0).  X u arrives as
// nparts partial n-vectors (the fused lambda launch, k_eapply<XU>, or the sparse row pass
// with nparts = 1).
template <int RW>
__global__ __launch_bounds__(kRsThreads) void k_cheb_init(
    const double *__restrict__ xu_part, int nparts, int n, int n_pad,
    const double *__restrict__ y, const DevScalars *sc, Key key, uint64_t t, const NidState *nid,
    double *x, double *r, double *d, double *b, int xcd) {
    if (nid->mode == 0) return;
    const int i = rs_block(xcd) * RW + (int)threadIdx.x;
    const double xu = part_rowsum_rw<RW>(xu_part, nparts, n_pad, rs_block(xcd) * RW);
    if ((int)threadIdx.x >= RW || i >= n_pad) return;
    double rhs = 0.0;
    if (i < n) {
        const double sig = sqrt(sc->sig2);
        const double delta = normal_at(key, t, KIND_DELTA, (uint64_t)i);
        rhs = y[i] / sig - (xu / sig + delta);  // k_form_m's right-hand side
    }
    const double d0 = rhs / nid->theta;
    r[i] = rhs;
    d[i] = d0;
    x[i] = d0;
    if (b) b[i] = rhs;
}

// Chebyshev step j (1 <= j <= K - 1): q = d + (sum of the E-apply partials) / sig2,
// r_j = r_{j-1} - q, d_j = rho_j rho_{j-1} d_{j-1} + (2 rho_j / delta) r_j, x_{j+1} = x_j + d_j.
template <int RW>
__global__ __launch_bounds__(kRsThreads) void k_cheb_step(
    const double *__restrict__ part, int nparts, int n_pad, const DevScalars *sc,
    const NidState *nid, int j, double *x, double *r, double *d, int phase, int xcd) {
    if ((phase == 1 ? nid->mode : nid->k2) <= j) return;
    const int i = rs_block(xcd) * RW + (int)threadIdx.x;
    const double e = part_rowsum_rw<RW>(part, nparts, n_pad, rs_block(xcd) * RW);
    if ((int)threadIdx.x >= RW || i >= n_pad) return;
    const double dv = d[i];
    const double qv = dv + e / sc->sig2;
    const double rv = r[i] - qv;
    const double s1 = nid->sigma1;
    const double rho0 = cheb_rho(s1, j - 1), rho1 = 1.0 / (2.0 * s1 - rho0);
    const double dn = rho1 * rho0 * dv + (2.0 * rho1 / nid->delta) * rv;
    r[i] = rv;
    d[i] = dn;
    x[i] += dn;
}

// The mixed plan's restart (k2 > 0): r = b - x - (the residual pass's E x partials) / sig2,
// the correction's first iterate d = r / theta added to x (x then holds x0 + c_1).
template <int RW>
__global__ __launch_bounds__(kRsThreads) void k_cheb_restart(
    const double *__restrict__ part, int nparts, int n_pad, const DevScalars *sc,
    const NidState *nid, const double *__restrict__ b, double *x, double *r, double *d, int xcd) {
    if (nid->k2 == 0 || nid->mode == 0) return;
    const int i = rs_block(xcd) * RW + (int)threadIdx.x;
    const double e = part_rowsum_rw<RW>(part, nparts, n_pad, rs_block(xcd) * RW);
    if ((int)threadIdx.x >= RW || i >= n_pad) return;
    const double xv = x[i];
    const double rv = b[i] - (xv + e / sc->sig2);
    const double dv = rv / nid->theta;
    r[i] = rv;
    d[i] = dv;
    x[i] = xv + dv;
}

// out[i] = sum of the nparts partials of row i (setup: power iteration on X X')
__global__ __launch_bounds__(64 * kRedWaves) void k_part_sum(const double *__restrict__ part,
                                                             int nparts, int n_pad,
                                                             double *__restrict__ out) {
    __shared__ double red[kRedWaves][64];
    const int i = blockIdx.x * 64 + (threadIdx.x & 63);
    const double v = part_rowsum(part, nparts, n_pad, i, red);
    if (threadIdx.x < 64 && i < n_pad) out[i] = v;
}

// M = U I - G (upper triangle, column-major ldm) from the packed Gram G (red2 layout)
__global__ __launch_bounds__(256) void k_shift_gram(const double *__restrict__ red2, int n_pad,
                                                    double U, double *__restrict__ M, int ldm) {
    const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= tri_count(n_pad)) return;
    int c = (int)((sqrt(8.0 * (double)idx + 1.0) - 1.0) * 0.5);
    while ((size_t)c * (c + 1) / 2 > idx) --c;
    while ((size_t)(c + 1) * (c + 2) / 2 <= idx) ++c;
    const int r = (int)(idx - (size_t)c * (c + 1) / 2);
    M[(size_t)r + (size_t)c * ldm] = (r == c ? U : 0.0) - red2[idx];
}

// ---------------------------------------------------------------------------------------
// One pass over dense X: part[wg][row] = sum over the workgroup's columns c of
//   X[row, c] D_c (X[:, c]' v).
// Workgroup g takes column chunks of kEaCols = 8 columns g, g + G, ...; thread t holds rows
// t + 256 m (m < NR = n_pad / 256) of the chunk in registers, so each column is read from
// HBM once for both its dot product and its update.  Dot products: per-thread partial sums,
// a fixed xor tree per wave, the four waves' sums added in order.
// ---------------------------------------------------------------------------------------
constexpr int kEaCols = 8;
constexpr int kEaThreads = 256;

// XU: the same pass forming X u (part[wg][row] = sum_c X[row, c] D_c, with D = u), for the
// right-hand side: no dot products.  T: the element type streamed (double, or float for the
// mixed plan's fp32 copy of X -- converted exactly to double, so the arithmetic is fp64).
template <int NR, bool XU, typename T>
__device__ __forceinline__ void eapply_body(const T *__restrict__ X, int ldx, int n_pad,
                                            int p_loc, const double *__restrict__ D,
                                            const double *__restrict__ v,
                                            double *__restrict__ part) {
    __shared__ double ws[4][kEaCols];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    double vr[NR], acc[NR];
#pragma unroll
    for (int m = 0; m < NR; ++m) {
        const int row = tid + kEaThreads * m;
        vr[m] = (!XU && row < n_pad) ? v[row] : 0.0;
        acc[m] = 0.0;
    }
    const int nchunk = (p_loc + kEaCols - 1) / kEaCols;
    for (int ch = blockIdx.x; ch < nchunk; ch += gridDim.x) {
        const int c0 = ch * kEaCols;
        // the chunk's elements in their stored type, every load in flight before the first use
        // (a conversion inside a guarded load makes the compiler wait for each load in turn:
        // the fp32 pass then ran at a third of the fp64 pass's rate)
        T raw[kEaCols][NR];
        if (c0 + kEaCols <= p_loc && NR * kEaThreads <= n_pad) {  // uniform: a full chunk
#pragma unroll
            for (int c = 0; c < kEaCols; ++c)
#pragma unroll
                for (int m = 0; m < NR; ++m)
                    raw[c][m] = __builtin_nontemporal_load(X + (size_t)(c0 + c) * ldx +
                                                           tid + kEaThreads * m);
        } else {
#pragma unroll
            for (int c = 0; c < kEaCols; ++c) {
                const bool ok = c0 + c < p_loc;
                const T *col = X + (size_t)(c0 + c) * ldx;
#pragma unroll
                for (int m = 0; m < NR; ++m) {
                    const int row = tid + kEaThreads * m;
                    raw[c][m] = (ok && row < n_pad) ? __builtin_nontemporal_load(col + row) : T(0);
                }
            }
        }
        double xv[kEaCols][NR];
#pragma unroll
        for (int c = 0; c < kEaCols; ++c)
#pragma unroll
            for (int m = 0; m < NR; ++m) xv[c][m] = (double)raw[c][m];
        if constexpr (XU) {
#pragma unroll
            for (int c = 0; c < kEaCols; ++c) {
                const double f = (c0 + c < p_loc) ? D[c0 + c] : 0.0;
#pragma unroll
                for (int m = 0; m < NR; ++m) acc[m] = __builtin_fma(xv[c][m], f, acc[m]);
            }
            continue;
        }
        double s[kEaCols];
#pragma unroll
        for (int c = 0; c < kEaCols; ++c) {
            double a = 0.0;
#pragma unroll
            for (int m = 0; m < NR; ++m) a = __builtin_fma(xv[c][m], vr[m], a);
            s[c] = wave_sum(a);
        }
        __syncthreads();  // the previous chunk's ws reads are done
        if (lane == 0)
#pragma unroll
            for (int c = 0; c < kEaCols; ++c) ws[wid][c] = s[c];
        __syncthreads();
#pragma unroll
        for (int c = 0; c < kEaCols; ++c) {
            const double dc = (c0 + c < p_loc) ? D[c0 + c] : 0.0;
            const double f = dc * (((ws[0][c] + ws[1][c]) + ws[2][c]) + ws[3][c]);
#pragma unroll
            for (int m = 0; m < NR; ++m) acc[m] = __builtin_fma(xv[c][m], f, acc[m]);
        }
    }
#pragma unroll
    for (int m = 0; m < NR; ++m) {
        const int row = tid + kEaThreads * m;
        if (row < n_pad) part[(size_t)blockIdx.x * n_pad + row] = acc[m];
    }
}

// KIND (launch_eapply): 0 product j of the first solve (X32 when the mixed plan was taken),
// 1 X u (XU), 2 the mixed plan's fp64 residual pass, 3 product j of its correction solve.
// Each launch returns at once unless the device's decision needs it (the gate).
template <int NR, int KIND>
__global__ __launch_bounds__(kEaThreads) void k_eapply(const double *__restrict__ X,
                                                       const float *__restrict__ X32, int ldx,
                                                       int n_pad, int p_loc,
                                                       const double *__restrict__ D,
                                                       const double *__restrict__ v,
                                                       const NidState *nid, int j,
                                                       double *__restrict__ part) {
    if constexpr (KIND == 1) {
        if (nid->mode == 0) return;
        eapply_body<NR, true, double>(X, ldx, n_pad, p_loc, D, v, part);
    } else if constexpr (KIND == 0) {
        if (nid->mode <= j) return;
        if (X32 && nid->k2 > 0)
            eapply_body<NR, false, float>(X32, ldx, n_pad, p_loc, D, v, part);
        else
            eapply_body<NR, false, double>(X, ldx, n_pad, p_loc, D, v, part);
    } else if constexpr (KIND == 2) {
        if (nid->k2 == 0 || nid->mode == 0) return;
        eapply_body<NR, false, double>(X, ldx, n_pad, p_loc, D, v, part);
    } else {
        if (nid->k2 <= j) return;
        eapply_body<NR, false, float>(X32, ldx, n_pad, p_loc, D, v, part);
    }
}

// X32 = fl32(X); *bad = 1 for an entry whose fp32 rounding is not within 2^-24 relative
// (beyond the normal range: the mixed plan is then not used)
__global__ __launch_bounds__(256) void k_cast_f32(const double *__restrict__ X, int ldx,
                                                  int n_pad, int ncols, float *__restrict__ X32,
                                                  int *bad) {
    const size_t tot = (size_t)n_pad * ncols;
    bool b = false;
    for (size_t e = (size_t)blockIdx.x * 256 + threadIdx.x; e < tot; e += (size_t)gridDim.x * 256) {
        const size_t c = e / n_pad, r = e % n_pad;
        const double x = X[c * ldx + r];
        const double ax = fabs(x);
        b |= !(ax <= 0x1p126) || (ax != 0.0 && ax < 0x1p-125);
        X32[c * ldx + r] = (float)x;
    }
    if (__any(b) && (threadIdx.x & 63) == 0) atomicOr(bad, 1);
}

// ---------------------------------------------------------------------------------------
// Sparse X (CSC + CSR): s_j = D_j (X_j' v) by columns (16 lanes per column), then
// part[row] = X_row . s by rows (a wave per row) -- two passes over the non-zeros.
// ---------------------------------------------------------------------------------------
constexpr int kSpEaLanes = 16;

__global__ __launch_bounds__(256) void k_sp_eapply_cols(const int *__restrict__ colptr,
                                                        const int *__restrict__ rowidx,
                                                        const double *__restrict__ cval,
                                                        int p_loc, const double *__restrict__ D,
                                                        const double *__restrict__ v,
                                                        const NidState *nid, int j,
                                                        double *__restrict__ s) {
    if (nid->mode <= j) return;
    const long gid = (long)blockIdx.x * 256 + threadIdx.x;
    const int c = (int)(gid / kSpEaLanes);
    const int q = (int)(gid % kSpEaLanes);
    double a = 0.0;
    if (c < p_loc)
        for (int k = colptr[c] + q; k < colptr[c + 1]; k += kSpEaLanes) a += cval[k] * v[rowidx[k]];
#pragma unroll
    for (int o = kSpEaLanes / 2; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
    if (q == 0 && c < p_loc) s[c] = D[c] * a;
}

__global__ __launch_bounds__(256) void k_sp_eapply_rows(const int *__restrict__ rowptr,
                                                        const int *__restrict__ colidx,
                                                        const double *__restrict__ rval,
                                                        int n_pad, const double *__restrict__ s,
                                                        const NidState *nid, int j, int pol,
                                                        double *__restrict__ out) {
    // pol 0: gated as an E-apply (step j); pol 1: X u for the right-hand side (mode != 0)
    if (pol == 0 ? nid->mode <= j : nid->mode == 0) return;
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n_pad) return;
    double a = 0.0;
    for (int k = rowptr[row] + lane; k < rowptr[row + 1]; k += 64) a += rval[k] * s[colidx[k]];
    a = wave_sum(a);
    if (lane == 0) out[row] = a;
}

// ---------------------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------------------
static int nid_cus() {
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

int eapply_parts(int p_loc, int n_pad) {
    (void)n_pad;
    const int nchunk = (p_loc + kEaCols - 1) / kEaCols;
    return std::max(1, std::min(nchunk, 2 * nid_cus()));
}

bool eapply_supported(int n_pad) { return n_pad <= 16 * kEaThreads; }


int nid_sum_groups(int p_loc) { return std::max(1, std::min(256, (p_loc + 255) / 256)); }

void launch_nid_sums(hipStream_t s, const double *D, const double *cn, int p_loc,
                     const DevScalars *sc, NidState *nid, int k_launched, int allow, int decide,
                     double *wg_part, double *red, double *eps_host) {
    const int G = nid_sum_groups(p_loc);
    k_nid_sums<<<G, kNidSumWG, 0, s>>>(D, cn, p_loc, sc, wg_part);
    k_nid_reduce<<<1, 64 * 5, 0, s>>>(wg_part, G, sc, k_launched, allow, decide, nid, red,
                                  eps_host, 0, 0ull);
}

void launch_nid_sums_decide(hipStream_t s, const double *D, const double *cn, int p_loc,
                            const DevScalars *sc, NidState *nid, int k_launched,
                            double *wg_part, double *red, double *host2, int allow_mixed,
                            unsigned long long tag_seq) {
    const int G = nid_sum_groups(p_loc);
    k_nid_sums<<<G, kNidSumWG, 0, s>>>(D, cn, p_loc, sc, wg_part);
    k_nid_reduce<<<1, 64 * 5, 0, s>>>(wg_part, G, sc, k_launched, 1, 2, nid, red, host2,
                                      allow_mixed, tag_seq);
}

void launch_nid_reduce(hipStream_t s, const double *wg_part, int G, const DevScalars *sc,
                       NidState *nid, double *red, int k_launched, double *host2,
                       int allow_mixed, unsigned long long tag_seq) {
    if (host2)
        k_nid_reduce<<<1, 64 * 5, 0, s>>>(wg_part, G, sc, k_launched, 1, 2, nid, red, host2,
                                          allow_mixed, tag_seq);
    else
        k_nid_reduce<<<1, 64 * 5, 0, s>>>(wg_part, G, sc, 0, 0, 0, nid, red, nullptr, 0, 0ull);
}

void launch_nid_decide_from(hipStream_t s, const double *red, const DevScalars *sc,
                            int k_launched, NidState *nid, double *host2,
                            unsigned long long tag_seq) {
    k_nid_decide_from<<<1, 64, 0, s>>>(red, sc, k_launched, nid, host2, tag_seq);
}

template <int KIND>
static void launch_pass(hipStream_t s, const double *X, const float *X32, int ldx, int n_pad,
                        int p_loc, const double *D, const double *v, const NidState *nid, int j,
                        double *part) {
    const int g = eapply_parts(p_loc, n_pad);
    const int nr = (n_pad + kEaThreads - 1) / kEaThreads;
    auto *kern = nr <= 1 ? k_eapply<1, KIND> : nr <= 2 ? k_eapply<2, KIND>
               : nr <= 4 ? k_eapply<4, KIND> : nr <= 8 ? k_eapply<8, KIND> : k_eapply<16, KIND>;
    if (KIND == 0) note_launch(KF_EAPPLY, (const void *)kern);
    kern<<<g, kEaThreads, 0, s>>>(X, X32, ldx, n_pad, p_loc, D, v, nid, j, part);
}

void launch_nid_xu(hipStream_t s, const double *X, int ldx, const double *u, int ncols,
                   int n_pad, const NidState *nid, double *part) {
    launch_pass<1>(s, X, nullptr, ldx, n_pad, ncols, u, nullptr, nid, 0, part);
}

void launch_cheb_init(hipStream_t s, const double *xu_part, int nparts, int n, int n_pad,
                      const double *y, const DevScalars *sc, uint64_t k0, uint64_t k1,
                      uint64_t t, const NidState *nid, double *x, double *r, double *d,
                      double *b) {
    if (rowsum_rw(nparts) == 8)
        k_cheb_init<8><<<(n_pad + 7) / 8, kRsThreads, 0, s>>>(xu_part, nparts, n, n_pad, y, sc,
                                                              Key{k0, k1}, t, nid, x, r, d, b,
                                                              g_rs_xcd);
    else
        k_cheb_init<64><<<(n_pad + 63) / 64, kRsThreads, 0, s>>>(xu_part, nparts, n, n_pad, y,
                                                                 sc, Key{k0, k1}, t, nid, x, r, d,
                                                                 b, g_rs_xcd);
}

void launch_cheb_step(hipStream_t s, const double *part, int nparts, int n_pad,
                      const DevScalars *sc, const NidState *nid, int j, double *x, double *r,
                      double *d, int phase) {
    if (rowsum_rw(nparts) == 8)
        k_cheb_step<8><<<(n_pad + 7) / 8, kRsThreads, 0, s>>>(part, nparts, n_pad, sc, nid, j, x,
                                                              r, d, phase, g_rs_xcd);
    else
        k_cheb_step<64><<<(n_pad + 63) / 64, kRsThreads, 0, s>>>(part, nparts, n_pad, sc, nid, j,
                                                                 x, r, d, phase, g_rs_xcd);
}

void launch_cheb_restart(hipStream_t s, const double *part, int nparts, int n_pad,
                         const DevScalars *sc, const NidState *nid, const double *b, double *x,
                         double *r, double *d) {
    if (rowsum_rw(nparts) == 8)
        k_cheb_restart<8><<<(n_pad + 7) / 8, kRsThreads, 0, s>>>(part, nparts, n_pad, sc, nid, b,
                                                                 x, r, d, g_rs_xcd);
    else
        k_cheb_restart<64><<<(n_pad + 63) / 64, kRsThreads, 0, s>>>(part, nparts, n_pad, sc, nid,
                                                                    b, x, r, d, g_rs_xcd);
}

void launch_eapply(hipStream_t s, const double *X, int ldx, int n_pad, int p_loc,
                   const double *D, const double *v, const NidState *nid, int j, double *part,
                   const float *X32, int kind) {
    switch (kind) {
        case 2: launch_pass<2>(s, X, X32, ldx, n_pad, p_loc, D, v, nid, j, part); break;
        case 3: launch_pass<3>(s, X, X32, ldx, n_pad, p_loc, D, v, nid, j, part); break;
        default: launch_pass<0>(s, X, X32, ldx, n_pad, p_loc, D, v, nid, j, part); break;
    }
}

void launch_cast_f32(hipStream_t s, const double *X, int ldx, int n_pad, int ncols, float *X32,
                     int *bad) {
    const size_t tot = (size_t)n_pad * ncols;
    const unsigned g = (unsigned)std::min<size_t>((tot + 255) / 256, 4096);
    k_cast_f32<<<g, 256, 0, s>>>(X, ldx, n_pad, ncols, X32, bad);
}

void launch_sp_eapply(hipStream_t s, const int *colptr, const int *rowidx, const double *cval,
                      const int *rowptr, const int *colidx, const double *rval, int p_loc,
                      int n_pad, const double *D, const double *v, const NidState *nid, int j,
                      double *scratch_p, double *out) {
    const long threads = (long)p_loc * kSpEaLanes;
    k_sp_eapply_cols<<<(unsigned)((threads + 255) / 256), 256, 0, s>>>(colptr, rowidx, cval,
                                                                       p_loc, D, v, nid, j,
                                                                       scratch_p);
    k_sp_eapply_rows<<<(n_pad + 3) / 4, 256, 0, s>>>(rowptr, colidx, rval, n_pad, scratch_p,
                                                     nid, j, 0, out);
}

void launch_part_sum(hipStream_t s, const double *part, int nparts, int n_pad, double *out) {
    k_part_sum<<<(n_pad + 63) / 64, 64 * kRedWaves, 0, s>>>(part, nparts, n_pad, out);
}

void launch_shift_gram(hipStream_t s, const double *red2, int n_pad, double U, double *M,
                       int ldm) {
    const size_t tot = tri_count(n_pad);
    k_shift_gram<<<(unsigned)((tot + 255) / 256), 256, 0, s>>>(red2, n_pad, U, M, ldm);
}

void launch_sp_nid_xu(hipStream_t s, const int *rowptr, const int *colidx, const double *rval,
                      int n_pad, const double *u, const NidState *nid, double *out) {
    k_sp_eapply_rows<<<(n_pad + 3) / 4, 256, 0, s>>>(rowptr, colidx, rval, n_pad, u, nid, 0, 1,
                                                     out);
}

// ---------------------------------------------------------------------------------------
// The split lambda + X u launch (bb_set_tuning key 7 = 3, the default) with the decision's
// bound sums folded into its stream role (they need D, which the launch writes)
// ---------------------------------------------------------------------------------------
// Mode 3: the draws and the X u stream as two roles of one grid.  Workgroups [0, ndraw) draw:
// each claims 32-coefficient chunks from a counter (any resident draw workgroup takes the next
// chunk, so the draws never wait on a workgroup that is not resident), draws them exactly as
// k_lambda_xw does, and releases the chunk's u with a flag (write-through stores, drained,
// then the flag, tagged with the launch's epoch: flags are never cleared).  Workgroups
// [ndraw, grid) stream X: unit q = (chunk q / 4, its 8-column quarter q % 4) for q = s, s + S,
// ... -- a fixed assignment, so each stream workgroup's partial n-vector (rows t + 256 m in
// thread t's registers) sums the same columns in the same order every launch (bitwise
// reproducible) -- waiting for a chunk's flag before its first unit.  With two draw and one
// stream workgroup per CU the stream's loads run beside the draws' VALU work instead of
// alternating with it inside each workgroup (mode 2).  Partials: S = the stream workgroups.
// out of line: the decision's code stays out of the draw role's register allocation
// (scalar arguments: a struct passed by reference would be copied to scratch memory)
__device__ __noinline__ void nid_fold_decide(const double *wg_part, int S, const DevScalars *sc,
                                             int k_launched, int allow_mixed, NidState *nid,
                                             double *red, double *host2,
                                             unsigned long long tag_seq) {
    nid_reduce_body<true>(wg_part, S, sc, k_launched, 1, 2, nid, red, host2, allow_mixed,
                          tag_seq);
}

template <int NR>
__device__ __forceinline__ void lambda_xs_body(const double *beta, int p_loc, int p_pad,
                                               uint64_t j0, const DevScalars *sc, Key key,
                                               uint64_t t, double *lam, double *D, double *u,
                                               double *lam_trace, uint32_t *err,
                                               const double *__restrict__ X, int ldx, int n_pad,
                                               int nchunk, double *__restrict__ xu_part,
                                               unsigned int *sync, unsigned int ep, int ndraw,
                                               NidFold fold) {
    constexpr int C = 32;
    const int tid = threadIdx.x;
    unsigned int *ctr = sync + nchunk;
    if ((int)blockIdx.x < ndraw) {
        __shared__ int claim;
        const double tau = sc->tau;
        for (;;) {
            if (tid == 0)
                claim = (int)__hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
            __syncthreads();
            const int ch = claim;
            __syncthreads();  // claim is rewritten by the next round
            if (ch >= nchunk) {
                // the last of the nchunk + ndraw claims re-arms the counter for the next launch
                if (tid == 0 && ch == nchunk + ndraw - 1)
                    __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return;
            }
            const int i = ch * C + tid / 8;
            const bool active = i < p_loc;
            const double b = active ? beta[i] : 0.0;
            const double x = stable_wave_draw(active, b * b / (tau * tau), 0.5 * sc->alpha, 1.0,
                                              key, t, j0 + (uint64_t)i, err);
            if ((tid % 8) == 0) {
                double uv = 0.0;
                if (active) {
                    const double l = 2 * x;
                    lam[i] = l;
                    if (lam_trace) lam_trace[i] = l;
                    const double d = (tau * tau) / l;
                    __hip_atomic_store(&D[i], d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    uv = sqrt(d) * normal_at(key, t, KIND_BETA_Z, j0 + (uint64_t)i);
                } else if (i < p_pad) {
                    lam[i] = 1.0;
                    __hip_atomic_store(&D[i], 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                if (i < p_pad)
                    __hip_atomic_store(&u[i], uv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) __hip_atomic_store(&sync[ch], ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    // ---- stream role ----
    const int sidx = (int)blockIdx.x - ndraw, S = (int)gridDim.x - ndraw;
    __shared__ double us[8];
    // the fold: the near-identity bound sums of this workgroup's columns (k_nid_sums' kNidTS + 1
    // per column, D_j |x_j|^2 over D_j > T_k and the trace).  Thread (column slot tid / 32,
    // threshold tid % 32) accumulates its slot's terms over the units in order -- a fixed order,
    // so the partials are reproducible -- and slot threads k == 0 the trace.
    const bool sums = fold.wg_part != nullptr;
    const double nthr = sums ? shard_threshold(sc->tau * sc->tau, tid & 31) : 0.0;
    double nacc = 0.0, ntr = 0.0;
    double a[NR];
#pragma unroll
    for (int m = 0; m < NR; ++m) a[m] = 0.0;
    const int nunit = nchunk * 4;
    int have = -1;  // the chunk whose flag this workgroup has seen
    for (int q = sidx; q < nunit; q += S) {
        const int ch = q >> 2, c0 = ch * C + (q & 3) * 8;
        if (ch != have) {
            if (tid == 0) {
                const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                while (__hip_atomic_load(&sync[ch], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) !=
                       ep) {
                    __builtin_amdgcn_s_sleep(2);
                    // bounded like every cross-workgroup wait (2 s): a launch that cannot make
                    // progress ends with error bit 16 instead of hanging the device
                    if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
                        atomicOr(err, 16u);
                        break;
                    }
                }
            }
            have = ch;
        }
        __syncthreads();  // the flag is seen; us of the previous unit is no longer read
        double ndv = 0.0, ncv = 0.0;
        if (sums && c0 + (tid >> 5) < p_loc) {
            ndv = __hip_atomic_load(&D[c0 + (tid >> 5)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ncv = fold.cn[c0 + (tid >> 5)];
        }
        if (tid < 8)
            us[tid] = c0 + tid < p_pad ? __hip_atomic_load(&u[c0 + tid], __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT)
                                       : 0.0;
        __syncthreads();
        if (sums) {
            const double v = ndv * ncv;
            if (ndv > nthr) nacc += v;
            ntr += v;
        }
        constexpr int CB = NR >= 16 ? 2 : 4;  // columns in flight (8 measured no faster)
#pragma unroll
        for (int cb = 0; cb < 8; cb += CB) {
            double xv[CB][NR];
#pragma unroll
            for (int k = 0; k < CB; ++k) {
                const int col = c0 + cb + k;
                const bool ok = col < p_loc;
                const double *xc = X + (size_t)col * ldx;
#pragma unroll
                for (int m = 0; m < NR; ++m) {
                    const int row = tid + 256 * m;
                    xv[k][m] = (ok && row < n_pad) ? __builtin_nontemporal_load(xc + row) : 0.0;
                }
            }
#pragma unroll
            for (int k = 0; k < CB; ++k) {
                const double f = us[cb + k];
#pragma unroll
                for (int m = 0; m < NR; ++m) a[m] = __builtin_fma(xv[k][m], f, a[m]);
            }
        }
    }
#pragma unroll
    for (int m = 0; m < NR; ++m) {
        const int row = tid + 256 * m;
        if (row < n_pad) xu_part[(size_t)sidx * n_pad + row] = a[m];
    }
    if (!sums) return;
    __shared__ double nsum[8][kNidTS + 1];
    nsum[tid >> 5][tid & 31] = nacc;
    if ((tid & 31) == 0) nsum[tid >> 5][kNidTS] = ntr;
    __syncthreads();
    if (tid <= kNidTS) {
        double sv = 0.0;
#pragma unroll
        for (int c = 0; c < 8; ++c) sv += nsum[c][tid];
        __hip_atomic_store(&fold.wg_part[(size_t)sidx * (kNidTS + 1) + tid], sv, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!fold.decide) return;
    // unsharded: the stream workgroup that finishes last adds the S partials (k_nid_reduce's
    // body over the write-through partials) and decides, then re-arms the count
    __shared__ int last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
        last = __hip_atomic_fetch_add(fold.cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
               (unsigned)S - 1;
    __syncthreads();
    if (!last) return;
    if (tid == 0) __hip_atomic_store(fold.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    nid_fold_decide(fold.wg_part, S, sc, fold.k_launched, fold.allow_mixed, fold.nid, fold.red,
                    fold.host2, fold.tag_seq);
}
template <int NR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 8))) void
k_lambda_xs(const double *beta, int p_loc, int p_pad, uint64_t j0, const DevScalars *sc, Key key,
            uint64_t t, double *lam, double *D, double *u, double *lam_trace, uint32_t *err,
            const double *__restrict__ X, int ldx, int n_pad, int nchunk,
            double *__restrict__ xu_part, unsigned int *sync, unsigned int ep, int ndraw,
            NidFold fold) {
    lambda_xs_body<NR>(beta, p_loc, p_pad, j0, sc, key, t, lam, D, u, lam_trace, err, X, ldx, n_pad,
                       nchunk, xu_part, sync, ep, ndraw, fold);
}

// the split launch needs its whole grid resident (three workgroups per CU)
// a flag per 32-coefficient chunk + the claim counter
int lambda_xs_sync_words(int p_pad) { return (p_pad + 31) / 32 + 1; }

int lambda_xs_resident(int nr) {
    static int cache[3] = {-1, -1, -1};
    static std::mutex mu;
    std::lock_guard<std::mutex> lk(mu);
    const int idx = nr <= 4 ? 0 : nr <= 8 ? 1 : 2;
    int &c = cache[idx];
    if (c < 0) {
        int nb = 0;
        const hipError_t e = idx == 0 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_lambda_xs<4>, 256, 0)
                           : idx == 1 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_lambda_xs<8>, 256, 0)
                                      : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_lambda_xs<16>, 256, 0);
        c = e == hipSuccess ? nb : 0;
    }
    return c;
}


int launch_lambda_xs(hipStream_t s, const double *beta, int p_loc, int p_pad, uint64_t j0,
                     const DevScalars *sc, uint64_t k0, uint64_t k1, uint64_t t, double *lam,
                     double *D, double *u, double *lam_trace, uint32_t *err, const double *X, int ldx, int n_pad,
                     int nchunk, double *xu_part, unsigned int *sync, unsigned int ep, int ndraw,
                     int nstream, const NidFold *fold) {
    const int nr = (n_pad + 255) / 256;
    NidFold f{};
    if (fold && fold->wg_part && (!fold->decide || fold->cnt)) f = *fold;
    auto *kk = nr <= 4 ? k_lambda_xs<4> : nr <= 8 ? k_lambda_xs<8> : k_lambda_xs<16>;
    note_launch(KF_LAMBDA, (const void *)kk);
    const Key key{k0, k1};
    kk<<<ndraw + nstream, 256, 0, s>>>(beta, p_loc, p_pad, j0, sc, key, t, lam, D, u, lam_trace,
                                       err, X, ldx, n_pad, nchunk, xu_part, sync, ep, ndraw, f);
    return f.wg_part ? (f.decide ? 2 : 1) : 0;
}

}  // namespace bb
