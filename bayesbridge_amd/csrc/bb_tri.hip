// bb_tri.hip -- triangle-mixture Gibbs update for bridge.reg.tri (gfx950).
//
// Reference: Code/C/BridgeRegression.cpp:97-147 (sample_u, sample_omega with shape),
// :405-433 (sample_beta), :235-286 (rtnorm_gibbs); driver BridgeWrapper.cpp:80-204.
//
// rtnorm_gibbs is a sequential coordinate sweep over the p coordinates z = V'beta; each
// step needs the tightest bounds over all p box constraints |beta_j| <= b_j.  One
// workgroup of 256 threads runs the whole update: thread j owns coefficients
// j + 256 k (b_j and beta_cur_j = (tV' z)_j stay in registers), the row v_i. of tV is
// prefetched one coordinate ahead, the bounds are DPP-reduced per 16-lane row, then per
// wave (max/min are exact, so any tree gives the CPU checker's value) and every lane
// evaluates the same truncated-normal draw redundantly: one barrier per coordinate.
// beta_cur is kept up to date incrementally
// (beta_cur_j += v_ij dz_i) instead of recomputing dot(v_j, z) per coordinate as :254-258
// does: the same quantity in O(p^2) instead of O(p^3) per pass (oracle/bb_oracle.c
// bbo_tri_update uses the identical update order).
//
// r.tnorm comes from the un-vendored RNG library; it is restated from Robert (1995):
// normal or uniform rejection when the standardised interval holds 0, else Robert's
// uniform / translated-exponential proposal.  Counter kinds 8 (omega), 9 (u), 10 (z_i).
#include <hip/hip_runtime.h>

#include "bb_kernels.h"
#include "bb_sampler.h"

namespace bb {

namespace {

constexpr int kTriNT = 256;
constexpr int kTriE = kTriMaxP / kTriNT;  // coefficients per thread
constexpr long kTnMaxAttempts = 1l << 22;
constexpr unsigned KIND_TRI_OMEGA = 8, KIND_TRI_U = 9, KIND_TRI_Z = 10;

// Attempt 0 of every coordinate's draw is precomputed in parallel before the coordinate
// loop (pre = {r0, r1, Box-Muller normal of (r0, r1)}), so the serial chain only runs
// Philox on a rejection.  Bit-identical to drawing it in place.
struct Pre {
    double r0, r1, x0;
};

__device__ __forceinline__ double readlane_dd(double v, int lane) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, lane);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ void attempt(Key key, uint64_t t, uint64_t i, uint64_t it, long k,
                                        const Pre &pre, double &r0, double &r1, double &x0,
                                        bool need_x) {
    if (k == 0) {
        r0 = pre.r0;
        r1 = pre.r1;
        x0 = pre.x0;
    } else {
        U4 r = uniforms(key, t, KIND_TRI_Z, i, it, (uint64_t)k);
        r0 = r.r[0];
        r1 = r.r[1];
        x0 = need_x ? bm_normal(r0, r1) : 0.0;
    }
}

// Force-inlined: the compiler outlined tnorm, and an out-of-line call inside the
// coordinate loop costs its prologue's s_waitcnt vmcnt(0), which drains the row prefetch
// on every coordinate.  k0 > 0 resumes the rejection loop at attempt k0 (k_tri_chain's
// fall-through after its parallel attempts; `pre` is then unused).
__device__ __forceinline__ double tn_pos(double a, double b, Key key, uint64_t t, uint64_t i,
                                         uint64_t it, const Pre &pre, uint32_t *err,
                                         long k0 = 0) {
    const double sq = sqrt(a * a + 4.0);
    const double as = 0.5 * (a + sq);
    const double thr = a + 2.0 / (a + sq) * exp(0.5 + 0.25 * (a * a - a * sq));
    for (long k = k0; k < kTnMaxAttempts; ++k) {
        double r0, r1, x0;
        attempt(key, t, i, it, k, pre, r0, r1, x0, false);
        if (b <= thr) {
            const double x = a + (b - a) * r0;
            if (r1 <= exp(0.5 * (a * a - x * x))) return x;
        } else {
            const double x = a - log(r0) / as;
            const double e = x - as;
            if (x <= b && r1 <= exp(-0.5 * e * e)) return x;
        }
    }
    atomicOr(err, 64u);
    return a;
}

__device__ __forceinline__ double tnorm(double lo, double hi, double mu, double sd, Key key,
                                        uint64_t t, uint64_t i, uint64_t it, const Pre &pre,
                                        uint32_t *err, long k0 = 0) {
    const double a = (lo - mu) / sd, b = (hi - mu) / sd;
    if (!(a < b)) {
        atomicOr(err, 128u);
        return lo;
    }
    if (a <= 0.0 && b >= 0.0) {
        const bool wide = (b - a) >= 2.5066282746310002;  // sqrt(2 pi)
        for (long k = k0; k < kTnMaxAttempts; ++k) {
            double r0, r1, x0;
            attempt(key, t, i, it, k, pre, r0, r1, x0, wide);
            if (wide) {
                if (x0 >= a && x0 <= b) return mu + sd * x0;
            } else {
                const double x = a + (b - a) * r0;
                if (r1 <= exp(-0.5 * x * x)) return mu + sd * x;
            }
        }
        atomicOr(err, 64u);
        return lo;
    }
    if (a > 0.0) return mu + sd * tn_pos(a, b, key, t, i, it, pre, err, k0);
    return mu - sd * tn_pos(-b, -a, key, t, i, it, pre, err, k0);
}

// The same draw with attempts 0 .. K-1 evaluated in parallel, attempt k in lane k from its
// precomputed (r0, r1, x0): the lowest accepted attempt is the sequential loop's answer;
// if none of the K is accepted the loop resumes at attempt K.  lo, hi, mu, sd uniform; every
// lane of the wave calls this.
template <int K>
__device__ __forceinline__ double tnorm_par(double lo, double hi, double mu, double sd,
                                            double r0, double r1, double x0, Key key,
                                            uint64_t t, uint64_t i, uint64_t it, uint32_t *err) {
    const int lane = threadIdx.x & 63;
    const double a = (lo - mu) / sd, b = (hi - mu) / sd;
    if (!(a < b)) {
        atomicOr(err, 128u);
        return lo;
    }
    bool acc = false;
    double val = 0.0;
    if (a <= 0.0 && b >= 0.0) {
        if ((b - a) >= 2.5066282746310002) {  // sqrt(2 pi)
            acc = x0 >= a && x0 <= b;
            val = mu + sd * x0;
        } else {
            const double x = a + (b - a) * r0;
            acc = r1 <= exp(-0.5 * x * x);
            val = mu + sd * x;
        }
    } else {
        const double pa = a > 0.0 ? a : -b, pb = a > 0.0 ? b : -a;  // tn_pos's (a, b)
        const double sq = sqrt(pa * pa + 4.0);
        const double as = 0.5 * (pa + sq);
        const double thr = pa + 2.0 / (pa + sq) * exp(0.5 + 0.25 * (pa * pa - pa * sq));
        double x;
        if (pb <= thr) {
            x = pa + (pb - pa) * r0;
            acc = r1 <= exp(0.5 * (pa * pa - x * x));
        } else {
            x = pa - log(r0) / as;
            const double e = x - as;
            acc = x <= pb && r1 <= exp(-0.5 * e * e);
        }
        val = a > 0.0 ? mu + sd * x : mu - sd * x;
    }
    const uint64_t m = __ballot(acc && lane < K);
    if (m) return readlane_dd(val, __ffsll((unsigned long long)m) - 1);
    return tnorm(lo, hi, mu, sd, key, t, i, it, Pre{0.0, 0.0, 0.0}, err, K);
}

// Row-of-16 max / min through DPP (quad xor 1, quad xor 2, half-row mirror, row mirror):
// every lane of a 16-lane row ends with the row's extreme.  v_max_f64 takes no DPP operand
// on gfx9, so each step moves the two halves with v_mov_b32_dpp.  Replaces a 6-step
// ds_bpermute butterfly per value (an LDS round trip per step).
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double row16_max(double v) {
    v = fmax(v, dpp_d<0xB1>(v));
    v = fmax(v, dpp_d<0x4E>(v));
    v = fmax(v, dpp_d<0x141>(v));
    return fmax(v, dpp_d<0x140>(v));
}
__device__ __forceinline__ double row16_min(double v) {
    v = fmin(v, dpp_d<0xB1>(v));
    v = fmin(v, dpp_d<0x4E>(v));
    v = fmin(v, dpp_d<0x141>(v));
    return fmin(v, dpp_d<0x140>(v));
}

// Combine the four row extremes of a wave (every lane holds its row's value) through
// scalar reads of lanes 0, 16, 32, 48: the wave's extreme, uniform in every lane.
__device__ __forceinline__ double readlane_d(double v, int lane) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, lane);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double rows_max(double v) {
    return fmax(fmax(readlane_d(v, 0), readlane_d(v, 16)),
                fmax(readlane_d(v, 32), readlane_d(v, 48)));
}
__device__ __forceinline__ double rows_min(double v) {
    return fmin(fmin(readlane_d(v, 0), readlane_d(v, 16)),
                fmin(readlane_d(v, 32), readlane_d(v, 48)));
}

// tVc: tV column-major (tVc[i + j p] = tV(i, j)); tVr: its transpose (tVr[i p + j] =
// tV(i, j)), so row i of tV is contiguous for the coordinate loop.
__global__ __launch_bounds__(kTriNT) void k_tri_update(
    double *beta, double *u, double *omega, double *shape, int p, const double *tVc,
    const double *tVr, const double *av, const double *dv, const double *Gf, const double *cv,
    int ortho, const DevScalars *sc, int betaburn, Key key, uint64_t t, double *tr_beta,
    double *tr_u, double *tr_omega, double *tr_shape, uint32_t *err) {
    __shared__ double sz[kTriMaxP];
    __shared__ double sb[kTriMaxP];
    __shared__ double sbnd[kTriMaxP];
    __shared__ Pre spre[kTriMaxP];
    // per-coordinate constants staged once: a global load inside the serial loop would put
    // a full memory latency on every coordinate's critical path
    __shared__ double sav[kTriMaxP], sdv[kTriMaxP];
    // per-wave partials, double-buffered by coordinate parity: one barrier per coordinate
    __shared__ double shmax[2][kTriNT / 64], shmin[2][kTriNT / 64];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const double tau = sc->tau, sig2 = sc->sig2, alpha = sc->alpha;

    double bj[kTriE], bcur[kTriE];
#pragma unroll
    for (int e = 0; e < kTriE; ++e) {
        const int j = tid + e * kTriNT;
        bj[e] = 0.0;
        if (j < p) {
            const double betaj = beta[j];
            // sample_omega (BridgeRegression.cpp:130-146)
            const double aj = exp(alpha * log(fabs(betaj) / ((1.0 - u[j]) * tau)));
            const double prob = alpha / (1.0 + alpha * aj);
            U4 r = uniforms(key, t, KIND_TRI_OMEGA, (uint64_t)j, 0, 0);
            double w, sh;
            if (r.r[0] > prob) {
                sh = 1.0;
                w = -log(r.r[1]);  // Ga(1, 1)
            } else {
                sh = 2.0;
                w = -log(r.r[1]) - log(r.r[2]);  // Ga(2, 1)
            }
            const double om = w + aj;
            // sample_u (:97-111): flat(0, right)
            const double right = 1.0 - fabs(betaj) / tau * exp(-1.0 * log(om) / alpha);
            U4 r2 = uniforms(key, t, KIND_TRI_U, (uint64_t)j, 0, 0);
            const double uj = right * r2.r[0];
            bj[e] = (1.0 - uj) * exp(log(om) / alpha) * tau;  // sample_beta :410-412
            sbnd[j] = bj[e];
            omega[j] = om;
            shape[j] = sh;
            u[j] = uj;
            if (tr_omega) tr_omega[j] = om;
            if (tr_shape) tr_shape[j] = sh;
            if (tr_u) tr_u[j] = uj;
            sb[j] = betaj;
            sav[j] = ortho ? cv[j] : av[j];
            sdv[j] = ortho ? Gf[(size_t)j * p + j] : dv[j];
        }
    }
    __syncthreads();
    const double sig = sqrt(sig2);
    // Every thread reduces the per-wave partials in the same order and evaluates the same
    // draw (uniform control flow, no divergence), so no broadcast barrier is needed; the
    // owner of a coefficient keeps the state it alone reads later.
    auto precompute = [&](int it) {
        for (int i = tid; i < p; i += kTriNT) {
            U4 r = uniforms(key, t, KIND_TRI_Z, (uint64_t)i, (uint64_t)it, 0);
            spre[i] = Pre{r.r[0], r.r[1], bm_normal(r.r[0], r.r[1])};
        }
    };
    if (ortho) {
        // sample_beta_ortho (BridgeRegression.cpp:362-403): coordinate Gibbs on beta itself,
        // m_j = (c_j - sum_{k != j} G_jk beta_k) / G_jj, one pass (its burn defaults to 0).
        // Gf is the full symmetric Gram, row j contiguous.
        precompute(0);
        __syncthreads();
        double gn[kTriE];
#pragma unroll
        for (int e = 0; e < kTriE; ++e) gn[e] = tid + e * kTriNT < p ? Gf[tid + e * kTriNT] : 0.0;
        for (int j = 0; j < p; ++j) {
            double g[kTriE];
#pragma unroll
            for (int e = 0; e < kTriE; ++e) g[e] = gn[e];
            if (j + 1 < p) {
#pragma unroll
                for (int e = 0; e < kTriE; ++e) {
                    const int k = tid + e * kTriNT;
                    gn[e] = k < p ? Gf[(size_t)(j + 1) * p + k] : 0.0;
                }
            }
            double part = 0.0;
#pragma unroll
            for (int e = 0; e < kTriE; ++e) {
                const int k = tid + e * kTriNT;
                if (k < p && k != j) part += g[e] * sb[k];
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
            if (lane == 0) shmax[j & 1][wv] = part;
            __syncthreads();
            double xb = 0.0;
#pragma unroll
            for (int w = 0; w < kTriNT / 64; ++w) xb += shmax[j & 1][w];
            if (tid == (j % kTriNT)) {  // the owner draws and keeps beta_j
                const double gjj = sdv[j];
                const double m = (sav[j] - xb) / gjj;
                const double v = sig2 / gjj;
                const double bnd = sbnd[j];
                sb[j] = tnorm(-1.0 * bnd, bnd, m, sqrt(v), key, t, (uint64_t)j, 0, spre[j], err);
            }
        }
        __syncthreads();
    } else {
        // the conditional mean a_i / d_i^2 and sd sigma / d_i of every coordinate, off the
        // serial chain (same expressions, so the same bits); sd < 0 flags d_i <= 1e-16
        for (int i = tid; i < p; i += kTriNT) {
            const double di = sdv[i];
            const bool ok = di > 1e-16;
            sav[i] = ok ? sav[i] / (di * di) : 0.0;
            sdv[i] = ok ? sig / di : -1.0;
        }
        __syncthreads();
    }
    for (int it = 0; it <= (ortho ? -1 : betaburn); ++it) {
        precompute(it);
        // z = tV beta (:246)
        for (int i = tid; i < p; i += kTriNT) {
            double s = 0.0;
            for (int j = 0; j < p; ++j) s += tVc[i + (size_t)j * p] * sb[j];
            sz[i] = s;
        }
        __syncthreads();
#pragma unroll
        for (int e = 0; e < kTriE; ++e) {
            const int j = tid + e * kTriNT;
            double s = 0.0;
            if (j < p)
                for (int k = 0; k < p; ++k) s += tVr[(size_t)k * p + j] * sz[k];
            bcur[e] = s;
        }
        double vn[kTriE];
#pragma unroll
        for (int e = 0; e < kTriE; ++e) {
            const int j = tid + e * kTriNT;
            vn[e] = j < p ? tVr[j] : 0.0;
        }
        for (int i = 0; i < p; ++i) {  // :250-283
            double v[kTriE];
#pragma unroll
            for (int e = 0; e < kTriE; ++e) v[e] = vn[e];
            if (i + 1 < p) {
#pragma unroll
                for (int e = 0; e < kTriE; ++e) {
                    const int j = tid + e * kTriNT;
                    vn[e] = j < p ? tVr[(size_t)(i + 1) * p + j] : 0.0;
                }
            }
            const double zi = sz[i];
            double lmax = -1.0 * 1.7976931348623157e308, rmin = 1.7976931348623157e308;
#pragma unroll
            for (int e = 0; e < kTriE; ++e) {
                const int j = tid + e * kTriNT;
                if (j < p) {
                    const double vji = v[e];
                    const double rji = bcur[e] - vji * zi;
                    const double dif = bj[e] - rji, sum = bj[e] + rji;
                    const double left = (vji > 0 ? -sum : -dif) / fabs(vji);
                    const double right = (vji > 0 ? dif : sum) / fabs(vji);
                    lmax = lmax > left ? lmax : left;
                    rmin = rmin < right ? rmin : right;
                }
            }
            lmax = rows_max(row16_max(lmax));
            rmin = rows_min(row16_min(rmin));
            if (lane == 0) {  // one partial per wave
                shmax[i & 1][wv] = lmax;
                shmin[i & 1][wv] = rmin;
            }
            // LDS-only barrier: __syncthreads() would also drain the row prefetch (vmcnt(0))
            // LDS writes visible, then the barrier, in ONE asm statement with a memory
            // clobber so no LDS access can be scheduled across the pair
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            double L = shmax[i & 1][0], R = shmin[i & 1][0];
#pragma unroll
            for (int w = 1; w < kTriNT / 64; ++w) {
                L = L > shmax[i & 1][w] ? L : shmax[i & 1][w];
                R = R < shmin[i & 1][w] ? R : shmin[i & 1][w];
            }
            const double sdi = sdv[i];
            double zn;
            if (sdi > 0.0) {
                zn = tnorm(L, R, sav[i], sdi, key, t, (uint64_t)i, (uint64_t)it, spre[i], err);
            } else {
                zn = L + (R - L) * spre[i].r0;
            }
            const double dz = zn - zi;
            if (tid == 0) sz[i] = zn;  // read again only after the loop's closing barrier
#pragma unroll
            for (int e = 0; e < kTriE; ++e) bcur[e] += v[e] * dz;
        }
        __syncthreads();
        // beta = tV' z (:285)
#pragma unroll
        for (int e = 0; e < kTriE; ++e) {
            const int j = tid + e * kTriNT;
            if (j < p) {
                double s = 0.0;
                for (int k = 0; k < p; ++k) s += tVr[(size_t)k * p + j] * sz[k];
                sb[j] = s;
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int e = 0; e < kTriE; ++e) {
        const int j = tid + e * kTriNT;
        if (j < p) {
            beta[j] = sb[j];
            if (tr_beta) tr_beta[j] = sb[j];
        }
    }
}

// ---------------------------------------------------------------------------
// Whole sweeps for small p (the reference's published designs, p = 10, 13): the general
// path's four launches per sweep (S_alpha / X beta partials, tau and sig2, k_tri_update,
// X beta) cost more than the arithmetic.  k_tri_chain keeps the chain in LDS and runs
// `count` sweeps per launch: all 512 threads for S_alpha / rss, two lanes for tau and sig2,
// then wave 0 alone (lane j = coefficient j) for omega, u and the coordinate passes, whose
// bound reductions are DPP + readlane inside the wave (no barrier per coordinate) and whose
// truncated-normal draws test kTcK attempts at once (tnorm_par).  While wave 0 runs the
// serial part, waves 1..7 draw every counter-only variate of the NEXT sweep into the other
// half of a double buffer: the tau / sig2 gamma variates, the omega / u uniforms and
// attempts 0..kTcK-1 of each coordinate's first-pass truncated normal.  The arithmetic is
// k_tri_update's, expression for expression.
// ---------------------------------------------------------------------------
constexpr int kTcNT = 512;
constexpr int kTcK = 16;                // parallel truncated-normal attempts
constexpr size_t kTcXLds = 96 * 1024;  // X staged in LDS up to this size
constexpr int kTcP = kTriChainMaxP;

__device__ __forceinline__ double wave_sum64(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

struct TcVariates {  // counter-only variates of one sweep
    double gt, gs;                 // Ga(tau shape, 1), Ga(sig2 shape, 1)
    double om[kTcP][3], uu[kTcP];  // omega: r0 and the Ga(1, 1) / Ga(2, 1) variates; u
    double r[kTcP][kTcK][2];       // attempt k of coordinate i (pass 0): r0, r1
    double x[kTcP][kTcK];          //   and its Box-Muller normal
};

// Item e of sweep tt's variates (e < 2 + p (1 + kTcK)).
__device__ __forceinline__ void tc_variate(TcVariates &v, int e, int p, double tau_shape,
                                           double sig2_shape, const Hyper &hy, Key key,
                                           uint64_t tt, uint32_t *err) {
    if (e == 0) {
        if (!hy.know_tau) v.gt = gamma1(tau_shape, key, tt, KIND_TAU, err);
    } else if (e == 1) {
        if (!hy.know_sig2) v.gs = gamma1(sig2_shape, key, tt, KIND_SIG2, err);
    } else if (e < 2 + p) {
        const int j = e - 2;
        const U4 r = uniforms(key, tt, KIND_TRI_OMEGA, (uint64_t)j, 0, 0);
        v.om[j][0] = r.r[0];
        v.om[j][1] = -log(r.r[1]);                // Ga(1, 1)
        v.om[j][2] = -log(r.r[1]) - log(r.r[2]);  // Ga(2, 1)
        v.uu[j] = uniforms(key, tt, KIND_TRI_U, (uint64_t)j, 0, 0).r[0];
    } else {
        const int q = e - 2 - p, i = q / kTcK, k = q % kTcK;
        const U4 r = uniforms(key, tt, KIND_TRI_Z, (uint64_t)i, 0, (uint64_t)k);
        v.r[i][k][0] = r.r[0];
        v.r[i][k][1] = r.r[1];
        v.x[i][k] = bm_normal(r.r[0], r.r[1]);
    }
}

__global__ __launch_bounds__(kTcNT) void k_tri_chain(
    const double *__restrict__ X, int ldx, int n, int p, const double *__restrict__ y,
    const double *__restrict__ tVc, const double *__restrict__ tVr,
    const double *__restrict__ av, const double *__restrict__ dv, const double *__restrict__ Gf,
    const double *__restrict__ cv, int ortho, int x_lds, double *beta,
    double *u, double *omega, double *shape, DevScalars *sc, Hyper hy, int betaburn, Key key,
    uint64_t t0, int count, int first_slot, int slot_step, int cap, double *tr_beta,
    double *tr_u, double *tr_omega, double *tr_shape, double *tr_sig2, double *tr_tau,
    double *tr_alpha, uint32_t *err) {
    extern __shared__ double sX[];
    __shared__ double sTc[kTcP * kTcP], sTr[kTcP * kTcP];
    __shared__ double sb[kTcP];
    __shared__ TcVariates vb[2];
    __shared__ double red[2][kTcNT / 64];
    __shared__ double s_tau, s_sig2;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    // orthogonal design: sTc holds the full symmetric Gram X'X (row j contiguous) instead
    for (int e = tid; e < p * p; e += kTcNT) {
        sTc[e] = ortho ? Gf[e] : tVc[e];
        if (!ortho) sTr[e] = tVr[e];
    }
    if (x_lds)
        for (int e = tid; e < n * p; e += kTcNT) sX[e] = X[(size_t)(e % n) + (size_t)(e / n) * ldx];
    const double *Xs = x_lds ? sX : X;
    const int lds_x = x_lds ? n : ldx;
    const bool act = wid == 0 && lane < p;  // wave 0, lane j = coefficient / coordinate j
    double uj = 0.0, om = 0.0, sh = 0.0, aj_c = 0.0, dj_c = 0.0;
    if (tid < p) {
        sb[tid] = beta[tid];
        uj = u[tid];
        aj_c = ortho ? cv[tid] : av[tid];          // ortho: c_j = (X'y)_j
        dj_c = ortho ? Gf[(size_t)tid * p + tid] : dv[tid];  //        G_jj
    }
    if (tid == 0) {
        s_tau = sc->tau;
        s_sig2 = sc->sig2;
    }
    const double alpha = sc->alpha;
    const double tau_shape = hy.nu_shape + ((double)p) / alpha;
    const double sig2_shape = hy.sig2_shape + 0.5 * (double)n;
    const int nvar = 2 + p * (1 + kTcK);
    for (int e = tid; e < nvar; e += kTcNT)  // sweep 0's variates
        tc_variate(vb[0], e, p, tau_shape, sig2_shape, hy, key, t0, err);
    __syncthreads();
    for (int k = 0; k < count; ++k) {
        TcVariates &v = vb[k & 1];
        const uint64_t t = t0 + (uint64_t)k;
        const int slot = first_slot < 0 ? -1 : (first_slot + k * slot_step) % cap;
        // ---- S_alpha = sum |beta_j|^alpha and rss = |y - X beta|^2 ----
        double sa = 0.0, rs = 0.0;
        if (tid < p) sa = exp(alpha * log(fabs(sb[tid])));
        for (int i = tid; i < n; i += kTcNT) {
            double xb = 0.0;
            for (int j = 0; j < p; ++j) xb += Xs[(size_t)i + (size_t)j * lds_x] * sb[j];
            const double r = y[i] - xb;
            rs += r * r;
        }
        sa = wave_sum64(sa);
        rs = wave_sum64(rs);
        if (lane == 0) {
            red[0][wid] = sa;
            red[1][wid] = rs;
        }
        __syncthreads();
        // tau | beta (wave 0) and sig2 | beta (wave 1), as k_scalars
        if (tid == 0 || tid == 64) {
            double S = red[tid == 0 ? 0 : 1][0];
#pragma unroll
            for (int w = 1; w < kTcNT / 64; ++w) S += red[tid == 0 ? 0 : 1][w];
            if (tid == 0) {
                if (!hy.know_tau) s_tau = exp(-1.0 * log(v.gt / (hy.nu_rate + S)) / alpha);
                if (slot >= 0) {
                    tr_tau[slot] = s_tau;
                    tr_alpha[slot] = alpha;
                }
            } else {
                if (!hy.know_sig2) s_sig2 = (hy.sig2_scale + 0.5 * S) / v.gs;
                if (slot >= 0) tr_sig2[slot] = s_sig2;
            }
        }
        __syncthreads();
        if (wid > 0) {
            // the next sweep's variates, off wave 0's serial chain
            if (k + 1 < count)
                for (int e = tid - 64; e < nvar; e += kTcNT - 64)
                    tc_variate(vb[(k + 1) & 1], e, p, tau_shape, sig2_shape, hy, key, t + 1, err);
        } else {
            const double tau = s_tau, sig2 = s_sig2, sig = sqrt(sig2);
            double bj = 0.0;
            if (act) {
                // sample_omega, sample_u, the bound of sample_beta (BridgeRegression.cpp:97-146,
                // :410-412)
                const double betaj = sb[lane];
                const double aj = exp(alpha * log(fabs(betaj) / ((1.0 - uj) * tau)));
                const double prob = alpha / (1.0 + alpha * aj);
                double w;
                if (v.om[lane][0] > prob) {
                    sh = 1.0;
                    w = v.om[lane][1];
                } else {
                    sh = 2.0;
                    w = v.om[lane][2];
                }
                om = w + aj;
                const double right = 1.0 - fabs(betaj) / tau * exp(-1.0 * log(om) / alpha);
                uj = right * v.uu[lane];
                bj = (1.0 - uj) * exp(log(om) / alpha) * tau;
                if (slot >= 0) {
                    tr_omega[(size_t)slot * p + lane] = om;
                    tr_shape[(size_t)slot * p + lane] = sh;
                    tr_u[(size_t)slot * p + lane] = uj;
                }
            }
            if (ortho) {
                // sample_beta_ortho (BridgeRegression.cpp:362-403), one coordinate pass as
                // k_tri_update's: m_j = (c_j - sum_{k != j} G_jk beta_k) / G_jj, sd
                // sqrt(sig2 / G_jj), truncated to |beta_j| <= b_j; attempts 0..kTcK-1 of
                // every coordinate precomputed by waves 1..7 during the previous sweep
                double bl = act ? sb[lane] : 0.0;
                for (int j = 0; j < p; ++j) {
                    const double prod = (act && lane != j) ? sTc[j * p + lane] * bl : 0.0;
                    const double xb = wave_sum64(prod);  // xor butterfly: the same bits in
                                                          // every lane
                    const double gjj = readlane_d(dj_c, j), bnd = readlane_d(bj, j);
                    const double m = (readlane_d(aj_c, j) - xb) / gjj;
                    const double sd = sqrt(sig2 / gjj);
                    const int ka = lane < kTcK ? lane : 0;
                    const double zn = tnorm_par<kTcK>(-1.0 * bnd, bnd, m, sd, v.r[j][ka][0],
                                                      v.r[j][ka][1], v.x[j][ka], key, t,
                                                      (uint64_t)j, 0, err);
                    if (lane == j) bl = zn;
                }
                if (act) {
                    sb[lane] = bl;
                    if (slot >= 0) tr_beta[(size_t)slot * p + lane] = bl;
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            } else {
            // conditional mean a_i / d_i^2 and sd sigma / d_i of coordinate i (lane i)
            const bool ok = dj_c > 1e-16;
            const double ci = ok ? aj_c / (dj_c * dj_c) : 0.0;
            const double si = ok ? sig / dj_c : -1.0;
            double zr = 0.0;
            for (int it = 0; it <= betaburn; ++it) {
                Pre pr{0.0, 0.0, 0.0};  // attempt 0 of coordinate `lane` (passes >= 1)
                if (it > 0 && act) {
                    const U4 q = uniforms(key, t, KIND_TRI_Z, (uint64_t)lane, (uint64_t)it, 0);
                    pr = Pre{q.r[0], q.r[1], bm_normal(q.r[0], q.r[1])};
                }
                // z = tV beta (:246), then beta_cur = tV' z, in k_tri_update's order
                zr = 0.0;
                if (act)
                    for (int j = 0; j < p; ++j) zr += sTc[lane + j * p] * sb[j];
                double bc = 0.0;
                for (int kk = 0; kk < p; ++kk) {
                    const double zk = readlane_d(zr, kk);
                    if (act) bc += sTr[kk * p + lane] * zk;
                }
                for (int i = 0; i < p; ++i) {  // :250-283
                    const double vi = act ? sTr[i * p + lane] : 0.0;
                    const double zi = readlane_d(zr, i);
                    double lmax = -1.0 * 1.7976931348623157e308, rmin = 1.7976931348623157e308;
                    if (act) {
                        const double rji = bc - vi * zi;
                        const double dif = bj - rji, sum = bj + rji;
                        const double left = (vi > 0 ? -sum : -dif) / fabs(vi);
                        const double right = (vi > 0 ? dif : sum) / fabs(vi);
                        lmax = lmax > left ? lmax : left;
                        rmin = rmin < right ? rmin : right;
                    }
                    const double L = rows_max(row16_max(lmax));
                    const double R = rows_min(row16_min(rmin));
                    const double sdi = readlane_d(si, i);
                    double zn;
                    if (it == 0) {
                        const int ka = lane < kTcK ? lane : 0;
                        if (sdi > 0.0)
                            zn = tnorm_par<kTcK>(L, R, readlane_d(ci, i), sdi, v.r[i][ka][0],
                                                 v.r[i][ka][1], v.x[i][ka], key, t, (uint64_t)i,
                                                 0, err);
                        else
                            zn = L + (R - L) * v.r[i][0][0];
                    } else {
                        const Pre pi{readlane_d(pr.r0, i), readlane_d(pr.r1, i),
                                     readlane_d(pr.x0, i)};
                        if (sdi > 0.0)
                            zn = tnorm(L, R, readlane_d(ci, i), sdi, key, t, (uint64_t)i,
                                       (uint64_t)it, pi, err);
                        else
                            zn = L + (R - L) * pi.r0;
                    }
                    bc += vi * (zn - zi);
                    if (lane == i) zr = zn;
                }
                // beta = tV' z (:285)
                double bn = 0.0;
                for (int kk = 0; kk < p; ++kk) {
                    const double zk = readlane_d(zr, kk);
                    if (act) bn += sTr[kk * p + lane] * zk;
                }
                if (act) sb[lane] = bn;
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // sb read by other lanes next
            }
            if (act && slot >= 0) tr_beta[(size_t)slot * p + lane] = sb[lane];
            }
        }
        __syncthreads();
    }
    if (act) {
        beta[lane] = sb[lane];
        u[lane] = uj;
        omega[lane] = om;
        shape[lane] = sh;
    }
    if (tid == 0) {
        sc->tau = s_tau;
        sc->sig2 = s_sig2;
    }
}

// Truncated normal / exponential batches behind the .C utilities rtnorm_left, rtnorm_both,
// rtnorm, rtexpon_rate_left, rtexpon_rate_both, rtexpon_rate (BridgeWrapper.cpp:762-935):
// one lane per draw; draw i uses counters (0, 10 << 56 | i, 0, k) for truncated-normal
// attempts and (0, 12 << 56 | i, 0, 0) for the exponential / untruncated normal.
constexpr unsigned KIND_TRUNC = 12;

__device__ double texpon(double left, double right, double rate, double u) {
    if (isinf(right)) return left - log(u) / rate;  // memoryless left truncation
    return left - log1p(u * expm1(-rate * (right - left))) / rate;  // inversion on [l, r]
}

__global__ __launch_bounds__(256) void k_trunc_batch(int mode, int num, double *x,
                                                     const double *p0, const double *p1,
                                                     const double *p2, const double *p3, Key key,
                                                     uint32_t *err) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= num) return;
    const double inf = __builtin_inf();
    U4 r = uniforms(key, 0, KIND_TRI_Z, (uint64_t)i, 0, 0);
    const Pre pre{r.r[0], r.r[1], bm_normal(r.r[0], r.r[1])};
    const U4 e = uniforms(key, 0, KIND_TRUNC, (uint64_t)i, 0, 0);
    double out;
    switch (mode) {
        case 0:  // rtnorm_left(left, mu, sig)
            out = tnorm(p0[i], inf, p1[i], p2[i], key, 0, i, 0, pre, err);
            break;
        case 1:  // rtnorm_both(left, right, mu, sig)
            out = tnorm(p0[i], p1[i], p2[i], p3[i], key, 0, i, 0, pre, err);
            break;
        case 2: {  // rtnorm(left, right, mu, sig), USE_R branch (:904-919)
            const double l = p0[i], rt = p1[i], mu = p2[i], sg = p3[i];
            if (isnan(l) || isnan(rt) || isnan(mu) || isnan(sg)) {
                out = __builtin_nan("");
            } else if (!isinf(l) && !isinf(rt)) {
                out = tnorm(l, rt, mu, sg, key, 0, i, 0, pre, err);
            } else if (!isinf(l) && rt == inf) {
                out = tnorm(l, inf, mu, sg, key, 0, i, 0, pre, err);
            } else if (l == -inf && !isinf(rt)) {
                out = -1.0 * tnorm(-1.0 * rt, inf, -1.0 * mu, sg, key, 0, i, 0, pre, err);
            } else if (l == -inf && rt == inf) {
                out = mu + sg * bm_normal(e.r[0], e.r[1]);
            } else {
                out = __builtin_nan("");
            }
            break;
        }
        case 3:  // rtexpon_rate_left(left, rate)
            out = texpon(p0[i], inf, p1[i], e.r[0]);
            break;
        case 4:  // rtexpon_rate_both(left, right, rate)
            out = texpon(p0[i], p1[i], p2[i], e.r[0]);
            break;
        default: {  // rtexpon_rate(left, right, rate) (:805-830)
            // the reference sets x = NaN and prints for a non-finite input, then the draw
            // below overwrites it (no else): a non-finite right means left truncation only
            const double l = p0[i], rt = p1[i], rate = p2[i];
            if (isnan(l) || isnan(rt) || isnan(rate) || isinf(l))
                atomicOr(err, 256u);  // the host prints the reference's stderr line
            out = texpon(l, isfinite(rt) ? rt : inf, rate, e.r[0]);
            break;
        }
    }
    x[i] = out;
}

// Right-truncated gamma (rrtgamma_rate, BridgeWrapper.cpp:944-962): Y = rate x ~ Ga(a, 1)
// restricted to (0, T], T = rate right_t; the four exact rejection regimes of
// oracle/bb_oracle.c bbo_rtgamma_std, attempt k on counters (0, 13 << 56 | i, k, 0).
constexpr unsigned KIND_RTGAMMA = 13;

__device__ double rtgamma_std(double a, double T, Key key, uint64_t i, uint32_t *err) {
    for (long k = 0; k < kTnMaxAttempts; ++k) {
        const U4 r = uniforms(key, 0, KIND_RTGAMMA, i, (uint64_t)k, 0);
        if (T >= a) {  // Marsaglia-Tsang draw, accept if it lands below T
            const double ap = a < 1.0 ? a + 1.0 : a;
            const double d = ap - 1.0 / 3.0, cc = 1.0 / sqrt(9.0 * d);
            const double x = bm_normal(r.r[0], r.r[1]);
            double v = 1.0 + cc * x;
            if (v <= 0.0) continue;
            v = v * v * v;
            const double x2 = x * x;
            if (!(r.r[2] < 1.0 - 0.0331 * x2 * x2) &&
                !(log(r.r[2]) < 0.5 * x2 + d * (1.0 - v + log(v))))
                continue;
            double y = d * v;
            if (a < 1.0) y *= pow(r.r[3], 1.0 / a);
            if (y <= T) return y;
        } else if (a <= 1.0) {  // power proposal, accept w.p. e^-y
            const double y = T * pow(r.r[0], 1.0 / a);
            if (r.r[1] <= exp(-y)) return y;
        } else if (T <= a - 1.0) {  // increasing log-concave: tangent envelope at T
            const double c = (a - 1.0) / T - 1.0;
            const double z = c > 0.0 ? -log1p(r.r[0] * expm1(-c * T)) / c : T * r.r[0];
            const double y = T - z;
            if (y > 0.0 && log(r.r[1]) <= (a - 1.0) * log(y / T) + z + c * z) return y;
        } else {  // mode inside (0, T): uniform proposal bounded at the mode
            const double m = a - 1.0;
            const double y = T * r.r[0];
            if (log(r.r[1]) <= (a - 1.0) * log(y / m) - (y - m)) return y;
        }
    }
    atomicOr(err, 64u);
    return T;
}

__global__ __launch_bounds__(256) void k_rrtgamma_batch(int num, double *x, const double *shape,
                                                        const double *rate,
                                                        const double *right_t, Key key,
                                                        uint32_t *err) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= num) return;
    x[i] = rtgamma_std(shape[i], rate[i] * right_t[i], key, (uint64_t)i, err) / rate[i];
}

}  // namespace

void launch_rrtgamma_batch(hipStream_t s, int num, double *x, const double *shape,
                           const double *rate, const double *right_t, uint64_t k0, uint64_t k1,
                           uint32_t *err) {
    if (num <= 0) return;
    hipLaunchKernelGGL(k_rrtgamma_batch, dim3((num + 255) / 256), dim3(256), 0, s, num, x, shape,
                       rate, right_t, Key{k0, k1}, err);
}

void launch_trunc_batch(hipStream_t s, int mode, int num, double *x, const double *p0,
                        const double *p1, const double *p2, const double *p3, uint64_t k0,
                        uint64_t k1, uint32_t *err) {
    if (num <= 0) return;
    hipLaunchKernelGGL(k_trunc_batch, dim3((num + 255) / 256), dim3(256), 0, s, mode, num, x, p0,
                       p1, p2, p3, Key{k0, k1}, err);
}

void launch_tri_update(hipStream_t s, double *beta, double *u, double *omega, double *shape,
                       int p, const double *tVc, const double *tVr, const double *a,
                       const double *d, const double *Gf, const double *c, int ortho,
                       const DevScalars *sc, int betaburn, uint64_t k0, uint64_t k1, uint64_t t,
                       double *tr_beta, double *tr_u, double *tr_omega, double *tr_shape,
                       uint32_t *err) {
    if (p < 1 || p > kTriMaxP) return;  // the engine checks p at setup
    hipLaunchKernelGGL(k_tri_update, dim3(1), dim3(kTriNT), 0, s, beta, u, omega, shape, p, tVc,
                       tVr, a, d, Gf, c, ortho, sc, betaburn, Key{k0, k1}, t, tr_beta, tr_u,
                       tr_omega, tr_shape, err);
}

void launch_tri_chain(hipStream_t s, const double *X, int ldx, int n, int p, const double *y,
                      const double *tVc, const double *tVr, const double *a, const double *d,
                      const double *Gf, const double *c, int ortho, double *beta, double *u, double *omega, double *shape, DevScalars *sc,
                      Hyper hy, int betaburn, uint64_t k0, uint64_t k1, uint64_t t0, int count,
                      int first_slot, int slot_step, int cap, double *tr_beta, double *tr_u,
                      double *tr_omega, double *tr_shape, double *tr_sig2, double *tr_tau,
                      double *tr_alpha, uint32_t *err) {
    if (count <= 0 || p < 1 || p > kTriChainMaxP) return;  // the engine checks p at setup
    const size_t xbytes = (size_t)n * p * sizeof(double);
    const int x_lds = xbytes <= kTcXLds;
    static const hipError_t attr = hipFuncSetAttribute(  // one-time opt-in above 64 KB
        (const void *)k_tri_chain, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kTcXLds);
    (void)attr;
    k_tri_chain<<<1, kTcNT, x_lds ? xbytes : 0, s>>>(
        X, ldx, n, p, y, tVc, tVr, a, d, Gf, c, ortho, x_lds, beta, u, omega, shape, sc, hy, betaburn,
        Key{k0, k1}, t0, count, first_slot, slot_step, cap, tr_beta, tr_u, tr_omega, tr_shape,
        tr_sig2, tr_tau, tr_alpha, err);
}

}  // namespace bb
