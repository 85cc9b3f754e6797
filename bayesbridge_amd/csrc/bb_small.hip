// bb_small.hip -- the whole stable Gibbs sweep for small p in ONE workgroup (gfx950).
//
// For the reference's published designs (diabetes 442 x 10, Boston 506 x 13: SURVEY.md s6)
// a sweep is a few microseconds of arithmetic, and a launch per step (~12 per sweep on the
// general path, with the p x p system padded to a 256 x 256 Cholesky) costs far more than
// the work.  k_small_chain runs `count` consecutive sweeps in one launch with the chain
// state in LDS, in the reference's order (Code/C/BridgeWrapper.cpp:266-298):
//   tau | beta and sig2 | beta       BridgeRegression.cpp:453-465, :436-450 (thread 0)
//   lambda | beta, tau               :506-510 (16-lane groups, retstable.cpp:94-271)
//   beta | rest                      :552-575 (A = G + diag(lambda sig2 / tau^2), A = U'U,
//                                    m = U^-1 U'^-1 c, beta = m + sig U^-1 z; one wave)
//                                    or the orthogonal design's :514-521
// with the same counters as the general path (t = t0 + k per sweep), so both draw the same
// chain up to summation order.  alpha known (the MH step runs on the general path).
#include <hip/hip_runtime.h>

#include "bb_kernels.h"
#include "bb_sampler.h"

namespace bb {

namespace {

constexpr int kSmallMaxP = kSmallChainMaxP;
constexpr size_t kSmallXLds = 112 * 1024;
constexpr int kSmallPre = 32;  // sweeps of counter-only variates drawn ahead  // X staged in LDS up to this size

__device__ __forceinline__ double wave_sum_all(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ double readlane_f64(double v, int lane) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, lane);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

}  // namespace

// tools/small_phase_bench.cpp builds this file with BB_SMALL_PHASES: thread 0 accumulates
// the realtime-clock ticks of each phase of the sweep into g_small_phase_ticks.
#ifdef BB_SMALL_PHASES
__device__ unsigned long long g_small_phase_ticks[4];
#define SMALL_PHASE(i)                                                  \
    do {                                                                \
        if (tid == 0) {                                                 \
            const unsigned long long now = wall_clock64();              \
            if ((i) > 0) g_small_phase_ticks[(i) - 1] += now - ph_t;    \
            ph_t = now;                                                 \
        }                                                               \
    } while (0)
// read (and zero) the accumulated ticks from the host
void small_phase_ticks(unsigned long long out[4]) {
    (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_small_phase_ticks), 4 * sizeof(*out));
    const unsigned long long zero[4] = {0, 0, 0, 0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_small_phase_ticks), zero, sizeof(zero));
}
#else
#define SMALL_PHASE(i) \
    do {               \
    } while (0)
#endif

// L lanes per coefficient in the lambda draw (stable_spec_draw<L, I>), the p x p system
// dynamic LDS holds
// X (n x p, column-major) when it fits, else X is read from HBM each sweep.
template <int NT, int L, int I>
__global__ __launch_bounds__(NT) void k_small_chain(
    const double *__restrict__ X, int ldx, int n, int p, const double *__restrict__ y,
    const double *__restrict__ G, int ldg, const double *__restrict__ cvec,
    const double *__restrict__ gdiag, int ortho, int x_lds, double *beta, double *lam,
    DevScalars *sc, Hyper hy, Key key, uint64_t t0, int count, int first_slot, int slot_step,
    int cap, double *tr_beta, double *tr_lam, double *tr_sig2, double *tr_tau, double *tr_alpha,
    uint32_t *err) {
    extern __shared__ double sX[];
    __shared__ double sU[kSmallMaxP][kSmallMaxP + 1];  // U, row-major (U[k][j])
    __shared__ double sG[kSmallMaxP][kSmallMaxP + 1];
    __shared__ double sb[kSmallMaxP], sl[kSmallMaxP], sc_[kSmallMaxP], sgd[kSmallMaxP];
    // Ga(shape, 1) variates of tau and sig2 and the beta normals of the next kSmallPre
    // sweeps: their shapes are constant along the chain (alpha known), so they depend on
    // their counters alone and come off the serial chain
    __shared__ double s_gt[kSmallPre], s_gs[kSmallPre], s_z[kSmallPre][kSmallMaxP];
    __shared__ double red[2][NT / 64];
    __shared__ double s_tau, s_sig2;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (int e = tid; e < p * p; e += NT) {
        const int r = e % p, c = e / p;
        const int lo = r < c ? r : c, hi = r < c ? c : r;  // G holds its upper triangle
        sG[r][c] = ortho ? 0.0 : G[(size_t)lo + (size_t)hi * ldg];
    }
    if (x_lds)
        for (int e = tid; e < n * p; e += NT) sX[e] = X[(size_t)(e % n) + (size_t)(e / n) * ldx];
    const double *Xs = x_lds ? sX : X;
    const int lds_x = x_lds ? n : ldx;
    if (tid < p) {
        sb[tid] = beta[tid];
        sc_[tid] = cvec[tid];
        sgd[tid] = ortho ? gdiag[tid] : 0.0;
    }
    if (tid == 0) {
        s_tau = sc->tau;
        s_sig2 = sc->sig2;
    }
    const double alpha = sc->alpha;
#ifdef BB_SMALL_PHASES
    unsigned long long ph_t = 0;
#endif
    __syncthreads();
    const double tau_shape = hy.nu_shape + ((double)p) / alpha;
    const double sig2_shape = hy.sig2_shape + 0.5 * (double)n;
    // upper-triangle entries owned by this thread: e = tid and tid + NT, e = j (j + 1) / 2 + i
    bool own[2];
    int oi[2], oj[2];
    double av[2] = {0.0, 0.0};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int e = tid + h * NT;
        own[h] = !ortho && e < p * (p + 1) / 2;
        int j = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
        while ((j + 1) * (j + 2) / 2 <= e) ++j;
        while (j * (j + 1) / 2 > e) --j;
        oj[h] = j;
        oi[h] = e - j * (j + 1) / 2;
    }
    for (int k = 0; k < count; ++k) {
        if (k % kSmallPre == 0) {
            // wave 0: tau's gamma variates, wave 1: sig2's, waves 2..: the normals
            const int nb = count - k < kSmallPre ? count - k : kSmallPre;
            if (wid == 0 && lane < nb && !hy.know_tau)
                s_gt[lane] = gamma1(tau_shape, key, t0 + (uint64_t)(k + lane), KIND_TAU, err);
            else if (wid == 1 && lane < nb && !hy.know_sig2)
                s_gs[lane] = gamma1(sig2_shape, key, t0 + (uint64_t)(k + lane), KIND_SIG2, err);
            for (int e = tid - 128; e >= 0 && e < nb * p; e += NT - 128) {
                const int kk = e / p, j = e % p;
                s_z[kk][j] = normal_at(key, t0 + (uint64_t)(k + kk), KIND_BETA_Z, (uint64_t)j);
            }
            __syncthreads();
        }
        const int kp = k % kSmallPre;
        SMALL_PHASE(0);
        const uint64_t t = t0 + (uint64_t)k;
        const int slot = first_slot < 0 ? -1 : (first_slot + k * slot_step) % cap;
        // ---- S_alpha = sum |beta_j|^alpha and rss = |y - X beta|^2 ----
        double sa = 0.0, rs = 0.0;
        if (tid < p) sa = exp(alpha * log(fabs(sb[tid])));
        for (int i = tid; i < n; i += NT) {
            double xb = 0.0;
            for (int j = 0; j < p; ++j) xb += Xs[(size_t)i + (size_t)j * lds_x] * sb[j];
            const double r = y[i] - xb;
            rs += r * r;
        }
        sa = wave_sum_all(sa);
        rs = wave_sum_all(rs);
        if (lane == 0) {
            red[0][wid] = sa;
            red[1][wid] = rs;
        }
        __syncthreads();
        SMALL_PHASE(1);
        // tau (wave 0) and sig2 (wave 1) are independent draws: BridgeRegression.cpp:453-465,
        // :436-450
        if (tid == 0 || tid == 64) {
            double S = red[tid == 0 ? 0 : 1][0];
#pragma unroll
            for (int w = 1; w < NT / 64; ++w) S += red[tid == 0 ? 0 : 1][w];
            if (tid == 0) {
                if (!hy.know_tau) {
                    const double nu = s_gt[kp] / (hy.nu_rate + S);
                    s_tau = exp(-1.0 * log(nu) / alpha);
                }
                if (slot >= 0) {
                    tr_tau[slot] = s_tau;
                    tr_alpha[slot] = alpha;
                }
            } else {
                if (!hy.know_sig2) s_sig2 = (hy.sig2_scale + 0.5 * S) / s_gs[kp];
                if (slot >= 0) tr_sig2[slot] = s_sig2;
            }
        }
        __syncthreads();
        SMALL_PHASE(2);
        const double tau = s_tau, sig2 = s_sig2;
        // ---- lambda_j = 2 retstable(beta_j^2 / tau^2, alpha / 2, 1) ----
        for (int jb = 0; jb < p; jb += NT / L) {
            const int j = jb + tid / L;
            const bool act = j < p;
            const double b = act ? sb[j] : 0.0;
            const double x = stable_spec_draw<L, I>(act, b * b / (tau * tau), 0.5 * alpha, 1.0,
                                                    key, t, (uint64_t)j, err);
            if (act && (tid % L) == 0) {
                sl[j] = 2 * x;
                if (slot >= 0) tr_lam[(size_t)slot * p + j] = 2 * x;
            }
        }
        __syncthreads();
        SMALL_PHASE(3);
        // ---- beta | rest ----
        if (ortho) {
            if (tid < p) {  // BridgeRegression.cpp:514-521
                const double uu = sgd[tid] + sl[tid] * sig2 / (tau * tau);
                const double sd = sqrt(sig2 / uu);
                const double m = sc_[tid] / uu;
                sb[tid] = m + sd * s_z[kp][tid];
            }
        } else {
            // A = G + diag(lambda sig2 / tau^2), factored right-looking as A = U'U with one
            // thread per upper-triangle entry (i, j) (two for the last 16 at p = 32): per
            // pivot k the owner of (k, k) takes the square root, the owners of row k divide
            // (row k of U goes to LDS), every trailing owner subtracts U(k, i) U(k, j) -- the
            // reference's operations entry by entry (BridgeRegression.cpp:560), two barriers
            // per pivot and no register arrays.  (One barrier per pivot -- trailing owners
            // subtracting a_ki a_kj / a_kk from a published unscaled row, one reciprocal square
            // root per pivot -- measured the same at C1 in three alternations, 27 176-27 186
            // against 27 152-27 188 sweeps/s, gpurun_out/r04q_*: the factor is not what bounds
            // the chain.)
            const double dl = tau * tau;
#pragma unroll
            for (int h = 0; h < 2; ++h)
                if (own[h]) {
                    const int i = oi[h], j = oj[h];
                    av[h] = sG[i][j] + (i == j ? sl[i] * sig2 / dl : 0.0);
                }
            for (int kk = 0; kk < p; ++kk) {
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    if (own[h] && oi[h] == kk && oj[h] == kk) {
                        if (!(av[h] > 0.0)) atomicOr(err, 8u);
                        av[h] = sqrt(av[h]);
                        sU[kk][kk] = av[h];
                    }
                __syncthreads();
                const double d = sU[kk][kk];
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    if (own[h] && oi[h] == kk && oj[h] > kk) {
                        av[h] = av[h] / d;
                        sU[kk][oj[h]] = av[h];
                    }
                __syncthreads();
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    if (own[h] && oi[h] > kk) av[h] -= sU[kk][oi[h]] * sU[kk][oj[h]];
            }
            if (wid == 0) {
                // m: U'v = c (forward), U m = v (backward); x: U x = z; lane j holds entry j
                double w = lane < p ? sc_[lane] : 0.0;
                double z = lane < p ? s_z[kp][lane] : 0.0;
                for (int kk = 0; kk < p; ++kk) {
                    const double vk = readlane_f64(w, kk) / sU[kk][kk];
                    if (lane > kk && lane < p) w -= sU[kk][lane] * vk;
                    if (lane == kk) w = vk;
                }
                for (int kk = p - 1; kk >= 0; --kk) {
                    const double ukk = sU[kk][kk];
                    const double mk = readlane_f64(w, kk) / ukk;
                    const double xk = readlane_f64(z, kk) / ukk;
                    if (lane < kk) {
                        const double ulk = sU[lane][kk];
                        w -= ulk * mk;
                        z -= ulk * xk;
                    }
                    if (lane == kk) {
                        w = mk;
                        z = xk;
                    }
                }
                if (lane < p) sb[lane] = w + sqrt(sig2) * z;
            }
        }
        __syncthreads();
        SMALL_PHASE(4);
        if (slot >= 0 && tid < p) tr_beta[(size_t)slot * p + tid] = sb[tid];
    }
    if (tid < p) {
        beta[tid] = sb[tid];
        lam[tid] = sl[tid];
    }
    if (tid == 0) {
        sc->tau = s_tau;
        sc->sig2 = s_sig2;
    }
}

// Dynamic LDS above the 64 KB default needs a per-kernel opt-in: done once for every
// instance (thread-safe static init), with the launch error checked by the caller.
template <int NT, int L, int I>
static void small_chain_lds_optin() {
    static const hipError_t rc = hipFuncSetAttribute(
        (const void *)k_small_chain<NT, L, I>, hipFuncAttributeMaxDynamicSharedMemorySize,
        kSmallXLds);
    (void)rc;
}

void launch_small_chain(hipStream_t s, const double *X, int ldx, int n, int p, const double *y,
                        const double *G, int ldg, const double *cvec, const double *gdiag,
                        int ortho, double *beta, double *lam, DevScalars *sc, Hyper hy,
                        uint64_t k0, uint64_t k1, uint64_t t0, int count, int first_slot,
                        int slot_step, int cap, double *tr_beta, double *tr_lam, double *tr_sig2,
                        double *tr_tau, double *tr_alpha, uint32_t *err) {
    if (count <= 0) return;
    const size_t xbytes = (size_t)n * p * sizeof(double);
    const int x_lds = xbytes <= kSmallXLds;
    const size_t shm = x_lds ? xbytes : 0;
    small_chain_lds_optin<512, 64, 16>();
    small_chain_lds_optin<512, 32, 8>();
    small_chain_lds_optin<512, 16, 8>();
    auto go = [&](auto kern, int nt) {
        kern<<<1, nt, shm, s>>>(X, ldx, n, p, y, G, ldg, cvec, gdiag, ortho, x_lds, beta, lam, sc,
                                hy, Key{k0, k1}, t0, count, first_slot, slot_step, cap, tr_beta,
                                tr_lam, tr_sig2, tr_tau, tr_alpha, err);
    };
    // lanes per coefficient: as many as the workgroup allows for p coefficients at once
    static_assert(kSmallMaxP == 32, "instances below cover p <= 32");
    if (p <= 8) go(k_small_chain<512, 64, 16>, 512);
    else if (p <= 16) go(k_small_chain<512, 32, 8>, 512);
    else go(k_small_chain<512, 16, 8>, 512);
}

}  // namespace bb
