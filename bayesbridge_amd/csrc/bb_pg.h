// bb_pg.h -- the Polya-Gamma PG(1, z) sampler (Devroye / Polson, Scott & Windle 2013), shared
// by k_pg (bb_logit.hip) and the lambda launch that draws omega alongside (bb_kernels.hip).
// The oracle restates the same expressions in the same order (oracle/bb_oracle.c, bbo_pg1).
#pragma once
#include <hip/hip_runtime.h>

#include "bb_sampler.h"

namespace bb {
namespace pg {

constexpr double kPgT = 0.64;  // Devroye's truncation point for J*(1, z)
constexpr unsigned kKindPg = 11, kKindPgIg = 12;
constexpr int kPgMaxAttempts = 1000, kPgMaxTerms = 1000;

__device__ __forceinline__ double pg_log_ncdf(double x) {
    return log(0.5 * erfc(-x * 0.70710678118654752440));
}

// n-th coefficient of the alternating series of the J*(1, 0) density at x
__device__ __forceinline__ double pg_a(int n, double x) {
    const double K = (n + 0.5) * kPi;
    if (x > kPgT) return K * exp(-0.5 * K * K * x);
    if (x > 0.0)
        return exp(-1.5 * (log(0.5 * kPi) + log(x)) + log(K) - 2.0 * (n + 0.5) * (n + 0.5) / x);
    return 0.0;
}

__device__ inline double pg_mass_texpon(double z) {
    const double t = kPgT;
    const double fz = 0.125 * kPi * kPi + 0.5 * z * z;
    const double b = sqrt(1.0 / t) * (t * z - 1.0);
    const double a = -sqrt(1.0 / t) * (t * z + 1.0);
    const double x0 = log(fz) + fz * t;
    const double xb = x0 - z + pg_log_ncdf(b);
    const double xa = x0 + z + pg_log_ncdf(a);
    const double qdivp = 4.0 / kPi * (exp(xb) + exp(xa));
    return 1.0 / (1.0 + qdivp);
}

// IG(1/z, 1) truncated to (0, t)
__device__ inline double pg_rtigauss(double z, Key key, uint64_t t, uint64_t i, uint64_t o, bool *fail) {
    const double tr = kPgT;
    for (uint64_t k = 0; k < (uint64_t)kPgMaxAttempts; ++k) {
        const U4 u = uniforms(key, t, kKindPgIg, i, o, k);
        if (z < 1.0 / tr) {
            const double E1 = -log(u.r[0]), E2 = -log(u.r[1]);
            if (E1 * E1 > 2.0 * E2 / tr) continue;
            const double d = 1.0 + E1 * tr;
            const double X = tr / (d * d);
            if (u.r[2] <= exp(-0.5 * z * z * X)) return X;
        } else {
            const double mu = 1.0 / z;
            double Y = bm_normal(u.r[0], u.r[1]);
            Y *= Y;
            const double half_mu = 0.5 * mu, mu_Y = mu * Y;
            double X = mu + half_mu * mu_Y - half_mu * sqrt(4.0 * mu_Y + mu_Y * mu_Y);
            if (u.r[2] > mu / (mu + X)) X = mu * mu / X;
            if (X <= tr) return X;
        }
    }
    *fail = true;
    return tr;
}

__device__ inline double pg1(double psi, Key key, uint64_t t, uint64_t i, bool *fail) {
    const double z = fabs(psi) * 0.5;
    const double fz = 0.125 * kPi * kPi + 0.5 * z * z;
    const double mass = pg_mass_texpon(z);
    for (uint64_t o = 0; o < (uint64_t)kPgMaxAttempts; ++o) {
        const U4 u = uniforms(key, t, kKindPg, i, o, 0);
        double X;
        if (u.r[0] < mass)
            X = kPgT + (-log(u.r[1])) / fz;
        else
            X = pg_rtigauss(z, key, t, i, o, fail);
        double S = pg_a(0, X);
        const double Y = u.r[2] * S;
        for (int n = 1; n < kPgMaxTerms; ++n) {
            if (n & 1) {
                S -= pg_a(n, X);
                if (Y <= S) return 0.25 * X;
            } else {
                S += pg_a(n, X);
                if (Y > S) break;
            }
        }
    }
    *fail = true;
    return 0.25;
}


}  // namespace pg

// omega_i ~ PG(1, psi_i) for i < n, 0 on the padding rows (i < n_pad)
__device__ __forceinline__ void pg_draw_at(int i, const double *__restrict__ psi, int n,
                                           int n_pad, Key key, uint64_t t,
                                           double *__restrict__ omega, uint32_t *err) {
    if (i >= n_pad) return;
    double w = 0.0;
    if (i < n) {
        bool fail = false;
        w = pg::pg1(psi[i], key, t, (uint64_t)i, &fail);
        if (fail) atomicOr(err, 32u);
    }
    omega[i] = w;
}

}  // namespace bb
