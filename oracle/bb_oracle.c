/*
 * bb_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference BayesBridge normal-mixture ("stable") Gibbs
 * sweep, used exclusively as the checker by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg.  Nothing in the product (bayesbridge_amd/,
 * BayesBridge.so) links, loads or calls this file.
 *
 * PARITY UNPINNED against the reference's own outputs: the reference ships no
 * golden vectors / fixtures for this path, R is not installed,
 * and the reference C++ cannot be built here (Code/C/retstable.h:7 includes the
 * un-vendored RNG.hpp; BridgeRegression.h:67-68 includes the un-vendored
 * Matrix.h / RNG.hpp).  This restatement is pinned instead by
 *   - Philox4x64-10 known-answer vectors (Random123 KAT) and numpy's
 *     independent Philox implementation (tests/test_oracle_cpu.py),
 *   - analytic properties of the exponentially tilted stable law
 *     (E[S] = a h^(a-1), Laplace transform exp(-((h+t)^a - h^a))),
 *   - closed-form Gaussian conditional moments of beta | rest, and
 *   - 1-D quadrature of the exact bridge posterior (known sig2, tau).
 *
 * Also restated here, same status: the triangle-mixture update (bbo_tri_update,
 * BridgeRegression.cpp:97-147, 235-286, 362-433) and the truncated-distribution .C
 * utilities (bbo_tnorm, bbo_trunc_batch, bbo_rrtgamma_batch, BridgeWrapper.cpp:762-962).
 * Their truncated normal / exponential / gamma draws come from the un-vendored RNG
 * library and are pinned distributionally (KS tests against scipy's truncnorm,
 * truncexpon and the truncated gamma CDF; exact 1-D bridge posterior for the triangle
 * chain: tests/test_triangle_cpu.py, tests/test_truncated_cpu.py).
 *
 * The reference draws its variates from R's RNG (absent).  Here every variate
 * is a pure function of a Philox counter (DESIGN.md "RNG counter layout"), the
 * same layout the HIP kernels use, so the GPU path and this oracle consume
 * identical uniforms on fixed seeds.
 *
 * Reference citations are relative to /root/reference/.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif
#define BBO_SQRT_PI 1.772453850905516027298167483341 /* retstable.cpp:14-16 */
#define BBO_SQRT2 1.41421356237309504880
#define BBO_PI_2 1.57079632679489661923

/* ----------------------------------------------------------------------- */
/* Philox4x64-10 (Salmon et al. 2011).  Independent of the product's copy. */
/* ----------------------------------------------------------------------- */
static inline void mulhilo64(uint64_t a, uint64_t b, uint64_t *hi, uint64_t *lo)
{
    __uint128_t p = (__uint128_t)a * (__uint128_t)b;
    *hi = (uint64_t)(p >> 64);
    *lo = (uint64_t)p;
}

void bbo_philox4x64(const uint64_t ctr_in[4], const uint64_t key_in[2], uint64_t out[4])
{
    uint64_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint64_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; ++r) {
        if (r > 0) {
            k0 += 0x9E3779B97F4A7C15ULL;
            k1 += 0xBB67AE8584CAA73BULL;
        }
        uint64_t hi0, lo0, hi1, lo1;
        mulhilo64(0xD2E7470EE14C6C93ULL, c0, &hi0, &lo0);
        mulhilo64(0xCA5A826395121157ULL, c2, &hi1, &lo1);
        uint64_t n0 = hi1 ^ c1 ^ k0;
        uint64_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* Counter layout: ctr = {t, (kind << 56) | j, a, b}; key = {seed, stream}. */
enum {
    BBO_KIND_LAMBDA_INNER = 1,
    BBO_KIND_LAMBDA_OUTER = 2,
    BBO_KIND_TAU = 3,
    BBO_KIND_SIG2 = 4,
    BBO_KIND_BETA_Z = 5,
    BBO_KIND_DELTA = 6,
    BBO_KIND_ALPHA = 7,
};

static inline void draw4(const uint64_t key[2], uint64_t t, unsigned kind, uint64_t j,
                         uint64_t a, uint64_t b, double u[4])
{
    uint64_t ctr[4] = {t, ((uint64_t)kind << 56) | j, a, b}, o[4];
    bbo_philox4x64(ctr, key, o);
    for (int i = 0; i < 4; ++i)
        u[i] = ((double)(o[i] >> 11) + 0.5) * 0x1.0p-53; /* open (0,1) */
}

static inline double bm_normal(double r0, double r1)
{
    return sqrt(-2.0 * log(r0)) * cos(2.0 * M_PI * r1);
}

void bbo_uniforms(const uint64_t key[2], uint64_t t, unsigned kind, uint64_t j,
                  uint64_t a, uint64_t b, double out[4])
{
    draw4(key, t, kind, j, a, b, out);
}

/* z_j ~ N(0,1) for j in [j0, j0+count): one Philox block per normal. */
void bbo_normals(double *out, long count, const uint64_t key[2], uint64_t t,
                 unsigned kind, uint64_t j0)
{
    for (long i = 0; i < count; ++i) {
        double u[4];
        draw4(key, t, kind, j0 + (uint64_t)i, 0, 0, u);
        out[i] = bm_normal(u[0], u[1]);
    }
}

/* ----------------------------------------------------------------------- */
/* Exponentially tilted positive stable sampler: Code/C/retstable.cpp.      */
/* ----------------------------------------------------------------------- */
static double sinc_MM(double x) /* retstable.cpp:18-29 */
{
    double ax = fabs(x);
    if (ax < 0.006) {
        if (x == 0.) return 1;
        double x2 = x * x;
        if (ax < 2e-4) return 1. - x2 / 6.;
        return 1. - x2 / 6. * (1 - x2 / 20.);
    }
    return sin(x) / x;
}

static double A_(double x, double alpha) /* retstable.cpp:40-47 (_A_3) */
{
    double Ia = 1. - alpha;
    return pow(Ia * sinc_MM(Ia * x), Ia) * pow(alpha * sinc_MM(alpha * x), alpha) / sinc_MM(x);
}

static double BdB0(double x, double alpha) /* retstable.cpp:73-77 */
{
    double Ia = 1. - alpha;
    double den = pow(sinc_MM(alpha * x), alpha) * pow(sinc_MM(Ia * x), Ia);
    return sinc_MM(x) / den;
}

/*
 * retstable.cpp:94-271.  Outer attempt o uses block (t, OUTER|j, o, 0); inner
 * attempt i of outer attempt o uses block (t, INNER|j, o, i).  Slots: inner
 * r0=V, r1=W, r2=W_ (or Box-Muller u1), r3=Box-Muller u2; outer r0=V_,
 * r1=unif / exp / Box-Muller u1, r2=Box-Muller u2.
 * *n_outer / *n_inner (may be NULL) return the attempts consumed.
 */
double bbo_retstable(double h, double alpha, double V0, const uint64_t key[2],
                     uint64_t t, uint64_t j, long *n_outer, long *n_inner)
{
    if (n_outer) *n_outer = 0;
    if (n_inner) *n_inner = 0;
    if (alpha == 1.) return V0; /* :104-110 */
    if (h < 0 || alpha < 0 || alpha > 1 || V0 < 0) { /* :112-115 (print only) */
        fprintf(stderr, "Problem with parameter.\n");
        fprintf(stderr, "V0: %g; h: %g; alpha: %g\n", V0, h, alpha);
    }
    const double c1 = sqrt(BBO_PI_2); /* :121-123 */
    const double c2 = 2. + c1;
    double b = (1. - alpha) / alpha;

    double lambda_alpha = pow(h, alpha) * V0; /* :131 */
    double gamma = lambda_alpha * alpha * (1. - alpha); /* :140-147 */
    double sgamma = sqrt(gamma);
    double c3 = c2 * sgamma;
    double xi = (1. + BBO_SQRT2 * c3) / M_PI;
    double psi = c3 * exp(-gamma * M_PI * M_PI / 8.) / BBO_SQRT_PI;
    double w1 = c1 * xi / sgamma;
    double w2 = 2. * BBO_SQRT_PI * psi;
    double w3 = xi * M_PI;
    double X = 0, c = 0, E = 0;
    long ninner = 0;

    for (uint64_t o = 0;; ++o) { /* outer loop :155-256 */
        double U = 0, z = 0, Z = 0;
        for (uint64_t i = 0;; ++i) { /* inner loop :162-207 */
            double r[4];
            draw4(key, t, BBO_KIND_LAMBDA_INNER, j, o, i, r);
            ++ninner;
            double V = r[0];
            if (gamma >= 1) {
                if (V < w1 / (w1 + w2)) U = fabs(bm_normal(r[2], r[3])) / sgamma;
                else {
                    double W_ = r[2];
                    U = M_PI * (1. - W_ * W_);
                }
            } else {
                double W_ = r[2];
                if (V < w3 / (w2 + w3)) U = M_PI * W_;
                else U = M_PI * (1. - W_ * W_);
            }
            double W = r[1];
            double zeta = sqrt(BdB0(U, alpha));
            z = 1 / (1 - pow(1 + alpha * zeta / sgamma, -1 / alpha));
            double rho = M_PI * exp(-lambda_alpha * (1. - 1. / (zeta * zeta))) /
                         ((1. + c1) * sgamma / zeta + z);
            double d = 0.;
            if (U >= 0 && gamma >= 1) d += xi * exp(-gamma * U * U / 2.);
            if (U > 0 && U < M_PI) d += psi / sqrt(M_PI - U);
            if (U >= 0 && U <= M_PI && gamma < 1) d += xi;
            rho *= d;
            Z = W * rho;
            if (U < M_PI && Z <= 1.) break;
        }
        double a = pow(A_(U, alpha), 1. / (1. - alpha)); /* :212-218 */
        double m = pow(b / a, alpha) * lambda_alpha;
        double delta = sqrt(m * alpha / a);
        double a1 = delta * c1;
        double a2 = delta;
        double a3 = z / a;
        double s = a1 + a2 + a3;

        double r[4];
        draw4(key, t, BBO_KIND_LAMBDA_OUTER, j, o, 0, r);
        double V_ = r[0], N_ = 0., E_ = 0.; /* :224-238 */
        if (V_ < a1 / s) {
            N_ = bm_normal(r[1], r[2]);
            X = m - delta * fabs(N_);
        } else {
            if (V_ < (a1 + a2) / s) X = m + delta * r[1];
            else {
                E_ = -log(r[1]);
                X = m + delta + E_ * a3;
            }
        }
        E = -log(Z); /* :239 */
        c = a * (X - m); /* :247-251 (incl. the "MYMY" h=0 guard) */
        c += (m != 0) ? h * (pow(X, -1. * b) - pow(m, -1. * b)) : 0.0;
        if (X < m) c -= N_ * N_ / 2.;
        else if (X > m + delta) c -= E_;
        if (X >= 0 && c <= E) { /* :256 */
            if (n_outer) *n_outer = (long)o + 1;
            if (n_inner) *n_inner = ninner;
            break;
        }
    }
    return exp(1 / alpha * log(V0) - b * log(X)); /* :270 */
}

/* BridgeWrapper.cpp:965-984 (batch .C entry), counters (t, j = i). */
void bbo_retstable_batch(double *x, const double *alpha, const double *V0, const double *h,
                         long num, const uint64_t key[2], uint64_t t)
{
    for (long i = 0; i < num; ++i)
        x[i] = bbo_retstable(h[i], alpha[i], V0[i], key, t, (uint64_t)i, NULL, NULL);
}

/* BridgeRegression.cpp:506-510; j0 = global index of beta[0] (column shards). */
void bbo_sample_lambda(double *lambda, const double *beta, long p, double alpha, double tau,
                       const uint64_t key[2], uint64_t t, uint64_t j0, long *attempts)
{
    long tot = 0;
    for (long j = 0; j < p; ++j) {
        long no = 0;
        lambda[j] = 2 * bbo_retstable(beta[j] * beta[j] / (tau * tau), 0.5 * alpha, 1.0, key, t,
                                      j0 + (uint64_t)j, &no, NULL);
        tot += no;
    }
    if (attempts) *attempts = tot;
}

/* ----------------------------------------------------------------------- */
/* Gamma / inverse gamma: the RNG contract gamma_rate / igamma.  */
/* Marsaglia-Tsang with one Philox block per attempt.                       */
/* ----------------------------------------------------------------------- */
double bbo_gamma1(double shape, const uint64_t key[2], uint64_t t, unsigned kind)
{
    double a = shape, boost = 1.0;
    if (a < 1.0) {
        double u[4];
        draw4(key, t, kind, 0, 0, 1, u);
        boost = pow(u[0], 1.0 / a);
        a += 1.0;
    }
    double d = a - 1.0 / 3.0;
    double cc = 1.0 / sqrt(9.0 * d);
    for (uint64_t k = 0;; ++k) {
        double u[4];
        draw4(key, t, kind, 0, k, 0, u);
        double x = bm_normal(u[0], u[1]);
        double v = 1.0 + cc * x;
        if (v <= 0.0) continue;
        v = v * v * v;
        double uu = u[2];
        double x2 = x * x;
        if (uu < 1.0 - 0.0331 * x2 * x2) return d * v * boost;
        if (log(uu) < 0.5 * x2 + d * (1.0 - v + log(v))) return d * v * boost;
    }
}

/* BridgeRegression.cpp:453-465: nu ~ Ga(nu_shape + p/alpha, rate = nu_rate + sum|b|^a). */
double bbo_tau_from_sum(double sum_abs_pow, long p, double alpha, double nu_shape, double nu_rate,
                        const uint64_t key[2], uint64_t t)
{
    double shape = nu_shape + ((double)p) / alpha;
    double rate = nu_rate + sum_abs_pow;
    double nu = bbo_gamma1(shape, key, t, BBO_KIND_TAU) / rate;
    return exp(-1.0 * log(nu) / alpha);
}

double bbo_sum_abs_pow(const double *beta, long p, double alpha)
{
    double rate = 0.0;
    for (long j = 0; j < p; ++j) rate += exp(alpha * log(fabs(beta[j])));
    return rate;
}

/* BridgeRegression.cpp:436-450: sig2 ~ IG(a + n/2, scale = b + rss/2). */
double bbo_sig2_from_rss(double rss, long n, double sig2_shape, double sig2_scale,
                         const uint64_t key[2], uint64_t t)
{
    double shape = sig2_shape + 0.5 * (double)n;
    double scale = sig2_scale + 0.5 * rss;
    return scale / bbo_gamma1(shape, key, t, BBO_KIND_SIG2);
}

/* BridgeRegression.cpp:469-476 */
static double llh_alpha_marg(double alpha, const double *s, long p)
{
    double pp = (double)p;
    double llh = pp * log(alpha) - pp * lgamma(1.0 / alpha);
    for (long i = 0; i < p; ++i) llh -= exp(alpha * s[i]);
    return llh;
}

static double log_dbeta(double x, double a, double b)
{
    return (a - 1.0) * log(x) + (b - 1.0) * log(1.0 - x) - (lgamma(a) + lgamma(b) - lgamma(a + b));
}

/* BridgeRegression.cpp:478-503 (random-walk MH on alpha, window ep).  s is scratch (p). */
double bbo_alpha_mh(double a_old, const double *beta, long p, double tau, double pr_a,
                    double pr_b, double ep, double *s, const uint64_t key[2], uint64_t t)
{
    for (long i = 0; i < p; ++i) s[i] = log(fabs(beta[i] / tau));
    double u[4];
    draw4(key, t, BBO_KIND_ALPHA, 0, 0, 0, u);
    double l_new = fmax(0.0, a_old - ep);
    double r_new = fmin(1.0, a_old + ep);
    double d_new = r_new - l_new;
    double a_new = l_new + d_new * u[0]; /* r.flat(l_new, r_new) */
    double l_old = fmax(0.0, a_new - ep);
    double r_old = fmin(1.0, a_new + ep);
    double d_old = r_old - l_old;
    double log_accept = llh_alpha_marg(a_new, s, p) - llh_alpha_marg(a_old, s, p) +
                        log_dbeta(a_new, pr_a, pr_b) - log_dbeta(a_old, pr_a, pr_b) +
                        log(d_old) - log(d_new);
    if (u[1] > exp(log_accept)) return a_old;
    return a_new;
}

/* ----------------------------------------------------------------------- */
/* Triangle-mixture sampler (bridge.reg.tri): BridgeRegression.cpp:97-147    */
/* (sample_u, sample_omega with shape), :405-433 (sample_beta), :235-286     */
/* (rtnorm_gibbs).  The truncated normal r.tnorm comes from the un-vendored  */
/* RNG library, so it is restated from Robert (1995): normal or uniform      */
/* rejection when the interval holds 0, else Robert's uniform / translated-  */
/* exponential choice.  Counter kinds 8 (omega), 9 (u), 10 (z_i attempts).   */
/* ----------------------------------------------------------------------- */
enum { BBO_KIND_TRI_OMEGA = 8, BBO_KIND_TRI_U = 9, BBO_KIND_TRI_Z = 10 };
#define BBO_TN_MAX_ATTEMPTS (1L << 22)

/* one-sided standard truncated normal on [a, b], 0 <= a < b (Robert 1995, prop. 2.3) */
static double tn_pos(double a, double b, const uint64_t key[2], uint64_t t, uint64_t i,
                     uint64_t it, int *fail)
{
    const double sq = sqrt(a * a + 4.0);
    const double as = 0.5 * (a + sq);
    const double thr = a + 2.0 / (a + sq) * exp(0.5 + 0.25 * (a * a - a * sq));
    for (long k = 0; k < BBO_TN_MAX_ATTEMPTS; ++k) {
        double r[4];
        draw4(key, t, BBO_KIND_TRI_Z, i, it, (uint64_t)k, r);
        if (b <= thr) {
            const double x = a + (b - a) * r[0];
            if (r[1] <= exp(0.5 * (a * a - x * x))) return x;
        } else {
            const double x = a - log(r[0]) / as;
            const double e = x - as;
            if (x <= b && r[1] <= exp(-0.5 * e * e)) return x;
        }
    }
    *fail = 1;
    return a;
}

/* r.tnorm(lo, hi, mu, sd) restated; attempts use counters (t, 10<<56 | i, it, k). */
double bbo_tnorm(double lo, double hi, double mu, double sd, const uint64_t key[2], uint64_t t,
                 uint64_t i, uint64_t it, int *fail)
{
    const double a = (lo - mu) / sd, b = (hi - mu) / sd;
    if (!(a < b)) {
        *fail = 2;
        return lo;
    }
    if (a <= 0.0 && b >= 0.0) {
        const int wide = (b - a) >= 2.5066282746310002; /* sqrt(2 pi) */
        for (long k = 0; k < BBO_TN_MAX_ATTEMPTS; ++k) {
            double r[4];
            draw4(key, t, BBO_KIND_TRI_Z, i, it, (uint64_t)k, r);
            if (wide) {
                const double x = bm_normal(r[0], r[1]);
                if (x >= a && x <= b) return mu + sd * x;
            } else {
                const double x = a + (b - a) * r[0];
                if (r[1] <= exp(-0.5 * x * x)) return mu + sd * x;
            }
        }
        *fail = 1;
        return lo;
    }
    if (a > 0.0) return mu + sd * tn_pos(a, b, key, t, i, it, fail);
    return mu - sd * tn_pos(-b, -a, key, t, i, it, fail);
}

/*
 * One sweep's omega, u and beta updates of the triangle sampler, given tau, sig2,
 * alpha.  tV is the p x p matrix V' of X = U diag(d) V' (column-major, tV[i + j p]),
 * a = d * U'y (BridgeRegression.cpp:47-57).  u holds the previous sweep's u on entry.
 * rtnorm_gibbs keeps beta_cur = tV' z up to date incrementally (beta_cur_j += v_ji dz_i)
 * instead of recomputing dot(v_j, z) for every i (:254-258): the same quantity, O(p^2)
 * instead of O(p^3) per pass.  Returns the number of failed truncated draws.
 */
long bbo_tri_update(double *beta, double *u, double *omega, double *shape, long p,
                    const double *tV, const double *a, const double *d, const double *G,
                    const double *c, int ortho, double tau, double sig2, double alpha,
                    int betaburn, const uint64_t key[2], uint64_t t, double *z, double *bcur,
                    double *b)
{
    long fails = 0;
    for (long j = 0; j < p; ++j) {
        double r[4];
        /* sample_omega :130-146 */
        const double aj = exp(alpha * log(fabs(beta[j]) / ((1.0 - u[j]) * tau)));
        const double prob = alpha / (1.0 + alpha * aj);
        draw4(key, t, BBO_KIND_TRI_OMEGA, (uint64_t)j, 0, 0, r);
        double w;
        if (r[0] > prob) {
            shape[j] = 1.0;
            w = -log(r[1]); /* Ga(1, 1) */
        } else {
            shape[j] = 2.0;
            w = -log(r[1]) - log(r[2]); /* Ga(2, 1) */
        }
        omega[j] = w + aj;
        /* sample_u :97-111: flat(0, right) */
        const double right = 1.0 - fabs(beta[j]) / tau * exp(-1.0 * log(omega[j]) / alpha);
        draw4(key, t, BBO_KIND_TRI_U, (uint64_t)j, 0, 0, r);
        u[j] = right * r[0];
        /* sample_beta :410-412 */
        b[j] = (1.0 - u[j]) * exp(log(omega[j]) / alpha) * tau;
    }
    const double sig = sqrt(sig2);
    if (ortho) {
        /* sample_beta_ortho (BridgeRegression.cpp:362-403), one pass: G is the full
         * p x p X'X, c = X'y. */
        for (long j = 0; j < p; ++j) {
            double xb = 0.0;
            for (long k = 0; k < p; ++k)
                if (k != j) xb += G[j * p + k] * beta[k];
            const double gjj = G[j * p + j];
            const double m = (c[j] - xb) / gjj, v = sig2 / gjj;
            int f = 0;
            beta[j] = bbo_tnorm(-1.0 * b[j], b[j], m, sqrt(v), key, t, (uint64_t)j, 0, &f);
            fails += f != 0;
        }
        return fails;
    }
    for (int it = 0; it <= betaburn; ++it) {
        for (long i = 0; i < p; ++i) { /* z = tV beta (:246) */
            double s = 0.0;
            for (long j = 0; j < p; ++j) s += tV[i + j * p] * beta[j];
            z[i] = s;
        }
        for (long j = 0; j < p; ++j) {
            double s = 0.0;
            for (long k = 0; k < p; ++k) s += tV[k + j * p] * z[k];
            bcur[j] = s;
        }
        for (long i = 0; i < p; ++i) { /* :250-283 */
            double lmax = -1.0 * 1.7976931348623157e308, rmin = 1.7976931348623157e308;
            const double zi = z[i];
            for (long j = 0; j < p; ++j) {
                const double vji = tV[i + j * p];
                const double rji = bcur[j] - vji * zi;
                const double dif = b[j] - rji, sum = b[j] + rji;
                const double left = (vji > 0 ? -sum : -dif) / fabs(vji);
                const double right = (vji > 0 ? dif : sum) / fabs(vji);
                lmax = lmax > left ? lmax : left;
                rmin = rmin < right ? rmin : right;
            }
            double zn;
            if (d[i] > 1e-16) {
                int f = 0;
                zn = bbo_tnorm(lmax, rmin, a[i] / (d[i] * d[i]), sig / d[i], key, t,
                               (uint64_t)i, (uint64_t)it, &f);
                fails += f != 0;
            } else {
                double r[4];
                draw4(key, t, BBO_KIND_TRI_Z, (uint64_t)i, (uint64_t)it, 0, r);
                zn = lmax + (rmin - lmax) * r[0];
            }
            const double dz = zn - zi;
            z[i] = zn;
            for (long j = 0; j < p; ++j) bcur[j] += tV[i + j * p] * dz;
        }
        for (long j = 0; j < p; ++j) { /* beta = tV' z (:285) */
            double s = 0.0;
            for (long k = 0; k < p; ++k) s += tV[k + j * p] * z[k];
            beta[j] = s;
        }
    }
    return fails;
}

/* ----------------------------------------------------------------------- */
/* Truncated-distribution .C utilities, BridgeWrapper.cpp:762-935.          */
/* Draw i: truncated-normal attempts on (0, 10<<56 | i, 0, k) (bbo_tnorm     */
/* with t = 0, it = 0), exponential / plain normal on (0, 12<<56 | i, 0, 0). */
/* ----------------------------------------------------------------------- */
static double bbo_texpon(double left, double right, double rate, double u)
{
    if (isinf(right)) return left - log(u) / rate;
    return left - log1p(u * expm1(-rate * (right - left))) / rate;
}

long bbo_trunc_batch(int mode, long num, double *x, const double *p0, const double *p1,
                     const double *p2, const double *p3, const uint64_t key[2])
{
    long fails = 0;
    const double inf = INFINITY;
    for (long i = 0; i < num; ++i) {
        double e[4];
        int f = 0;
        draw4(key, 0, 12, (uint64_t)i, 0, 0, e);
        switch (mode) {
        case 0: x[i] = bbo_tnorm(p0[i], inf, p1[i], p2[i], key, 0, i, 0, &f); break;
        case 1: x[i] = bbo_tnorm(p0[i], p1[i], p2[i], p3[i], key, 0, i, 0, &f); break;
        case 2: {
            const double l = p0[i], r = p1[i], mu = p2[i], sg = p3[i];
            if (isnan(l) || isnan(r) || isnan(mu) || isnan(sg)) x[i] = NAN;
            else if (!isinf(l) && !isinf(r)) x[i] = bbo_tnorm(l, r, mu, sg, key, 0, i, 0, &f);
            else if (!isinf(l) && r == inf) x[i] = bbo_tnorm(l, inf, mu, sg, key, 0, i, 0, &f);
            else if (l == -inf && !isinf(r))
                x[i] = -1.0 * bbo_tnorm(-1.0 * r, inf, -1.0 * mu, sg, key, 0, i, 0, &f);
            else if (l == -inf && r == inf) x[i] = mu + sg * bm_normal(e[0], e[1]);
            else x[i] = NAN;
            break;
        }
        case 3: x[i] = bbo_texpon(p0[i], inf, p1[i], e[0]); break;
        case 4: x[i] = bbo_texpon(p0[i], p1[i], p2[i], e[0]); break;
        default: {
            /* BridgeWrapper.cpp:816-828: the NaN set for a non-finite input is overwritten by
             * the draw (no else); a non-finite right is left truncation only */
            const double l = p0[i], r = p1[i], rate = p2[i];
            x[i] = bbo_texpon(l, isfinite(r) ? r : inf, rate, e[0]);
        }
        }
        fails += f != 0;
    }
    return fails;
}

/* ----------------------------------------------------------------------- */
/* Right-truncated gamma for rrtgamma_rate, BridgeWrapper.cpp:944-962:      */
/* x ~ Ga(shape, rate) restricted to (0, right_t].  r.rtgamma_rate comes from */
/* the un-vendored RNG library; restated as an exact rejection sampler on    */
/* Y = rate * x ~ Ga(a, 1) | Y <= T, T = rate * right_t, attempt k on        */
/* (0, 13<<56 | i, k, 0):                                                    */
/*   T >= a      : Marsaglia-Tsang draw (one block), accept if Y <= T        */
/*   a <= 1      : Y = T U^(1/a), accept w.p. e^-Y                            */
/*   T <= a - 1  : increasing log-concave density: Y = T - Z, Z ~ Exp(c) on   */
/*                 [0, T], c = (a-1)/T - 1 (tangent envelope at T)          */
/*   otherwise   : uniform on (0, T], bound at the mode a - 1                 */
/* ----------------------------------------------------------------------- */
double bbo_rtgamma_std(double a, double T, const uint64_t key[2], uint64_t i, int *fail)
{
    for (long k = 0; k < BBO_TN_MAX_ATTEMPTS; ++k) {
        double r[4];
        draw4(key, 0, 13, i, (uint64_t)k, 0, r);
        if (T >= a) {
            const double ap = a < 1.0 ? a + 1.0 : a;
            const double d = ap - 1.0 / 3.0, cc = 1.0 / sqrt(9.0 * d);
            const double x = bm_normal(r[0], r[1]);
            double v = 1.0 + cc * x;
            if (v <= 0.0) continue;
            v = v * v * v;
            const double x2 = x * x;
            if (!(r[2] < 1.0 - 0.0331 * x2 * x2) && !(log(r[2]) < 0.5 * x2 + d * (1.0 - v + log(v))))
                continue;
            double y = d * v;
            if (a < 1.0) y *= pow(r[3], 1.0 / a);
            if (y <= T) return y;
        } else if (a <= 1.0) {
            const double y = T * pow(r[0], 1.0 / a);
            if (r[1] <= exp(-y)) return y;
        } else if (T <= a - 1.0) {
            const double c = (a - 1.0) / T - 1.0;
            const double z = c > 0.0 ? -log1p(r[0] * expm1(-c * T)) / c : T * r[0];
            const double y = T - z;
            if (y > 0.0 && log(r[1]) <= (a - 1.0) * log(y / T) + z + c * z) return y;
        } else {
            const double m = a - 1.0;
            const double y = T * r[0];
            if (log(r[1]) <= (a - 1.0) * log(y / m) - (y - m)) return y;
        }
    }
    *fail = 1;
    return T;
}

long bbo_rrtgamma_batch(long num, double *x, const double *shape, const double *rate,
                        const double *right_t, const uint64_t key[2])
{
    long fails = 0;
    for (long i = 0; i < num; ++i) {
        int f = 0;
        x[i] = bbo_rtgamma_std(shape[i], rate[i] * right_t[i], key, (uint64_t)i, &f) / rate[i];
        fails += f;
    }
    return fails;
}

/* ----------------------------------------------------------------------- */
/* Polya-Gamma PG(1, z) draws for the logistic bridge (BASELINE config C4).  */
/* ----------------------------------------------------------------------- */
/*
 * No reference counterpart (the reference has no logistic model).  This is
 * the published exact sampler of Polson, Scott & Windle (2013, JASA 108:1339-1349,
 * "Bayesian inference for logistic models using Polya-Gamma latent variables", Algorithms
 * 1-2 and the appendix): PG(1, z) = J*(1, z/2) / 4, J* drawn by Devroye's alternating-series
 * method with the truncation point t = 0.64 -- a proposal mixing an exponential tail on
 * (t, inf) and an inverse-Gaussian body on (0, t), accepted by the alternating series of
 * the J* density.  PARITY UNPINNED against any reference implementation; pinned by the
 * exact moments E = tanh(z/2)/(2z), Var = (sinh z - z) / (4 z^3 cosh^2(z/2)), the Laplace
 * transform cosh(z/2) / cosh(sqrt((z^2/2 + s)/2)) and a two-sample KS test against the
 * infinite-convolution definition (tests/test_logit_cpu.py).
 *
 * Counter-based like every draw here: outer attempt o uses block (t, kind 11, i, o, 0) =
 * {mixture choice, exponential, series uniform}; the inverse-Gaussian body's sub-attempt k
 * uses block (t, kind 12, i, o, k).  The GPU kernel (bb_logit.hip) evaluates the same
 * expressions in the same order.
 */
#define BBO_PG_T 0.64
#define BBO_KIND_PG 11
#define BBO_KIND_PG_IG 12
#define BBO_PG_MAX_ATTEMPTS 1000
#define BBO_PG_MAX_TERMS 1000

static double pg_log_ncdf(double x) { return log(0.5 * erfc(-x * 0.70710678118654752440)); }

/* n-th coefficient of the alternating series of the J*(1, 0) density at x */
static double pg_a(int n, double x)
{
    const double K = (n + 0.5) * M_PI;
    if (x > BBO_PG_T) return K * exp(-0.5 * K * K * x);
    if (x > 0.0)
        return exp(-1.5 * (log(0.5 * M_PI) + log(x)) + log(K) - 2.0 * (n + 0.5) * (n + 0.5) / x);
    return 0.0;
}

/* probability of the exponential piece: p / (p + q) */
static double pg_mass_texpon(double z)
{
    const double t = BBO_PG_T;
    const double fz = 0.125 * M_PI * M_PI + 0.5 * z * z;
    const double b = sqrt(1.0 / t) * (t * z - 1.0);
    const double a = -sqrt(1.0 / t) * (t * z + 1.0);
    const double x0 = log(fz) + fz * t;
    const double xb = x0 - z + pg_log_ncdf(b);
    const double xa = x0 + z + pg_log_ncdf(a);
    const double qdivp = 4.0 / M_PI * (exp(xb) + exp(xa));
    return 1.0 / (1.0 + qdivp);
}

/* inverse-Gaussian IG(1/z, 1) truncated to (0, t) */
static double pg_rtigauss(double z, const uint64_t key[2], uint64_t t, uint64_t i, uint64_t o,
                          int *fail)
{
    const double tr = BBO_PG_T;
    for (uint64_t k = 0; k < BBO_PG_MAX_ATTEMPTS; ++k) {
        double u[4];
        draw4(key, t, BBO_KIND_PG_IG, i, o, k, u);
        if (z < 1.0 / tr) {
            /* mean above t: 1/X from a truncated chi-square(1) by rejection, then the
             * exp(-z^2 X / 2) tilt */
            const double E1 = -log(u[0]), E2 = -log(u[1]);
            if (E1 * E1 > 2.0 * E2 / tr) continue;
            const double d = 1.0 + E1 * tr;
            const double X = tr / (d * d);
            if (u[2] <= exp(-0.5 * z * z * X)) return X;
        } else {
            /* mean below t: Michael-Schucany-Haas inverse-Gaussian draw until X < t */
            const double mu = 1.0 / z;
            double Y = bm_normal(u[0], u[1]);
            Y *= Y;
            const double half_mu = 0.5 * mu, mu_Y = mu * Y;
            double X = mu + half_mu * mu_Y - half_mu * sqrt(4.0 * mu_Y + mu_Y * mu_Y);
            if (u[2] > mu / (mu + X)) X = mu * mu / X;
            if (X <= tr) return X;
        }
    }
    *fail = 1;
    return tr;
}

double bbo_pg1(double psi, const uint64_t key[2], uint64_t t, uint64_t i, int *fail)
{
    const double z = fabs(psi) * 0.5;
    const double fz = 0.125 * M_PI * M_PI + 0.5 * z * z;
    const double mass = pg_mass_texpon(z);
    for (uint64_t o = 0; o < BBO_PG_MAX_ATTEMPTS; ++o) {
        double u[4];
        draw4(key, t, BBO_KIND_PG, i, o, 0, u);
        double X;
        if (u[0] < mass)
            X = BBO_PG_T + (-log(u[1])) / fz;
        else
            X = pg_rtigauss(z, key, t, i, o, fail);
        double S = pg_a(0, X);
        const double Y = u[2] * S;
        for (int n = 1; n < BBO_PG_MAX_TERMS; ++n) {
            if (n & 1) {
                S -= pg_a(n, X);
                if (Y <= S) return 0.25 * X;
            } else {
                S += pg_a(n, X);
                if (Y > S) break;
            }
        }
    }
    *fail = 1;
    return 0.25;
}

/* omega_i ~ PG(1, psi_i), i = 0 .. n-1; returns the number of failed draws */
long bbo_pg_batch(double *omega, const double *psi, long n, const uint64_t key[2], uint64_t t)
{
    long fails = 0;
    for (long i = 0; i < n; ++i) {
        int f = 0;
        omega[i] = bbo_pg1(psi[i], key, t, (uint64_t)i, &f);
        fails += f;
    }
    return fails;
}
