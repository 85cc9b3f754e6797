/*
 * bb_cpu_chain.c -- TEST INFRASTRUCTURE / CPU BASELINE ONLY.
 *
 * A compiled, reference-literal CPU restatement of the stable Gibbs driver
 * bridge_regression_stable (Code/C/BridgeWrapper.cpp:207-313; the orthogonal twin
 * :434-537) with the reference's own dense linear algebra: X'X and X'y once
 * (BridgeRegression.cpp:24-25), then per sweep
 *   tau | beta     BridgeRegression.cpp:453-465   (bbo_tau_from_sum)
 *   sig2 | beta    :436-450, rss by dgemv          (bbo_sig2_from_rss)
 *   lambda | beta  :506-510 -> retstable.cpp:94-271 (bbo_retstable)
 *   beta | rest    :552-575: A = X'X + diag(lambda sig2 / tau^2), dpotrf 'U',
 *                  two triangular solves for the mean, one for U^-1 z
 * or, for p > n, the exact Woodbury form of the same conditional (DESIGN.md s6:
 * dsyrk of X diag(sqrt D), an n x n dpotrf, dgemv for X u and X'w) -- the algorithm
 * the GPU path runs, so the two time the same arithmetic.
 *
 * It is bench.py's compiled cpu_baseline ("the build's C++ restatement
 * ... linked to an available LAPACK", timed at 1 core and all cores) and is checked
 * against oracle/gibbs.py, the Python restatement, on the same Philox counters
 * (tests/test_cpu_chain.py).  Nothing in the product links or loads it.
 *
 * Variates: the oracle's (bb_oracle.c), i.e. the GPU path's counter layout
 * (DESIGN.md s2), so a chain here equals oracle/gibbs.py's up to LAPACK rounding.
 * LAPACK/BLAS: the OpenBLAS that scipy ships (scipy_ prefixed symbols), the only
 * LAPACK in this image.  With threads > 1 the BLAS runs that many threads and the
 * p independent lambda draws are split over OpenMP threads (counter-based draws:
 * identical results for any thread count).
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* bb_oracle.c */
double bbo_retstable(double h, double alpha, double V0, const uint64_t key[2], uint64_t t,
                     uint64_t j, long *n_outer, long *n_inner);
void bbo_normals(double *out, long count, const uint64_t key[2], uint64_t t, unsigned kind,
                 uint64_t j0);
double bbo_tau_from_sum(double sum_abs_pow, long p, double alpha, double nu_shape,
                        double nu_rate, const uint64_t key[2], uint64_t t);
double bbo_sum_abs_pow(const double *beta, long p, double alpha);
double bbo_sig2_from_rss(double rss, long n, double sig2_shape, double sig2_scale,
                         const uint64_t key[2], uint64_t t);

#define KIND_BETA_Z 5
#define KIND_DELTA 6

/* scipy's OpenBLAS (LP64, Fortran calling convention; trailing hidden string lengths) */
void scipy_dpotrf_(const char *uplo, const int *n, double *a, const int *lda, int *info,
                   size_t);
void scipy_dtrsm_(const char *side, const char *uplo, const char *transa, const char *diag,
                  const int *m, const int *n, const double *alpha, const double *a,
                  const int *lda, double *b, const int *ldb, size_t, size_t, size_t, size_t);
void scipy_dsyrk_(const char *uplo, const char *trans, const int *n, const int *k,
                  const double *alpha, const double *a, const int *lda, const double *beta,
                  double *c, const int *ldc, size_t, size_t);
void scipy_dgemm_(const char *ta, const char *tb, const int *m, const int *n, const int *k,
                  const double *alpha, const double *a, const int *lda, const double *b,
                  const int *ldb, const double *beta, double *c, const int *ldc, size_t,
                  size_t);
void scipy_dgemv_(const char *trans, const int *m, const int *n, const double *alpha,
                  const double *a, const int *lda, const double *x, const int *incx,
                  const double *beta, double *y, const int *incy, size_t);
void scipy_openblas_set_num_threads(int);

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

/* y <- alpha op(A) x + beta y, A m x n column-major */
static void gemv(char tr, int m, int n, double alpha, const double *A, const double *x,
                 double beta, double *y)
{
    const int one = 1;
    scipy_dgemv_(&tr, &m, &n, &alpha, A, &m, x, &one, &beta, y, &one, 1);
}

/* solve op(U) x = b in place, U upper triangular m x m (lda m), nrhs = 1 */
static void trsv_u(char tr, int m, const double *U, double *b)
{
    const int one = 1;
    const double done = 1.0;
    scipy_dtrsm_("L", "U", &tr, "N", &m, &one, &done, U, &m, b, &m, 1, 1, 1, 1);
}

/* BridgeRegression.cpp:506-510, lambda_j = 2 retstable(beta_j^2 / tau^2, alpha / 2, 1) */
static void draw_lambda(double *lam, const double *beta, long p, double alpha, double tau,
                        const uint64_t key[2], uint64_t t)
{
#pragma omp parallel for schedule(dynamic, 64)
    for (long j = 0; j < p; ++j)
        lam[j] = 2 * bbo_retstable(beta[j] * beta[j] / (tau * tau), 0.5 * alpha, 1.0, key, t,
                                   (uint64_t)j, NULL, NULL);
}

typedef struct {
    int n, p, method; /* method 0 chol (p x p), 1 woodbury (n x n), 2 ortho */
    const double *X, *y;
    double alpha, nu_shape, nu_rate, sig2_shape, sig2_scale, true_sig2;
    uint64_t key[2];
    /* work */
    double *G, *c, *A, *r, *z, *d, *D, *u, *v, *Y, *M, *w, *tmp;
} Chain;

static double draw_sig2(Chain *ch, const double *beta, uint64_t t)
{
    if (ch->true_sig2 > 0) return ch->true_sig2;
    memcpy(ch->r, ch->y, sizeof(double) * ch->n);
    gemv('N', ch->n, ch->p, -1.0, ch->X, beta, 1.0, ch->r); /* r = y - X beta */
    double rss = 0.0;
    for (int i = 0; i < ch->n; ++i) rss += ch->r[i] * ch->r[i];
    return bbo_sig2_from_rss(rss, ch->n, ch->sig2_shape, ch->sig2_scale, ch->key, t);
}

static double draw_tau(Chain *ch, const double *beta, uint64_t t)
{
    return bbo_tau_from_sum(bbo_sum_abs_pow(beta, ch->p, ch->alpha), ch->p, ch->alpha,
                            ch->nu_shape, ch->nu_rate, ch->key, t);
}

/* BridgeRegression.cpp:552-575.  Returns LAPACK's info (0 = success). */
static int beta_chol(Chain *ch, const double *lam, double sig2, double tau, uint64_t t,
                     double *beta)
{
    const int p = ch->p;
    const size_t pp = (size_t)p * p;
    memcpy(ch->A, ch->G, sizeof(double) * pp); /* VInv = XX + diag(lambda sig2/tau^2) */
    const double f = sig2 / (tau * tau);
    for (int j = 0; j < p; ++j) ch->A[(size_t)j * p + j] += lam[j] * f;
    int info = 0;
    scipy_dpotrf_("U", &p, ch->A, &p, &info, 1); /* chol(U, VInv, 'U') */
    if (info) return info;
    memcpy(beta, ch->c, sizeof(double) * p); /* m = U^-1 U'^-1 Xy */
    trsv_u('T', p, ch->A, beta);
    trsv_u('N', p, ch->A, beta);
    bbo_normals(ch->z, p, ch->key, t, KIND_BETA_Z, 0);
    trsv_u('N', p, ch->A, ch->z); /* U^-1 z */
    const double s = sqrt(sig2);
    for (int j = 0; j < p; ++j) beta[j] += s * ch->z[j];
    return 0;
}

/* The same conditional for p > n (Bhattacharya et al. 2016):
 * u = sqrt(D) z, v = X u / sig + delta, M = I + X D X' / sig2 = U'U,
 * w = M^-1 (y / sig - v), beta = u + D X'w / sig. */
static int beta_woodbury(Chain *ch, const double *lam, double sig2, double tau, uint64_t t,
                         double *beta)
{
    const int n = ch->n, p = ch->p;
    const double sig = sqrt(sig2);
    bbo_normals(ch->z, p, ch->key, t, KIND_BETA_Z, 0);
    bbo_normals(ch->d, n, ch->key, t, KIND_DELTA, 0);
#pragma omp parallel for schedule(static)
    for (long j = 0; j < p; ++j) {
        const double Dj = tau * tau / lam[j], sj = sqrt(Dj);
        ch->D[j] = Dj;
        ch->u[j] = sj * ch->z[j];
        const double *xs = ch->X + (size_t)j * n;
        double *ys = ch->Y + (size_t)j * n;
        for (int i = 0; i < n; ++i) ys[i] = xs[i] * sj; /* Y = X diag(sqrt D) */
    }
    gemv('N', n, p, 1.0 / sig, ch->X, ch->u, 0.0, ch->v);
    for (int i = 0; i < n; ++i) ch->v[i] += ch->d[i];
    const double a = 1.0 / sig2, zero = 0.0;
    scipy_dsyrk_("U", "N", &n, &p, &a, ch->Y, &n, &zero, ch->M, &n, 1, 1);
    for (int i = 0; i < n; ++i) ch->M[(size_t)i * n + i] += 1.0;
    int info = 0;
    scipy_dpotrf_("U", &n, ch->M, &n, &info, 1);
    if (info) return info;
    for (int i = 0; i < n; ++i) ch->w[i] = ch->y[i] / sig - ch->v[i];
    trsv_u('T', n, ch->M, ch->w);
    trsv_u('N', n, ch->M, ch->w);
    gemv('T', n, p, 1.0, ch->X, ch->w, 0.0, ch->tmp); /* X'w */
    for (int j = 0; j < p; ++j) beta[j] = ch->u[j] + ch->D[j] * ch->tmp[j] / sig;
    return 0;
}

/* BridgeRegression.cpp:514-521 */
static void beta_ortho(Chain *ch, const double *lam, double sig2, double tau, uint64_t t,
                       double *beta)
{
    bbo_normals(ch->z, ch->p, ch->key, t, KIND_BETA_Z, 0);
    for (int j = 0; j < ch->p; ++j) {
        const double uj = ch->G[(size_t)j * ch->p + j] + lam[j] * sig2 / (tau * tau);
        beta[j] = ch->c[j] / uj + sqrt(sig2 / uj) * ch->z[j];
    }
}

static int draw_beta(Chain *ch, const double *lam, double sig2, double tau, uint64_t t,
                     double *beta)
{
    if (ch->method == 0) return beta_chol(ch, lam, sig2, tau, t, beta);
    if (ch->method == 1) return beta_woodbury(ch, lam, sig2, tau, t, beta);
    beta_ortho(ch, lam, sig2, tau, t, beta);
    return 0;
}

/*
 * The stable chain with alpha known, as oracle/gibbs.py bridge_regression_stable restates
 * the driver: beta0 = least squares for p <= n (0 otherwise), the pre-burn tau draw (non
 * ortho), burn + 1 burn-in sweeps in slot 0, then M - 1 MCMC sweeps; the ortho driver draws
 * tau -> lambda -> sig2 -> beta.  Outputs (any may be NULL): beta_out P x M, tau_out and
 * sig2_out M.  Returns the post-burn wall seconds (the reference's `runtime`), or a
 * negative value on failure (-1 allocation, -(1 + info) LAPACK).
 */
double bbc_stable_chain(int method, const double *X, const double *y, int n, int p, double alpha,
                        double nu_shape, double nu_rate, double sig2_shape, double sig2_scale,
                        double true_sig2, int burn, int M, uint64_t seed, uint64_t stream,
                        int threads, double *beta_out, double *tau_out, double *sig2_out)
{
    if (threads < 1) threads = 1;
    scipy_openblas_set_num_threads(threads);
    omp_set_num_threads(threads);
    Chain ch = {0};
    ch.n = n;
    ch.p = p;
    ch.method = method;
    ch.X = X;
    ch.y = y;
    ch.alpha = alpha;
    ch.nu_shape = nu_shape;
    ch.nu_rate = nu_rate;
    ch.sig2_shape = sig2_shape;
    ch.sig2_scale = sig2_scale;
    ch.true_sig2 = true_sig2;
    ch.key[0] = seed;
    ch.key[1] = stream;
    const size_t pp = (size_t)p * p, np_ = (size_t)n * p, nn = (size_t)n * n;
    const int need_G = method != 1;
    double *beta = calloc(p, sizeof(double)), *lam = calloc(p, sizeof(double));
    ch.c = calloc(p, sizeof(double));
    ch.r = calloc(n, sizeof(double));
    ch.z = calloc(p, sizeof(double));
    ch.d = calloc(n, sizeof(double));
    ch.tmp = calloc(p > n ? p : n, sizeof(double));
    if (need_G) {
        ch.G = malloc(sizeof(double) * pp);
        ch.A = malloc(sizeof(double) * pp);
    } else {
        ch.D = calloc(p, sizeof(double));
        ch.u = calloc(p, sizeof(double));
        ch.v = calloc(n, sizeof(double));
        ch.Y = malloc(sizeof(double) * np_);
        ch.M = malloc(sizeof(double) * nn);
        ch.w = calloc(n, sizeof(double));
    }
    double rt = -1.0;
    if (!beta || !lam || !ch.c || !ch.r || !ch.z || !ch.d || !ch.tmp ||
        (need_G && (!ch.G || !ch.A)) ||
        (!need_G && (!ch.D || !ch.u || !ch.v || !ch.Y || !ch.M || !ch.w)))
        goto done;
    gemv('T', n, p, 1.0, X, y, 0.0, ch.c); /* Xy = X'y (BridgeRegression.cpp:25) */
    if (need_G) {                          /* XX = X'X (:24) */
        const double one = 1.0, zero = 0.0;
        scipy_dgemm_("T", "N", &p, &p, &n, &one, X, &n, X, &n, &zero, ch.G, &p, 1, 1);
    }
    /* beta0: least squares when X'X is invertible (:79-91), else 0 */
    if (method == 0 && p <= n) {
        memcpy(ch.A, ch.G, sizeof(double) * pp);
        int info = 0;
        scipy_dpotrf_("U", &p, ch.A, &p, &info, 1);
        if (info == 0) {
            memcpy(beta, ch.c, sizeof(double) * p);
            trsv_u('T', p, ch.A, beta);
            trsv_u('N', p, ch.A, beta);
        }
    }
    const int ortho = method == 2;
    double tau = 0.0, sig2 = true_sig2 > 0 ? true_sig2 : 0.0;
    if (!ortho) tau = draw_tau(&ch, beta, 0); /* BridgeWrapper.cpp:262 */
    int info = 0;
    for (int i = 0; i <= burn && !info; ++i) {
        const uint64_t t = 1 + (uint64_t)i;
        if (ortho) { /* :493-503 */
            tau = draw_tau(&ch, beta, t);
            draw_lambda(lam, beta, p, alpha, tau, ch.key, t);
            sig2 = draw_sig2(&ch, beta, t);
        } else { /* :266-276 */
            tau = draw_tau(&ch, beta, t);
            sig2 = draw_sig2(&ch, beta, t);
            draw_lambda(lam, beta, p, alpha, tau, ch.key, t);
        }
        info = draw_beta(&ch, lam, sig2, tau, t, beta);
    }
    if (beta_out) memcpy(beta_out, beta, sizeof(double) * p);
    if (tau_out) tau_out[0] = tau;
    if (sig2_out) sig2_out[0] = sig2;
    const double t0 = now_s();
    for (int i = 1; i < M && !info; ++i) { /* :287-298 */
        const uint64_t t = (uint64_t)burn + 1 + (uint64_t)i;
        if (ortho) {
            tau = draw_tau(&ch, beta, t);
            draw_lambda(lam, beta, p, alpha, tau, ch.key, t);
            sig2 = draw_sig2(&ch, beta, t);
        } else {
            tau = draw_tau(&ch, beta, t);
            sig2 = draw_sig2(&ch, beta, t);
            draw_lambda(lam, beta, p, alpha, tau, ch.key, t);
        }
        info = draw_beta(&ch, lam, sig2, tau, t, beta);
        if (beta_out) memcpy(beta_out + (size_t)i * p, beta, sizeof(double) * p);
        if (tau_out) tau_out[i] = tau;
        if (sig2_out) sig2_out[i] = sig2;
    }
    rt = info ? -(1.0 + info) : now_s() - t0;
done:
    free(beta);
    free(lam);
    free(ch.c);
    free(ch.r);
    free(ch.z);
    free(ch.d);
    free(ch.tmp);
    free(ch.G);
    free(ch.A);
    free(ch.D);
    free(ch.u);
    free(ch.v);
    free(ch.Y);
    free(ch.M);
    free(ch.w);
    return rt;
}

/* ------------------------------------------------------------------------------------ */
/* BASELINE config C4 (no reference counterpart): the logistic bridge by Polya-Gamma      */
/* latents, oracle/gibbs.py logit_sweep / bridge_regression_logit compiled:               */
/*   tau | beta (BridgeRegression.cpp:453-465), lambda | beta, tau (:506-510),            */
/*   omega_i ~ PG(1, x_i'beta) (bbo_pg1), beta | omega, lambda, tau by the reference's    */
/*   sample_beta_stable map (:552-575) with sig2 = 1, X'X -> X'Omega X (dsyrk of          */
/*   diag(sqrt omega) X) and X'y -> X'(y - 1/2).                                          */
/* beta0 = 0, the pre-burn tau draw at t = 0, burn + 1 sweeps in slot 0, MCMC sweep i at   */
/* t = burn + 1 + i.  Returns the post-burn seconds, or < 0 on failure (-1 allocation,    */
/* -2 a PG draw failed, -(1 + info) LAPACK).                                              */
/* ------------------------------------------------------------------------------------ */
long bbo_pg_batch(double *omega, const double *psi, long n, const uint64_t key[2], uint64_t t);
double bbo_pg1(double psi, const uint64_t key[2], uint64_t t, uint64_t i, int *fail);

double bbc_logit_chain(const double *X, const double *y, int n, int p, double alpha,
                       double nu_shape, double nu_rate, int burn, int M, uint64_t seed,
                       uint64_t stream, int threads, double *beta_out, double *tau_out)
{
    if (threads < 1) threads = 1;
    scipy_openblas_set_num_threads(threads);
    omp_set_num_threads(threads);
    Chain ch = {0};
    ch.n = n;
    ch.p = p;
    ch.method = 0;
    ch.X = X;
    ch.y = y;
    ch.alpha = alpha;
    ch.nu_shape = nu_shape;
    ch.nu_rate = nu_rate;
    ch.key[0] = seed;
    ch.key[1] = stream;
    const size_t pp = (size_t)p * p, np_ = (size_t)n * p;
    double *beta = calloc(p, sizeof(double)), *lam = calloc(p, sizeof(double));
    double *psi = calloc(n, sizeof(double)), *om = calloc(n, sizeof(double));
    double *kap = calloc(n, sizeof(double)), *Yw = malloc(sizeof(double) * np_);
    ch.c = calloc(p, sizeof(double));
    ch.z = calloc(p, sizeof(double));
    ch.G = malloc(sizeof(double) * pp);
    ch.A = malloc(sizeof(double) * pp);
    double rt = -1.0;
    long fails = 0;
    int info = 0;
    if (!beta || !lam || !psi || !om || !kap || !Yw || !ch.c || !ch.z || !ch.G || !ch.A)
        goto done;
    for (int i = 0; i < n; ++i) kap[i] = y[i] - 0.5;
    gemv('T', n, p, 1.0, X, kap, 0.0, ch.c); /* X'(y - 1/2) */
    double tau = draw_tau(&ch, beta, 0);
    double t0 = 0.0;
    for (int s = -1 - burn; s < M && !info && !fails; ++s) {
        /* s < 0: burn-in sweep (slot 0, t = burn + 2 + s); s = 0 starts the clock; s >= 1: MCMC */
        if (s == 0) {
            if (beta_out) memcpy(beta_out, beta, sizeof(double) * p);
            if (tau_out) tau_out[0] = tau;
            t0 = now_s();
            continue;
        }
        const uint64_t t = s < 0 ? (uint64_t)(burn + 2 + s) : (uint64_t)burn + 1 + (uint64_t)s;
        tau = draw_tau(&ch, beta, t);
        draw_lambda(lam, beta, p, alpha, tau, ch.key, t);
        gemv('N', n, p, 1.0, X, beta, 0.0, psi); /* x_i'beta */
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : fails)
        for (long i = 0; i < n; ++i) {
            int f = 0;
            om[i] = bbo_pg1(psi[i], ch.key, t, (uint64_t)i, &f);
            fails += f;
        }
#pragma omp parallel for schedule(static)
        for (long j = 0; j < p; ++j) { /* Yw = diag(sqrt omega) X */
            const double *xs = X + (size_t)j * n;
            double *ys = Yw + (size_t)j * n;
            for (int i = 0; i < n; ++i) ys[i] = xs[i] * sqrt(om[i]);
        }
        const double one = 1.0, zero = 0.0;
        scipy_dsyrk_("U", "T", &p, &n, &one, Yw, &n, &zero, ch.G, &p, 1, 1); /* X'Omega X */
        info = beta_chol(&ch, lam, 1.0, tau, t, beta);
        if (s >= 1) {
            if (beta_out) memcpy(beta_out + (size_t)s * p, beta, sizeof(double) * p);
            if (tau_out) tau_out[s] = tau;
        }
    }
    rt = fails ? -2.0 : info ? -(1.0 + info) : now_s() - t0;
done:
    free(beta);
    free(lam);
    free(psi);
    free(om);
    free(kap);
    free(Yw);
    free(ch.c);
    free(ch.z);
    free(ch.G);
    free(ch.A);
    return rt;
}

/* ------------------------------------------------------------------------------------ */
/* BASELINE config C5 (no reference counterpart): the stable chain on a sparse CSC design */
/* (p > n), the exact Woodbury form of BridgeRegression.cpp:552-575 as beta_woodbury above */
/* with the three passes over X done sparse: X beta and X u by CSR rows, X'w by CSC       */
/* columns, and the n x n Gram X diag(D) X' by output column (CSR row c x the CSC columns  */
/* it touches, OpenMP over columns), then dpotrf.  Driver as bbc_stable_chain (beta0 = 0, */
/* pre-burn tau, burn + 1 sweeps in slot 0).  Returns post-burn seconds or < 0.           */
/* ------------------------------------------------------------------------------------ */
double bbc_sparse_chain(const int *colptr, const int *rowidx, const double *val, const double *y,
                        int n, int p, double alpha, double nu_shape, double nu_rate,
                        double sig2_shape, double sig2_scale, int burn, int M, uint64_t seed,
                        uint64_t stream, int threads, double *beta_out, double *tau_out,
                        double *sig2_out)
{
    if (threads < 1) threads = 1;
    scipy_openblas_set_num_threads(threads);
    omp_set_num_threads(threads);
    Chain ch = {0};
    ch.n = n;
    ch.p = p;
    ch.alpha = alpha;
    ch.nu_shape = nu_shape;
    ch.nu_rate = nu_rate;
    ch.sig2_shape = sig2_shape;
    ch.sig2_scale = sig2_scale;
    ch.key[0] = seed;
    ch.key[1] = stream;
    const long nnz = colptr[p];
    const size_t nn = (size_t)n * n;
    int *rowptr = calloc((size_t)n + 1, sizeof(int)), *colidx = malloc(sizeof(int) * (nnz + 1));
    double *rval = malloc(sizeof(double) * (nnz + 1));
    double *beta = calloc(p, sizeof(double)), *lam = calloc(p, sizeof(double));
    double *D = calloc(p, sizeof(double)), *u = calloc(p, sizeof(double));
    double *z = calloc(p, sizeof(double)), *xtw = calloc(p, sizeof(double));
    double *r = calloc(n, sizeof(double)), *v = calloc(n, sizeof(double));
    double *d = calloc(n, sizeof(double)), *w = calloc(n, sizeof(double));
    double *Mm = malloc(sizeof(double) * nn);
    double rt = -1.0;
    int info = 0;
    if (!rowptr || !colidx || !rval || !beta || !lam || !D || !u || !z || !xtw || !r || !v ||
        !d || !w || !Mm)
        goto done;
    /* CSR copy (entries of a row in column order) */
    for (long q = 0; q < nnz; ++q) ++rowptr[rowidx[q] + 1];
    for (int i = 0; i < n; ++i) rowptr[i + 1] += rowptr[i];
    {
        int *next = malloc(sizeof(int) * (size_t)n);
        if (!next) goto done;
        memcpy(next, rowptr, sizeof(int) * (size_t)n);
        for (int j = 0; j < p; ++j)
            for (int q = colptr[j]; q < colptr[j + 1]; ++q) {
                const int k = next[rowidx[q]]++;
                colidx[k] = j;
                rval[k] = val[q];
            }
        free(next);
    }
    double tau = draw_tau(&ch, beta, 0), sig2 = 0.0;
    double t0 = 0.0;
    for (int s = -1 - burn; s < M && !info; ++s) {
        if (s == 0) {
            if (beta_out) memcpy(beta_out, beta, sizeof(double) * p);
            if (tau_out) tau_out[0] = tau;
            if (sig2_out) sig2_out[0] = sig2;
            t0 = now_s();
            continue;
        }
        const uint64_t t = s < 0 ? (uint64_t)(burn + 2 + s) : (uint64_t)burn + 1 + (uint64_t)s;
        tau = draw_tau(&ch, beta, t);
        double rss = 0.0; /* r = y - X beta by CSR rows */
#pragma omp parallel for schedule(static) reduction(+ : rss)
        for (int i = 0; i < n; ++i) {
            double a = 0.0;
            for (int k = rowptr[i]; k < rowptr[i + 1]; ++k) a += rval[k] * beta[colidx[k]];
            const double ri = y[i] - a;
            rss += ri * ri;
        }
        sig2 = bbo_sig2_from_rss(rss, n, sig2_shape, sig2_scale, ch.key, t);
        draw_lambda(lam, beta, p, alpha, tau, ch.key, t);
        /* beta | rest, Woodbury: u = sqrt(D) z, v = X u / sig + delta, M = I + X D X' / sig2 */
        const double sig = sqrt(sig2);
        bbo_normals(z, p, ch.key, t, KIND_BETA_Z, 0);
        bbo_normals(d, n, ch.key, t, KIND_DELTA, 0);
#pragma omp parallel for schedule(static)
        for (long j = 0; j < p; ++j) {
            D[j] = tau * tau / lam[j];
            u[j] = sqrt(D[j]) * z[j];
        }
#pragma omp parallel for schedule(static)
        for (int i = 0; i < n; ++i) {
            double a = 0.0;
            for (int k = rowptr[i]; k < rowptr[i + 1]; ++k) a += rval[k] * u[colidx[k]];
            v[i] = a / sig + d[i];
        }
        /* upper triangle, column c: M[r][c] = sum_j X_rj X_cj D_j / sig2 over j in row c */
#pragma omp parallel for schedule(dynamic, 16)
        for (int c = 0; c < n; ++c) {
            double *mc = Mm + (size_t)c * n;
            memset(mc, 0, sizeof(double) * (size_t)(c + 1));
            for (int k = rowptr[c]; k < rowptr[c + 1]; ++k) {
                const int j = colidx[k];
                const double f = rval[k] * D[j];
                for (int q = colptr[j]; q < colptr[j + 1] && rowidx[q] <= c; ++q)
                    mc[rowidx[q]] += val[q] * f;
            }
            for (int rr = 0; rr <= c; ++rr) mc[rr] /= sig2;
            mc[c] += 1.0;
        }
        scipy_dpotrf_("U", &n, Mm, &n, &info, 1);
        if (info) break;
        for (int i = 0; i < n; ++i) w[i] = y[i] / sig - v[i];
        trsv_u('T', n, Mm, w);
        trsv_u('N', n, Mm, w);
#pragma omp parallel for schedule(static)
        for (long j = 0; j < p; ++j) { /* X'w by CSC columns, beta = u + D X'w / sig */
            double a = 0.0;
            for (int q = colptr[j]; q < colptr[j + 1]; ++q) a += val[q] * w[rowidx[q]];
            xtw[j] = a;
            beta[j] = u[j] + D[j] * a / sig;
        }
        if (s >= 1) {
            if (beta_out) memcpy(beta_out + (size_t)s * p, beta, sizeof(double) * p);
            if (tau_out) tau_out[s] = tau;
            if (sig2_out) sig2_out[s] = sig2;
        }
    }
    rt = info ? -(1.0 + info) : now_s() - t0;
done:
    free(rowptr);
    free(colidx);
    free(rval);
    free(beta);
    free(lam);
    free(D);
    free(u);
    free(z);
    free(xtw);
    free(r);
    free(v);
    free(d);
    free(w);
    free(Mm);
    return rt;
}
