// bb_kernels.h -- host-side launch wrappers for the gfx950 kernels of the stable sweep.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <cmath>

namespace bb {

struct Key;

// Chain scalars kept on the device (read by kernels, written by the scalar draws).
struct DevScalars {
    double tau, sig2, alpha;
    double s_abs_pow;  // last sum |beta|^alpha (diagnostic)
    double rss;        // last residual sum of squares (diagnostic)
    double pad[3];
};

// Hyper-parameters of bridge.reg.stb (BridgeWrapper.R:194-201).
struct Hyper {
    double sig2_shape, sig2_scale, nu_shape, nu_rate, alpha_a, alpha_b;
    int know_tau, know_sig2, know_alpha;
};

constexpr int kGramTile = 128;  // Gram output tile (rows of X per tile)
constexpr int kGramBK = 16;     // Gram K step
constexpr int kNB = 64;         // Cholesky block
constexpr int kXvCols = 256;    // columns per block of the X.v partial-sum kernel (at most)
constexpr int kXvMinCols = 32;  // ... and at least (small grids split the columns finer)
constexpr int kXvRows = 512;    // rows per block of the X.v partial-sum kernel
constexpr int kTriMaxP = 2048;  // triangle-mixture sampler: coefficients in one workgroup

// Packed upper triangle, column-major: element (r, c), r <= c, at c (c + 1) / 2 + r.  The
// Woodbury Gram travels in this form (red2), so its all-reduce moves n(n+1)/2 doubles.
__host__ __device__ inline size_t tri_index(int r, int c) { return (size_t)c * (c + 1) / 2 + r; }
__host__ __device__ inline size_t tri_count(int n) { return (size_t)n * (n + 1) / 2; }

enum LambdaMode { LAMBDA_ONLY = 0, LAMBDA_WOODBURY = 1 };

// Per-sweep choice between the two exact solves of the Woodbury system (bb_nid.hip, DESIGN.md
// s6.5): mode 0 = Gram + Cholesky, mode K > 0 = Chebyshev iteration with K iterates on the
// certified spectrum interval [1, 1 + eps].  Written on the device every sweep by
// k_nid_reduce (k_nid_decide_from for shards); the kernels of the path not taken return at
// once.
// k2 > 0: the mixed-precision plan of an unsharded dense engine: mode = K1
// iterates on M~ = I + X~ D X~' / sig2 (X~ = X rounded to fp32), one fp64 residual pass, then
// k2 iterates on M~ from that residual; theta / delta / sigma1 are then those of [1, 1 + eps +
// eta], eta >= |E - E~| certified.
struct NidState {
    double eps, theta, delta, sigma1;
    int mode, k2;
    unsigned long long n_cheb, n_products, n_chol;  // sweeps per path, fp64 E-apply passes run
    double lambda_x;  // certified upper bound on lambda_max(X X') (0: none; setup)
    double eta;       // the mixed plan's certified |E - E~| (0 on an fp64 sweep)
    unsigned long long n_mixed, n_products32;  // mixed-plan sweeps, fp32 E-apply passes run
    // the plans' cost model (s, set at setup from the shape): an fp64 / fp32 pass over X and
    // the per-iterate step launch
    double c64, c32, cstep;
};
constexpr double kNidTol = 1.3877787807814457e-17;  // 2^-56: bound on the relative error

// Chebyshev scalars of the interval [1, 1 + eps]
struct ChebConst {
    double theta, delta, sigma1;
};
__host__ __device__ inline ChebConst cheb_const(double eps) {
    ChebConst c;
    c.theta = 1.0 + 0.5 * eps;
    c.delta = 0.5 * eps;
    c.sigma1 = c.delta > 0.0 ? c.theta / c.delta : 0.0;
    return c;
}
// smallest K (1 <= K <= kmax) with sqrt(1 + eps) / T_K(sigma1) <= tol, else 0 (the bound on
// |w - x_K| / |w| of K Chebyshev iterates from x_0 = 0 on the spectrum interval [1, 1 + eps])
__host__ __device__ inline int cheb_iterations(double eps, int kmax, double tol) {
    if (!(eps >= 0.0) || !(eps < 1e300)) return 0;
    if (eps == 0.0) return kmax >= 1 ? 1 : 0;  // E = 0: x_1 = r / theta = r exactly
    const ChebConst c = cheb_const(eps);
    const double lim = sqrt(1.0 + eps) / tol;
    double tm1 = 1.0, tk = c.sigma1;  // T_0, T_1
    for (int k = 1; k <= kmax; ++k) {
        if (tk >= lim) return k;
        const double tn = 2.0 * c.sigma1 * tk - tm1;
        tm1 = tk;
        tk = tn;
    }
    return 0;
}

// a kernel of the Gram + Cholesky path: skip it when the sweep took the Chebyshev path
__device__ __forceinline__ bool gated(const int *gate) { return gate && *gate != 0; }

// The kernel instance most recently launched (this process) per roofline family: bench.py
// matches the committed PMC summaries by this exact instance (bb_kernel_instance)
enum KernelFamily { KF_LAMBDA, KF_GRAM, KF_REDUCE, KF_CHOL, KF_SOLVE, KF_BETA, KF_EAPPLY, KF_COUNT };
void note_launch(KernelFamily f, const void *kernel);
const void *launched_instance(int f);

int eapply_parts(int p_loc, int n_pad);  // E-apply partial n-vectors (one per workgroup)
bool eapply_supported(int n_pad);        // dense E-apply register tiling covers n_pad
// the decision's bound sums (bb_nid.hip): G = nid_sum_groups(p_loc) workgroup partials
// (wg_part, G x (kNidTS + 1)) reduced in order into red (kNidTS + 2: [S_k | trace | Lambda]);
// decide != 0: the unsharded decision at once (eps into the host-mapped eps_host); a shard
// exchanges red, then launch_nid_decide_from (host2 = host-mapped [eps, mode, k2, tag]; tag_seq
// != 0: the tag word (seq << 16 | mode << 8 | k2) the host polls for the decision)
constexpr int kNidTS = 32;
int nid_sum_groups(int p_loc);
void launch_nid_sums(hipStream_t s, const double *D, const double *cn, int p_loc,
                     const DevScalars *sc, NidState *nid, int k_launched, int allow, int decide,
                     double *wg_part, double *red, double *eps_host);
// unsharded, synchronous protocol: the sums and the decision, [eps, mode] into host2
// allow_mixed: the engine holds an fp32 copy of X and may take the mixed-precision plan
// (host2[2] = its k2, 0 for the fp64 plan)
void launch_nid_sums_decide(hipStream_t s, const double *D, const double *cn, int p_loc,
                            const DevScalars *sc, NidState *nid, int k_launched,
                            double *wg_part, double *red, double *host2, int allow_mixed = 0,
                            unsigned long long tag_seq = 0);
// the reduction of G partials the split lambda launch wrote (a shard: alone; host2 given:
// and the unsharded decision, as launch_nid_sums_decide)
void launch_nid_reduce(hipStream_t s, const double *wg_part, int G, const DevScalars *sc,
                       NidState *nid, double *red, int k_launched = 0, double *host2 = nullptr,
                       int allow_mixed = 0, unsigned long long tag_seq = 0);
// The bound sums folded into the split lambda launch's stream role (wg_part: one kNidTS + 1
// partial per stream workgroup); decide: the last stream workgroup (cnt, zeroed, re-armed by
// it) reduces them into red and makes the unsharded decision (launch_nid_sums_decide's)
struct NidFold {
    const double *cn = nullptr;
    double *wg_part = nullptr;
    unsigned int *cnt = nullptr;
    int decide = 0, k_launched = 0, allow_mixed = 0;
    NidState *nid = nullptr;
    double *red = nullptr, *host2 = nullptr;
    unsigned long long tag_seq = 0;
};
void launch_nid_decide_from(hipStream_t s, const double *red, const DevScalars *sc,
                            int k_launched, NidState *nid, double *host2,
                            unsigned long long tag_seq = 0);
void launch_nid_xu(hipStream_t s, const double *X, int ldx, const double *u, int ncols,
                   int n_pad, const NidState *nid, double *part);
// b (optional): the right-hand side, kept for the mixed plan's residual pass
void launch_cheb_init(hipStream_t s, const double *xu_part, int nparts, int n, int n_pad,
                      const double *y, const DevScalars *sc, uint64_t k0, uint64_t k1,
                      uint64_t t, const NidState *nid, double *x, double *r, double *d,
                      double *b = nullptr);
// phase 1: step j of the first solve (runs if mode > j); phase 2: step j of the mixed plan's
// correction solve (runs if k2 > j)
void launch_cheb_step(hipStream_t s, const double *part, int nparts, int n_pad,
                      const DevScalars *sc, const NidState *nid, int j, double *x, double *r,
                      double *d, int phase = 1);
// the mixed plan's restart: r = b - x - (E x) / sig2 from the fp64 residual pass's partials,
// d = r / theta, x += d (runs if k2 > 0 and mode > 0)
void launch_cheb_restart(hipStream_t s, const double *part, int nparts, int n_pad,
                         const DevScalars *sc, const NidState *nid, const double *b, double *x,
                         double *r, double *d);
// One pass over X: part = X D X' v partials.  kind 0: product j of the first solve (runs if
// mode > j; streams X32 when the sweep took the mixed plan and X32 is given); 2: the mixed
// plan's fp64 residual pass (v = the iterate; runs if k2 > 0 and mode > 0); 3: product j of
// the correction solve (X32; runs if k2 > j)
void launch_eapply(hipStream_t s, const double *X, int ldx, int n_pad, int p_loc,
                   const double *D, const double *v, const NidState *nid, int j, double *part,
                   const float *X32 = nullptr, int kind = 0);
// X32 = X rounded to fp32 (n_pad x ncols, ld ldx); *bad = 1 if an entry is outside the range
// where the rounding error is <= 2^-24 |x| (|x| > 2^126 or 0 < |x| < 2^-125)
void launch_cast_f32(hipStream_t s, const double *X, int ldx, int n_pad, int ncols, float *X32,
                     int *bad);
constexpr double kU32 = 5.9604644775390625e-08;  // 2^-24: fp32 unit roundoff
void launch_sp_eapply(hipStream_t s, const int *colptr, const int *rowidx, const double *cval,
                      const int *rowptr, const int *colidx, const double *rval, int p_loc,
                      int n_pad, const double *D, const double *v, const NidState *nid, int j,
                      double *scratch_p, double *out);
void launch_part_sum(hipStream_t s, const double *part, int nparts, int n_pad, double *out);
void launch_shift_gram(hipStream_t s, const double *red2, int n_pad, double U, double *M,
                       int ldm);
void launch_sp_nid_xu(hipStream_t s, const int *rowptr, const int *colidx, const double *rval,
                      int n_pad, const double *u, const NidState *nid, double *out);

// Number of lanes cooperating on one tilted-stable draw for a problem of `count` draws.
int stable_group_for(long count);
bool stable_noinline_for(long count);

void launch_retstable_batch(hipStream_t s, double *x, const double *alpha, const double *V0,
                            const double *h, int num, uint64_t k0, uint64_t k1, uint64_t t,
                            int group, uint32_t *err);

// lambda (LAMBDA_ONLY) and omega ~ PG(1, psi) in one launch when p_loc takes the
// speculative lambda kernel; false (nothing launched) otherwise
bool launch_lambda_pg(hipStream_t s, const double *beta, int p_loc, int p_pad, uint64_t j0,
                      const DevScalars *sc, uint64_t k0, uint64_t k1, uint64_t t, int group,
                      double *lam, double *lam_trace, const double *psi, int n, int n_pad,
                      double *omega, uint32_t *err);
void launch_lambda(hipStream_t s, const double *beta, int p_loc, int p_pad, uint64_t j0,
                   const DevScalars *sc, uint64_t k0, uint64_t k1, uint64_t t, int mode,
                   int group, double *lam, double *D, double *u, double *lam_trace,
                   uint32_t *err);

// lambda (LAMBDA_WOODBURY) fused with the X u pass (dense, bb_kernels.hip k_lambda_xu):
// returns the partial n-vectors written to xu_part (xu_part holds lambda_xu_parts of them),
// 0 when the shape does not take the fused launch (nothing launched)
int lambda_xu_parts(int p_loc, int p_pad, int n_pad);
int launch_lambda_xu(hipStream_t s, const double *beta, int p_loc, int p_pad, uint64_t j0,
                     const DevScalars *sc, uint64_t k0, uint64_t k1, uint64_t t, double *lam,
                     double *D, double *u, double *lam_trace, uint32_t *err, const double *X,
                     int ldx, int n_pad, double *xu_part, unsigned int *sync = nullptr,
                     unsigned int ep = 0, const NidFold *fold = nullptr, int *folded = nullptr);
// the split launch (key 7 = 3; bb_nid.hip): ndraw drawing and nstream streaming workgroups;
// returns 0, or 1 / 2 when the bound sums were folded in (2: and the unsharded decision made)
int launch_lambda_xs(hipStream_t s, const double *beta, int p_loc, int p_pad, uint64_t j0,
                     const DevScalars *sc, uint64_t k0, uint64_t k1, uint64_t t, double *lam,
                     double *D, double *u, double *lam_trace, uint32_t *err, const double *X,
                     int ldx, int n_pad, int nchunk, double *xu_part, unsigned int *sync,
                     unsigned int ep, int ndraw, int nstream, const NidFold *fold);
int lambda_xs_resident(int nr);  // k_lambda_xs workgroups resident per CU
// words of the split launch's (key 7 mode 3) synchronisation buffer, zeroed before first use
int lambda_xs_sync_words(int p_pad);
extern int g_lam_xu;
extern int g_lam_wave;  // wave-adaptive draw in the fused lambda + X u launch (key 13)
extern int g_lam_lend;  // the continuous-batching launch lends its tail lanes (key 15)

void launch_lambda_variant(hipStream_t s, const double *beta, int p, const DevScalars *sc,
                           uint64_t k0, uint64_t k1, uint64_t t, int group, int noinline,
                           double *lam, uint32_t *err);

// slabs[s] (ld = ldo) gets the upper triangle (column-major) of Y diag(w) Y' over
// K-range s; Y is n_pad x K column-major with ld = ldy (n_pad multiple of 128).
int gram_splits_for(int n_pad, int K);
void launch_gram(hipStream_t s, const double *Y, int ldy, const double *w, int n_pad, int K,
                 int S, double *slabs, int ldo, size_t slab_stride, const int *gate = nullptr);

// part[cb * n_pad + r] = sum over columns j of chunk cb of X[r, j] * v[j].
int xv_chunks(int ncols, int n_pad);  // X.v partials launch_xv writes (= k_pre's nparts)
int xv_chunks_max(int ncols);         // upper bound over n_pad, for allocation
void launch_xv(hipStream_t s, const double *X, int ldx, const double *v, int ncols, int n_pad,
               double *part, const int *gate = nullptr);

// red1 = [S_alpha partials (nbS) | sum_q part[q] (n_pad)].
int pre_blocks_s(int p_loc);
void launch_pre(hipStream_t s, const double *part, int nparts, int n_pad, const double *beta,
                int p_loc, const DevScalars *sc, double *red1, int nbS);

// tau / sig2 draws from red1 (tau_only: initial draw at t = 0).
void launch_scalars(hipStream_t s, const double *red1, int nbS, const double *y, int n,
                    int p, DevScalars *sc, Hyper hy, uint64_t k0, uint64_t k1, uint64_t t,
                    double *tau_tr, double *sig2_tr, double *alpha_tr, int tau_only,
                    uint32_t *err);

// red2 = [sum_s slabs, upper triangle | sum_q xu_part (n_pad)]; packed = 1: the triangle is
// packed (tri_index, the Woodbury red2), 0: full column-major n_pad^2 (lower part zero).
void launch_slab_sum(hipStream_t s, const double *slabs, int S, size_t slab_stride, int n_pad,
                     const double *xu_part, int nxu, double *red2, int packed, const int *gate = nullptr);

// M (upper, ld = ldm) = I + red2 / sig2; column rhs_col = y/sig - (xu/sig + delta).
void launch_form_m(hipStream_t s, const double *red2, int n, int n_pad, const double *y,
                   const DevScalars *sc, uint64_t k0, uint64_t k1, uint64_t t, double *M,
                   int ldm, int rhs_col, const int *gate = nullptr);

// A (upper) = G + diag(lambda sig2 / tau^2) (or G alone if lam == nullptr); column
// rhs_col = c.  Padding: identity.
// Bridge EM maximisation system over the p_pad index space (mask 0 / padding coordinates
// become identity rows with a zero right-hand side); dlam = c2 lam per coordinate or null.
void launch_em_form(hipStream_t s, const double *G, int ldg, const double *dlam, const int *mask,
                    const double *b, int p, int p_pad, double *A, int lda, int rhs_col);
// Conjugate gradients on that system from x (in/out); work: 3 n doubles; *out_it = iterations.
void launch_em_cg(hipStream_t s, const double *A, int lda, int n, const double *b, double *x,
                  double tol, int max_it, double *work, int *out_it);
// Batched bridge EM (direct solves) for p <= 128: one workgroup per ratio (a thread per row), the EM
// loop entirely on the device.  beta_out: count x p; solves_out: count (-1: not PD).
void launch_em_batch(hipStream_t s, const double *G, int ldg, const double *b, int p,
                     const double *ratios, const double *lambda_max, int count, double alpha,
                     double tol, int max_iter, double *beta_out, int *solves_out);
// The same EM for any p: a workgroup per ratio r0 .. r0 + count - 1, each with a p_pad x
// p_pad system in scratch (count slices; p_pad a multiple of em_tile()), vecs: 3 p_pad
// doubles and masks: p_pad ints per workgroup.  Tiled Cholesky over LDS tiles.
void launch_em_batch_tiled(hipStream_t s, const double *G, int ldg, const double *b, int p,
                           int p_pad, const double *ratios, const double *lambda_max, int r0,
                           int count, double alpha, double tol, int max_iter, double *scratch,
                           double *vecs, int *masks, double *beta_out, int *solves_out);
int em_tile();
// packed != 0: G is the packed upper triangle (tri_index, as k_oz_crt writes it)
void launch_form_a(hipStream_t s, const double *G, int ldg, const double *lam,
                   const DevScalars *sc, const double *c, int p, int p_pad, double *A, int lda,
                   int rhs_col, int packed = 0);

// In-place upper Cholesky A = U'U of the leading m_pad x m_pad block with the
// forward solve U'^-1 folded into the nrhs_blocks column blocks that follow (one persistent
// launch, k_chol_persistent).  Wd: m_pad/kNB blocks of kNB x kNB receiving U_kk^-T (used by
// chol_bsolve).  flags: chol_flag_words(m_pad, nrhs_blocks) unsigned ints of scratch (set-once
// flags tagged with a per-buffer epoch; zeroed only when first seen).  trace: optional
// timestamps (bb_bench_chol).
size_t chol_flag_words(int m_pad, int nrhs_blocks);
extern int g_bsolve_ll;  // the persistent backward solve's tagged-word hand-off (key 20)
// doubles of the Wd buffer chol_factor needs (W_k blocks + scratch tiles)
size_t chol_wd_words(int m_pad);
extern int g_bxb_nt;  // non-temporal X loads in k_beta_wb_xb (bb_set_tuning key 2)
extern int g_rs_xcd;  // XCD-aware row blocks of the partial row sums (key 12)
extern int g_nid_force_k;  // forced Chebyshev iterate count, 0 = certified (key 16)
void nid_set_force_k(int k);
extern int g_lam_occ;  // lambda launches at 4 waves per SIMD (bb_set_tuning key 4)
extern int g_lam_lanes;  // lanes per coefficient of k_lambda_spec, 0 = default (key 5)
// k_chol_persistent chain variant: 1 (default) or the pipelined 2 / 3, for A/B
extern int g_chol_version;
void chol_factor(hipStream_t s, double *A, int lda, int m_pad, int nrhs_blocks, uint32_t *err,
                 double *Wd, unsigned int *flags, unsigned long long *trace = nullptr, const int *gate = nullptr);


// Backward solve U W = Y (Y, W: m_pad x nrhs <= 2, ld = m_pad); Y may be overwritten.
// With the flag buffer of the factorisation just run (chol_factor with nrhs_blocks = 1) and
// an error word: one persistent launch; otherwise (or beyond one workgroup per CU) one
// launch per kBsNB blocks.
void chol_bsolve(hipStream_t s, const double *A, int lda, int m_pad, const double *Wd,
                 double *Y, double *W, int nrhs, unsigned int *flags = nullptr,
                 uint32_t *err = nullptr, const int *gate = nullptr);

// beta_j = u_j + D_j (X_j . w) / sig (Woodbury update); writes beta and trace.
void launch_beta_woodbury(hipStream_t s, const double *X, int ldx, int n_pad, const double *w,
                          const double *u, const double *D, const DevScalars *sc, int p_loc,
                          double *beta, double *beta_trace);

// Fused variant for n_pad <= 2048: also writes the X beta partials part[g * n_pad + r]
// (g < beta_xb_parts(p_loc)) that k_pre sums, so no separate X beta pass is needed.
int beta_xb_parts(int p_loc);
bool beta_xb_supported(int n_pad);
void launch_beta_woodbury_xb(hipStream_t s, const double *X, int ldx, int n_pad, const double *w,
                             const double *u, const double *D, const DevScalars *sc, int p_loc,
                             double *beta, double *beta_trace, double *part);

// Build the 2-RHS backward-solve input [U'^-1 c | z] (chol path).
void launch_chol_rhs(hipStream_t s, const double *A, int lda, int rhs_col, int p, int p_pad,
                     uint64_t k0, uint64_t k1, uint64_t t, double *Y2);

// beta = m + sqrt(sig2) x (chol path) from W2 = [m | x].
void launch_beta_chol(hipStream_t s, const double *W2, int p_pad, const DevScalars *sc, int p,
                      double *beta, double *beta_trace);

// Orthogonal design: beta_i ~ N(c_i/u_i, sig2/u_i), u_i = G_ii + lambda_i sig2/tau^2.
void launch_beta_ortho(hipStream_t s, const double *gdiag, const double *c, const double *lam,
                       const DevScalars *sc, int p, uint64_t j0, uint64_t k0, uint64_t k1,
                       uint64_t t, double *beta, double *beta_trace);

// alpha | beta, tau random-walk MH (world == 1).
void launch_alpha_mh(hipStream_t s, const double *beta, int p, DevScalars *sc, double pr_a,
                     double pr_b, uint64_t k0, uint64_t k1, uint64_t t, double *alpha_tr);
// the alpha MH step of a column-sharded chain: per-shard sums, then (after the exchange of
// the two sums) the decision with the global p
void launch_alpha_sums(hipStream_t s, const double *beta, int p_loc, const DevScalars *sc,
                       uint64_t k0, uint64_t k1, uint64_t t, double *sums);
void launch_alpha_decide(hipStream_t s, const double *sums, int p, DevScalars *sc, double pr_a,
                         double pr_b, uint64_t k0, uint64_t k1, uint64_t t, double *alpha_tr);

// Triangle-mixture update (bb_tri.hip): omega, u and the rtnorm_gibbs beta passes of one
// sweep of bridge.reg.tri, given sc->tau, sig2, alpha; ortho != 0: the orthogonal-design
// variant's coordinate Gibbs on beta (full Gram Gf, c = X'y).  p <= kTriMaxP.  err bits: 64 a
// truncated draw exhausted its attempts, 128 an empty truncation interval.
void launch_tri_update(hipStream_t s, double *beta, double *u, double *omega, double *shape,
                       int p, const double *tVc, const double *tVr, const double *a,
                       const double *d, const double *Gf, const double *c, int ortho,
                       const DevScalars *sc, int betaburn, uint64_t k0, uint64_t k1, uint64_t t,
                       double *tr_beta, double *tr_u, double *tr_omega, double *tr_shape,
                       uint32_t *err);

// Truncated normal / exponential batches (bb_tri.hip) for the .C utilities: mode 0
// rtnorm_left(l, mu, sig), 1 rtnorm_both(l, r, mu, sig), 2 rtnorm(l, r, mu, sig), 3
// rtexpon_rate_left(l, rate), 4 rtexpon_rate_both(l, r, rate), 5 rtexpon_rate(l, r, rate).
// err bits: 64 rejection cap, 128 empty interval, 256 non-finite rtexpon_rate input.
void launch_trunc_batch(hipStream_t s, int mode, int num, double *x, const double *p0,
                        const double *p1, const double *p2, const double *p3, uint64_t k0,
                        uint64_t k1, uint32_t *err);

// Right-truncated gamma batch (rrtgamma_rate): x_i ~ Ga(shape_i, rate_i) on (0, right_t_i].
void launch_rrtgamma_batch(hipStream_t s, int num, double *x, const double *shape,
                           const double *rate, const double *right_t, uint64_t k0, uint64_t k1,
                           uint32_t *err);

// Logistic bridge (bb_logit.hip): omega_i ~ PG(1, psi_i) for i < n (0 on padding rows),
// err bit 32 when a draw exhausted its attempts; kappa = y - 1/2.
void launch_pg(hipStream_t s, const double *psi, int n, int n_pad, uint64_t k0, uint64_t k1,
               uint64_t t, double *omega, uint32_t *err);
void launch_kappa(hipStream_t s, const double *y, int n, int n_pad, double *kappa);

// Small-p fused chain (bb_small.hip): `count` whole sweeps (tau, sig2, lambda, beta by the
// p x p Cholesky draw, or the orthogonal-design draw) in ONE single-workgroup launch, for
// p <= kSmallChainMaxP and alpha known.  Sweep k uses counter t0 + k and trace slot
// (first_slot + k slot_step) % cap (first_slot < 0: none).
constexpr int kSmallChainMaxP = 32;
void launch_small_chain(hipStream_t s, const double *X, int ldx, int n, int p, const double *y,
                        const double *G, int ldg, const double *cvec, const double *gdiag,
                        int ortho, double *beta, double *lam, DevScalars *sc, Hyper hy,
                        uint64_t k0, uint64_t k1, uint64_t t0, int count, int first_slot,
                        int slot_step, int cap, double *tr_beta, double *tr_lam, double *tr_sig2,
                        double *tr_tau, double *tr_alpha, uint32_t *err);

// Whole triangle-mixture sweeps (non-orthogonal design, alpha known, p <= kTriChainMaxP) in
// one single-workgroup launch (bb_tri.hip k_tri_chain): S_alpha / rss, tau and sig2, then
// omega, u and the rtnorm_gibbs passes of launch_tri_update in one wave, `count` sweeps from
// t0 with the trace-slot convention of launch_small_chain.
constexpr int kTriChainMaxP = 32;
void launch_tri_chain(hipStream_t s, const double *X, int ldx, int n, int p, const double *y,
                      const double *tVc, const double *tVr, const double *a, const double *d,
                      const double *Gf, const double *c, int ortho, double *beta, double *u, double *omega, double *shape, DevScalars *sc,
                      Hyper hy, int betaburn, uint64_t k0, uint64_t k1, uint64_t t0, int count,
                      int first_slot, int slot_step, int cap, double *tr_beta, double *tr_u,
                      double *tr_omega, double *tr_shape, double *tr_sig2, double *tr_tau,
                      double *tr_alpha, uint32_t *err);

// Copy the scalars into trace slots (known parameters / alpha when known).
void launch_record_scalars(hipStream_t s, const DevScalars *sc, double *tau_tr,
                           double *sig2_tr, double *alpha_tr);

// Element-wise helpers.
void launch_copy_cols(hipStream_t s, const double *src, int lds, double *dst, int ldd, int rows,
                      int cols);
void launch_gdiag(hipStream_t s, const double *G, int ldg, int p, double *d);
void launch_sum_into(hipStream_t s, const double *a, double *b, size_t n);
void launch_transpose(hipStream_t s, const double *src, int lds, int rows, int cols, double *dst,
                      int ldd);
void launch_coldot(hipStream_t s, const double *X, int ldx, int n_pad, const double *v, int ncols,
                   double *out);
void launch_colnorm2(hipStream_t s, const double *X, int ldx, int n_pad, int ncols, double *out);

}  // namespace bb
