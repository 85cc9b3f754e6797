/*
 * bayesbridge.h -- C ABI of the MI355X-native BayesBridge drop-in (BayesBridge.so).
 *
 * Part 1: the reference's own .C() entry points for the normal-mixture
 * ("stable") path, with identical names, argument order and meaning, so that
 * the reference R front end (`.C("bridge_reg_stable", ..., PACKAGE="BayesBridge")`,
 * Code/C/BridgeWrapper.R:220-228 and :534) binds them unchanged.
 *
 * Part 2: bb_* extensions (seeding, device engine for benchmarks / multi-GPU,
 * diagnostics).  Plain pointers and sizes only; no torch or HIP types.
 *
 * Error behaviour follows the reference: the .C entry points never throw or
 * return a status; problems are printed and partial traces are returned
 * (Code/C/BridgeWrapper.cpp:300-304).  bb_* functions return 0 on success and
 * a negative code on failure (message via bb_last_error()).
 */
#ifndef BAYESBRIDGE_AMD_H
#define BAYESBRIDGE_AMD_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------ */
/* Part 1: reference .C entry points                                         */
/* ------------------------------------------------------------------------ */

/*
 * Gibbs sampler for Bayesian bridge regression, normal-mixture ("stable")
 * representation.  Replaces Code/C/BridgeWrapper.h:205-226 (declaration) /
 * Code/C/BridgeWrapper.cpp:659-732 (implementation), which drives
 * bridge_regression_stable (:207-313) or bridge_regression_stable_ortho (:434-537).
 *
 * Outputs (caller-allocated, column-major as R passes them):
 *   betap, lambdap : P x M  (sample i at offset i*P)
 *   sig2p, taup, alphap : M
 *   runtime : post-burn-in wall seconds (the reference reports post-burn CPU
 *             seconds from clock())
 * Inputs: yp (N), Xp (N x P column-major), hyper-parameters as in
 * bridge.reg.stb (BridgeWrapper.R:194-234); true_* > 0 fixes that parameter.
 * `ortho` is declared `const bool*` in the reference but R passes
 * as.integer(ortho) (4 bytes); this implementation reads it as an int.
 */
void bridge_reg_stable(double *betap, double *lambdap, double *sig2p, double *taup,
                       double *alphap, const double *yp, const double *Xp,
                       const double *sig2_shape, const double *sig2_scale,
                       const double *nu_shape, const double *nu_rate, const double *alpha_a,
                       const double *alpha_b, const double *true_sig2, const double *true_tau,
                       const double *true_alpha, const int *P, const int *N, const int *M,
                       const int *burn, double *runtime, const int *ortho);

/*
 * Batch exponentially tilted positive alpha-stable draws (Devroye 2009 double
 * rejection): x[i] has Laplace transform exp(-V0[i]((h[i]+t)^alpha[i] - h[i]^alpha[i])).
 * Replaces Code/C/BridgeWrapper.h:244 / BridgeWrapper.cpp:965-984, which loops
 * retstable_LD(h, alpha, RNG&, V0) of Code/C/retstable.cpp:94-271.
 */
void retstable_LD(double *x, double *alpha, double *V0, double *h, int *num);

/*
 * Bridge EM point estimate (sig = 1, tau = ratio): replaces Code/C/BridgeWrapper.cpp:544-568
 * (decl. BridgeWrapper.h:166-176; algorithm BR::EM, BridgeRegression.cpp:600-708), called
 * by bridge.EM (BridgeWrapper.R:89-133) and trace.beta (bridge-trace.R).  betap (P) gets
 * the estimate; max_iter is the iteration cap on entry and the number of solves on return
 * (-1 after an error, which prints "Aborting EM.").  `use_cg` is declared `const bool*`
 * in the reference but R passes as.integer(use.cg); it is read as an int.
 */
void bridge_EM(double *betap, const double *yp, const double *Xp, const double *ratio,
               const double *alpha, const int *P, const int *N, const double *lambda_max,
               const double *tol, int *max_iter, const int *use_cg);

/*
 * Triangle-mixture Gibbs sampler: replaces Code/C/BridgeWrapper.cpp:572-657 (decl.
 * BridgeWrapper.h:178-203; driver :80-204; conditionals BridgeRegression.cpp:97-147,
 * 235-286, 405-465), called by bridge.reg.tri (BridgeWrapper.R:139-186) with 26 args.
 * betap, up, omegap, shapep are P x M column-major traces; sig2p, taup, alphap are M.
 * Requires P <= N and P <= 2048 (the reference's svd(X, 'A') indexing breaks for P > N).
 * `ortho` and `use_hmc` are declared `const bool*` but R passes integers; both are read
 * as ints.  ortho != 0 runs the orthogonal-design triangle driver (bridge_regression_ortho,
 * BridgeWrapper.cpp:320-432).  use_hmc is ignored: the reference forces it false
 * (BridgeRegression.cpp:418).
 */
void bridge_regression(double *betap, double *up, double *omegap, double *shapep,
                       double *sig2p, double *taup, double *alphap, const double *yp,
                       const double *Xp, const double *sig2_shape, const double *sig2_scale,
                       const double *nu_shape, const double *nu_rate, const double *alpha_a,
                       const double *alpha_b, const double *true_sig2, const double *true_tau,
                       const double *true_alpha, const int *P, const int *N, const int *M,
                       const int *burn, double *runtime, const int *ortho,
                       const int *betaburn, const int *use_hmc);

/*
 * Truncated-distribution utilities: replace Code/C/BridgeWrapper.cpp:762-935 (decl.
 * BridgeWrapper.h:230-242), called by rtexp.left / rtexp.both / rtexp and rtnorm.left /
 * rtnorm.both / rtruncated.norm (BridgeWrapper.R:290-474).  x[i] gets one draw per
 * parameter set i; draws run on the device, one lane each.  r.tnorm / r.texpon_rate come
 * from the un-vendored RNG library and are restated.  rtnorm and
 * rtexpon_rate follow the reference's USE_R special-value handling (NaN in, NaN out;
 * rtexpon_rate prints its "caught non finite left value" line to stderr).
 */
void rtnorm_left(double *x, double *left, double *mu, double *sig, int *num);
void rtnorm_both(double *x, double *left, double *right, double *mu, double *sig, int *num);
void rtnorm(double *x, double *left, double *right, double *mu, double *sig, int *num);
void rtexpon_rate_left(double *x, double *left, double *rate, int *num);
void rtexpon_rate_both(double *x, double *left, double *right, double *rate, int *num);
void rtexpon_rate(double *x, double *left, double *right, double *rate, int *num);
/* Right-truncated gamma: replaces BridgeWrapper.cpp:944-962 (decl. BridgeWrapper.h:242),
 * called by rrtgamma (BridgeWrapper.R:482-509); `scale` is the shape (the reference's
 * parameter name).  x[i] ~ Ga(scale[i], rate[i]) restricted to (0, right_t[i]]. */
void rrtgamma_rate(double *x, double *scale, double *rate, double *right_t, int *num);
/* BridgeWrapper.cpp:738-756: R special-value marshalling test (host only). */
void mytest(int *out, double *x);

/*
 * bridge_reg_stable for a sparse design given in compressed-sparse-column form, the
 * layout of R's Matrix::dgCMatrix (X@p = Xcolptr, P + 1 entries; X@i = Xrowidx, 0-based
 * rows strictly increasing within a column; X@x = Xval).  Same outputs, hyper-parameters
 * and semantics as bridge_reg_stable on the dense X (BridgeWrapper.cpp:659-732); there is
 * no reference counterpart (BASELINE config C5).  For P > N (non-ortho) the Woodbury draw
 * runs on the CSC/CSR design with a pair-list sparse Gram; otherwise X is
 * densified and the dense path runs.
 */
void bridge_reg_stable_csc(double *betap, double *lambdap, double *sig2p, double *taup,
                           double *alphap, const double *yp, const int *Xcolptr,
                           const int *Xrowidx, const double *Xval, const double *sig2_shape,
                           const double *sig2_scale, const double *nu_shape,
                           const double *nu_rate, const double *alpha_a, const double *alpha_b,
                           const double *true_sig2, const double *true_tau,
                           const double *true_alpha, const int *P, const int *N, const int *M,
                           const int *burn, double *runtime, const int *ortho);

/*
 * Logistic bridge regression by Polya-Gamma augmentation (BASELINE config C4; no reference
 * counterpart): y_i in {0, 1} ~ Bernoulli(1 / (1 + exp(-x_i'beta))), bridge prior
 * exp(-sum |beta_j / tau|^alpha).  Per sweep: tau | beta and lambda | beta, tau as in
 * bridge_reg_stable (BridgeRegression.cpp:453-465, 506-510), omega_i ~ PG(1, x_i'beta),
 * beta ~ N(A^-1 X'(y - 1/2), A^-1) with A = X'Omega X + diag(lambda / tau^2) (the
 * reference's sample_beta_stable with sig2 = 1).  Layout, trace slots, burn-in and
 * error behaviour as bridge_reg_stable; there is no sig2.  Unknown alpha (true_alpha <= 0)
 * runs the reference's MH step with the (alpha_a, alpha_b) prior.
 */
void bridge_reg_logit(double *betap, double *lambdap, double *taup, double *alphap,
                      const double *yp, const double *Xp, const double *nu_shape,
                      const double *nu_rate, const double *alpha_a, const double *alpha_b,
                      const double *true_tau, const double *true_alpha, const int *P,
                      const int *N, const int *M, const int *burn, double *runtime);

/* ------------------------------------------------------------------------ */
/* Part 2: extensions                                                        */
/* ------------------------------------------------------------------------ */

/* Library / device information. */
const char *bb_version(void);
const char *bb_last_error(void);
int bb_device_count(void);

/*
 * RNG seeding.  Every variate is Philox4x64-10 of a counter; the key
 * is (seed, stream).  bb_set_seed sets the seed and resets the stream to 0; each
 * .C call consumes one stream value.  When the library runs inside R (the
 * symbols GetRNGstate / unif_rand / PutRNGstate resolve), the seed is instead
 * drawn from R's RNG on every .C call, so set.seed() reproduces results.
 */
void bb_set_seed(uint64_t seed);
void bb_get_rng_state(uint64_t *seed, uint64_t *stream);
void bb_set_rng_state(uint64_t seed, uint64_t stream);
void bb_use_r_rng(int enable); /* default 1: use R's RNG when present */

/* Select the device used by the .C entry points (default 0). */
int bb_set_device(int device);

/* Verbosity of the reference-style progress messages (0 silences them). */
void bb_set_verbose(int verbose);

/*
 * Device engine: one Gibbs chain on one GPU, holding a column shard
 * [j0, j0 + p_local) of an N x P problem.  Used by bench.py, the multi-GPU path
 * and the tests.  Sweeps are enqueued asynchronously on the engine's stream.
 */
typedef struct bb_engine bb_engine;

typedef struct bb_config {
    int n;              /* rows */
    int p;              /* global number of columns */
    int p_local;        /* columns held by this engine (== p unless sharded) */
    int j0;             /* global index of this engine's first column */
    int rank, world;    /* shard id and count (world > 1 requires a communicator) */
    double sig2_shape, sig2_scale, nu_shape, nu_rate, alpha_a, alpha_b;
    double true_sig2, true_tau, true_alpha;
    int ortho;          /* orthogonal-design variant (sample_beta_stable_ortho) */
    int method;         /* 0 auto (chol if p <= n else woodbury), 1 chol, 2 woodbury,
                           4 triangle mixture (bridge.reg.tri; p <= n, p <= 2048);
                           5 sparse Woodbury is selected by bb_engine_create_csc;
                           6 logistic bridge (Polya-Gamma; y in {0, 1}) */
    int trace_capacity; /* number of trace slots kept on device (>= 1) */
    uint64_t seed, stream;
    int device;
    int gram_mode;      /* Woodbury Gram X diag(D) X' and the logistic X'Omega X: 0 fp64 MFMA,
                           1 Ozaki-II on int8 MFMA (fp64-accurate); default 1 */
    int betaburn;       /* triangle method: rtnorm_gibbs passes per sweep - 1 */
} bb_config;

void bb_config_default(bb_config *cfg);

/* Create: X_local is N x p_local column-major (host), y is N (host). */
int bb_engine_create(const bb_config *cfg, const double *X_local, const double *y,
                     bb_engine **out);
void bb_engine_destroy(bb_engine *e);

/* Create from a CSC design (the engine's p_local columns; colptr has p_local + 1 entries,
 * canonical row order): the sparse Woodbury engine (method 5).  Builds the Gram pair list
 * on the device at setup; fails (-1, bb_last_error) if it does not fit in HBM. */
int bb_engine_create_csc(const bb_config *cfg, const int *colptr, const int *rowidx,
                         const double *val, const double *y, bb_engine **out);
/* Number of off-diagonal Gram pairs (X_rj X_cj != 0, r < c) of a sparse engine, else -1. */
long long bb_engine_sparse_pairs(const bb_engine *e);
/* Sparse engine layout: pair count, nnz of the shard, largest row nnz, and whether the
 * by-column Gram kernel runs (1: every row has <= 8192 non-zeros) or the general one (0). */
int bb_engine_sparse_info(const bb_engine *e, long long *pairs, long long *nnz, int *max_row,
                          int *col_mode);

/*
 * RCCL communicator for world > 1: rank 0 calls bb_comm_unique_id, the bytes are
 * broadcast out of band (torch.distributed store), every rank calls
 * bb_engine_comm_init.  id_bytes is bb_comm_id_size() bytes.
 */
int bb_comm_id_size(void);
int bb_comm_unique_id(void *id_bytes);
int bb_engine_comm_init(bb_engine *e, const void *id_bytes);

/*
 * Initialise the chain state as the reference does (BridgeWrapper.cpp:242-262):
 * beta = least squares (0 when X'X is singular or p > n), alpha = 0.5 (or
 * true_alpha), then the pre-burn tau draw (non-ortho only).
 */
int bb_engine_init_state(bb_engine *e);

/*
 * Enqueue `count` sweeps starting at global sweep index t0 (t = 1 + i for burn-in
 * sweep i, t = burn + 1 + i for MCMC sweep i; BridgeWrapper.cpp:266,287).  Sweep k
 * records its state in trace slot first_slot + k * slot_step (mod trace_capacity);
 * first_slot < 0 records nothing.  Burn-in uses slot_step 0 (everything in slot 0,
 * as the reference does).  mcmc_phase selects the (alpha_b, alpha_b) prior pair of
 * the reference's MCMC loop (BridgeWrapper.cpp:294) over (alpha_a, alpha_b) (:272).
 */
int bb_engine_run(bb_engine *e, uint64_t t0, int count, int first_slot, int slot_step,
                  int mcmc_phase);
int bb_engine_sync(bb_engine *e);

/* Copy trace slots [slot0, slot0 + count) to host buffers (any may be NULL).
 * beta/lambda are p_local x count. */
int bb_engine_get_trace(bb_engine *e, int slot0, int count, double *beta, double *lambda,
                        double *sig2, double *tau, double *alpha);

/* Current chain state (beta, lambda: p_local; scalars). */
int bb_engine_get_state(bb_engine *e, double *beta, double *lambda, double *tau,
                        double *sig2, double *alpha);
/* Overwrite the current chain state (teacher forcing in tests). */
int bb_engine_set_state(bb_engine *e, const double *beta, double tau, double sig2,
                        double alpha);

/*
 * Shard group: `count` engines with cfg.rank = 0..count-1 and cfg.world = count, each
 * holding a column shard of one p > n chain.  Two kinds share the type:
 *   - bb_group_create: every member on ONE device, driven by one host thread, the per-sweep
 *     exchanges done as on-device sums (the sharded decomposition on a single GPU; RCCL
 *     cannot place two ranks on one device);
 *   - bb_group_create_rccl: members on DISTINCT devices, communicators from
 *     ncclCommInitAll lent to the members, each member's sweeps enqueued by its own host
 *     thread inside bb_group_run (the single-process multi-GPU path of the .C entry points).
 */
typedef struct bb_group bb_group;
/* Batch of truncated draws (mode 0..5 = rtnorm_left, rtnorm_both, rtnorm,
 * rtexpon_rate_left, rtexpon_rate_both, rtexpon_rate; parameters in the .C order, unused
 * ones NULL) under key (seed, stream).  Returns 0, or -2 if a draw failed. */
int bb_trunc_batch(int mode, int num, double *x, const double *p0, const double *p1,
                   const double *p2, const double *p3, uint64_t seed, uint64_t stream);

/* omega_i ~ PG(1, psi_i), i < n, under key (seed, stream) and sweep counter t -- the
 * logistic path's Polya-Gamma kernel (tests).  Returns 0, or -2 if a draw failed. */
int bb_pg_batch(double *omega, const double *psi, int n, uint64_t seed, uint64_t stream,
                uint64_t t);

/* rrtgamma_rate under an explicit key (seed, stream). */
int bb_rrtgamma_batch(int num, double *x, const double *shape, const double *rate,
                      const double *right_t, uint64_t seed, uint64_t stream);

/* Triangle method (cfg.method == 4): u and shape traces (omega comes back as `lambda`
 * from bb_engine_get_trace), and the design basis X = U diag(d) V' the engine computed
 * at setup: tV (P x P column-major, row i = i-th right singular vector), a = V'X'y, d. */
int bb_engine_get_tri_trace(bb_engine *e, int slot0, int count, double *u, double *shape);
int bb_engine_get_tri_basis(bb_engine *e, double *tV, double *a, double *d);
/* Triangle method: overwrite the latent u (P) -- teacher-forced tests. */
int bb_engine_set_tri_state(bb_engine *e, const double *u);

int bb_group_create(bb_engine **engines, int count, bb_group **out);
/* The group over engines on DISTINCT devices, exchanging with RCCL (see above).  R calls .C
 * from one process, so this is the multi-GPU path of the .C entry points; bb_group_run
 * starts one enqueue thread per member and joins them before it returns. */
int bb_group_create_rccl(bb_engine **engines, int count, bb_group **out);
void bb_group_destroy(bb_group *g);
int bb_group_init_state(bb_group *g);
int bb_group_run(bb_group *g, uint64_t t0, int count, int first_slot, int slot_step,
                 int mcmc_phase);
int bb_group_sync(bb_group *g);

/*
 * .C driver controls.  bb_set_device_count(k) lets bridge_reg_stable / bridge_reg_stable_csc
 * shard the columns of a p > n problem (stable mixture: Woodbury or orthogonal design, alpha
 * known or drawn by MH) over up to k visible devices in one process (>= 4096 columns per
 * device, an RCCL group; 0: every visible device).  The default is 1 (opt-in): a sharded
 * chain sums its Gram in another fp64 order, and p > n chains amplify roundoff, so a trace
 * depends on the device count.  Traces live on the device in a ring of at most `bytes` per
 * engine (default
 * 1 GiB), copied out to the caller's P x M buffers whenever it fills, so M is not bounded by
 * HBM.  Every 10 sweeps the driver polls R's interrupt (R_CheckUserInterrupt under
 * R_ToplevelExec, as BridgeWrapper.cpp:273-275 polls), stops, releases the device, returns
 * the samples drawn so far and re-raises the interrupt in R.
 */
void bb_set_device_count(int count);
/* Chain variant of the device Cholesky (k_chol_persistent): 1 = the default chain, 2 and 3 =
 * the pipelined chains (measured slower); for A/B measurements.  Returns 0, or -1 for another value; version 0
 * changes nothing and returns the variant in use. */
int bb_set_chol_version(int version);
void bb_set_trace_budget(long long bytes);
/* A/B tuning knobs (measurement tools only).  key 1: the Ozaki residue-plane stores
 * non-temporal (value 1), ordinary (0), or non-temporal stores and X loads (2, the default);
 * key 2: non-temporal X loads in the fused beta / X.beta pass (1, the default) or ordinary (0);
 * key 3: the sparse Gram kernel: lanes per entry (0), the same with non-temporal pair-list
 * loads (1), or the flat chunked pair stream with 8 (2) or 16 (3, the default) pairs per lane;
 * key 4: occupancy of the lambda launches, bit 0 = k_lambda_spec and bit 1 = k_lambda_cb
 * capped at 128 VGPRs for 4 waves per SIMD instead of their register-minimal 3 (default 2:
 * k_lambda_cb only: 4 % faster at C5 than 3 waves); bit 2: k_lambda_cb with the sampler
 * bodies inlined (3 waves per SIMD) instead, 6 % faster at C5 than the out-of-line instance at
 * 4 waves; bit 3: that launch also for 40000 < p <= 50000 (7 % faster than the speculative
 * launch there); default 12 (bits 2 and 3); the draws are the same;
 * key 5: lanes per coefficient of the speculative lambda launch (0 = the size-based default);
 * key 6: the most Chebyshev iterations a Woodbury sweep may take on the near-identity path
 * (default 16; 0 = every sweep forms the Gram and factors it);
 * key 7: a dense Woodbury sweep that may take the near-identity path draws lambda and forms
 * the X u partials in one launch (1: up to 3 workgroups per CU looping over column chunks;
 * 2: one workgroup per chunk, drawing then streaming; 3, the default: two drawing and one
 * streaming workgroup per CU, the stream following per-chunk flags) or in two (0); the draws
 * are the same;
 * key 8: an unsharded Woodbury engine decides each sweep's path as a column shard does (the
 * host waits for the decision, then launches that path only: 1, the default, with the
 * Chebyshev solve's first kernels enqueued before the wait and returning at once unless the
 * device decided so; 2: without them) or launches both
 * paths with the kernels of the one not taken returning at once (0); the draws are the same
 * except on sweeps where mode 0's launch hint fell short (it then takes the factor);
 * key 9 (testing): 1 makes an engine with world == 1 that owns a communicator (a 1-rank RCCL
 * comm, bb_engine_comm_init) or belongs to an on-device shard group run the column-shard
 * near-identity protocol of world > 1 (bound sums exchanged, the decision from them, X u and
 * every product E d exchanged), so each of its exchanges executes on one GPU (default 0).
 * key 10: the mixed-precision near-identity plan of unsharded dense Woodbury engines
 * (products over an fp32 copy of X, one fp64 residual pass, the same certified bound; 1, the
 * default) or fp64 products only (0);
 * key 11: the host learns a synchronous near-identity decision by polling the tag word the
 * decision kernel stores into coherent host memory (1, the default) or by waiting on an event
 * recorded behind it (0);
 * key 12: the partial row sums of the Chebyshev kernels read row blocks placed so that
 * neighbouring blocks share an XCD (1, the default) or in dispatch order (0);
 * key 13: the fused lambda + X u launch with 8 lanes per coefficient deals the lanes of a
 * wave's finished draws to its unfinished ones (1, the default) or keeps fixed 8-lane groups
 * (0);
 * key 15: the continuous-batching lambda launch with its sampler inlined lends the lanes of a
 * wave's idle groups to its unfinished draws once its range is used up (1, the default) or
 * lets every group finish its own draw (0); under keys 11-15 the draws are the same;
 * key 16 (benchmarking only): K > 0 makes every near-identity sweep run K Chebyshev iterates
 * (at most key 6's cap) instead of its certified count, for timing a C3 rank's product count
 * on a narrower proxy; the solve is then not certified (default 0, the current device only);
 * key 17: the split lambda launch (key 7 = 3) also forms the near-identity decision's bound
 * sums, reduced and decided on by one small launch after it (1, the default), or, unsharded,
 * reduces them and decides in its last workgroup as well (2), or separate launches form them
 * (0); the decision and the chain are the same bits in every mode (the bound is rounded up to
 * 12 significant bits, so the sums' order does not reach it);
 * key 20: the persistent backward solve hands each solved block to the next as 64-bit words
 * tagged with the solve's epoch, polled directly (1, the default), or behind a flag (0); the
 * same bits.
 * A negative value changes nothing.  Returns the previous value, or -1 for an unknown key. */
int bb_set_tuning(int key, int value);
/* Test hook: the k-th interrupt poll from now reports an interrupt (k >= 0; -1 clears). */
void bb_debug_interrupt_after(int polls);
/* Last .C sampler call: devices used, trace ring slots, whether it was interrupted. */
int bb_last_call_info(int *devices, int *trace_capacity, int *interrupted);
/* Test hook: member `member` of the NEXT RCCL shard-group run throws before its sweep `sweep`
 * (-1 clears).  The group then aborts every communicator, returns -1 and refuses further runs. */
void bb_debug_fail_member(int member, int sweep);

/*
 * .C-callable forms of the controls.  R's .C passes every argument as a pointer (the
 * reference's whole .C surface is pointer-only, BridgeWrapper.h:164-245), so a by-value
 * `int` control called from R would receive the ADDRESS of the R integer.  From R:
 *   .C("bb_set_device_count_C", 0L)       # shard p > n chains over every visible device
 *   .C("bb_set_device_count_C", 1L)       # one device (the default)
 *   .C("bb_last_call_info_C", devices = 0L, capacity = 0L, interrupted = 0L)$devices
 * R integers are 32-bit and R doubles carry integers exactly up to 2^53, so the 64-bit seed,
 * stream and byte counts are passed as doubles.
 */
void bb_set_device_count_C(const int *count);
void bb_get_device_count_C(int *count);
/* Devices a bridge_reg_stable call of this shape would use with `nvisible` devices
 * visible (nvisible < 0: the devices actually visible). */
void bb_plan_devices_C(const int *n, const int *p, const int *ortho, const int *nvisible,
                       int *devices);
void bb_set_device_C(const int *device, int *status); /* status: 0, or -1 (invalid device) */
void bb_set_verbose_C(const int *verbose);
void bb_use_r_rng_C(const int *enable);
void bb_set_seed_C(const double *seed);
void bb_set_rng_state_C(const double *seed, const double *stream);
void bb_get_rng_state_C(double *seed, double *stream);
void bb_set_trace_budget_C(const double *bytes);
void bb_last_call_info_C(int *devices, int *trace_capacity, int *interrupted);

/* Which beta-step path the engine uses: 1 chol (p <= n), 2 woodbury, 3 ortho, 4 triangle,
 * 5 sparse woodbury, 6 logistic. */
int bb_engine_method(const bb_engine *e);
/* Logistic engine: the current Polya-Gamma latents omega (N). */
int bb_engine_get_omega(bb_engine *e, double *omega);
/* Gram implementation in use on the Woodbury path: 0 fp64 MFMA, 1 Ozaki-II int8. */
int bb_engine_gram_mode(const bb_engine *e);

/* Per-kernel timing with HIP events on the engine's stream.  enable: 0 off, 1 only the
 * timed phase is bracketed (two events per sweep, for timed runs), 2 every phase start.
 * kernel_times: average ms of the timed phase (first output) and of the event-covered part
 * of a sweep.  The timed phase is the Gram GEMM unless bb_engine_set_timed_phase chose
 * another (an index 0 .. bb_phase_count()-2 of bb_phase_name). */
int bb_engine_enable_timing(bb_engine *e, int enable);
int bb_engine_set_timed_phase(bb_engine *e, int phase);
/* enable = 1: bracket the timed phase in every stride-th sweep only (default 1: every sweep);
 * an event pair costs ~6 us of stream time per bracketed sweep (kernel boundaries the
 * hardware cannot overlap), 1-2 % of a near-identity C3 sweep */
int bb_engine_set_timing_stride(bb_engine *e, int stride);
int bb_engine_kernel_times(bb_engine *e, double *gram_ms_avg, double *sweep_ms_avg,
                           int *samples);
int bb_engine_reset_timing(bb_engine *e);
/* Average milliseconds per sweep spent in each phase (ms[0 .. bb_phase_count()-1]),
 * measured between HIP events recorded at phase starts on the engine stream. */
int bb_engine_phase_times(bb_engine *e, double *ms, int cap, int *samples);
int bb_phase_count(void);
const char *bb_phase_name(int i);

/* The near-identity path's setup: the certified bound lambda_x >= lambda_max(X X') (0: none)
 * and the most Chebyshev iterations a sweep may take (cost model and bb_set_tuning key 6; -1:
 * no near-identity path). */
int bb_engine_nid_bound(bb_engine *e, double *lambda_x, int *kmax);
/* Number of timed-phase brackets (launches of the timed phase) recorded since the last reset. */
int bb_engine_timed_brackets(bb_engine *e, int *count);
/* Near-identity solve of the Woodbury system: sweeps that took the Chebyshev
 * path, E-apply passes they ran, sweeps that formed the Gram and factored it (counts since the
 * engine was created), and the eps = tr(X D X') / sig2 bound and mode of the latest sweep (-1
 * when the engine has no near-identity path: sharded, p <= n or n > 4096 dense). */
int bb_engine_nid_stats(bb_engine *e, unsigned long long *cheb_sweeps,
                        unsigned long long *products, unsigned long long *chol_sweeps,
                        double *eps, int *mode);

/* Launch counts since the engine was created: sweeps whose lambda draws were launched together
 * with the X u stream of the near-identity solve (k_lambda_xu), and sweeps whose
 * lambda draws were a launch of their own. */
int bb_engine_launch_counts(bb_engine *e, unsigned long long *lambda_xu,
                            unsigned long long *lambda_alone);

/* The kernel instance this process most recently launched for a roofline phase ("lambda",
 * "gram", "reduce", "chol", "solve", "beta", "eapply"), demangled without its parameter list
 * ("bb::k_eapply<8, false>"), into buf.  Returns 0, or -1 if none was launched. */
int bb_kernel_instance(const char *phase, char *buf, int len);

/* The mixed-precision near-identity plan: sweeps that took it and the fp32
 * E-apply passes they ran (counts since creation), the latest sweep's certified |E - E~| and
 * correction iterates (0: that sweep took the fp64 plan or the factor), and whether the engine
 * holds the fp32 copy of X at all. */
int bb_engine_nid_mixed(bb_engine *e, unsigned long long *mixed_sweeps,
                        unsigned long long *products32, double *eta, int *k2, int *holds_x32);

/* Error flags raised on device (rejection-loop caps, non-SPD factorisations). */
int bb_engine_error_flags(bb_engine *e, uint32_t *flags);

/* ---- kernel-level entry points (tests / microbenchmarks) ---- */

/* Tilted-stable batch with explicit key and counter base t (host buffers). */
int bb_retstable_batch(double *x, const double *alpha, const double *V0, const double *h,
                       int num, uint64_t seed, uint64_t stream, uint64_t t, int group);

/* lambda_j = 2 * retstable(beta_j^2/tau^2, alpha/2, 1) for global j = j0 + i. */
int bb_sample_lambda(double *lambda, const double *beta, int p, double alpha, double tau,
                     uint64_t seed, uint64_t stream, uint64_t t, uint64_t j0, int group);

/* Microbenchmark of the lambda kernel: average ms over `reps` launches (sweep indices
 * t = 2 .. reps+1, key (1, 0)) for an explicit group size and inlining variant; the
 * last launch's draws are returned in lambda_out (may be NULL). */
int bb_bench_lambda(const double *beta, int p, double alpha, double tau, int group,
                    int noinline, int reps, double *ms_avg, double *lambda_out);

/* Microbenchmark of the blocked Cholesky (m x m SPD test matrix, 1 RHS): average ms of
 * chol_factor and of chol_bsolve over `reps` runs.  If `trace` is not NULL it receives
 * 32 * ceil(m/64) stamps of an extra traced factorisation: per block step, 8 points of the
 * chain workgroup's critical path (elimination start / done / W stored / hand-off acquired
 * / tiles loaded / U formed / next diagonal block formed / released) in s_memrealtime ticks
 * (100 MHz), the same 8 points in shader clocks (s_memtime), then the diagonal
 * elimination's 8 producer-group starts and 8 ends (s_memrealtime). */
int bb_bench_chol(int m, int reps, double *ms_factor, double *ms_solve,
                  unsigned long long *trace);

/* Gram C = Y diag(w) Y' (Y: n x k column-major) via the fp64 MFMA kernel;
 * C is n x n column-major, full symmetric result. */
int bb_gram(double *C, const double *Y, const double *w, int n, int k);

/* Microbenchmark of the Ozaki int8 GEMM alone on random residues (n x k, nsplit K splits, 0 =
 * automatic); dbg != 0 selects timing ablations (results then meaningless), except dbg = 999
 * (the production kernel with every pass from K chunk 0), dbg = 1000 + L (the production
 * kernel with the diagonal pairs' K lead set to L / 1000 of the pass) and dbg = 1000000 +
 * 1000 T + L (lead L / 1000, start shift T / 1000 of a pass per earlier diagonal-pair round). */
int bb_bench_ozaki(int n, int k, int nsplit, int dbg, int reps, double *ms);

/* The same Gram through the Ozaki-II int8 path (w >= 0): exact integer Gram of the
 * row-scaled, fp64-rounded Y diag(sqrt(w)), rounded once to fp64. */
int bb_gram_ozaki(double *C, const double *Y, const double *w, int n, int k);

/* Sparse Gram of a CSC design (n x p): C = X diag(D) X' (n x n column-major, full
 * symmetric) and xu = X u (n; u and xu may be NULL), through the engine's pair-list
 * kernels. */
int bb_sparse_gram(double *C, double *xu, const int *colptr, const int *rowidx, const double *val,
                   const double *D, const double *u, int n, int p);
/* Microbenchmark of the sparse Gram: average ms of the pair-list kernel and of the CSR row
 * pass (diagonal + X u) over `reps` launches; pairs receives the pair count. */
int bb_bench_sparse_gram(const int *colptr, const int *rowidx, const double *val, const double *D,
                         int n, int p, int reps, double *ms_gram, double *ms_rows,
                         long long *pairs);

/* SPD solve via the blocked device Cholesky: A (m x m, column-major, only the
 * upper triangle read) -> x = A^-1 b for nrhs right-hand sides (m x nrhs). */
int bb_chol_solve(double *x, const double *A, const double *b, int m, int nrhs);

/* bridge_EM without the .C marshalling: returns the solve count (as bridge_EM's max_iter),
 * the EM iteration count when every coefficient was dropped, or -1 (bb_last_error()). */
int bb_bridge_em(double *beta, const double *y, const double *X, int n, int p, double ratio,
                 double alpha, double lambda_max, double tol, int max_iter, int use_cg);

/* trace.beta on the device (Code/R/bridge-trace.R:25-54): bridge EM (direct solves) for
 * every ratio of a grid in ONE launch, a workgroup per ratio (the system in LDS for
 * p <= 128, in a per-ratio global slice with a tiled Cholesky above; the ratios then run in
 * chunks that fit half the free device memory, at most 16 GiB).  beta: count x p (row r for ratios[r]),
 * solves: count (bb_bridge_em's return per ratio).  Returns 0 or -1 (bb_last_error()). */
int bb_bridge_em_batch(double *beta, int *solves, const double *y, const double *X, int n,
                       int p, const double *ratios, const double *lambda_max, int count,
                       double alpha, double tol, int max_iter);

#ifdef __cplusplus
}
#endif

#endif /* BAYESBRIDGE_AMD_H */
