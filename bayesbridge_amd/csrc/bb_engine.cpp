// bb_engine.cpp -- host side of the MI355X BayesBridge drop-in: the Gibbs driver
// (restating Code/C/BridgeWrapper.cpp:207-313 and :434-537) over the HIP kernels of
// bb_kernels.hip, RCCL for column-sharded multi-GPU runs, and the extern "C" entry
// points declared in include/bayesbridge.h.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cxxabi.h>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <atomic>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/bayesbridge.h"
#include "bb_kernels.h"
#include "bb_ozaki.h"
#include "bb_sparse.h"

using namespace bb;

namespace {

thread_local std::string g_last_error;
std::mutex g_mu;
uint64_t g_seed = 0xB4E5B41D6EULL;
uint64_t g_stream = 0;
int g_device = 0;
int g_verbose = 1;
int g_use_r_rng = 1;
// bb_debug_fail_member: member `g_debug_fail_member` of the next RCCL group run throws
// before its sweep `g_debug_fail_sweep` (test hook for the group's failure handling)
std::atomic<int> g_debug_fail_member{-1}, g_debug_fail_sweep{-1};

void set_error(const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
}

struct HipError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

#define HIPCHECK(x)                                                                       \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            char b_[512];                                                                 \
            snprintf(b_, sizeof(b_), "HIP error %s at %s:%d: %s", hipGetErrorName(e_),    \
                     __FILE__, __LINE__, #x);                                             \
            throw HipError(b_);                                                           \
        }                                                                                 \
    } while (0)

#define NCCLCHECK(x)                                                                      \
    do {                                                                                  \
        ncclResult_t r_ = (x);                                                            \
        if (r_ != ncclSuccess) {                                                          \
            char b_[512];                                                                 \
            snprintf(b_, sizeof(b_), "RCCL error %s at %s:%d", ncclGetErrorString(r_),    \
                     __FILE__, __LINE__);                                                 \
            throw HipError(b_);                                                           \
        }                                                                                 \
    } while (0)

inline int round_up(int x, int m) { return ((x + m - 1) / m) * m; }

template <typename T>
T *dalloc(size_t count, std::vector<void *> &owned) {
    void *p = nullptr;
    if (count == 0) count = 1;
    HIPCHECK(hipMalloc(&p, count * sizeof(T)));
    HIPCHECK(hipMemset(p, 0, count * sizeof(T)));
    // the engine's streams are non-blocking: the zero fill must land before their first use
    HIPCHECK(hipDeviceSynchronize());
    owned.push_back(p);
    return (T *)p;
}

// R's RNG, resolved at run time when this library is loaded inside R.
struct RRng {
    void (*get)(void) = nullptr;
    void (*put)(void) = nullptr;
    double (*unif)(void) = nullptr;
    bool tried = false;
    bool ok() {
        if (!tried) {
            tried = true;
            get = (void (*)(void))dlsym(RTLD_DEFAULT, "GetRNGstate");
            put = (void (*)(void))dlsym(RTLD_DEFAULT, "PutRNGstate");
            unif = (double (*)(void))dlsym(RTLD_DEFAULT, "unif_rand");
        }
        return get && put && unif;
    }
} g_rrng;

// Key for one .C call: from R's RNG if present, else (seed, stream++).
void next_call_key(uint64_t *k0, uint64_t *k1) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_use_r_rng && g_rrng.ok()) {
        g_rrng.get();
        uint64_t a = (uint64_t)(g_rrng.unif() * 4294967296.0);
        uint64_t b = (uint64_t)(g_rrng.unif() * 4294967296.0);
        uint64_t c = (uint64_t)(g_rrng.unif() * 4294967296.0);
        g_rrng.put();
        *k0 = (a << 32) ^ b;
        *k1 = c;
        return;
    }
    *k0 = g_seed;
    *k1 = g_stream++;
}

// ---------------------------------------------------------------------------
// Sparse design (CSC input): CSC + CSR copies on the device and the Gram pair list
// (bb_sparse.h).  Built once at setup; X is constant over a chain.
// ---------------------------------------------------------------------------
// The canonical dgCMatrix form every CSC entry point requires (colptr[0] = 0,
// non-decreasing, rows in [0, n), strictly increasing within a column); throws otherwise.
// Both .C CSC paths (sparse engine and densified dense path) run it, so a malformed matrix
// is refused the same way whichever path its shape selects.
static void csc_validate(int n, int p, const int *cp, const int *ri) {
    if (cp[0] != 0) throw HipError("CSC: colptr[0] must be 0");
    for (int j = 0; j < p; ++j) {
        if (cp[j + 1] < cp[j]) throw HipError("CSC: colptr must be non-decreasing");
        for (int q = cp[j]; q < cp[j + 1]; ++q) {
            if (ri[q] < 0 || ri[q] >= n) throw HipError("CSC: row index out of range");
            if (q > cp[j] && ri[q] <= ri[q - 1])
                throw HipError("CSC: row indices must be strictly increasing within a "
                               "column (canonical dgCMatrix form)");
        }
    }
}

struct SparseDesign {
    int n = 0, n_pad = 0, p = 0;
    long nnz = 0;
    size_t pairs = 0;
    int *colptr = nullptr, *rowidx = nullptr, *rowptr = nullptr, *colidx = nullptr,
        *cpos = nullptr, *pj = nullptr;
    double *cval = nullptr, *rval = nullptr, *prod = nullptr;
    unsigned *estart = nullptr;
    unsigned short *pidx = nullptr;
    int max_row = 0;        // largest row nnz
    bool col_mode = false;  // by-column Gram kernel (max_row <= kSpColMaxRow)

    // Validates the CSC (colptr[0] = 0, non-decreasing, rows in [0, n), strictly increasing
    // within a column -- R's dgCMatrix is in this canonical form), transposes it on the host
    // into a CSR with each entry's CSC position, uploads both and builds the pair list.
    void build(hipStream_t s, int n_, int n_pad_, int p_, const int *cp, const int *ri,
               const double *cv, std::vector<void *> &owned) {
        n = n_;
        n_pad = n_pad_;
        p = p_;
        csc_validate(n, p, cp, ri);
        nnz = cp[p];
        std::vector<int> rp(n_pad + 1, 0), ci(nnz > 0 ? nnz : 1), pos(nnz > 0 ? nnz : 1);
        std::vector<double> rv(nnz > 0 ? nnz : 1);
        for (long q = 0; q < nnz; ++q) ++rp[ri[q] + 1];
        max_row = 0;
        for (int r = 0; r < n_pad; ++r) max_row = std::max(max_row, rp[r + 1]);
        col_mode = max_row <= kSpColMaxRow;
        for (int r = 0; r < n_pad; ++r) rp[r + 1] += rp[r];
        std::vector<int> next(rp.begin(), rp.end() - 1);
        for (int j = 0; j < p; ++j)
            for (int q = cp[j]; q < cp[j + 1]; ++q) {
                const int k = next[ri[q]]++;
                ci[k] = j;
                rv[k] = cv[q];
                pos[k] = q;
            }
        colptr = dalloc<int>(p + 1, owned);
        rowidx = dalloc<int>(nnz, owned);
        cval = dalloc<double>(nnz, owned);
        rowptr = dalloc<int>(n_pad + 1, owned);
        colidx = dalloc<int>(nnz, owned);
        rval = dalloc<double>(nnz, owned);
        cpos = dalloc<int>(nnz, owned);
        HIPCHECK(hipMemcpy(colptr, cp, (size_t)(p + 1) * sizeof(int), hipMemcpyHostToDevice));
        if (nnz > 0) {
            HIPCHECK(hipMemcpy(rowidx, ri, (size_t)nnz * sizeof(int), hipMemcpyHostToDevice));
            HIPCHECK(hipMemcpy(cval, cv, (size_t)nnz * sizeof(double), hipMemcpyHostToDevice));
            HIPCHECK(hipMemcpy(colidx, ci.data(), (size_t)nnz * sizeof(int), hipMemcpyHostToDevice));
            HIPCHECK(hipMemcpy(rval, rv.data(), (size_t)nnz * sizeof(double), hipMemcpyHostToDevice));
            HIPCHECK(hipMemcpy(cpos, pos.data(), (size_t)nnz * sizeof(int), hipMemcpyHostToDevice));
        }
        HIPCHECK(hipMemcpy(rowptr, rp.data(), (size_t)(n_pad + 1) * sizeof(int),
                           hipMemcpyHostToDevice));
        // pair counts per output column, host scan, then the pair list itself
        unsigned long long *dcnt = nullptr, *dbase = nullptr;
        HIPCHECK(hipMalloc(&dcnt, (size_t)n_pad * sizeof(unsigned long long)));
        launch_sp_count(s, rowptr, colidx, cpos, colptr, n_pad, dcnt);
        std::vector<unsigned long long> cnt(n_pad), base(n_pad);
        HIPCHECK(hipMemcpyAsync(cnt.data(), dcnt, cnt.size() * sizeof(unsigned long long),
                                hipMemcpyDeviceToHost, s));
        HIPCHECK(hipStreamSynchronize(s));
        (void)hipFree(dcnt);
        unsigned long long tot = 0;
        for (int c = 0; c < n_pad; ++c) {
            base[c] = tot;
            tot += cnt[c];
        }
        if (tot > 0xFFFFFF00ull)
            throw HipError("sparse Gram: more than 2^32 - 1 column pairs (X too dense for the "
                           "pair-list Gram; use the dense entry point)");
        pairs = (size_t)tot;
        size_t fr = 0, total_mem = 0;
        HIPCHECK(hipMemGetInfo(&fr, &total_mem));
        const size_t need = pairs * (sizeof(double) + (col_mode ? 2 : sizeof(int))) +
                            (tri_count(n_pad) + 1) * sizeof(unsigned);
        if (need + (size_t(1) << 28) > fr) {
            char b[256];
            snprintf(b, sizeof(b), "sparse Gram: pair list needs %.2f GB, %.2f GB free", need / 1e9,
                     fr / 1e9);
            throw HipError(b);
        }
        estart = dalloc<unsigned>(tri_count(n_pad) + 1, owned);
        prod = dalloc<double>(pairs, owned);
        if (col_mode)
            pidx = dalloc<unsigned short>(pairs, owned);
        else
            pj = dalloc<int>(pairs, owned);
        HIPCHECK(hipMalloc(&dbase, (size_t)n_pad * sizeof(unsigned long long)));
        HIPCHECK(hipMemcpyAsync(dbase, base.data(), base.size() * sizeof(unsigned long long),
                                hipMemcpyHostToDevice, s));
        launch_sp_build(s, rowptr, colidx, cpos, rval, colptr, rowidx, cval, n_pad, dbase, estart,
                        prod, pj, pidx);
        const unsigned last = (unsigned)tot;
        HIPCHECK(hipMemcpyAsync(estart + tri_count(n_pad), &last, sizeof(unsigned),
                                hipMemcpyHostToDevice, s));
        HIPCHECK(hipStreamSynchronize(s));
        (void)hipFree(dbase);
    }

    // tri (packed upper triangle of X diag(D) X', n_pad wide) and xu = X u
    void gram(hipStream_t s, const double *D, const double *u, double *tri, double *xu,
              const int *gate = nullptr) const {
        if (col_mode) {
            launch_sp_gram_col(s, rowptr, colidx, rval, estart, prod, pidx, D, u, n_pad, max_row,
                               tri, xu, gate);
        } else {
            launch_sp_gram(s, estart, prod, pj, D, n_pad, tri, gate);
            launch_sp_rows(s, rowptr, colidx, rval, n_pad, u, D, xu, tri, gate);
        }
    }
};

}  // namespace

// ---------------------------------------------------------------------------
// Engine
// ---------------------------------------------------------------------------
enum Phase {
    PH_PRE, PH_SCALARS, PH_LAMBDA, PH_PG, PH_OZPREP, PH_GRAM, PH_XU, PH_REDUCE, PH_FORM, PH_CHOL,
    PH_SOLVE, PH_BETA, PH_XB, PH_ALPHA, PH_NID, PH_EAPPLY, PH_END, PH_COUNT
};
// "gram" times the Gram GEMM kernel alone (k_gram, or k_oz_gemm after "ozprep" = row scales
// + residues); "reduce" is the split/slab combine (k_slab_sum or the CRT k_oz_crt); "nid" the
// near-identity decision, X u and Chebyshev recurrences, "eapply" its passes over X
// (bb_nid.hip).

// Chebyshev iterations the near-identity solve may take per sweep (bb_set_tuning key 6; 0
// turns the path off: every sweep forms the Gram and factors it)
int g_nid_kmax = 16;
// bb_set_tuning key 8: an unsharded engine decides like a shard (the host waits for each
// sweep's decision, then launches only that path: 1, the default) or launches both paths
// gated with the hint of nid_launch_count (0).  Measured at the driver's settings (round 4,
// gpurun_out/r04f_*): C3 1781 against 1746-1749 sweeps/s, C2 5840 against 5519, C5 1672
// against 1636 -- the host's wake-up and first launch cost less than the gated no-ops.
int g_nid_sync = 1;
// bb_set_tuning key 9 (testing): an engine with world == 1 that owns a communicator (a 1-rank
// RCCL comm) or belongs to an on-device shard group runs the world > 1 near-identity stage
// sequence (bound-sum exchange, k_nid_decide_from, X u and per-product exchanges), so every
// exchange call site of that protocol executes on a one-GPU box
int g_shard_proto = 0;
// bb_set_tuning key 10: the mixed-precision near-identity plan of unsharded
// dense engines: products over an fp32 copy of X with one fp64 residual pass (1, the default)
// or fp64 products only (0)
int g_nid_mixed = 1;
// bb_set_tuning key 11: the host learns a synchronous decision by polling its tag word in
// coherent host memory (1, the default) or by an event recorded behind the decision kernel
// (0).  The event's marker left the device idle ~4 us per sweep: C3 at the driver's settings
// 2010 against 1995 sweeps/s, 1000 sweeps after 100 1370 against 1367 (gpurun_out/ab_*).
int g_nid_poll = 1;
// bb_set_tuning key 17: under the synchronous protocol the split lambda launch (key 7 = 3)
// forms the decision's bound sums in its stream role, k_nid_reduce adds them and decides
// (1, the default); 2: unsharded, the launch's last stream workgroup reduces and decides too;
// 0: k_nid_sums + k_nid_reduce after the launch
int g_nid_fold = 1;
static const char *kPhaseNames[PH_COUNT] = {"pre", "scalars", "lambda", "pg", "ozprep", "gram",
                                            "xu", "reduce", "form", "chol", "solve", "beta",
                                            "xb", "alpha", "nid", "eapply", "end"};

struct bb_engine {
    bb_config cfg{};
    int n = 0, p = 0, p_loc = 0, n_pad = 0, p_pad = 0;
    // p x p systems (methods 1, 6): factored at round_up(p, 64) inside the p_pad-strided
    // buffers, so a p = 64 design is one block step, not p_pad / 64 = 4
    int chol_m = 0;
    int method = 0;  // 1 chol, 2 woodbury, 3 ortho, 4 triangle mixture, 5 sparse woodbury,
                     // 6 logistic (Polya-Gamma)
    int group = 1;
    bool fused = false;  // small p: whole sweeps in one launch (bb_small.hip)
    SparseDesign spd;  // method 5: CSC/CSR design and the Gram pair list
    Hyper hy{};
    hipStream_t stream = nullptr;
    std::vector<void *> owned;

    double *X = nullptr, *y = nullptr;
    double *beta = nullptr, *lam = nullptr, *D = nullptr, *u = nullptr;
    DevScalars *sc = nullptr;
    uint32_t *err = nullptr;
    double *xb_part = nullptr, *red1 = nullptr;
    double *red3 = nullptr;  // sharded alpha MH: [S(alpha_new), S(alpha_old)]
    int nparts = 0, nbS = 0;
    bool xb_stale = false;  // a fused run left the X beta partials behind beta
    // woodbury
    double *slabs = nullptr, *xu_part = nullptr, *red2 = nullptr, *M = nullptr, *w = nullptr,
           *Wd = nullptr;
    unsigned int *flags = nullptr;
    int S = 1;
    size_t slab_stride = 0;
    // Ozaki-II Gram (gram_mode 1)
    int n_oz = 0, oz_b = 0, oz_S = 1;
    double *oz_xmax = nullptr, *oz_rscale = nullptr;
    double *oz_rowmax = nullptr;  // per chunk-group row maxima (launch_oz_scale scratch)
    int *oz_escale = nullptr;
    int8_t *oz_R = nullptr, *oz_P = nullptr;
    // logistic: X' resident for X'Omega X, omega, kappa = y - 1/2, the per-sweep Gram
    double *Xt = nullptr, *omega = nullptr, *kappa = nullptr, *Gw = nullptr;
    // chol / ortho
    double *G = nullptr, *cvec = nullptr, *A = nullptr, *Y2 = nullptr, *W2 = nullptr,
           *gdiag = nullptr;
    // triangle mixture: design basis (bb_tri.hip), omega in lam, shape in D, u in u
    double *tVc = nullptr, *tVr = nullptr, *tri_a = nullptr, *tri_d = nullptr,
           *tri_G = nullptr;
    double *tr_u = nullptr, *tr_shape = nullptr;
    std::vector<double> h_tV, h_a, h_d;
    // traces
    double *tr_beta = nullptr, *tr_lam = nullptr, *tr_sig2 = nullptr, *tr_tau = nullptr,
           *tr_alpha = nullptr;
    int cap = 1;
    // near-identity solve of the Woodbury system (bb_nid.hip): column norms,
    // the device decision word, Chebyshev vectors (x is w), E-apply partials, the host-mapped
    // eps of the latest decided sweep (the launch hint) and the enqueue throttle
    double *cn = nullptr;
    NidState *nid = nullptr;
    double *ch_r = nullptr, *ch_d = nullptr, *ea_part = nullptr, *sp_s = nullptr,
           *nid_xu = nullptr;
    double *eps_host = nullptr;  // ring of kNidRing: eps of sweep q in slot q % kNidRing
    // the mixed-precision plan (unsharded dense engines): X rounded to fp32 (n_pad x p_loc,
    // ld n_pad; nullptr when not held), the right-hand side kept for the residual pass, and the
    // correction iterates the latest sweep's decision asked for (0: the fp64 plan)
    float *X32 = nullptr;
    double *ch_b = nullptr;
    int nid_k2 = 0;
    double nid_cost[3] = {0.0, 0.0, 0.0};  // NidState c64, c32, cstep (s)
    int ea_parts = 1;
    int nid_kmax = 0;  // iterations beyond which the Gram + Cholesky path is cheaper (model)
    double lambda_x = 0.0;  // certified lambda_max(X X') bound (0: none)
    // decided-sweep events (after the decision of sweep q, slot q % kNidRing) and the number of
    // Woodbury sweeps enqueued since init_state (q)
    hipEvent_t nid_ev[8] = {};
    long nid_seq = 0;
    // column shards (world > 1): the bound sums exchanged before the decision, the reduced
    // X u / E d vector, the decision event the host waits on, whether this sweep took the
    // Chebyshev path, and membership of an on-device shard group (its exchanges are the
    // group's reduce; RCCL ranks and RCCL group members exchange through their communicator)
    double *nid_red = nullptr, *nid_sum = nullptr, *nid_wg = nullptr;
    hipEvent_t nid_sev = nullptr;
    bool nid_only = false;
    bool group_member = false;
    int nid_last = -1;  // the previous sweep's decided K (-1: none since init_state)
    // communicator (own_comm false: lent by an RCCL shard group, which destroys it)
    ncclComm_t comm = nullptr;
    bool own_comm = true;
    // timing: per-sweep event marks at phase starts, on the engine stream
    bool timing = false;
    int timing_level = 2;  // 1: one phase's bracket only (timed_phase), 2: every phase
    int timed_phase = PH_GRAM;
    int timing_stride = 1;  // level 1: bracket every timing_stride-th sweep
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::vector<std::pair<int, int>>> sweep_marks;  // (phase, event)
    size_t ev_next = 0;

    void mark(int phase) {
        if (!timing) return;
        // level 1: only the timed phase's bracket (its start and the next mark), so a timed
        // run carries two events per sweep instead of one per phase
        if (timing_level == 1) {
            if ((sweep_marks.size() - 1) % (size_t)timing_stride != 0) return;
            const bool open = !sweep_marks.back().empty() &&
                              sweep_marks.back().back().first == timed_phase;
            if (phase != timed_phase && !open) return;
        }
        int e0 = ev();
        HIPCHECK(hipEventRecord(ev_pool[e0], stream));
        sweep_marks.back().push_back({phase, e0});
    }

    ~bb_engine() {
        if (stream) (void)hipStreamSynchronize(stream);
        if (comm && own_comm) ncclCommDestroy(comm);
        for (auto e : ev_pool) (void)hipEventDestroy(e);
        for (auto e : nid_ev)
            if (e) (void)hipEventDestroy(e);
        if (nid_sev) (void)hipEventDestroy(nid_sev);
        if (eps_host) (void)hipHostFree(eps_host);
        for (void *q : owned) (void)hipFree(q);
        if (stream) (void)hipStreamDestroy(stream);
    }

    int ev() {
        if (ev_next == ev_pool.size()) {
            hipEvent_t e;
            HIPCHECK(hipEventCreate(&e));
            ev_pool.push_back(e);
        }
        return (int)ev_next++;
    }

    void allreduce(double *buf, size_t count) {
        if (cfg.world <= 1 && !comm) return;  // a 1-rank communicator still runs (testing)
        if (!comm) throw HipError("world > 1 but no communicator (call bb_engine_comm_init)");
        NCCLCHECK(ncclAllReduce(buf, buf, count, ncclFloat64, ncclSum, comm, stream));
    }

    double *slot_ptr(double *base, int slot, int stride) {
        if (slot < 0 || base == nullptr) return nullptr;
        return base + (size_t)(slot % cap) * stride;
    }

    bool woodbury() const { return method == 2 || method == 5; }

    // the near-identity path: an unsharded Woodbury engine (a one-member RCCL group included:
    // nothing is exchanged) decides on the device against a launch hint; column shards
    // (world > 1, exchanging through a communicator or an on-device group) decide from the
    // reduced bound sums and the host waits for that decision (nid_sync)
    bool nid_enabled() const {
        return nid != nullptr && (cfg.world == 1 || comm != nullptr || group_member) &&
               std::min(g_nid_kmax, nid_kmax) > 0;
    }
    // this engine runs the column-shard protocol of the near-identity solve (exchanged bound
    // sums, the decision from them, exchanged X u and products): world > 1, or world == 1 with
    // a communicator / in a group when forced for testing (g_shard_proto)
    bool sharded() const {
        return cfg.world > 1 || (g_shard_proto && (comm != nullptr || group_member));
    }
    bool nid_sync() const { return (sharded() || g_nid_sync) && nid_enabled(); }
    // the mixed-precision plan may be chosen by this engine's decision: an unsharded dense
    // engine that holds X32 (shards and shard-group members decide the fp64 plan only, so
    // every rank runs the same collectives)
    bool mixed_ok() const {
        return X32 != nullptr && g_nid_mixed && !sharded() && !group_member && method == 2;
    }
    // the exchanged vectors are single n-vectors on a shard; an unsharded engine in the
    // synchronous mode reads the partials directly
    bool nid_vec() const { return sharded() || method == 5; }

    // Cost model of the two exact solves, from the round-3/4 measured rates:
    // a Chebyshev solve of K iterates reads X K times (the X u pass and K - 1 products, ~6 TB/s
    // dense, ~3 TB/s for the sparse gathers, plus ~10 us of launches and the recurrence per
    // pass); the Gram + Cholesky path costs the Gram (Ozaki int8 GEMM at ~2.6 POP/s and its
    // 24 B per X element of residue traffic at ~5 TB/s; the fp64 MFMA Gram at ~33 TF/s; the
    // sparse pair stream at ~4 TB/s) plus ~19 us per 64-column block step of the factor and
    // solve.  Returns the largest K for which the Chebyshev solve is the cheaper one.
    int nid_kmax_model() const {
        double t_pass, t_chol;
        const double steps = n_pad / 64.0;
        if (method == 5) {
            t_pass = 24.0 * (double)spd.nnz / 3.0e12 + 10e-6;
            t_chol = 10.0 * (double)spd.pairs / 4.0e12 + steps * 21e-6 + 60e-6;
        } else {
            t_pass = 8.0 * n_pad * (double)p_loc / 6.0e12 + 10e-6;
            const double gram = cfg.gram_mode == 1
                ? 16.0 * (double)n_pad * n_pad * p_pad / 2.6e15 + 24.0 * (double)n_pad * p_pad / 5.0e12
                : 2.0 * (double)n_pad * n_pad * p_pad / 33e12;
            t_chol = gram + steps * 19e-6 + 40e-6;
        }
        if (cfg.world > 1) {
            // shards: an n-vector all-reduce per pass; the packed Gram's all-reduce (~100 GB/s
            // effective over xGMI rings) and the replicated factor on the other side
            t_pass += 25e-6;
            t_chol += 8.0 * (double)red2_count() / 100e9 + 25e-6;
        }
        return (int)std::min(64.0, std::floor(t_chol / t_pass));
    }

    // Chebyshev iterations to launch for Woodbury sweep q: from eps of sweep q - kNidLag
    // (host-mapped ring; the host waits for that sweep's decision, so it stays at most
    // kNidLag sweeps ahead of the device -- no bubble, the device has that many queued) with
    // an 8x growth margin; the first kNidLag sweeps after init_state: the maximum; beyond the
    // maximum: 0 (only the Gram + Cholesky path is launched).  The device decides sweep q
    // itself (k_nid_reduce): K iterates needed > launched makes it take the Gram + Cholesky
    // path, never a wrong w.  The hint is eps of a fixed earlier sweep, so the path a sweep
    // takes -- and its bits -- depend only on the chain, not on host / device timing.
    static constexpr int kNidRing = 8, kNidLag = 3;
    int nid_launch_count() {
        const int kmax = std::min(g_nid_kmax, nid_kmax);
        if (nid_seq < kNidLag) return kmax;
        const long q = nid_seq - kNidLag;
        wait_event(nid_ev[q % kNidRing]);
        const double h = ((volatile double *)eps_host)[q % kNidRing];
        if (!(h >= 0.0)) return kmax;
        return cheb_iterations(8.0 * h, kmax, kNidTol);
    }

    // decision kernel of a Woodbury sweep (eps is tracked even when only the Gram + Cholesky
    // path is launched, so the hint follows the chain back into the near-identity regime)
    int nid_begin(int kl) {
        if (!nid_enabled()) return 0;
        mark(PH_NID);
        const long q = nid_seq++;
        launch_nid_sums(stream, D, cn, p_loc, sc, nid, kl, kl > 0, 1, nid_wg, nid_red,
                        eps_dev + q % kNidRing);
        hipEvent_t &ev = nid_ev[q % kNidRing];
        if (!ev) HIPCHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        HIPCHECK(hipEventRecord(ev, stream));
        return kl;
    }
    double *eps_dev = nullptr;  // device view of eps_host

    // the Chebyshev solve (kl iterations launched, the device runs mode of them); x is w
    void nid_solve(uint64_t t, int kl) {
        mark(PH_NID);
        if (method == 5)
            launch_cheb_init(stream, nid_xu, 1, n, n_pad, y, sc, cfg.seed, cfg.stream, t, nid, w,
                             ch_r, ch_d);
        else
            launch_cheb_init(stream, nid_xu, xu_fused ? xu_fused : ea_parts, n, n_pad, y, sc,
                             cfg.seed, cfg.stream, t, nid, w, ch_r, ch_d);
        for (int j = 1; j < kl; ++j) {
            mark(PH_EAPPLY);
            if (method == 5)
                launch_sp_eapply(stream, spd.colptr, spd.rowidx, spd.cval, spd.rowptr, spd.colidx,
                                 spd.rval, p_loc, n_pad, D, ch_d, nid, j, sp_s, ea_part);
            else
                launch_eapply(stream, X, n_pad, n_pad, p_loc, D, ch_d, nid, j, ea_part);
            mark(PH_NID);
            launch_cheb_step(stream, ea_part, method == 5 ? 1 : ea_parts, n_pad, sc, nid, j, w,
                             ch_r, ch_d);
        }
    }

    // ---- column shards (nid_sync): the stages between the exchanges of a Woodbury sweep ----
    static constexpr int kNidRed = kNidTS + 2;
    // this shard's bound sums into nid_red (exchanged: kNidRed doubles); an unsharded engine
    // decides in the same launch (its sums need no exchange)
    // folded: the split lambda launch formed the sums (1: its nstream partials in nid_wg, reduced
    // here; 2: reduced and decided as well)
    void nidx_partials(int folded = 0, int nstream = 0) {
        mark(PH_NID);
        if (folded == 2) return;
        if (folded == 1 && sharded())
            launch_nid_reduce(stream, nid_wg, nstream, sc, nid, nid_red);
        else if (folded == 1)
            launch_nid_reduce(stream, nid_wg, nstream, sc, nid, nid_red,
                              std::min(g_nid_kmax, nid_kmax), eps_dev + kNidRing,
                              mixed_ok() ? 1 : 0, ++nid_dseq);
        else if (sharded())
            launch_nid_sums(stream, D, cn, p_loc, sc, nid, 0, 0, 0, nid_wg, nid_red, nullptr);
        else
            launch_nid_sums_decide(stream, D, cn, p_loc, sc, nid, std::min(g_nid_kmax, nid_kmax),
                                   nid_wg, nid_red, eps_dev + kNidRing, mixed_ok() ? 1 : 0,
                                   ++nid_dseq);
    }
    // the decision from the reduced sums (identical on every rank), then wait for it
    void nidx_decide_launch() {
        if (sharded())
            launch_nid_decide_from(stream, nid_red, sc, std::min(g_nid_kmax, nid_kmax), nid,
                                   eps_dev + kNidRing, ++nid_dseq);
        if (g_nid_poll) return;
        if (!nid_sev) HIPCHECK(hipEventCreateWithFlags(&nid_sev, hipEventDisableTiming));
        HIPCHECK(hipEventRecord(nid_sev, stream));
    }
    int nidx_decide_read() {
        int mode, k2;
        if (g_nid_poll) {
            const unsigned long long tag = wait_tag(nid_dseq);
            mode = (int)((tag >> 8) & 0xff);
            k2 = (int)(tag & 0xff);
        } else {
            wait_event(nid_sev);
            mode = (int)((volatile double *)eps_host)[kNidRing + 1];
            k2 = (int)((volatile double *)eps_host)[kNidRing + 2];
        }
        nid_k2 = mixed_ok() ? k2 : 0;
        return mode;
    }
    // Poll the decision's tag word (host2[3]: seq << 16 | mode << 8 | k2, one 64-bit store by
    // the decision kernel into coherent host memory) until it carries decision seq.  Every
    // 1024 polls the stream is queried: a device error surfaces as the HIP error, and a drained
    // stream without the tag is an error (never a silent wrong path); a shard-group member
    // gives up when another member failed (wait_event).
    unsigned long long wait_tag(unsigned long long seq) {
        const unsigned long long *tp = (const unsigned long long *)(eps_host + kNidRing + 3);
        const unsigned long long want = seq & 0xffffffffffffull;
        for (long spin = 0;; ++spin) {
            const unsigned long long v = __atomic_load_n(tp, __ATOMIC_ACQUIRE);
            if ((v >> 16) == want) return v;
            if ((spin & 1023) != 1023) {
                __builtin_ia32_pause();
                continue;
            }
            if (stop && stop->load(std::memory_order_relaxed))
                throw HipError("stopped: another member of the shard group failed");
            const hipError_t q = hipStreamQuery(stream);
            if (q == hipSuccess) {
                const unsigned long long w = __atomic_load_n(tp, __ATOMIC_ACQUIRE);
                if ((w >> 16) == want) return w;
                throw HipError("near-identity decision tag not written by the drained stream");
            }
            if (q != hipErrorNotReady) HIPCHECK(q);
            if (spin > 65536) std::this_thread::yield();
        }
    }
    unsigned long long nid_dseq = 0;  // decisions launched with a tag
    // Block the host until ev completes.  A member of an RCCL group (stop != nullptr) polls
    // instead, so that it gives up when another member failed: that member's all-reduces are
    // never posted, so an event behind them never completes (the group then aborts the
    // communicators once every member thread has returned, bb_group_run).
    void wait_event(hipEvent_t ev) {
        if (!stop) {
            HIPCHECK(hipEventSynchronize(ev));
            return;
        }
        for (long spin = 0;; ++spin) {
            const hipError_t q = hipEventQuery(ev);
            if (q == hipSuccess) return;
            if (q != hipErrorNotReady) HIPCHECK(q);
            if (stop->load(std::memory_order_relaxed))
                throw HipError("stopped: another member of the shard group failed");
            if (spin > 64) std::this_thread::yield();
        }
    }
    // this shard's X u into nid_sum (exchanged: n_pad)
    void nidx_xu() {
        mark(PH_NID);
        if (method == 5) {
            launch_sp_nid_xu(stream, spd.rowptr, spd.colidx, spd.rval, n_pad, u, nid, nid_sum);
        } else {
            if (!xu_fused) launch_nid_xu(stream, X, n_pad, u, p_loc, n_pad, nid, nid_xu);
            if (nid_vec())
                launch_part_sum(stream, nid_xu, xu_fused ? xu_fused : ea_parts, n_pad, nid_sum);
        }
    }
    void nidx_init(uint64_t t) {
        if (nid_vec())
            launch_cheb_init(stream, nid_sum, 1, n, n_pad, y, sc, cfg.seed, cfg.stream, t, nid,
                             w, ch_r, ch_d);
        else
            launch_cheb_init(stream, nid_xu, xu_fused ? xu_fused : ea_parts, n, n_pad, y, sc,
                             cfg.seed, cfg.stream, t, nid, w, ch_r, ch_d,
                             mixed_ok() ? ch_b : nullptr);
    }
    // the mixed plan's residual pass, restart and correction solve (k2 iterates), after the
    // first solve's products
    void nidx_mixed_tail(int k2) {
        mark(PH_EAPPLY);
        launch_eapply(stream, X, n_pad, n_pad, p_loc, D, w, nid, 0, ea_part, X32, 2);
        mark(PH_NID);
        launch_cheb_restart(stream, ea_part, ea_parts, n_pad, sc, nid, ch_b, w, ch_r, ch_d);
        for (int j = 1; j < k2; ++j) {
            mark(PH_EAPPLY);
            launch_eapply(stream, X, n_pad, n_pad, p_loc, D, ch_d, nid, j, ea_part, X32, 3);
            mark(PH_NID);
            launch_cheb_step(stream, ea_part, ea_parts, n_pad, sc, nid, j, w, ch_r, ch_d, 2);
        }
    }
    // this shard's E d of step j into nid_sum (exchanged: n_pad)
    void nidx_eapply(int j) {
        mark(PH_EAPPLY);
        if (method == 5) {
            launch_sp_eapply(stream, spd.colptr, spd.rowidx, spd.cval, spd.rowptr, spd.colidx,
                             spd.rval, p_loc, n_pad, D, ch_d, nid, j, sp_s, nid_sum);
        } else {
            launch_eapply(stream, X, n_pad, n_pad, p_loc, D, ch_d, nid, j, ea_part,
                          mixed_ok() ? X32 : nullptr);
            if (nid_vec()) launch_part_sum(stream, ea_part, ea_parts, n_pad, nid_sum);
        }
    }
    void nidx_step(int j) {
        mark(PH_NID);
        if (nid_vec())
            launch_cheb_step(stream, nid_sum, 1, n_pad, sc, nid, j, w, ch_r, ch_d);
        else
            launch_cheb_step(stream, ea_part, ea_parts, n_pad, sc, nid, j, w, ch_r, ch_d);
    }
    // a shard's Woodbury sweep between phase b and phase c, through exchange(buf, count)
    template <class Exchange>
    void shard_solve(uint64_t t, Exchange exchange) {
        if (!nid_sync()) {
            exchange(red2, red2_count());
            return;
        }
        exchange(nid_red, (size_t)kNidRed);
        nidx_decide_launch();
        // The start of the Chebyshev solve is enqueued before the host waits for the
        // decision -- X u, the initial iterate and one product, each returning at once unless
        // the device decided so -- so the device runs them while the host wakes up (no bubble
        // on the common near-identity sweep); the rest follows the decision.  A shard's two
        // exchanges among them run on every rank whatever the decision (the same sequence of
        // collectives everywhere; on a factor sweep they carry unused vectors).
        const int spec = g_nid_sync != 2 ? 2 : 0;
        if (spec) {
            nidx_xu();
            if (sharded()) exchange(nid_sum, (size_t)n_pad);
            nidx_init(t);
            nidx_eapply(1);
            if (sharded()) exchange(nid_sum, (size_t)n_pad);
            nidx_step(1);
        }
        const int K = nidx_decide_read();
        nid_only = K > 0;
        nid_last = K;
        if (K > 0) {
            if (!spec) {
                nidx_xu();
                exchange(nid_sum, (size_t)n_pad);
                nidx_init(t);
            }
            for (int j = spec ? spec : 1; j < K; ++j) {
                nidx_eapply(j);
                exchange(nid_sum, (size_t)n_pad);
                nidx_step(j);
            }
            if (nid_k2 > 0) nidx_mixed_tail(nid_k2);  // unsharded: exchange() is a no-op
        } else {
            wb_gram(nullptr);
            exchange(red2, red2_count());
        }
    }

    // X beta of the current beta into the partials k_pre sums next
    void xbeta() {
        xb_stale = false;
        if (method == 5) {
            launch_sp_rows(stream, spd.rowptr, spd.colidx, spd.rval, n_pad, beta, nullptr,
                           xb_part, nullptr);
            nparts = 1;
        } else {
            launch_xv(stream, X, n_pad, beta, p_loc, n_pad, xb_part);
            nparts = xv_chunks(p_loc, n_pad);
        }
    }

    void pre_and_scalars(uint64_t t, int slot, int tau_only) {
        if (xb_stale) xbeta();
        launch_pre(stream, xb_part, nparts, n_pad, beta, p_loc, sc, red1, nbS);
        allreduce(red1, (size_t)nbS + n_pad);
        launch_scalars(stream, red1, nbS, y, n, p, sc, hy, cfg.seed, cfg.stream, t,
                       slot_ptr(tr_tau, slot, 1), slot_ptr(tr_sig2, slot, 1),
                       slot_ptr(tr_alpha, slot, 1), tau_only, err);
    }

    // A sweep is three phases separated by the two exchange points of the column-sharded
    // decomposition: red1 = [S_alpha partials | X beta] and
    // red2 = [partial Gram | X u].  Single engines and RCCL ranks run them back to back
    // through allreduce(); a shard group (bb_group_*) interleaves its members' phases.
    void phase_a(uint64_t t) {
        (void)t;
        if (timing) sweep_marks.emplace_back();
        mark(PH_PRE);
        if (xb_stale) xbeta();
        launch_pre(stream, xb_part, nparts, n_pad, beta, p_loc, sc, red1, nbS);
    }

    // this shard's (or the whole) Gram X D X' with X u into red2 (packed upper triangle, then
    // the n-vector); gate: the near-identity decision word (its kernels skip on mode != 0)
    void wb_gram(const int *gate) {
        if (method == 5) {
            mark(PH_GRAM);
            spd.gram(stream, D, u, red2, red2 + tri_count(n_pad), gate);
            return;
        }
        if (cfg.gram_mode == 1) {
            mark(PH_OZPREP);
            launch_oz_scale(stream, D, p_pad, oz_xmax, n_oz, oz_b, oz_rowmax, oz_rscale,
                            oz_escale, gate);
            // the residue pass over X also forms the X u partials
            launch_oz_residues(stream, X, n_pad, n_pad, n_oz, p_pad, D, oz_rscale, oz_R, u,
                               xu_part, gate);
            mark(PH_GRAM);
            launch_oz_gemm(stream, oz_R, n_oz, p_pad, oz_S, oz_P, 0, kOzLeadDefault, -1, gate);
        } else {
            mark(PH_GRAM);
            launch_gram(stream, X, n_pad, D, n_pad, p_pad, S, slabs, n_pad, slab_stride, gate);
            mark(PH_XU);
            launch_xv(stream, X, n_pad, u, p_pad, n_pad, xu_part, gate);
        }
        mark(PH_REDUCE);
        if (cfg.gram_mode == 1)
            launch_oz_crt(stream, oz_P, oz_S, n_oz, n_pad, oz_escale, xu_part,
                          oz_xu_parts(p_pad, n_oz), red2, gate);
        else
            launch_slab_sum(stream, slabs, S, slab_stride, n_pad, xu_part, xv_chunks(p_pad, n_pad),
                            red2, 1, gate);
    }

    void phase_b(uint64_t t, int slot) {
        mark(PH_SCALARS);
        launch_scalars(stream, red1, nbS, y, n, p, sc, hy, cfg.seed, cfg.stream, t,
                       slot_ptr(tr_tau, slot, 1), slot_ptr(tr_sig2, slot, 1),
                       slot_ptr(tr_alpha, slot, 1), 0, err);
        double *trl = slot_ptr(tr_lam, slot, p_loc);
        mark(PH_LAMBDA);
        if (method == 5 || method == 2) {
            const bool sync = nid_sync();
            const int kl = (!sync && nid_enabled()) ? nid_launch_count() : 0;
            // a sweep that may take the Chebyshev path draws lambda and forms the X u partials
            // in one launch (k_lambda_xu, dense); under the synchronous protocol unless the
            // previous sweep took the factor (then X u would be streamed for nothing: the
            // residue pass forms it; a sweep that turns back to the Chebyshev path streams X u
            // in its own pass)
            xu_fused = 0;
            int folded = 0;
            if (method == 2 && (sync ? nid_last != 0 : kl > 0)) {
                // under the synchronous protocol the split launch also forms the bound sums
                // (and, unsharded, decides): k_nid_sums / k_nid_reduce are not launched
                NidFold fold;
                if (sync && g_nid_fold) {
                    fold.cn = cn;
                    fold.wg_part = nid_wg;
                    fold.cnt = lam_sync + lambda_xs_sync_words(p_pad);
                    fold.decide = (!sharded() && g_nid_fold == 2) ? 1 : 0;
                    fold.k_launched = std::min(g_nid_kmax, nid_kmax);
                    fold.allow_mixed = mixed_ok() ? 1 : 0;
                    fold.nid = nid;
                    fold.red = nid_red;
                    fold.host2 = eps_dev + kNidRing;
                    fold.tag_seq = nid_dseq + 1;
                }
                xu_fused = launch_lambda_xu(stream, beta, p_loc, p_pad, (uint64_t)cfg.j0, sc,
                                            cfg.seed, cfg.stream, t, lam, D, u, trl, err, X,
                                            n_pad, n_pad, nid_xu, lam_sync, ++lam_ep, &fold,
                                            &folded);
                if (folded == 2) ++nid_dseq;
            }
            if (!xu_fused)
                launch_lambda(stream, beta, p_loc, p_pad, (uint64_t)cfg.j0, sc, cfg.seed,
                              cfg.stream, t, LAMBDA_WOODBURY, group, lam, D, u, trl, err);
            ++(xu_fused ? n_lambda_xu : n_lambda_alone);
            nid_only = false;
            if (sync) {
                // a shard: the bound sums now, the path after their exchange (shard_solve)
                nid_kl = 0;
                nidx_partials(folded, xu_fused);
                return;
            }
            nid_kl = nid_begin(kl);
            wb_gram(nid_kl ? &nid->mode : nullptr);
            if (nid_kl && !xu_fused) {
                mark(PH_NID);
                if (method == 5)
                    launch_sp_nid_xu(stream, spd.rowptr, spd.colidx, spd.rval, n_pad, u, nid,
                                     nid_xu);
                else
                    launch_nid_xu(stream, X, n_pad, u, p_loc, n_pad, nid, nid_xu);
            }
        } else if (method == 6) {
            // omega_i ~ PG(1, x_i' beta), x_i' beta from red1 (k_pre's row sums): drawn by
            // trailing workgroups of the speculative lambda launch.  The logistic engine caps
            // p at 16384 (engine create), inside that launch's range (kLamSpecMax).
            if (!launch_lambda_pg(stream, beta, p_loc, p_pad, 0, sc, cfg.seed, cfg.stream, t,
                                  group, lam, trl, red1 + nbS, n, n_pad, omega, err))
                throw HipError("logistic sweep: p beyond the fused lambda / Polya-Gamma launch");
            if (cfg.gram_mode == 1) {
                // X'Omega X = Y Y', Y = X' diag(sqrt(omega)): the Ozaki-II Gram of the
                // resident transpose (rows = coefficients, K = observations)
                mark(PH_OZPREP);
                launch_oz_scale(stream, omega, n_pad, oz_xmax, n_oz, oz_b, oz_rowmax, oz_rscale,
                                oz_escale);
                launch_oz_residues(stream, Xt, p_pad, p_pad, n_oz, n_pad, omega, oz_rscale, oz_R,
                                   nullptr, nullptr);
                mark(PH_GRAM);
                launch_oz_gemm(stream, oz_R, n_oz, n_pad, oz_S, oz_P);
                mark(PH_REDUCE);
                launch_oz_crt(stream, oz_P, oz_S, n_oz, p_pad, oz_escale, nullptr, 0, Gw);
            } else {
                mark(PH_GRAM);
                launch_gram(stream, Xt, p_pad, omega, p_pad, n_pad, S, slabs, p_pad, slab_stride);
                mark(PH_REDUCE);
                launch_slab_sum(stream, slabs, S, slab_stride, p_pad, nullptr, 0, Gw, 0);
            }
        } else if (method == 4) {
            // BridgeWrapper.cpp:166-168: omega, u, then the rtnorm_gibbs beta passes
            mark(PH_BETA);
            launch_tri_update(stream, beta, u, lam, D, p, tVc, tVr, tri_a, tri_d, tri_G, cvec,
                              cfg.ortho, sc, cfg.betaburn, cfg.seed, cfg.stream, t,
                              slot_ptr(tr_beta, slot, p_loc), slot_ptr(tr_u, slot, p_loc), trl,
                              slot_ptr(tr_shape, slot, p_loc), err);
        } else {
            launch_lambda(stream, beta, p_loc, p_pad, (uint64_t)cfg.j0, sc, cfg.seed, cfg.stream, t, LAMBDA_ONLY,
                          group, lam, nullptr, nullptr, trl, err);
        }
    }

    void phase_c(uint64_t t, int slot, int mcmc_phase) {
        double *trb = slot_ptr(tr_beta, slot, p_loc);
        bool xb_fused = false;
        if (method == 5 || method == 2) {
            // w = M^-1 (y / sig - v): the Gram + Cholesky path, or (nid_kl > 0 and the device
            // decided so) the Chebyshev solve -- the kernels of the other path return at once
            // (a shard that took the Chebyshev path solved it in shard_solve: nid_only)
            const int *gate = nid_kl ? &nid->mode : nullptr;
            if (!nid_only) {
                mark(PH_FORM);
                launch_form_m(stream, red2, n, n_pad, y, sc, cfg.seed, cfg.stream, t, M, n_pad,
                              n_pad, gate);
                mark(PH_CHOL);
                chol_factor(stream, M, n_pad, n_pad, 1, err, Wd, flags, nullptr, gate);
                mark(PH_SOLVE);
                chol_bsolve(stream, M, n_pad, n_pad, Wd, M + (size_t)n_pad * n_pad, w, 1, flags,
                            err, gate);
            }
            if (nid_kl) nid_solve(t, nid_kl);
        }
        if (method == 5) {
            mark(PH_BETA);
            launch_sp_beta(stream, spd.colptr, spd.rowidx, spd.cval, p_loc, w, u, D, sc, beta, trb);
        } else if (method == 2) {
            mark(PH_BETA);
            if (beta_xb_supported(n_pad)) {
                // beta and the X beta partials of the next sweep in one pass over X
                launch_beta_woodbury_xb(stream, X, n_pad, n_pad, w, u, D, sc, p_loc, beta, trb,
                                        xb_part);
                nparts = beta_xb_parts(p_loc);
                xb_fused = true;
            } else {
                launch_beta_woodbury(stream, X, n_pad, n_pad, w, u, D, sc, p_loc, beta, trb);
            }
        } else if (method == 1 || method == 6) {
            // logistic: A = X'Omega X + diag(lambda / tau^2) (sig2 = 1), c = X'kappa
            mark(PH_FORM);
            const int m = chol_m;  // round_up(p, 64) <= p_pad
            launch_form_a(stream, method == 6 ? Gw : G, p_pad, lam, sc, cvec, p, m, A, p_pad, m,
                          method == 6 && cfg.gram_mode == 1);
            mark(PH_CHOL);
            chol_factor(stream, A, p_pad, m, 1, err, Wd, flags);
            mark(PH_SOLVE);
            launch_chol_rhs(stream, A, p_pad, m, p, m, cfg.seed, cfg.stream, t, Y2);
            chol_bsolve(stream, A, p_pad, m, Wd, Y2, W2, 2, flags, err);
            mark(PH_BETA);
            launch_beta_chol(stream, W2, m, sc, p, beta, trb);
        } else if (method == 3) {
            mark(PH_BETA);
            launch_beta_ortho(stream, gdiag, cvec, lam, sc, p_loc, (uint64_t)cfg.j0, cfg.seed,
                              cfg.stream, t, beta, trb);
        }
        if (!xb_fused) {
            mark(PH_XB);
            xbeta();
        }
        if (!hy.know_alpha) {
            mark(PH_ALPHA);
            if (cfg.world > 1) {
                // a column shard: this shard's two sums, exchanged (red3) before phase_d
                launch_alpha_sums(stream, beta, p_loc, sc, cfg.seed, cfg.stream, t, red3);
                return;
            }
            // BridgeWrapper.cpp:272 (burn-in: alpha_a, alpha_b), :294 (MCMC: alpha_b, alpha_b
            // -- reference quirk kept), ortho :499/:519 (alpha_a, alpha_b).
            launch_alpha_mh(stream, beta, p, sc, alpha_prior_a(mcmc_phase), hy.alpha_b, cfg.seed,
                            cfg.stream, t, slot_ptr(tr_alpha, slot, 1));
        }
        mark(PH_END);
    }

    // triangle driver: (alpha_a, alpha_b) in both loops (BridgeWrapper.cpp:146,173)
    double alpha_prior_a(int mcmc_phase) const {
        return ((method <= 2 || method == 5) && mcmc_phase) ? hy.alpha_b : hy.alpha_a;
    }
    // a sharded chain with alpha unknown exchanges the MH sums between phase_c and phase_d
    bool alpha_exchange() const { return !hy.know_alpha && cfg.world > 1; }

    void phase_d(uint64_t t, int slot, int mcmc_phase) {
        if (!alpha_exchange()) return;
        launch_alpha_decide(stream, red3, p, sc, alpha_prior_a(mcmc_phase), hy.alpha_b, cfg.seed,
                            cfg.stream, t, slot_ptr(tr_alpha, slot, 1));
        mark(PH_END);
    }

    size_t red1_count() const { return (size_t)nbS + n_pad; }
    size_t red2_count() const { return tri_count(n_pad) + n_pad; }

    // RCCL shard-group members (bb_group_run): the group's stop flag, raised when another
    // member failed (its collectives will never be matched, so enqueueing more is pointless),
    // and the sweep index at which this member fails on purpose (bb_debug_fail_member)
    const std::atomic<bool> *stop = nullptr;
    int fail_at = -1;
    int nid_kl = 0;  // Chebyshev iterations launched for the sweep being enqueued
    int xu_fused = 0;  // X u partials formed by this sweep's lambda launch (k_lambda_xu), or 0
    unsigned int *lam_sync = nullptr;  // the split lambda launch's chunk flags and counter
    unsigned int lam_ep = 0;           // its launch epoch (flags are never cleared)
    unsigned long long n_lambda_xu = 0, n_lambda_alone = 0;  // Woodbury lambda launches by kind

    // `count` sweeps from t0 into slots first_slot + k slot_step (mod cap)
    void run(uint64_t t0, int count, int first_slot, int slot_step, int mcmc_phase) {
        if (fused) {
            if (timing) {
                sweep_marks.emplace_back();
                mark(PH_BETA);
            }
            if (method == 4)
                launch_tri_chain(stream, X, n_pad, n, p, y, tVc, tVr, tri_a, tri_d, tri_G, cvec,
                                 cfg.ortho, beta, u, lam,
                                 D, sc, hy, cfg.betaburn, cfg.seed, cfg.stream, t0, count,
                                 first_slot, slot_step, cap, tr_beta, tr_u, tr_lam, tr_shape,
                                 tr_sig2, tr_tau, tr_alpha, err);
            else
                launch_small_chain(stream, X, n_pad, n, p, y, G, p_pad, cvec, gdiag, method == 3,
                                   beta, lam, sc, hy, cfg.seed, cfg.stream, t0, count,
                                   first_slot, slot_step, cap, tr_beta, tr_lam, tr_sig2, tr_tau,
                                   tr_alpha, err);
            if (timing) mark(PH_END);
            xb_stale = true;  // X beta partials refreshed only if a general sweep needs them
            return;
        }
        for (int k = 0; k < count; ++k) {
            if (stop && stop->load(std::memory_order_relaxed)) break;
            if (k == fail_at) throw HipError("injected failure (bb_debug_fail_member)");
            const int slot = first_slot < 0 ? -1 : first_slot + k * slot_step;
            sweep(t0 + (uint64_t)k, slot, mcmc_phase);
        }
    }

    void sweep(uint64_t t, int slot, int mcmc_phase) {
        phase_a(t);
        allreduce(red1, red1_count());
        phase_b(t, slot);
        if (woodbury())
            shard_solve(t, [this](double *buf, size_t count) { allreduce(buf, count); });
        phase_c(t, slot, mcmc_phase);
        if (alpha_exchange()) {
            allreduce(red3, 2);
            phase_d(t, slot, mcmc_phase);
        }
    }

    uint32_t read_err() {
        uint32_t f = 0;
        HIPCHECK(hipMemcpyAsync(&f, err, sizeof(f), hipMemcpyDeviceToHost, stream));
        HIPCHECK(hipStreamSynchronize(stream));
        return f;
    }
    void clear_err() { HIPCHECK(hipMemsetAsync(err, 0, sizeof(uint32_t), stream)); }
};

namespace {

// Right singular vectors and singular values of X (n x p, column-major, n >= p) without
// forming X'X, whose condition number is the square of X's: Householder QR X = Q R on the
// host, then one-sided (Hestenes) Jacobi on the columns of R until every pair is orthogonal
// to fp64 precision.  R V = U diag(d) gives X = (Q U) diag(d) V'.  O(n p^2 + sweeps p^3).
void svd_right(const double *Xh, int n, int p, std::vector<double> &V, std::vector<double> &d) {
    std::vector<double> A(Xh, Xh + (size_t)n * p);
    auto col = [&](int j) { return &A[(size_t)j * n]; };
    for (int k = 0; k < p && k < n; ++k) {
        double *ak = col(k);
        double nrm = 0.0;
        for (int i = k; i < n; ++i) nrm += ak[i] * ak[i];
        nrm = sqrt(nrm);
        if (nrm == 0.0) continue;
        const double alpha = ak[k] >= 0 ? -nrm : nrm;
        ak[k] -= alpha;  // v = x - alpha e1 (stored in place)
        double vv = 0.0;
        for (int i = k; i < n; ++i) vv += ak[i] * ak[i];
        for (int j = k + 1; j < p; ++j) {
            double *aj = col(j);
            double sdot = 0.0;
            for (int i = k; i < n; ++i) sdot += ak[i] * aj[i];
            const double f = 2.0 * sdot / vv;
            for (int i = k; i < n; ++i) aj[i] -= f * ak[i];
        }
        ak[k] = alpha;
        for (int i = k + 1; i < n; ++i) ak[i] = 0.0;
    }
    // W = R (p x p), V = I
    std::vector<double> W((size_t)p * p, 0.0);
    for (int j = 0; j < p; ++j)
        for (int i = 0; i <= j && i < n; ++i) W[(size_t)j * p + i] = A[(size_t)j * n + i];
    V.assign((size_t)p * p, 0.0);
    for (int i = 0; i < p; ++i) V[(size_t)i * p + i] = 1.0;
    std::vector<double> nrm2(p);
    for (int sweep = 0; sweep < 80; ++sweep) {
        long rotated = 0;
        // squared column norms, refreshed every sweep and carried through each rotation
        // (||w_i'||^2 = a - t c, ||w_j'||^2 = b + t c)
        for (int j = 0; j < p; ++j) {
            double s2 = 0.0;
            for (int k = 0; k < p; ++k) s2 += W[(size_t)j * p + k] * W[(size_t)j * p + k];
            nrm2[j] = s2;
        }
        for (int i = 0; i < p - 1; ++i) {
            double *wi = &W[(size_t)i * p], *vi = &V[(size_t)i * p];
            for (int j = i + 1; j < p; ++j) {
                double *wj = &W[(size_t)j * p], *vj = &V[(size_t)j * p];
                const double a = nrm2[i], b = nrm2[j];
                double c = 0.0;
                for (int k = 0; k < p; ++k) c += wi[k] * wj[k];
                if (c == 0.0 || fabs(c) <= 1e-15 * sqrt(a * b)) continue;
                ++rotated;
                const double zeta = (b - a) / (2.0 * c);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                const double cs = 1.0 / sqrt(1.0 + t * t), sn = cs * t;
                nrm2[i] = a - t * c;
                nrm2[j] = b + t * c;
                for (int k = 0; k < p; ++k) {
                    const double x = wi[k], y = wj[k];
                    wi[k] = cs * x - sn * y;
                    wj[k] = sn * x + cs * y;
                    const double u = vi[k], w = vj[k];
                    vi[k] = cs * u - sn * w;
                    vj[k] = sn * u + cs * w;
                }
            }
        }
        if (rotated == 0) break;
    }
    d.resize(p);
    for (int j = 0; j < p; ++j) {
        double s2 = 0.0;
        for (int k = 0; k < p; ++k) s2 += W[(size_t)j * p + k] * W[(size_t)j * p + k];
        d[j] = sqrt(s2);
    }
}

// X = U diag(d) V' (BridgeRegression.cpp:47-57, svd 'S' for n > p): tV = V' with singular
// values in decreasing order, each right singular vector signed so its largest-magnitude
// entry is positive; a = d * U'y = V' X'y.
void tri_setup(bb_engine *e, const double *Xh) {
    const int p = e->p, pp = e->p_pad;
    std::vector<double> Gp((size_t)pp * pp), c(pp);
    HIPCHECK(hipStreamSynchronize(e->stream));
    HIPCHECK(hipMemcpy(Gp.data(), e->G, Gp.size() * sizeof(double), hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(c.data(), e->cvec, (size_t)pp * sizeof(double), hipMemcpyDeviceToHost));
    std::vector<double> G((size_t)p * p);
    for (int j = 0; j < p; ++j)
        for (int i = 0; i < p; ++i) {  // the device Gram holds the upper triangle
            const int r = i < j ? i : j, q = i < j ? j : i;
            G[(size_t)j * p + i] = Gp[(size_t)q * pp + r];
        }
    std::vector<double> V, sv;
    svd_right(Xh, e->n, p, V, sv);
    std::vector<int> ord(p);
    for (int i = 0; i < p; ++i) ord[i] = i;
    std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return sv[x] > sv[y]; });
    e->h_tV.assign((size_t)p * p, 0.0);
    e->h_a.assign(p, 0.0);
    e->h_d.assign(p, 0.0);
    std::vector<double> tVr((size_t)p * p);
    for (int i = 0; i < p; ++i) {
        const double *v = &V[(size_t)ord[i] * p];
        int jm = 0;
        for (int j = 1; j < p; ++j)
            if (fabs(v[j]) > fabs(v[jm])) jm = j;
        const double sg = v[jm] < 0 ? -1.0 : 1.0;
        double a = 0.0;
        for (int j = 0; j < p; ++j) {
            const double x = sg * v[j];
            e->h_tV[i + (size_t)j * p] = x;
            tVr[(size_t)i * p + j] = x;
            a += x * c[j];
        }
        e->h_a[i] = a;
        e->h_d[i] = sv[ord[i]];
    }
    auto &o = e->owned;
    e->tVc = dalloc<double>((size_t)p * p, o);
    e->tVr = dalloc<double>((size_t)p * p, o);
    e->tri_a = dalloc<double>(p, o);
    e->tri_d = dalloc<double>(p, o);
    HIPCHECK(hipMemcpy(e->tVc, e->h_tV.data(), (size_t)p * p * sizeof(double),
                       hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(e->tVr, tVr.data(), (size_t)p * p * sizeof(double), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(e->tri_a, e->h_a.data(), (size_t)p * sizeof(double), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(e->tri_d, e->h_d.data(), (size_t)p * sizeof(double), hipMemcpyHostToDevice));
    e->tri_G = dalloc<double>((size_t)p * p, o);  // full symmetric X'X (ortho variant)
    HIPCHECK(hipMemcpy(e->tri_G, G.data(), (size_t)p * p * sizeof(double), hipMemcpyHostToDevice));
    e->tr_u = dalloc<double>((size_t)p * e->cap, o);
    e->tr_shape = dalloc<double>((size_t)p * e->cap, o);
}

struct SparseIn {
    const int *colptr, *rowidx;
    const double *val;
};

// Certified upper bound Lambda >= lambda_max(X X') for the near-identity bound (bb_nid.hip
// k_nid_reduce): 40 power iterations on X X' (the E-apply pass with D = 1) give the Rayleigh
// quotient rho; U = 1.02 rho is certified by factoring U I - X X' (the Gram with D = 1, the
// device Cholesky): a non-positive pivot (error bit 8) raises U by 25 %, at most six times,
// after which the bound is left out (Lambda = 0: the trace bound alone).  The factor's
// backward error (~n u |A|) is far below the 2 % margin.  Setup only, ~10 ms at C3.
void nid_certify_lambda(bb_engine *e) {
    const int n_pad = e->n_pad, p_pad = e->p_pad;
    hipStream_t s = e->stream;
    double *ones = nullptr;
    NidState *gate = nullptr;
    HIPCHECK(hipMalloc(&ones, (size_t)p_pad * sizeof(double)));
    HIPCHECK(hipMalloc(&gate, sizeof(NidState)));
    std::vector<double> h1(p_pad, 0.0);
    for (int j = 0; j < e->p_loc; ++j) h1[j] = 1.0;
    HIPCHECK(hipMemcpyAsync(ones, h1.data(), h1.size() * sizeof(double), hipMemcpyHostToDevice, s));
    NidState g{};
    g.mode = 64;  // every pass of the power iteration runs
    HIPCHECK(hipMemcpyAsync(gate, &g, sizeof(g), hipMemcpyHostToDevice, s));
    std::vector<double> v(n_pad, 0.0), w(n_pad);
    double nv = 0.0;
    for (int i = 0; i < e->n; ++i) {
        v[i] = std::cos(0.7 * i + 0.3) + 0.5 * std::sin(1.3 * i * i + 0.1);
        nv += v[i] * v[i];
    }
    for (auto &x : v) x /= std::sqrt(nv);
    double rho = 0.0;
    for (int it = 0; it < 40; ++it) {
        HIPCHECK(hipMemcpyAsync(e->ch_d, v.data(), n_pad * sizeof(double), hipMemcpyHostToDevice, s));
        if (e->method == 5)
            launch_sp_eapply(s, e->spd.colptr, e->spd.rowidx, e->spd.cval, e->spd.rowptr,
                             e->spd.colidx, e->spd.rval, e->p_loc, n_pad, ones, e->ch_d, gate, 0,
                             e->sp_s, e->ea_part);
        else
            launch_eapply(s, e->X, n_pad, n_pad, e->p_loc, ones, e->ch_d, gate, 0, e->ea_part);
        launch_part_sum(s, e->ea_part, e->method == 5 ? 1 : e->ea_parts, n_pad, e->ch_r);
        HIPCHECK(hipMemcpyAsync(w.data(), e->ch_r, n_pad * sizeof(double), hipMemcpyDeviceToHost, s));
        HIPCHECK(hipStreamSynchronize(s));
        double vw = 0.0, ww = 0.0;
        for (int i = 0; i < n_pad; ++i) {
            vw += v[i] * w[i];
            ww += w[i] * w[i];
        }
        rho = vw;
        if (!(ww > 0.0)) break;
        for (int i = 0; i < n_pad; ++i) v[i] = w[i] / std::sqrt(ww);
    }
    double lam = 0.0;
    if (rho > 0.0 && std::isfinite(rho)) {
        // the Gram X X' into red2 (packed upper triangle)
        if (e->method == 5) {
            e->spd.gram(s, ones, ones, e->red2, e->red2 + tri_count(n_pad));
        } else if (e->cfg.gram_mode == 1) {
            launch_oz_scale(s, ones, p_pad, e->oz_xmax, e->n_oz, e->oz_b, e->oz_rowmax,
                            e->oz_rscale, e->oz_escale);
            launch_oz_residues(s, e->X, n_pad, n_pad, e->n_oz, p_pad, ones, e->oz_rscale, e->oz_R);
            launch_oz_gemm(s, e->oz_R, e->n_oz, p_pad, e->oz_S, e->oz_P);
            launch_oz_crt(s, e->oz_P, e->oz_S, e->n_oz, n_pad, e->oz_escale, nullptr, 0, e->red2);
        } else {
            launch_gram(s, e->X, n_pad, ones, n_pad, p_pad, e->S, e->slabs, n_pad, e->slab_stride);
            launch_slab_sum(s, e->slabs, e->S, e->slab_stride, n_pad, nullptr, 0, e->red2, 1);
        }
        double U = 1.02 * rho;
        for (int attempt = 0; attempt < 7 && lam == 0.0; ++attempt, U *= 1.25) {
            e->clear_err();
            launch_shift_gram(s, e->red2, n_pad, U, e->M, n_pad);
            chol_factor(s, e->M, n_pad, n_pad, 1, e->err, e->Wd, e->flags);
            if ((e->read_err() & (8u | 16u)) == 0) lam = U * (1.0 + 1e-9);
        }
        e->clear_err();
    }
    HIPCHECK(hipMemsetAsync(e->nid, 0, sizeof(NidState), s));
    HIPCHECK(hipMemcpyAsync(&e->nid->lambda_x, &lam, sizeof(double), hipMemcpyHostToDevice, s));
    HIPCHECK(hipMemcpyAsync(&e->nid->c64, e->nid_cost, sizeof(e->nid_cost), hipMemcpyHostToDevice,
                            s));
    HIPCHECK(hipStreamSynchronize(s));
    e->lambda_x = lam;
    (void)hipFree(ones);
    (void)hipFree(gate);
}

void engine_setup(bb_engine *e, const double *Xh, const double *yh, const SparseIn *spin) {
    const bb_config &c = e->cfg;
    e->n = c.n;
    e->p = c.p;
    e->p_loc = c.p_local;
    e->n_pad = round_up(c.n, kGramTile);
    e->p_pad = round_up(c.p_local, 256);
    e->chol_m = round_up(c.p_local, kNB);
    e->cap = c.trace_capacity < 1 ? 1 : c.trace_capacity;
    e->hy = Hyper{c.sig2_shape, c.sig2_scale, c.nu_shape, c.nu_rate, c.alpha_a, c.alpha_b,
                  c.true_tau > 0, c.true_sig2 > 0, c.true_alpha > 0};
    if (spin) {
        if (c.ortho || c.method == 1 || c.method == 3 || c.method == 4 || c.method == 6)
            throw HipError("a CSC design runs the Woodbury (p > n) draw only");
        e->method = 5;
    } else if (c.method == 6) {
        e->method = 6;
        e->hy.know_sig2 = 1;  // the PG mixture has unit scale
        // X'Omega X runs over K = n_pad rows: pad to 512 so the Gram can split K 16 ways
        e->n_pad = round_up(c.n, 512);
        if (c.world > 1) throw HipError("the logistic path runs on one device (world == 1)");
        if (c.ortho) throw HipError("the logistic path has no orthogonal-design variant");
        if (c.p > 16384) throw HipError("logistic path limited to p <= 16384");
    } else if (c.method == 4) e->method = 4;
    else if (c.ortho) e->method = 3;
    else if (c.method == 1 || (c.method == 0 && c.p <= c.n)) e->method = 1;
    else e->method = 2;
    // column shards: the p > n Woodbury draws (dense, sparse) and the orthogonal design
    // (per-coefficient draws, p > n); alpha known or unknown (the MH sums are exchanged)
    if (c.world > 1 && !e->woodbury() && !(e->method == 3 && c.p > c.n))
        throw HipError("column sharding (world > 1) is implemented for the p > n paths only "
                       "(Woodbury, sparse Woodbury, orthogonal design)");
    if (e->method == 4 && (c.p > c.n || c.p > kTriMaxP))
        throw HipError("triangle sampler needs p <= n and p <= 2048");
    if (e->method == 1 && c.p > 16384) throw HipError("p x p Cholesky path limited to p <= 16384");
    if (e->woodbury() && e->n_pad > 8192)
        throw HipError("Woodbury path limited to n <= 8192 in this build");

    HIPCHECK(hipSetDevice(c.device));
    HIPCHECK(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
    auto &o = e->owned;
    const int n_pad = e->n_pad, p_pad = e->p_pad;
    if (spin) {
        e->spd.build(e->stream, c.n, n_pad, c.p_local, spin->colptr, spin->rowidx, spin->val, o);
    } else {
        e->X = dalloc<double>((size_t)n_pad * p_pad, o);
        HIPCHECK(hipMemcpy2D(e->X, (size_t)n_pad * sizeof(double), Xh,
                             (size_t)c.n * sizeof(double), (size_t)c.n * sizeof(double),
                             (size_t)c.p_local, hipMemcpyHostToDevice));
    }
    e->y = dalloc<double>(n_pad, o);
    HIPCHECK(hipMemcpy(e->y, yh, (size_t)c.n * sizeof(double), hipMemcpyHostToDevice));
    e->beta = dalloc<double>(p_pad, o);
    e->lam = dalloc<double>(p_pad, o);
    e->D = dalloc<double>(p_pad, o);
    e->u = dalloc<double>(p_pad, o);
    e->sc = dalloc<DevScalars>(1, o);
    e->err = dalloc<uint32_t>(4, o);
    e->nparts = xv_chunks(p_pad, n_pad);
    e->xb_part = dalloc<double>(
        (size_t)std::max(e->method == 5 ? 1 : xv_chunks_max(p_pad), beta_xb_parts(c.p_local)) *
            n_pad,
        o);
    e->nbS = pre_blocks_s(c.p_local);
    e->red1 = dalloc<double>((size_t)e->nbS + n_pad, o);
    e->red3 = dalloc<double>(2, o);
    e->group = stable_group_for(c.p_local);
    e->tr_beta = dalloc<double>((size_t)c.p_local * e->cap, o);
    e->tr_lam = dalloc<double>((size_t)c.p_local * e->cap, o);
    e->tr_sig2 = dalloc<double>(e->cap, o);
    e->tr_tau = dalloc<double>(e->cap, o);
    e->tr_alpha = dalloc<double>(e->cap, o);

    if (e->method == 2) {
        if (c.gram_mode == 1) {
            e->n_oz = oz_rows(n_pad);
            const int nkc = p_pad / kOzKC;
            e->oz_b = oz_bits_for(p_pad);
            e->oz_S = oz_splits_for(e->n_oz, nkc);
            e->oz_xmax = dalloc<double>((size_t)nkc * e->n_oz, o);
            e->oz_rowmax = dalloc<double>((size_t)oz_bound_groups(p_pad) * e->n_oz, o);
            e->oz_rscale = dalloc<double>(e->n_oz, o);
            e->oz_escale = dalloc<int>(e->n_oz, o);
            e->oz_R = dalloc<int8_t>(oz_residue_bytes(e->n_oz, p_pad), o);
            e->oz_P = dalloc<int8_t>(oz_partial_bytes(e->n_oz, e->oz_S), o);
            launch_oz_xmax(e->stream, e->X, n_pad, n_pad, e->n_oz, p_pad, e->oz_xmax);
        } else {
            e->S = gram_splits_for(n_pad, p_pad);
            e->slab_stride = (size_t)n_pad * n_pad;
            e->slabs = dalloc<double>(e->slab_stride * e->S, o);
        }
        e->xu_part = dalloc<double>((size_t)xv_chunks_max(p_pad) * n_pad, o);
    }
    if (e->woodbury()) {
        e->red2 = dalloc<double>(tri_count(n_pad) + n_pad, o);
        e->M = dalloc<double>((size_t)n_pad * (n_pad + kNB), o);
        e->w = dalloc<double>(n_pad, o);
        // near-identity solve (bb_nid.hip); the dense E-apply keeps its rows in registers up
        // to n_pad = 4096
        if (e->method == 5 || eapply_supported(n_pad)) {
            e->cn = dalloc<double>(p_pad, o);
            if (e->method == 5) {
                std::vector<double> h(c.p_local, 0.0);
                for (int j = 0; j < c.p_local; ++j)
                    for (int q = spin->colptr[j]; q < spin->colptr[j + 1]; ++q)
                        h[j] += spin->val[q] * spin->val[q];
                HIPCHECK(hipMemcpy(e->cn, h.data(), h.size() * sizeof(double),
                                   hipMemcpyHostToDevice));
                e->sp_s = dalloc<double>(p_pad, o);
                e->ea_parts = 1;
                e->ea_part = dalloc<double>(n_pad, o);
                e->nid_xu = dalloc<double>(n_pad, o);
            } else {
                launch_colnorm2(e->stream, e->X, n_pad, n_pad, c.p_local, e->cn);
                e->ea_parts = eapply_parts(c.p_local, n_pad);
                e->ea_part = dalloc<double>((size_t)e->ea_parts * n_pad, o);
                const int xp = std::max(e->ea_parts, lambda_xu_parts(c.p_local, p_pad, n_pad));
                e->nid_xu = dalloc<double>((size_t)xp * n_pad, o);
                // + the folded decision's count (the last word)
                const int sw = lambda_xs_sync_words(p_pad) + 1;
                e->lam_sync = dalloc<unsigned int>(sw, o);
                HIPCHECK(hipMemsetAsync(e->lam_sync, 0, sizeof(unsigned int) * sw, e->stream));
            }
            e->nid = dalloc<NidState>(1, o);
            {
                // the Chebyshev plans' cost model (bb_nid.hip nid_plan_mixed; copied into the
                // NidState by nid_certify_lambda): a pass streams X at ~6.2 TB/s plus ~4 us of
                // launch and partials; a step launch ~6 us
                const double bytes = (double)n_pad * (double)c.p_local;
                e->nid_cost[0] = 8.0 * bytes / 6.2e12 + 4e-6;
                e->nid_cost[1] = 4.0 * bytes / 6.2e12 + 4e-6;
                e->nid_cost[2] = 6e-6;
            }
            e->ch_r = dalloc<double>(n_pad, o);
            e->ch_d = dalloc<double>(n_pad, o);
            e->nid_red = dalloc<double>(bb_engine::kNidRed, o);
            // k_nid_sums' partials, or the split lambda launch's (one per stream workgroup)
            e->nid_wg = dalloc<double>(
                (size_t)std::max(nid_sum_groups(c.p_local), 1024) * (kNidTS + 1), o);
            e->nid_sum = dalloc<double>(n_pad, o);
            // the hint ring, then [eps, mode, k2, tag] of the sweep being decided (coherent:
            // the host polls the tag while the device runs on)
            const int nh = bb_engine::kNidRing + 4;
            HIPCHECK(hipHostMalloc((void **)&e->eps_host, nh * sizeof(double),
                                   hipHostMallocMapped | hipHostMallocCoherent));
            for (int q = 0; q < nh; ++q) e->eps_host[q] = -1.0;  // no observation yet
            *(unsigned long long *)(e->eps_host + bb_engine::kNidRing + 3) = 0ull;
            HIPCHECK(hipHostGetDevicePointer((void **)&e->eps_dev, e->eps_host, 0));
            e->nid_kmax = e->nid_kmax_model();
            // the mixed-precision plan's fp32 copy of X (unsharded dense engines; 4 B per
            // element: 400 MB at C3), unless an entry is outside fp32's normal range
            // Only when the plan can be used (key 10 on, a Chebyshev path at all), and never
            // at the price of the engine: a failed allocation keeps the fp64 plan.
            if (e->method == 2 && c.world == 1 && g_nid_mixed && e->nid_kmax > 0) {
                void *x32 = nullptr;
                if (hipMalloc(&x32, (size_t)n_pad * p_pad * sizeof(float)) != hipSuccess) {
                    (void)hipGetLastError();  // clear the sticky out-of-memory status
                    x32 = nullptr;
                }
                if (x32) {
                    e->ch_b = dalloc<double>(n_pad, o);
                    int *bad = dalloc<int>(1, o);
                    HIPCHECK(hipMemsetAsync(bad, 0, sizeof(int), e->stream));
                    launch_cast_f32(e->stream, e->X, n_pad, n_pad, c.p_local, (float *)x32, bad);
                    int hb = 0;
                    HIPCHECK(hipMemcpyAsync(&hb, bad, sizeof(int), hipMemcpyDeviceToHost, e->stream));
                    HIPCHECK(hipStreamSynchronize(e->stream));
                    if (hb) {
                        (void)hipFree(x32);  // an entry outside fp32's normal range
                    } else {
                        o.push_back(x32);
                        e->X32 = (float *)x32;
                    }
                }
            }
        }
    }
    // X'X / X'y when the chol or ortho path needs them, or for the least-squares start.
    const bool small = c.p <= c.n && c.world == 1 && e->method != 5 && e->method != 6;
    // the Cholesky scratch covers the n x n (Woodbury) and any p x p (chol, LS start) system
    const int m_sys = (e->woodbury() && !small) ? n_pad : (n_pad > p_pad ? n_pad : p_pad);
    e->Wd = dalloc<double>(chol_wd_words(m_sys), o);
    e->flags = dalloc<unsigned int>(chol_flag_words(m_sys, 1), o);
    if (e->method == 6) {
        // logistic: X' resident (p_pad x n_pad), K-split slabs of X'Omega X, c = X'kappa
        e->Xt = dalloc<double>((size_t)p_pad * n_pad, o);
        launch_transpose(e->stream, e->X, n_pad, n_pad, p_pad, e->Xt, p_pad);
        if (c.gram_mode == 1) {
            // Ozaki-II X'Omega X (packed upper triangle into Gw): rows = p_pad, K = n_pad
            e->n_oz = oz_rows(p_pad);
            const int nkc = n_pad / kOzKC;
            e->oz_b = oz_bits_for(n_pad);
            e->oz_S = oz_splits_for(e->n_oz, nkc);
            e->oz_xmax = dalloc<double>((size_t)nkc * e->n_oz, o);
            e->oz_rowmax = dalloc<double>((size_t)oz_bound_groups(n_pad) * e->n_oz, o);
            e->oz_rscale = dalloc<double>(e->n_oz, o);
            e->oz_escale = dalloc<int>(e->n_oz, o);
            e->oz_R = dalloc<int8_t>(oz_residue_bytes(e->n_oz, n_pad), o);
            e->oz_P = dalloc<int8_t>(oz_partial_bytes(e->n_oz, e->oz_S), o);
            launch_oz_xmax(e->stream, e->Xt, p_pad, p_pad, e->n_oz, n_pad, e->oz_xmax);
        } else {
            e->S = gram_splits_for(p_pad, n_pad);
            e->slab_stride = (size_t)p_pad * p_pad;
            e->slabs = dalloc<double>(e->slab_stride * e->S, o);
        }
        e->Gw = dalloc<double>(std::max((size_t)p_pad * p_pad, tri_count(p_pad)) + p_pad, o);
        e->omega = dalloc<double>(n_pad, o);
        e->kappa = dalloc<double>(n_pad, o);
        launch_kappa(e->stream, e->y, c.n, n_pad, e->kappa);
        e->cvec = dalloc<double>(p_pad, o);
        launch_coldot(e->stream, e->X, n_pad, n_pad, e->kappa, c.p_local, e->cvec);
        e->A = dalloc<double>((size_t)p_pad * (p_pad + kNB), o);
        e->Y2 = dalloc<double>((size_t)2 * p_pad, o);
        e->W2 = dalloc<double>((size_t)2 * p_pad, o);
    } else if ((e->method != 2 && e->method != 5) || small) {
        e->cvec = dalloc<double>(p_pad, o);
        launch_coldot(e->stream, e->X, n_pad, n_pad, e->y, c.p_local, e->cvec);
        e->gdiag = dalloc<double>(p_pad, o);
        if (small) {
            // G = X'X: transpose X (n_pad x p_pad) into Xt (p_pad x n_pad), Gram over rows.
            double *Xt = nullptr;
            HIPCHECK(hipMalloc(&Xt, (size_t)p_pad * n_pad * sizeof(double)));
            launch_transpose(e->stream, e->X, n_pad, n_pad, p_pad, Xt, p_pad);
            double *ones = nullptr;
            HIPCHECK(hipMalloc(&ones, (size_t)n_pad * sizeof(double)));
            std::vector<double> h1(n_pad, 1.0);
            HIPCHECK(hipMemcpyAsync(ones, h1.data(), n_pad * sizeof(double),
                                    hipMemcpyHostToDevice, e->stream));
            const int Sg = gram_splits_for(p_pad, n_pad);
            double *sl = nullptr;
            HIPCHECK(hipMalloc(&sl, (size_t)Sg * p_pad * p_pad * sizeof(double)));
            launch_gram(e->stream, Xt, p_pad, ones, p_pad, n_pad, Sg, sl, p_pad,
                        (size_t)p_pad * p_pad);
            double *red = nullptr;
            HIPCHECK(hipMalloc(&red, ((size_t)p_pad * p_pad + p_pad) * sizeof(double)));
            launch_slab_sum(e->stream, sl, Sg, (size_t)p_pad * p_pad, p_pad, nullptr, 0, red, 0);
            e->G = dalloc<double>((size_t)p_pad * p_pad, o);
            HIPCHECK(hipMemcpyAsync(e->G, red, (size_t)p_pad * p_pad * sizeof(double),
                                    hipMemcpyDeviceToDevice, e->stream));
            HIPCHECK(hipStreamSynchronize(e->stream));
            (void)hipFree(Xt);
            (void)hipFree(ones);
            (void)hipFree(sl);
            (void)hipFree(red);
            launch_gdiag(e->stream, e->G, p_pad, c.p_local, e->gdiag);
            e->A = dalloc<double>((size_t)p_pad * (p_pad + kNB), o);
            e->Y2 = dalloc<double>((size_t)2 * p_pad, o);
            e->W2 = dalloc<double>((size_t)2 * p_pad, o);
        } else {
            launch_colnorm2(e->stream, e->X, n_pad, n_pad, c.p_local, e->gdiag);
        }
    }
    if (e->method == 4) tri_setup(e, Xh);
    // small p, one device, alpha known: whole sweeps in one single-workgroup launch
    e->fused = (e->method == 1 || e->method == 3) && c.p <= kSmallChainMaxP && c.world == 1 &&
               e->hy.know_alpha && e->cvec && e->gdiag && (e->method == 3 || e->G);
    if (e->method == 4)  // bb_tri.hip k_tri_chain (general and orthogonal designs)
        e->fused = c.p <= kTriChainMaxP && c.world == 1 && e->hy.know_alpha &&
                   (!c.ortho || (e->tri_G && e->cvec));
    if (e->nid) nid_certify_lambda(e);
    HIPCHECK(hipStreamSynchronize(e->stream));
}

void engine_init_state_local(bb_engine *e) {
    const bb_config &c = e->cfg;
    e->nid_seq = 0;  // the near-identity launch hint restarts with the chain
    e->nid_last = -1;
    // least squares start (BridgeWrapper.cpp:242-244, BridgeRegression.cpp:79-91)
    bool ls_ok = false;
    if (e->G != nullptr) {
        e->clear_err();
        const int m = e->chol_m ? e->chol_m : e->p_pad;
        launch_form_a(e->stream, e->G, e->p_pad, nullptr, e->sc, e->cvec, e->p, m, e->A,
                      e->p_pad, m);
        chol_factor(e->stream, e->A, e->p_pad, m, 1, e->err, e->Wd, e->flags);
        HIPCHECK(hipMemcpyAsync(e->Y2, e->A + (size_t)m * e->p_pad, m * sizeof(double),
                                hipMemcpyDeviceToDevice, e->stream));
        chol_bsolve(e->stream, e->A, e->p_pad, m, e->Wd, e->Y2, e->W2, 1, e->flags, e->err);
        uint32_t f = e->read_err();
        ls_ok = (f & 8u) == 0;
        if (ls_ok) {
            HIPCHECK(hipMemcpyAsync(e->beta, e->W2, (size_t)e->p * sizeof(double),
                                    hipMemcpyDeviceToDevice, e->stream));
        }
        e->clear_err();
    }
    if (!ls_ok) {
        HIPCHECK(hipMemsetAsync(e->beta, 0, (size_t)e->p_pad * sizeof(double), e->stream));
        if (g_verbose && c.rank == 0 && e->method != 6) {
            printf("Warning: cannot calculate least squares estimate; X'X is singular.\n");
            printf("Warning: setting least squares estimate to 0.0.\n");
        }
    }
    DevScalars s{};
    s.alpha = c.true_alpha > 0 ? c.true_alpha : 0.5;
    s.sig2 = e->method == 6 ? 1.0 : (c.true_sig2 > 0 ? c.true_sig2 : 0.0);
    s.tau = c.true_tau > 0 ? c.true_tau : 0.0;
    HIPCHECK(hipMemcpyAsync(e->sc, &s, sizeof(s), hipMemcpyHostToDevice, e->stream));
    if (e->method == 4) {  // BridgeWrapper.cpp:123 u[0].fill(0.5); omega starts at 1.0 (:604)
        std::vector<double> h(e->p_pad, 0.5);
        HIPCHECK(hipMemcpyAsync(e->u, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice,
                                e->stream));
        std::vector<double> h1(e->p_pad, 1.0);
        HIPCHECK(hipMemcpyAsync(e->lam, h1.data(), h1.size() * sizeof(double),
                                hipMemcpyHostToDevice, e->stream));
        HIPCHECK(hipMemcpyAsync(e->tr_u, h.data(), (size_t)e->p_loc * sizeof(double),
                                hipMemcpyHostToDevice, e->stream));
        HIPCHECK(hipMemcpyAsync(e->tr_lam, h1.data(), (size_t)e->p_loc * sizeof(double),
                                hipMemcpyHostToDevice, e->stream));
        HIPCHECK(hipStreamSynchronize(e->stream));
    }
    // trace slot 0 holds the starting values (as the reference's slot 0 before burn-in)
    HIPCHECK(hipMemcpyAsync(e->tr_beta, e->beta, (size_t)e->p_loc * sizeof(double),
                            hipMemcpyDeviceToDevice, e->stream));
    e->xbeta();
    launch_record_scalars(e->stream, e->sc, e->tr_tau, e->tr_sig2, e->tr_alpha);
}

void engine_init_state(bb_engine *e) {
    engine_init_state_local(e);
    if (e->method == 4 && e->cfg.ortho) {
        // triangle ortho driver draws sig2 then tau before burn-in (BridgeWrapper.cpp:374-375)
        if (!e->hy.know_tau || !e->hy.know_sig2) e->pre_and_scalars(0, 0, 0);
    } else if (e->method != 3 && !e->hy.know_tau) {
        e->pre_and_scalars(0, 0, 1);  // :262
    }
    HIPCHECK(hipStreamSynchronize(e->stream));
}

// one contiguous run of trace-ring doubles to the host (one copy, not one per sample)
void ring_copy(double *dst, const double *src, size_t count) {
    HIPCHECK(hipMemcpy(dst, src, count * sizeof(double), hipMemcpyDeviceToHost));
}

}  // namespace

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

const char *bb_version(void) { return "bayesbridge_amd 0.1 (gfx950)"; }
const char *bb_last_error(void) { return g_last_error.c_str(); }

int bb_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

void bb_set_seed(uint64_t seed) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_seed = seed;
    g_stream = 0;
}
void bb_get_rng_state(uint64_t *seed, uint64_t *stream) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (seed) *seed = g_seed;
    if (stream) *stream = g_stream;
}
void bb_set_rng_state(uint64_t seed, uint64_t stream) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_seed = seed;
    g_stream = stream;
}
void bb_use_r_rng(int enable) { g_use_r_rng = enable; }
int bb_set_device(int device) {
    if (device < 0 || device >= bb_device_count()) {
        set_error("invalid device %d", device);
        return -1;
    }
    g_device = device;
    return 0;
}
void bb_set_verbose(int verbose) { g_verbose = verbose; }

void bb_config_default(bb_config *c) {
    memset(c, 0, sizeof(*c));
    c->world = 1;
    c->sig2_shape = 0.0;
    c->sig2_scale = 0.0;
    c->nu_shape = 2.0;
    c->nu_rate = 2.0;
    c->alpha_a = 1.0;
    c->alpha_b = 1.0;
    c->true_alpha = 0.5;
    c->trace_capacity = 1;
    c->seed = 0xB4E5B41D6EULL;
    // Woodbury Gram: Ozaki-II int8 (fp64-accurate, ~2x faster at C3); cfg.gram_mode = 0
    // selects the fp64 MFMA Gram
    c->gram_mode = 1;
}

int bb_engine_create(const bb_config *cfg, const double *X_local, const double *y,
                     bb_engine **out) {
    *out = nullptr;
    bb_engine *e = new bb_engine();
    try {
        e->cfg = *cfg;
        if (e->cfg.p_local <= 0) e->cfg.p_local = e->cfg.p;
        if (e->cfg.world < 1) e->cfg.world = 1;
        if (cfg->n <= 0 || cfg->p <= 0) throw HipError("n and p must be positive");
        engine_setup(e, X_local, y, nullptr);
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        delete e;
        return -1;
    }
    *out = e;
    return 0;
}

int bb_engine_create_csc(const bb_config *cfg, const int *colptr, const int *rowidx,
                         const double *val, const double *y, bb_engine **out) {
    *out = nullptr;
    bb_engine *e = new bb_engine();
    try {
        e->cfg = *cfg;
        if (e->cfg.p_local <= 0) e->cfg.p_local = e->cfg.p;
        if (e->cfg.world < 1) e->cfg.world = 1;
        if (cfg->n <= 0 || cfg->p <= 0) throw HipError("n and p must be positive");
        SparseIn sp{colptr, rowidx, val};
        engine_setup(e, nullptr, y, &sp);
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        delete e;
        return -1;
    }
    *out = e;
    return 0;
}

long long bb_engine_sparse_pairs(const bb_engine *e) {
    return e->method == 5 ? (long long)e->spd.pairs : -1;
}

int bb_engine_sparse_info(const bb_engine *e, long long *pairs, long long *nnz, int *max_row,
                          int *col_mode) {
    if (e->method != 5) {
        set_error("not a sparse-design engine");
        return -1;
    }
    if (pairs) *pairs = (long long)e->spd.pairs;
    if (nnz) *nnz = (long long)e->spd.nnz;
    if (max_row) *max_row = e->spd.max_row;
    if (col_mode) *col_mode = e->spd.col_mode ? 1 : 0;
    return 0;
}

void bb_engine_destroy(bb_engine *e) { delete e; }

int bb_comm_id_size(void) { return (int)sizeof(ncclUniqueId); }
int bb_comm_unique_id(void *id_bytes) {
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) {
        set_error("ncclGetUniqueId failed");
        return -1;
    }
    memcpy(id_bytes, &id, sizeof(id));
    return 0;
}
// Every shard must cap the Chebyshev iterations alike, or ranks deciding from the same reduced
// sums would take different paths and post different collectives (a hang, or buffers mixed
// between exchanges).  The cost model's inputs differ between shards (p_loc, p_pad, the sparse
// non-zeros and pairs), so the ranks take the least of their caps: here through the
// new communicator, for groups in group_create.
static void agree_kmax_ranks(bb_engine *e) {
    double *buf = nullptr;
    HIPCHECK(hipMalloc(&buf, sizeof(double)));
    const double mine = e->nid ? (double)e->nid_kmax : 0.0;
    double got = mine;
    try {
        HIPCHECK(hipMemcpyAsync(buf, &mine, sizeof(double), hipMemcpyHostToDevice, e->stream));
        NCCLCHECK(ncclAllReduce(buf, buf, 1, ncclFloat64, ncclMin, e->comm, e->stream));
        HIPCHECK(hipMemcpyAsync(&got, buf, sizeof(double), hipMemcpyDeviceToHost, e->stream));
        HIPCHECK(hipStreamSynchronize(e->stream));
    } catch (...) {
        (void)hipFree(buf);
        throw;
    }
    (void)hipFree(buf);
    if (e->nid) e->nid_kmax = (int)got;
}

int bb_engine_comm_init(bb_engine *e, const void *id_bytes) {
    try {
        HIPCHECK(hipSetDevice(e->cfg.device));
        ncclUniqueId id;
        memcpy(&id, id_bytes, sizeof(id));
        NCCLCHECK(ncclCommInitRank(&e->comm, e->cfg.world, id, e->cfg.rank));
        agree_kmax_ranks(e);
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        return -1;
    }
    return 0;
}

int bb_engine_init_state(bb_engine *e) {
    try {
        HIPCHECK(hipSetDevice(e->cfg.device));
        engine_init_state(e);
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        return -1;
    }
    return 0;
}

int bb_engine_run(bb_engine *e, uint64_t t0, int count, int first_slot, int slot_step,
                  int mcmc_phase) {
    try {
        HIPCHECK(hipSetDevice(e->cfg.device));
        e->run(t0, count, first_slot, slot_step, mcmc_phase);
        HIPCHECK(hipGetLastError());
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        return -1;
    }
    return 0;
}

int bb_engine_sync(bb_engine *e) {
    try {
        HIPCHECK(hipStreamSynchronize(e->stream));
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        return -1;
    }
    return 0;
}

int bb_engine_get_trace(bb_engine *e, int slot0, int count, double *beta, double *lambda,
                        double *sig2, double *tau, double *alpha) {
    try {
        HIPCHECK(hipStreamSynchronize(e->stream));
        const size_t pl = (size_t)e->p_loc;
        // slots [slot0, slot0 + count) of the ring: at most two contiguous runs per trace
        for (int k = 0; k < count;) {
            const int s = (slot0 + k) % e->cap;
            const int run = std::min(count - k, e->cap - s);
            if (beta) ring_copy(beta + k * pl, e->tr_beta + s * pl, run * pl);
            if (lambda) ring_copy(lambda + k * pl, e->tr_lam + s * pl, run * pl);
            if (sig2) ring_copy(sig2 + k, e->tr_sig2 + s, run);
            if (tau) ring_copy(tau + k, e->tr_tau + s, run);
            if (alpha) ring_copy(alpha + k, e->tr_alpha + s, run);
            k += run;
        }
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        return -1;
    }
    return 0;
}

int bb_engine_get_state(bb_engine *e, double *beta, double *lambda, double *tau, double *sig2,
                        double *alpha) {
    try {
        HIPCHECK(hipStreamSynchronize(e->stream));
        if (beta)
            HIPCHECK(hipMemcpy(beta, e->beta, (size_t)e->p_loc * sizeof(double),
                               hipMemcpyDeviceToHost));
        if (lambda)
            HIPCHECK(hipMemcpy(lambda, e->lam, (size_t)e->p_loc * sizeof(double),
                               hipMemcpyDeviceToHost));
        DevScalars s;
        HIPCHECK(hipMemcpy(&s, e->sc, sizeof(s), hipMemcpyDeviceToHost));
        if (tau) *tau = s.tau;
        if (sig2) *sig2 = s.sig2;
        if (alpha) *alpha = s.alpha;
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        return -1;
    }
    return 0;
}

int bb_engine_set_state(bb_engine *e, const double *beta, double tau, double sig2,
                        double alpha) {
    try {
        HIPCHECK(hipStreamSynchronize(e->stream));
        HIPCHECK(hipMemcpy(e->beta, beta, (size_t)e->p_loc * sizeof(double),
                           hipMemcpyHostToDevice));
        DevScalars s;
        HIPCHECK(hipMemcpy(&s, e->sc, sizeof(s), hipMemcpyDeviceToHost));
        s.tau = tau;
        s.sig2 = sig2;
        s.alpha = alpha;
        HIPCHECK(hipMemcpy(e->sc, &s, sizeof(s), hipMemcpyHostToDevice));
        e->xbeta();
        HIPCHECK(hipStreamSynchronize(e->stream));
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        return -1;
    }
    return 0;
}

int bb_engine_method(const bb_engine *e) { return e->method; }

int bb_engine_get_omega(bb_engine *e, double *omega) {
    try {
        if (e->method != 6) throw HipError("not a logistic engine");
        HIPCHECK(hipStreamSynchronize(e->stream));
        HIPCHECK(hipMemcpy(omega, e->omega, (size_t)e->n * sizeof(double), hipMemcpyDeviceToHost));
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        return -1;
    }
    return 0;
}

int bb_engine_get_tri_trace(bb_engine *e, int slot0, int count, double *u, double *shape) {
    try {
        if (e->method != 4) throw HipError("not a triangle-method engine");
        HIPCHECK(hipStreamSynchronize(e->stream));
        const size_t pl = (size_t)e->p_loc;
        for (int k = 0; k < count;) {
            const int s = (slot0 + k) % e->cap;
            const int run = std::min(count - k, e->cap - s);
            if (u) ring_copy(u + k * pl, e->tr_u + s * pl, run * pl);
            if (shape) ring_copy(shape + k * pl, e->tr_shape + s * pl, run * pl);
            k += run;
        }
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        return -1;
    }
    return 0;
}

int bb_engine_set_tri_state(bb_engine *e, const double *u) {
    try {
        if (e->method != 4) throw HipError("not a triangle-method engine");
        HIPCHECK(hipStreamSynchronize(e->stream));
        HIPCHECK(hipMemcpy(e->u, u, (size_t)e->p_loc * sizeof(double), hipMemcpyHostToDevice));
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        return -1;
    }
    return 0;
}

int bb_engine_get_tri_basis(bb_engine *e, double *tV, double *a, double *d) {
    if (e->method != 4) {
        set_error("not a triangle-method engine");
        return -1;
    }
    if (tV) memcpy(tV, e->h_tV.data(), e->h_tV.size() * sizeof(double));
    if (a) memcpy(a, e->h_a.data(), e->h_a.size() * sizeof(double));
    if (d) memcpy(d, e->h_d.data(), e->h_d.size() * sizeof(double));
    return 0;
}
int bb_engine_gram_mode(const bb_engine *e) { return e->cfg.gram_mode; }

int bb_engine_enable_timing(bb_engine *e, int enable) {
    e->timing = enable != 0;
    e->timing_level = enable == 1 ? 1 : 2;
    return 0;
}

int bb_engine_set_timed_phase(bb_engine *e, int phase) {
    if (phase < 0 || phase >= PH_END) {
        set_error("bb_engine_set_timed_phase: phase %d out of range", phase);
        return -1;
    }
    e->timed_phase = phase;
    return 0;
}

int bb_engine_set_timing_stride(bb_engine *e, int stride) {
    if (stride < 1) {
        set_error("bb_engine_set_timing_stride: stride %d < 1", stride);
        return -1;
    }
    e->timing_stride = stride;
    return 0;
}

int bb_engine_reset_timing(bb_engine *e) {
    (void)hipStreamSynchronize(e->stream);
    e->sweep_marks.clear();
    e->ev_next = 0;
    return 0;
}

int bb_engine_phase_times(bb_engine *e, double *ms, int cap, int *samples) {
    try {
        HIPCHECK(hipStreamSynchronize(e->stream));
        std::vector<double> acc(PH_COUNT, 0.0);
        for (auto &marks : e->sweep_marks)
            for (size_t i = 0; i + 1 < marks.size(); ++i) {
                float v = 0;
                HIPCHECK(hipEventElapsedTime(&v, e->ev_pool[marks[i].second],
                                             e->ev_pool[marks[i + 1].second]));
                acc[marks[i].first] += v;
            }
        const double ns = e->sweep_marks.empty() ? 1.0 : (double)e->sweep_marks.size();
        for (int i = 0; i < cap && i < PH_COUNT; ++i) ms[i] = acc[i] / ns;
        if (samples) *samples = (int)e->sweep_marks.size();
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        return -1;
    }
    return 0;
}

const char *bb_phase_name(int i) { return (i >= 0 && i < PH_COUNT) ? kPhaseNames[i] : ""; }
int bb_phase_count(void) { return PH_COUNT; }

int bb_engine_kernel_times(bb_engine *e, double *gram_ms_avg, double *sweep_ms_avg,
                           int *samples) {
    try {
        HIPCHECK(hipStreamSynchronize(e->stream));
        double g = 0, s = 0;
        int ng = 0, ns = 0;
        for (auto &marks : e->sweep_marks) {
            for (size_t i = 0; i + 1 < marks.size(); ++i)
                if (marks[i].first == e->timed_phase) {
                    float v = 0;
                    HIPCHECK(hipEventElapsedTime(&v, e->ev_pool[marks[i].second],
                                                 e->ev_pool[marks[i + 1].second]));
                    g += v;
                    ++ng;
                }
            if (marks.size() >= 2) {
                float v = 0;
                HIPCHECK(hipEventElapsedTime(&v, e->ev_pool[marks.front().second],
                                             e->ev_pool[marks.back().second]));
                s += v;
                ++ns;
            }
        }
        if (gram_ms_avg) *gram_ms_avg = ng ? g / ng : 0.0;
        if (sweep_ms_avg) *sweep_ms_avg = ns ? s / ns : 0.0;
        if (samples) *samples = ns;
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        return -1;
    }
    return 0;
}

int bb_engine_timed_brackets(bb_engine *e, int *count) {
    int ng = 0;
    for (auto &marks : e->sweep_marks)
        for (size_t i = 0; i + 1 < marks.size(); ++i)
            if (marks[i].first == e->timed_phase) ++ng;
    *count = ng;
    return 0;
}

int bb_engine_nid_mixed(bb_engine *e, unsigned long long *mixed_sweeps,
                        unsigned long long *products32, double *eta, int *k2, int *holds_x32) {
    try {
        NidState h{};
        if (e->nid) {
            HIPCHECK(hipMemcpyAsync(&h, e->nid, sizeof(h), hipMemcpyDeviceToHost, e->stream));
            HIPCHECK(hipStreamSynchronize(e->stream));
        }
        if (mixed_sweeps) *mixed_sweeps = h.n_mixed;
        if (products32) *products32 = h.n_products32;
        if (eta) *eta = h.eta;
        if (k2) *k2 = h.k2;
        if (holds_x32) *holds_x32 = e->X32 != nullptr;
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        return -1;
    }
    return 0;
}

int bb_engine_nid_bound(bb_engine *e, double *lambda_x, int *kmax) {
    if (lambda_x) *lambda_x = e->lambda_x;
    if (kmax) *kmax = e->nid ? std::min(g_nid_kmax, e->nid_kmax) : -1;
    return 0;
}

int bb_engine_nid_stats(bb_engine *e, unsigned long long *cheb_sweeps,
                        unsigned long long *products, unsigned long long *chol_sweeps,
                        double *eps, int *mode) {
    try {
        NidState h{};
        if (e->nid) {
            HIPCHECK(hipMemcpyAsync(&h, e->nid, sizeof(h), hipMemcpyDeviceToHost, e->stream));
            HIPCHECK(hipStreamSynchronize(e->stream));
        }
        if (cheb_sweeps) *cheb_sweeps = h.n_cheb;
        if (products) *products = h.n_products;
        if (chol_sweeps) *chol_sweeps = h.n_chol;
        if (eps) *eps = e->nid ? h.eps : -1.0;
        if (mode) *mode = e->nid ? h.mode : -1;
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        return -1;
    }
    return 0;
}

int bb_kernel_instance(const char *phase, char *buf, int len) {
    static const char *kFam[KF_COUNT] = {"lambda", "gram", "reduce", "chol", "solve", "beta",
                                         "eapply"};
    if (!phase || !buf || len <= 0) return -1;
    buf[0] = 0;
    int f = -1;
    for (int i = 0; i < KF_COUNT; ++i)
        if (!strcmp(phase, kFam[i])) f = i;
    const void *k = launched_instance(f);
    if (!k) return -1;
    const char *mangled = hipKernelNameRefByPtr(k, nullptr);
    if (!mangled) return -1;
    int st = 0;
    char *dem = abi::__cxa_demangle(mangled, nullptr, nullptr, &st);
    std::string name = (st == 0 && dem) ? dem : mangled;
    free(dem);
    // "void bb::k_eapply<8, false>(double const*, ...)" -> "bb::k_eapply<8, false>" (the form
    // tools/profile_summary.py gives rocprofv3's kernel names)
    if (name.rfind("void ", 0) == 0) name = name.substr(5);
    int depth = 0;
    for (size_t i = 0; i < name.size(); ++i) {
        if (name[i] == '<') ++depth;
        if (name[i] == '>') --depth;
        if (name[i] == '(' && depth == 0) {
            name.resize(i);
            break;
        }
    }
    snprintf(buf, (size_t)len, "%s", name.c_str());
    return 0;
}

int bb_engine_launch_counts(bb_engine *e, unsigned long long *lambda_xu,
                            unsigned long long *lambda_alone) {
    if (lambda_xu) *lambda_xu = e->n_lambda_xu;
    if (lambda_alone) *lambda_alone = e->n_lambda_alone;
    return 0;
}

int bb_engine_error_flags(bb_engine *e, uint32_t *flags) {
    try {
        *flags = e->read_err();
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        return -1;
    }
    return 0;
}

// ---------------------------------------------------------------------------
// Shard groups: several column-shard engines driven by ONE host thread, interleaving their
// phases around the two per-sweep exchanges.  Two exchange modes:
//   - on-device sums: every member on one device (tests the sharded decomposition on one
//     GPU -- RCCL cannot place two ranks on one device);
//   - RCCL: members on distinct devices with communicators from ncclCommInitAll, each
//     exchange one ncclGroupStart / ncclAllReduce per member / ncclGroupEnd on the members'
//     streams.  This is the single-process multi-GPU path behind the .C entry points: R
//     calls .C from one process (BridgeWrapper.R:220-228), SURVEY.md 5 "distributed comm
//     backend".
// ---------------------------------------------------------------------------
struct bb_group {
    std::vector<bb_engine *> members;
    bool rccl = false;
    std::vector<ncclComm_t> comms;
    hipStream_t stream = nullptr;
    hipEvent_t ev = nullptr;
    std::vector<hipEvent_t> mev;
    double *tmp = nullptr;
    size_t tmp_count = 0;
    // an RCCL member failed mid-run: the communicators were aborted (the other members'
    // pending all-reduces can never be matched), so nothing may wait on the streams again
    bool poisoned = false;
    ~bb_group() {
        for (auto *m : members) {
            (void)hipSetDevice(m->cfg.device);
            if (!poisoned) (void)hipStreamSynchronize(m->stream);
            if (rccl) m->comm = nullptr;  // lent by this group
            m->stop = nullptr;
            m->group_member = false;
        }
        for (auto c : comms)
            if (c) ncclCommDestroy(c);
        if (!members.empty()) (void)hipSetDevice(members[0]->cfg.device);
        if (stream && !poisoned) (void)hipStreamSynchronize(stream);
        if (tmp) (void)hipFree(tmp);
        if (ev) (void)hipEventDestroy(ev);
        for (auto e : mev) (void)hipEventDestroy(e);
        if (stream) (void)hipStreamDestroy(stream);
    }
    // sum buf(member) over members, result written back to every member's buf
    void reduce(double *bb_engine::*buf, size_t count) {
        if (rccl) {
            NCCLCHECK(ncclGroupStart());
            for (size_t i = 0; i < members.size(); ++i)
                NCCLCHECK(ncclAllReduce(members[i]->*buf, members[i]->*buf, count, ncclFloat64,
                                        ncclSum, comms[i], members[i]->stream));
            NCCLCHECK(ncclGroupEnd());
            return;
        }
        HIPCHECK(hipSetDevice(members[0]->cfg.device));
        for (size_t i = 0; i < members.size(); ++i) {
            HIPCHECK(hipEventRecord(mev[i], members[i]->stream));
            HIPCHECK(hipStreamWaitEvent(stream, mev[i], 0));
        }
        HIPCHECK(hipMemcpyAsync(tmp, members[0]->*buf, count * sizeof(double),
                                hipMemcpyDeviceToDevice, stream));
        for (size_t i = 1; i < members.size(); ++i)
            launch_sum_into(stream, members[i]->*buf, tmp, count);
        for (size_t i = 0; i < members.size(); ++i)
            HIPCHECK(hipMemcpyAsync(members[i]->*buf, tmp, count * sizeof(double),
                                    hipMemcpyDeviceToDevice, stream));
        HIPCHECK(hipEventRecord(ev, stream));
        for (auto *m : members) HIPCHECK(hipStreamWaitEvent(m->stream, ev, 0));
    }
    void on(bb_engine *m) { HIPCHECK(hipSetDevice(m->cfg.device)); }
};

namespace {

bb_group *group_create(bb_engine **engines, int count, bool rccl) {
    bb_group *g = new bb_group();
    try {
        if (count < 1) throw HipError("empty group");
        for (int i = 0; i < count; ++i) {
            if (engines[i]->cfg.world != count || engines[i]->cfg.rank != i)
                throw HipError("group member rank/world mismatch");
            for (int k = 0; k < i; ++k)
                if ((engines[k]->cfg.device == engines[i]->cfg.device) == rccl)
                    throw HipError(rccl ? "an RCCL group needs its members on distinct devices"
                                        : "an on-device group needs its members on one device "
                                          "(use an RCCL group across devices)");
            if (engines[i]->comm) throw HipError("group members must not own a communicator");
            g->members.push_back(engines[i]);
        }
        size_t c = 0;
        for (auto *m : g->members) {
            c = std::max(c, m->red1_count());
            if (m->woodbury()) c = std::max(c, m->red2_count());
        }
        g->tmp_count = c;
        // one iteration cap for every member (see agree_kmax_ranks); members disagreeing on
        // whether the near-identity path exists at all (n_pad decides it) cannot be grouped
        int kmin = 1 << 30;
        for (auto *m : g->members) {
            if ((m->nid != nullptr) != (g->members[0]->nid != nullptr))
                throw HipError("group members disagree on the near-identity solve (n differs?)");
            if (m->nid) kmin = std::min(kmin, m->nid_kmax);
        }
        for (auto *m : g->members)
            if (m->nid) m->nid_kmax = kmin;
        if (rccl) {
            g->rccl = true;
            std::vector<int> devs(count);
            for (int i = 0; i < count; ++i) devs[i] = engines[i]->cfg.device;
            g->comms.assign(count, nullptr);
            NCCLCHECK(ncclCommInitAll(g->comms.data(), count, devs.data()));
            // each member runs whole sweeps on its own host thread (bb_group_run) and
            // exchanges through its own communicator, as one rank of a multi-process job
            for (int i = 0; i < count; ++i) {
                engines[i]->comm = g->comms[i];
                engines[i]->own_comm = false;
            }
        } else {
            HIPCHECK(hipSetDevice(engines[0]->cfg.device));
            HIPCHECK(hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking));
            HIPCHECK(hipEventCreateWithFlags(&g->ev, hipEventDisableTiming));
            for (int i = 0; i < count; ++i) {
                hipEvent_t e;
                HIPCHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
                g->mev.push_back(e);
            }
            HIPCHECK(hipMalloc(&g->tmp, c * sizeof(double)));
            for (int i = 0; i < count; ++i) engines[i]->group_member = true;
        }
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        delete g;
        return nullptr;
    }
    return g;
}

}  // namespace

extern "C" {

int bb_group_create(bb_engine **engines, int count, bb_group **out) {
    *out = group_create(engines, count, false);
    return *out ? 0 : -1;
}

int bb_group_create_rccl(bb_engine **engines, int count, bb_group **out) {
    *out = group_create(engines, count, true);
    return *out ? 0 : -1;
}

void bb_group_destroy(bb_group *g) { delete g; }

int bb_group_run(bb_group *g, uint64_t t0, int count, int first_slot, int slot_step,
                 int mcmc_phase) {
    if (g->poisoned) {
        set_error("shard group unusable: a member failed in an earlier run and its "
                  "communicators were aborted");
        return -1;
    }
    if (g->rccl) {
        // one enqueue thread per device: member i runs its `count` sweeps exactly as rank i
        // of a one-process-per-GPU job would (phase a, all-reduce, phase b, all-reduce,
        // phase c on its own stream and communicator), so the host cost per sweep does not
        // grow with the device count
        const size_t k = g->members.size();
        std::vector<std::string> errs(k);
        std::vector<std::thread> th;
        std::atomic<bool> stop{false};
        const int fail_member = g_debug_fail_member.exchange(-1), fail_sweep = g_debug_fail_sweep.load();
        th.reserve(k);
        for (size_t i = 0; i < k; ++i)
            th.emplace_back([&, i] {
                bb_engine *m = g->members[i];
                m->stop = &stop;
                m->fail_at = (int)i == fail_member ? fail_sweep : -1;
                try {
                    HIPCHECK(hipSetDevice(m->cfg.device));
                    m->run(t0, count, first_slot, slot_step, mcmc_phase);
                    HIPCHECK(hipGetLastError());
                } catch (std::exception &ex) {
                    errs[i] = ex.what();
                    stop.store(true);  // the others stop enqueueing sweeps
                }
                m->fail_at = -1;
            });
        for (auto &t : th) t.join();
        for (size_t i = 0; i < k; ++i)
            if (!errs[i].empty()) {
                set_error("group member %zu: %s", i, errs[i].c_str());
                // A member stopped part-way through its sweeps, so the all-reduces the others
                // already enqueued can never be matched: abort every communicator (their
                // pending collectives return) and poison the group, so that neither this call
                // nor the destructor waits on those streams.
                for (auto &c : g->comms)
                    if (c) {
                        (void)ncclCommAbort(c);
                        c = nullptr;
                    }
                for (auto *m : g->members) m->comm = nullptr;
                g->poisoned = true;
                return -1;
            }
        return 0;
    }
    try {
        for (int k = 0; k < count; ++k) {
            const uint64_t t = t0 + (uint64_t)k;
            const int slot = first_slot < 0 ? -1 : first_slot + k * slot_step;
            for (auto *m : g->members) {
                g->on(m);
                m->phase_a(t);
            }
            g->reduce(&bb_engine::red1, g->members[0]->red1_count());
            for (auto *m : g->members) {
                g->on(m);
                m->phase_b(t, slot);
            }
            bb_engine *m0 = g->members[0];
            if (m0->woodbury() && m0->nid_sync()) {
                // the stages of bb_engine::shard_solve, each over all members, with the
                // group's reduce as the exchange; every member decides from the same reduced
                // sums, so member 0's decision is every member's
                g->reduce(&bb_engine::nid_red, (size_t)bb_engine::kNidRed);
                for (auto *m : g->members) {
                    g->on(m);
                    m->nidx_decide_launch();
                }
                const int K = m0->nidx_decide_read();
                for (auto *m : g->members) {
                    // every member decided from the same reduced sums with the same cap: a
                    // member whose device mode differed would skip both solves (stale w)
                    if (m != m0 && m->nidx_decide_read() != K)
                        throw HipError("shard group members decided different near-identity "
                                       "paths");
                    m->nid_only = K > 0;
                    m->nid_last = K;
                }
                if (K > 0) {
                    for (auto *m : g->members) {
                        g->on(m);
                        m->nidx_xu();
                    }
                    g->reduce(&bb_engine::nid_sum, (size_t)m0->n_pad);
                    for (auto *m : g->members) {
                        g->on(m);
                        m->nidx_init(t);
                    }
                    for (int j = 1; j < K; ++j) {
                        for (auto *m : g->members) {
                            g->on(m);
                            m->nidx_eapply(j);
                        }
                        g->reduce(&bb_engine::nid_sum, (size_t)m0->n_pad);
                        for (auto *m : g->members) {
                            g->on(m);
                            m->nidx_step(j);
                        }
                    }
                } else {
                    for (auto *m : g->members) {
                        g->on(m);
                        m->wb_gram(nullptr);
                    }
                    g->reduce(&bb_engine::red2, m0->red2_count());
                }
            } else if (m0->woodbury()) {
                g->reduce(&bb_engine::red2, m0->red2_count());
            }
            // phase c holds the persistent Cholesky / backward-solve kernels, which need every
            // workgroup of their grid resident at once: two members' launches on the shared
            // device must not overlap (two C3-sized factorisations side by side each hold part
            // of the CUs and wait on tiles owned by workgroups that cannot start), so the
            // members' phase c run one after another
            for (size_t i = 0; i < g->members.size(); ++i) {
                bb_engine *m = g->members[i];
                g->on(m);
                if (i > 0) HIPCHECK(hipStreamWaitEvent(m->stream, g->mev[i - 1], 0));
                m->phase_c(t, slot, mcmc_phase);
                if (i + 1 < g->members.size()) HIPCHECK(hipEventRecord(g->mev[i], m->stream));
            }
            if (g->members[0]->alpha_exchange()) {
                g->reduce(&bb_engine::red3, 2);
                for (auto *m : g->members) {
                    g->on(m);
                    m->phase_d(t, slot, mcmc_phase);
                }
            }
        }
        HIPCHECK(hipGetLastError());
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        return -1;
    }
    return 0;
}

int bb_group_sync(bb_group *g) {
    if (g->poisoned) {
        set_error("shard group unusable: a member failed and its communicators were aborted");
        return -1;
    }
    try {
        for (auto *m : g->members) {
            g->on(m);
            HIPCHECK(hipStreamSynchronize(m->stream));
        }
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        return -1;
    }
    return 0;
}

int bb_group_init_state(bb_group *g) {
    // p > n (Woodbury) start: beta = 0, then the pre-burn tau draw from the summed red1
    try {
        for (auto *m : g->members) {
            if (m->G != nullptr) throw HipError("group init supports the p > n path only");
            g->on(m);
            engine_init_state_local(m);
        }
        bool draw_tau = g->members[0]->method != 3 && !g->members[0]->hy.know_tau;
        if (draw_tau) {
            for (auto *m : g->members) {
                g->on(m);
                launch_pre(m->stream, m->xb_part, m->nparts, m->n_pad, m->beta, m->p_loc, m->sc,
                           m->red1, m->nbS);
            }
            g->reduce(&bb_engine::red1, g->members[0]->red1_count());
            for (auto *m : g->members) {
                g->on(m);
                launch_scalars(m->stream, m->red1, m->nbS, m->y, m->n, m->p, m->sc, m->hy,
                               m->cfg.seed, m->cfg.stream, 0, m->tr_tau, m->tr_sig2,
                               m->tr_alpha, 1, m->err);
            }
        }
        for (auto *m : g->members) {
            g->on(m);
            HIPCHECK(hipStreamSynchronize(m->stream));
        }
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        return -1;
    }
    return 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// kernel-level entry points
// ---------------------------------------------------------------------------
int bb_retstable_batch(double *x, const double *alpha, const double *V0, const double *h, int num,
                       uint64_t seed, uint64_t stream, uint64_t t, int group) {
    if (num <= 0) return 0;
    std::vector<void *> owned;
    int rc = 0;
    try {
        HIPCHECK(hipSetDevice(g_device));
        double *da = dalloc<double>(num, owned), *dv = dalloc<double>(num, owned),
               *dh = dalloc<double>(num, owned), *dx = dalloc<double>(num, owned);
        uint32_t *de = dalloc<uint32_t>(1, owned);
        HIPCHECK(hipMemcpy(da, alpha, num * sizeof(double), hipMemcpyHostToDevice));
        HIPCHECK(hipMemcpy(dv, V0, num * sizeof(double), hipMemcpyHostToDevice));
        HIPCHECK(hipMemcpy(dh, h, num * sizeof(double), hipMemcpyHostToDevice));
        if (group <= 0) group = stable_group_for(num);
        launch_retstable_batch(0, dx, da, dv, dh, num, seed, stream, t, group, de);
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipMemcpy(x, dx, num * sizeof(double), hipMemcpyDeviceToHost));
        uint32_t f = 0;
        HIPCHECK(hipMemcpy(&f, de, sizeof(f), hipMemcpyDeviceToHost));
        if (f & 4u) {
            fprintf(stderr, "Problem with parameter.\n");  // retstable.cpp:112-115
        }
        rc = (int)(f & ~4u) ? -2 : 0;
        if (rc) set_error("retstable: rejection cap reached (flags %u)", f);
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        rc = -1;
    }
    for (void *q : owned) (void)hipFree(q);
    return rc;
}

int bb_pg_batch(double *omega, const double *psi, int n, uint64_t seed, uint64_t stream,
                uint64_t t) {
    if (n <= 0) return 0;
    std::vector<void *> owned;
    int rc = 0;
    try {
        HIPCHECK(hipSetDevice(g_device));
        double *dp = dalloc<double>(n, owned), *dw = dalloc<double>(n, owned);
        uint32_t *de = dalloc<uint32_t>(1, owned);
        HIPCHECK(hipMemcpy(dp, psi, (size_t)n * sizeof(double), hipMemcpyHostToDevice));
        launch_pg(0, dp, n, n, seed, stream, t, dw, de);
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipMemcpy(omega, dw, (size_t)n * sizeof(double), hipMemcpyDeviceToHost));
        uint32_t f = 0;
        HIPCHECK(hipMemcpy(&f, de, sizeof(f), hipMemcpyDeviceToHost));
        if (f) {
            set_error("pg: rejection cap reached (flags %u)", f);
            rc = -2;
        }
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        rc = -1;
    }
    for (void *q : owned) (void)hipFree(q);
    return rc;
}

int bb_trunc_batch(int mode, int num, double *x, const double *p0, const double *p1,
                   const double *p2, const double *p3, uint64_t seed, uint64_t stream) {
    if (num <= 0) return 0;
    if (mode < 0 || mode > 5) {
        set_error("bb_trunc_batch: invalid mode %d", mode);
        return -1;
    }
    static const int nparams[6] = {3, 4, 4, 2, 3, 3};
    const double *src[4] = {p0, p1, p2, p3};
    std::vector<void *> owned;
    int rc = 0;
    try {
        HIPCHECK(hipSetDevice(g_device));
        double *dp[4] = {nullptr, nullptr, nullptr, nullptr};
        for (int k = 0; k < nparams[mode]; ++k) {
            dp[k] = dalloc<double>(num, owned);
            HIPCHECK(hipMemcpy(dp[k], src[k], num * sizeof(double), hipMemcpyHostToDevice));
        }
        double *dx = dalloc<double>(num, owned);
        uint32_t *de = dalloc<uint32_t>(1, owned);
        launch_trunc_batch(0, mode, num, dx, dp[0], dp[1], dp[2], dp[3], seed, stream, de);
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipMemcpy(x, dx, num * sizeof(double), hipMemcpyDeviceToHost));
        uint32_t f = 0;
        HIPCHECK(hipMemcpy(&f, de, sizeof(f), hipMemcpyDeviceToHost));
        if (f & 256u) {  // BridgeWrapper.cpp:815-822
            for (int i = 0; i < num; ++i)
                if (std::isnan(p0[i]) || std::isnan(p1[i]) || std::isnan(p2[i]) ||
                    std::isinf(p0[i]))
                    fprintf(stderr, "rtexpon_rate: caught non finite left value: %g; x[i] = %g.\n",
                            p0[i], (double)NAN);  // printed before the draw overwrites it
        }
        rc = (f & (64u | 128u)) ? -2 : 0;
        if (rc) set_error("truncated draw: %s (flags %u)",
                          (f & 128u) ? "empty truncation interval" : "rejection cap reached", f);
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        rc = -1;
    }
    for (void *q : owned) (void)hipFree(q);
    return rc;
}

int bb_rrtgamma_batch(int num, double *x, const double *shape, const double *rate,
                      const double *right_t, uint64_t seed, uint64_t stream) {
    if (num <= 0) return 0;
    std::vector<void *> owned;
    int rc = 0;
    try {
        HIPCHECK(hipSetDevice(g_device));
        const double *src[3] = {shape, rate, right_t};
        double *dp[3];
        for (int k = 0; k < 3; ++k) {
            dp[k] = dalloc<double>(num, owned);
            HIPCHECK(hipMemcpy(dp[k], src[k], num * sizeof(double), hipMemcpyHostToDevice));
        }
        double *dx = dalloc<double>(num, owned);
        uint32_t *de = dalloc<uint32_t>(1, owned);
        launch_rrtgamma_batch(0, num, dx, dp[0], dp[1], dp[2], seed, stream, de);
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipMemcpy(x, dx, num * sizeof(double), hipMemcpyDeviceToHost));
        uint32_t f = 0;
        HIPCHECK(hipMemcpy(&f, de, sizeof(f), hipMemcpyDeviceToHost));
        rc = f ? -2 : 0;
        if (rc) set_error("rrtgamma: rejection cap reached (flags %u)", f);
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        rc = -1;
    }
    for (void *q : owned) (void)hipFree(q);
    return rc;
}

int bb_sample_lambda(double *lambda, const double *beta, int p, double alpha, double tau,
                     uint64_t seed, uint64_t stream, uint64_t t, uint64_t j0, int group) {
    if (p <= 0) return 0;
    std::vector<void *> owned;
    int rc = 0;
    try {
        HIPCHECK(hipSetDevice(g_device));
        double *db = dalloc<double>(p, owned), *dl = dalloc<double>(p, owned);
        DevScalars *dsc = dalloc<DevScalars>(1, owned);
        uint32_t *de = dalloc<uint32_t>(1, owned);
        DevScalars s{};
        s.tau = tau;
        s.alpha = alpha;
        HIPCHECK(hipMemcpy(dsc, &s, sizeof(s), hipMemcpyHostToDevice));
        HIPCHECK(hipMemcpy(db, beta, p * sizeof(double), hipMemcpyHostToDevice));
        if (group <= 0) group = stable_group_for(p);
        launch_lambda(0, db, p, p, j0, dsc, seed, stream, t, LAMBDA_ONLY, group, dl, nullptr,
                      nullptr, nullptr, de);
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipMemcpy(lambda, dl, p * sizeof(double), hipMemcpyDeviceToHost));
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        rc = -1;
    }
    for (void *q : owned) (void)hipFree(q);
    return rc;
}

int bb_bench_lambda(const double *beta, int p, double alpha, double tau, int group,
                    int noinline, int reps, double *ms_avg, double *lambda_out) {
    std::vector<void *> owned;
    int rc = 0;
    try {
        HIPCHECK(hipSetDevice(g_device));
        double *db = dalloc<double>(p, owned), *dl = dalloc<double>(p, owned);
        DevScalars *dsc = dalloc<DevScalars>(1, owned);
        uint32_t *de = dalloc<uint32_t>(1, owned);
        DevScalars s{};
        s.tau = tau;
        s.alpha = alpha;
        HIPCHECK(hipMemcpy(dsc, &s, sizeof(s), hipMemcpyHostToDevice));
        HIPCHECK(hipMemcpy(db, beta, p * sizeof(double), hipMemcpyHostToDevice));
        hipEvent_t e0, e1;
        HIPCHECK(hipEventCreate(&e0));
        HIPCHECK(hipEventCreate(&e1));
        launch_lambda_variant(0, db, p, dsc, 1, 0, 1, group, noinline, dl, de);  // warm
        HIPCHECK(hipEventRecord(e0, 0));
        for (int r = 0; r < reps; ++r)
            launch_lambda_variant(0, db, p, dsc, 1, 0, 2 + r, group, noinline, dl, de);
        HIPCHECK(hipEventRecord(e1, 0));
        HIPCHECK(hipEventSynchronize(e1));
        float ms = 0;
        HIPCHECK(hipEventElapsedTime(&ms, e0, e1));
        *ms_avg = ms / reps;
        if (lambda_out)
            HIPCHECK(hipMemcpy(lambda_out, dl, p * sizeof(double), hipMemcpyDeviceToHost));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        rc = -1;
    }
    for (void *q : owned) (void)hipFree(q);
    return rc;
}

int bb_bench_chol(int m, int reps, double *ms_factor, double *ms_solve,
                  unsigned long long *trace) {
    std::vector<void *> owned;
    int rc = 0;
    try {
        HIPCHECK(hipSetDevice(g_device));
        const int m_pad = round_up(m, kNB);
        // SPD test matrix: I * m + small symmetric perturbation, built on the host once
        std::vector<double> h((size_t)m_pad * (m_pad + kNB), 0.0);
        for (int c = 0; c < m_pad; ++c)
            for (int r = 0; r <= c; ++r)
                h[(size_t)r + (size_t)c * m_pad] =
                    (r == c) ? (double)m_pad : 0.5 * std::sin(0.37 * r + 0.11 * c);
        for (int r = 0; r < m_pad; ++r) h[(size_t)r + (size_t)m_pad * m_pad] = 1.0;
        double *src = dalloc<double>(h.size(), owned), *dA = dalloc<double>(h.size(), owned);
        HIPCHECK(hipMemcpy(src, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice));
        double *Wd = dalloc<double>(chol_wd_words(m_pad), owned);
        unsigned int *fl = dalloc<unsigned int>(chol_flag_words(m_pad, 1), owned);
        double *W = dalloc<double>((size_t)m_pad, owned);
        uint32_t *de = dalloc<uint32_t>(1, owned);
        hipEvent_t e0, e1, e2;
        HIPCHECK(hipEventCreate(&e0));
        HIPCHECK(hipEventCreate(&e1));
        HIPCHECK(hipEventCreate(&e2));
        double tf = 0, ts = 0;
        for (int it = 0; it <= reps; ++it) {
            HIPCHECK(hipMemcpyAsync(dA, src, h.size() * sizeof(double), hipMemcpyDeviceToDevice, 0));
            HIPCHECK(hipEventRecord(e0, 0));
            chol_factor(0, dA, m_pad, m_pad, 1, de, Wd, fl);
            HIPCHECK(hipEventRecord(e1, 0));
            chol_bsolve(0, dA, m_pad, m_pad, Wd, dA + (size_t)m_pad * m_pad, W, 1, fl, de);
            HIPCHECK(hipEventRecord(e2, 0));
            HIPCHECK(hipEventSynchronize(e2));
            float a = 0, b = 0;
            HIPCHECK(hipEventElapsedTime(&a, e0, e1));
            HIPCHECK(hipEventElapsedTime(&b, e1, e2));
            if (it > 0) {
                tf += a;
                ts += b;
            }
        }
        *ms_factor = tf / reps;
        *ms_solve = ts / reps;
        if (trace) {
            const size_t nts = (size_t)32 * (m_pad / kNB + 1);
            unsigned long long *dt = dalloc<unsigned long long>(nts, owned);
            HIPCHECK(hipMemset(dt, 0, nts * sizeof(unsigned long long)));
            HIPCHECK(hipMemcpy(dA, src, h.size() * sizeof(double), hipMemcpyDeviceToDevice));
            chol_factor(0, dA, m_pad, m_pad, 1, de, Wd, fl, dt);
            HIPCHECK(hipDeviceSynchronize());
            HIPCHECK(hipMemcpy(trace, dt, nts * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        }
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        (void)hipEventDestroy(e2);
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        rc = -1;
    }
    for (void *q : owned) (void)hipFree(q);
    return rc;
}

int bb_gram(double *C, const double *Yh, const double *wh, int n, int k) {
    std::vector<void *> owned;
    int rc = 0;
    try {
        HIPCHECK(hipSetDevice(g_device));
        const int n_pad = round_up(n, kGramTile);
        const int k_pad = round_up(k, 256);
        double *dY = dalloc<double>((size_t)n_pad * k_pad, owned);
        double *dw = dalloc<double>(k_pad, owned);
        HIPCHECK(hipMemcpy2D(dY, (size_t)n_pad * sizeof(double), Yh, (size_t)n * sizeof(double),
                             (size_t)n * sizeof(double), (size_t)k, hipMemcpyHostToDevice));
        HIPCHECK(hipMemcpy(dw, wh, (size_t)k * sizeof(double), hipMemcpyHostToDevice));
        const int S = gram_splits_for(n_pad, k_pad);
        const size_t stride = (size_t)n_pad * n_pad;
        double *sl = dalloc<double>(stride * S, owned);
        double *red = dalloc<double>(stride + n_pad, owned);
        launch_gram(0, dY, n_pad, dw, n_pad, k_pad, S, sl, n_pad, stride);
        launch_slab_sum(0, sl, S, stride, n_pad, nullptr, 0, red, 1);
        HIPCHECK(hipGetLastError());
        std::vector<double> h(tri_count(n_pad));
        HIPCHECK(hipMemcpy(h.data(), red, h.size() * sizeof(double), hipMemcpyDeviceToHost));
        for (int c = 0; c < n; ++c)
            for (int r = 0; r < n; ++r)
                C[(size_t)r + (size_t)c * n] = r <= c ? h[tri_index(r, c)] : h[tri_index(c, r)];
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        rc = -1;
    }
    for (void *q : owned) (void)hipFree(q);
    return rc;
}

int bb_gram_ozaki(double *C, const double *Yh, const double *wh, int n, int k) {
    std::vector<void *> owned;
    int rc = 0;
    try {
        HIPCHECK(hipSetDevice(g_device));
        const int n_pad = round_up(n, kGramTile);
        const int n_oz = oz_rows(n_pad);
        const int k_pad = round_up(k, 256);
        const int nkc = k_pad / kOzKC;
        double *dY = dalloc<double>((size_t)n_pad * k_pad, owned);
        double *dw = dalloc<double>(k_pad, owned);
        HIPCHECK(hipMemcpy2D(dY, (size_t)n_pad * sizeof(double), Yh, (size_t)n * sizeof(double),
                             (size_t)n * sizeof(double), (size_t)k, hipMemcpyHostToDevice));
        HIPCHECK(hipMemcpy(dw, wh, (size_t)k * sizeof(double), hipMemcpyHostToDevice));
        const int b = oz_bits_for(k_pad);
        const int S = oz_splits_for(n_oz, nkc);
        double *xmax = dalloc<double>((size_t)nkc * n_oz, owned);
        double *rowmax = dalloc<double>((size_t)oz_bound_groups(k_pad) * n_oz, owned);
        double *rscale = dalloc<double>(n_oz, owned);
        int *escale = dalloc<int>(n_oz, owned);
        int8_t *R = dalloc<int8_t>(oz_residue_bytes(n_oz, k_pad), owned);
        int8_t *P = dalloc<int8_t>(oz_partial_bytes(n_oz, S), owned);
        const size_t stride = (size_t)n_pad * n_pad;
        double *red = dalloc<double>(stride + n_pad, owned);
        launch_oz_xmax(0, dY, n_pad, n_pad, n_oz, k_pad, xmax);
        launch_oz_scale(0, dw, k_pad, xmax, n_oz, b, rowmax, rscale, escale);
        launch_oz_residues(0, dY, n_pad, n_pad, n_oz, k_pad, dw, rscale, R);
        launch_oz_gemm(0, R, n_oz, k_pad, S, P);
        launch_oz_crt(0, P, S, n_oz, n_pad, escale, nullptr, 0, red);
        HIPCHECK(hipGetLastError());
        std::vector<double> h(tri_count(n_pad));
        HIPCHECK(hipMemcpy(h.data(), red, h.size() * sizeof(double), hipMemcpyDeviceToHost));
        for (int c = 0; c < n; ++c)
            for (int r = 0; r < n; ++r)
                C[(size_t)r + (size_t)c * n] = r <= c ? h[tri_index(r, c)] : h[tri_index(c, r)];
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        rc = -1;
    }
    for (void *q : owned) (void)hipFree(q);
    return rc;
}

int bb_sparse_gram(double *C, double *xu, const int *colptr, const int *rowidx, const double *val,
                   const double *D, const double *u, int n, int p) {
    std::vector<void *> owned;
    int rc = 0;
    try {
        HIPCHECK(hipSetDevice(g_device));
        const int n_pad = round_up(n, kGramTile);
        SparseDesign sd;
        sd.build(0, n, n_pad, p, colptr, rowidx, val, owned);
        double *dD = dalloc<double>(p, owned), *du = dalloc<double>(p, owned);
        HIPCHECK(hipMemcpy(dD, D, (size_t)p * sizeof(double), hipMemcpyHostToDevice));
        if (u) HIPCHECK(hipMemcpy(du, u, (size_t)p * sizeof(double), hipMemcpyHostToDevice));
        double *tri = dalloc<double>(tri_count(n_pad), owned);
        double *dxu = dalloc<double>(n_pad, owned);
        sd.gram(0, dD, du, tri, dxu);
        HIPCHECK(hipGetLastError());
        std::vector<double> h(tri_count(n_pad));
        HIPCHECK(hipMemcpy(h.data(), tri, h.size() * sizeof(double), hipMemcpyDeviceToHost));
        for (int c = 0; c < n; ++c)
            for (int r = 0; r < n; ++r)
                C[(size_t)r + (size_t)c * n] = r <= c ? h[tri_index(r, c)] : h[tri_index(c, r)];
        if (xu) HIPCHECK(hipMemcpy(xu, dxu, (size_t)n * sizeof(double), hipMemcpyDeviceToHost));
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        rc = -1;
    }
    for (void *q : owned) (void)hipFree(q);
    return rc;
}

int bb_bench_sparse_gram(const int *colptr, const int *rowidx, const double *val, const double *D,
                         int n, int p, int reps, double *ms_gram, double *ms_rows,
                         long long *pairs) {
    std::vector<void *> owned;
    int rc = 0;
    try {
        HIPCHECK(hipSetDevice(g_device));
        const int n_pad = round_up(n, kGramTile);
        SparseDesign sd;
        sd.build(0, n, n_pad, p, colptr, rowidx, val, owned);
        double *dD = dalloc<double>(p, owned), *du = dalloc<double>(p, owned);
        HIPCHECK(hipMemcpy(dD, D, (size_t)p * sizeof(double), hipMemcpyHostToDevice));
        double *tri = dalloc<double>(tri_count(n_pad), owned);
        double *dxu = dalloc<double>(n_pad, owned);
        hipEvent_t e0, e1, e2;
        HIPCHECK(hipEventCreate(&e0));
        HIPCHECK(hipEventCreate(&e1));
        HIPCHECK(hipEventCreate(&e2));
        sd.gram(0, dD, du, tri, dxu);  // warm
        float tg = 0, tr = 0;
        for (int r = 0; r < reps; ++r) {
            HIPCHECK(hipEventRecord(e0, 0));
            if (sd.col_mode)
                sd.gram(0, dD, du, tri, dxu);
            else
                launch_sp_gram(0, sd.estart, sd.prod, sd.pj, dD, n_pad, tri);
            HIPCHECK(hipEventRecord(e1, 0));
            if (!sd.col_mode)
                launch_sp_rows(0, sd.rowptr, sd.colidx, sd.rval, n_pad, du, dD, dxu, tri);
            HIPCHECK(hipEventRecord(e2, 0));
            HIPCHECK(hipEventSynchronize(e2));
            float a = 0, b = 0;
            HIPCHECK(hipEventElapsedTime(&a, e0, e1));
            HIPCHECK(hipEventElapsedTime(&b, e1, e2));
            tg += a;
            tr += b;
        }
        *ms_gram = tg / reps;
        *ms_rows = tr / reps;
        if (pairs) *pairs = (long long)sd.pairs;
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        (void)hipEventDestroy(e2);
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        rc = -1;
    }
    for (void *q : owned) (void)hipFree(q);
    return rc;
}

int bb_bench_ozaki(int n, int k, int nsplit, int dbg, int reps, double *ms) {
    std::vector<void *> owned;
    int rc = 0;
    try {
        HIPCHECK(hipSetDevice(g_device));
        const int n_oz = oz_rows(round_up(n, kGramTile));
        const int k_pad = round_up(k, 256);
        const int S = nsplit > 0 ? nsplit : oz_splits_for(n_oz, k_pad / kOzKC);
        int8_t *R = dalloc<int8_t>(oz_residue_bytes(n_oz, k_pad), owned);
        int8_t *P = dalloc<int8_t>(oz_partial_bytes(n_oz, S), owned);
        // random residues in [-120, 120]
        std::vector<int8_t> h(oz_residue_bytes(n_oz, k_pad));
        uint64_t st = 0x9E3779B97F4A7C15ULL;
        for (auto &v : h) {
            st = st * 6364136223846793005ULL + 1442695040888963407ULL;
            v = (int8_t)((int)((st >> 33) % 241) - 120);
        }
        HIPCHECK(hipMemcpy(R, h.data(), h.size(), hipMemcpyHostToDevice));
        hipEvent_t e0, e1;
        HIPCHECK(hipEventCreate(&e0));
        HIPCHECK(hipEventCreate(&e1));
        // dbg 999: production kernel without K rotation; 1000 + L: with pair lead L / 1000;
        // 1000000 + 1000 T + L: lead L / 1000 and late shift T / 1000
        int lead = kOzLeadDefault, late = -1;
        if (dbg == 999 || (dbg >= 1000 && dbg < 2000)) {
            lead = dbg == 999 ? -1 : dbg - 1000;
            dbg = 0;
        } else if (dbg >= 1000000) {
            lead = dbg % 1000;
            late = (dbg / 1000) % 1000;
            dbg = 0;
        }
        launch_oz_gemm(0, R, n_oz, k_pad, S, P, dbg, lead, late);
        HIPCHECK(hipEventRecord(e0, 0));
        for (int r = 0; r < reps; ++r) launch_oz_gemm(0, R, n_oz, k_pad, S, P, dbg, lead, late);
        HIPCHECK(hipEventRecord(e1, 0));
        HIPCHECK(hipEventSynchronize(e1));
        float t = 0;
        HIPCHECK(hipEventElapsedTime(&t, e0, e1));
        *ms = t / reps;
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        rc = -1;
    }
    for (void *q : owned) (void)hipFree(q);
    return rc;
}

int bb_chol_solve(double *x, const double *Ah, const double *bh, int m, int nrhs) {
    std::vector<void *> owned;
    int rc = 0;
    try {
        if (nrhs < 1 || nrhs > 2) throw HipError("nrhs must be 1 or 2");
        HIPCHECK(hipSetDevice(g_device));
        const int m_pad = round_up(m, kNB);
        double *dA = dalloc<double>((size_t)m_pad * (m_pad + kNB), owned);
        // identity padding, then the user block and the RHS (forward-solved in place)
        std::vector<double> h((size_t)m_pad * (m_pad + kNB), 0.0);
        for (int c = 0; c < m_pad; ++c)
            for (int r = 0; r <= c; ++r)
                h[(size_t)r + (size_t)c * m_pad] =
                    (r < m && c < m) ? Ah[(size_t)r + (size_t)c * m] : (r == c ? 1.0 : 0.0);
        for (int q = 0; q < nrhs; ++q)
            for (int r = 0; r < m; ++r) h[(size_t)r + (size_t)(m_pad + q) * m_pad] = bh[r + (size_t)q * m];
        HIPCHECK(hipMemcpy(dA, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice));
        double *Wd = dalloc<double>(chol_wd_words(m_pad), owned);
        unsigned int *fl = dalloc<unsigned int>(chol_flag_words(m_pad, 1), owned);
        double *W = dalloc<double>((size_t)m_pad * nrhs, owned);
        uint32_t *de = dalloc<uint32_t>(1, owned);
        chol_factor(0, dA, m_pad, m_pad, 1, de, Wd, fl);
        chol_bsolve(0, dA, m_pad, m_pad, Wd, dA + (size_t)m_pad * m_pad, W, nrhs, fl, de);
        HIPCHECK(hipGetLastError());
        std::vector<double> hw((size_t)m_pad * nrhs);
        HIPCHECK(hipMemcpy(hw.data(), W, hw.size() * sizeof(double), hipMemcpyDeviceToHost));
        for (int q = 0; q < nrhs; ++q)
            for (int r = 0; r < m; ++r) x[r + (size_t)q * m] = hw[r + (size_t)q * m_pad];
        uint32_t f = 0;
        HIPCHECK(hipMemcpy(&f, de, sizeof(f), hipMemcpyDeviceToHost));
        if (f & 8u) {
            set_error("matrix is not positive definite");
            rc = -3;
        }
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        rc = -1;
    }
    for (void *q : owned) (void)hipFree(q);
    return rc;
}

// ---------------------------------------------------------------------------
// Bridge EM (restating BR::EM, Code/C/BridgeRegression.cpp:600-708, with sig = 1 and
// tau = ratio as the EM wrapper passes them, BridgeWrapper.cpp:57-73).  X'X and X'y are
// formed once on the device; every maximisation step assembles the masked system on the
// device (k_em_form), factors it with the persistent Cholesky and back-solves, or runs
// conjugate gradients (k_em_cg).  The expectation step (lambda_j, the active set, the
// distance) is an O(p) host loop over the same order as the reference.
// Returns the number of "solves" (total_iter) or, when every coefficient was dropped, the
// EM iteration count (the reference's early `return iter`); -1 after an error.
// ---------------------------------------------------------------------------
int bb_bridge_em(double *beta_out, const double *yh, const double *Xh, int n, int p, double ratio,
                 double alpha, double lambda_max, double tol, int max_iter, int use_cg) {
    std::vector<void *> owned;
    int ret = -1;
    std::fill(beta_out, beta_out + p, 0.0);
    try {
        HIPCHECK(hipSetDevice(g_device));
        const int n_pad = round_up(n, kGramTile), p_pad = round_up(p, 256);
        double *dX = dalloc<double>((size_t)n_pad * p_pad, owned);
        double *dy = dalloc<double>(n_pad, owned);
        HIPCHECK(hipMemcpy2D(dX, (size_t)n_pad * sizeof(double), Xh, (size_t)n * sizeof(double),
                             (size_t)n * sizeof(double), (size_t)p, hipMemcpyHostToDevice));
        HIPCHECK(hipMemcpy(dy, yh, (size_t)n * sizeof(double), hipMemcpyHostToDevice));
        // G = X'X (transpose, Gram over rows with unit weights), b = X'y
        double *Xt = dalloc<double>((size_t)p_pad * n_pad, owned);
        launch_transpose(0, dX, n_pad, n_pad, p_pad, Xt, p_pad);
        double *ones = dalloc<double>(n_pad, owned);
        {
            std::vector<double> h1(n_pad, 1.0);
            HIPCHECK(hipMemcpy(ones, h1.data(), n_pad * sizeof(double), hipMemcpyHostToDevice));
        }
        const int Sg = gram_splits_for(p_pad, n_pad);
        const size_t gstride = (size_t)p_pad * p_pad;
        double *sl = dalloc<double>(gstride * Sg, owned);
        launch_gram(0, Xt, p_pad, ones, p_pad, n_pad, Sg, sl, p_pad, gstride);
        double *G = dalloc<double>(gstride + p_pad, owned);
        launch_slab_sum(0, sl, Sg, gstride, p_pad, nullptr, 0, G, 0);
        double *bvec = dalloc<double>(p_pad, owned);
        launch_coldot(0, dX, n_pad, n_pad, dy, p, bvec);
        double *A = dalloc<double>((size_t)p_pad * (p_pad + kNB), owned);
        double *Wd = dalloc<double>(chol_wd_words(p_pad), owned);
        unsigned int *fl = dalloc<unsigned int>(chol_flag_words(p_pad, 1), owned);
        double *W = dalloc<double>(p_pad, owned);
        double *dlam = dalloc<double>(p_pad, owned);
        int *dmask = dalloc<int>(p_pad, owned);
        double *work = dalloc<double>((size_t)3 * p_pad, owned);
        int *dit = dalloc<int>(1, owned);
        uint32_t *de = dalloc<uint32_t>(1, owned);

        std::vector<int> mask(p, 1);
        std::vector<double> nb(p_pad, 0.0), ob(p, 0.0), lam(p_pad, 0.0);
        auto upload_mask = [&]() {
            std::vector<int> m(p_pad, 0);
            std::copy(mask.begin(), mask.end(), m.begin());
            HIPCHECK(hipMemcpy(dmask, m.data(), p_pad * sizeof(int), hipMemcpyHostToDevice));
        };
        // direct maximisation: A = XX_act (+ c2 diag(lam)), solve by Cholesky (symsolve)
        auto solve_direct = [&](bool with_lam) {
            launch_em_form(0, G, p_pad, with_lam ? dlam : nullptr, dmask, bvec, p, p_pad, A,
                           p_pad, p_pad);
            HIPCHECK(hipMemset(de, 0, sizeof(uint32_t)));
            chol_factor(0, A, p_pad, p_pad, 1, de, Wd, fl);
            chol_bsolve(0, A, p_pad, p_pad, Wd, A + (size_t)p_pad * p_pad, W, 1, fl, de);
            HIPCHECK(hipGetLastError());
            uint32_t f = 0;
            HIPCHECK(hipMemcpy(&f, de, sizeof(f), hipMemcpyDeviceToHost));
            if (f & 8u) throw HipError("symsolve: matrix is not positive definite");
            if (f) throw HipError("device solver reported an error");
            HIPCHECK(hipMemcpy(nb.data(), W, p_pad * sizeof(double), hipMemcpyDeviceToHost));
        };
        const double sig = 1.0, tau = ratio;
        const double c1 = alpha * std::exp((2 - alpha) * (std::log(tau) - std::log(sig)));
        const double c2 = std::exp(-2 * (std::log(tau) - std::log(sig)));
        int pa = p;             // active count
        long total_iter = p;    // the first symsolve
        upload_mask();
        solve_direct(false);    // one maximisation step with A = X'X
        double dist = tol + 1.0;
        int iter = 0;
        while (dist > tol && iter < max_iter) {
            // expectation step over the active coordinates, in order
            int num = 0;
            for (int j = 0; j < p; ++j) {
                if (!mask[j]) continue;
                const double l = c1 * std::exp((alpha - 2) * std::log(std::fabs(nb[j])));
                if (l < lambda_max) {
                    lam[j] = c2 * l;
                    ob[j] = nb[j];
                    ++num;
                } else {
                    mask[j] = 0;
                }
            }
            if (num < pa) {
                if (num == 0) {
                    ret = iter;
                    for (void *q : owned) (void)hipFree(q);
                    owned.clear();
                    return ret;
                }
                pa = num;
                upload_mask();
            }
            HIPCHECK(hipMemcpy(dlam, lam.data(), p_pad * sizeof(double), hipMemcpyHostToDevice));
            if (!use_cg) {
                solve_direct(true);
                total_iter += pa;
            } else {
                // x0 = old beta on the active set (0 elsewhere)
                std::vector<double> x0(p_pad, 0.0);
                for (int j = 0; j < p; ++j)
                    if (mask[j]) x0[j] = ob[j];
                HIPCHECK(hipMemcpy(W, x0.data(), p_pad * sizeof(double), hipMemcpyHostToDevice));
                launch_em_form(0, G, p_pad, dlam, dmask, bvec, p, p_pad, A, p_pad, p_pad);
                launch_em_cg(0, A, p_pad, p_pad, A + (size_t)p_pad * p_pad, W, tol, pa, work,
                             dit);
                HIPCHECK(hipGetLastError());
                int it = 0;
                HIPCHECK(hipMemcpy(&it, dit, sizeof(int), hipMemcpyDeviceToHost));
                HIPCHECK(hipMemcpy(nb.data(), W, p_pad * sizeof(double), hipMemcpyDeviceToHost));
                total_iter += it;
            }
            double d2 = 0.0;
            for (int j = 0; j < p; ++j)
                if (mask[j]) d2 += (nb[j] - ob[j]) * (nb[j] - ob[j]);
            dist = std::sqrt(d2);
            ++iter;
        }
        for (int j = 0; j < p; ++j) beta_out[j] = mask[j] ? nb[j] : 0.0;
        ret = (int)total_iter;
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        std::fill(beta_out, beta_out + p, 0.0);
        ret = -1;
    }
    for (void *q : owned) (void)hipFree(q);
    return ret;
}

// Batched EM over `count` ratios (trace.beta), direct solves: X'X and X'y once, then one
// launch in which a workgroup per ratio runs the whole EM -- k_em_batch (system in LDS) for
// p <= 128, k_em_batch_tiled (system in a global scratch slice per ratio, tiled Cholesky)
// above, the ratios in chunks whose scratch fits min(free / 2, 16 GiB).
// beta: count x p (row r = ratio r); solves: count (as bb_bridge_em returns, -1 on a
// non positive-definite system).  Returns 0, or -1 with bb_last_error().
int bb_bridge_em_batch(double *beta, int *solves, const double *yh, const double *Xh, int n,
                       int p, const double *ratios, const double *lambda_max, int count,
                       double alpha, double tol, int max_iter) {
    std::vector<void *> owned;
    int rc = 0;
    try {
        if (p < 1) throw HipError("bb_bridge_em_batch: needs p >= 1");
        if (count < 1) throw HipError("bb_bridge_em_batch: empty ratio grid");
        HIPCHECK(hipSetDevice(g_device));
        const int n_pad = round_up(n, kGramTile), p_pad = round_up(p, 256);
        double *dX = dalloc<double>((size_t)n_pad * p_pad, owned);
        double *dy = dalloc<double>(n_pad, owned);
        HIPCHECK(hipMemcpy2D(dX, (size_t)n_pad * sizeof(double), Xh, (size_t)n * sizeof(double),
                             (size_t)n * sizeof(double), (size_t)p, hipMemcpyHostToDevice));
        HIPCHECK(hipMemcpy(dy, yh, (size_t)n * sizeof(double), hipMemcpyHostToDevice));
        double *Xt = dalloc<double>((size_t)p_pad * n_pad, owned);
        launch_transpose(0, dX, n_pad, n_pad, p_pad, Xt, p_pad);
        double *ones = dalloc<double>(n_pad, owned);
        {
            std::vector<double> h1(n_pad, 1.0);
            HIPCHECK(hipMemcpy(ones, h1.data(), n_pad * sizeof(double), hipMemcpyHostToDevice));
        }
        const int Sg = gram_splits_for(p_pad, n_pad);
        const size_t gstride = (size_t)p_pad * p_pad;
        double *sl = dalloc<double>(gstride * Sg, owned);
        launch_gram(0, Xt, p_pad, ones, p_pad, n_pad, Sg, sl, p_pad, gstride);
        double *G = dalloc<double>(gstride + p_pad, owned);
        launch_slab_sum(0, sl, Sg, gstride, p_pad, nullptr, 0, G, 0);
        double *bvec = dalloc<double>(p_pad, owned);
        launch_coldot(0, dX, n_pad, n_pad, dy, p, bvec);
        double *dr = dalloc<double>(count, owned), *dl = dalloc<double>(count, owned);
        HIPCHECK(hipMemcpy(dr, ratios, count * sizeof(double), hipMemcpyHostToDevice));
        HIPCHECK(hipMemcpy(dl, lambda_max, count * sizeof(double), hipMemcpyHostToDevice));
        double *db = dalloc<double>((size_t)count * p, owned);
        int *ds = dalloc<int>(count, owned);
        if (p <= 128) {
            launch_em_batch(0, G, p_pad, bvec, p, dr, dl, count, alpha, tol, max_iter, db, ds);
            HIPCHECK(hipGetLastError());
        } else {
            const int pe = round_up(p, em_tile());
            const size_t per = (size_t)pe * pe * sizeof(double);
            size_t fr = 0, tot = 0;
            HIPCHECK(hipMemGetInfo(&fr, &tot));
            const size_t budget = std::min(fr / 2, (size_t)16 << 30);
            const int chunk = (int)std::max<size_t>(1, std::min<size_t>(count, budget / per));
            if (per > fr) throw HipError("bb_bridge_em_batch: p x p system does not fit");
            double *scr = dalloc<double>((size_t)chunk * pe * pe, owned);
            double *vec = dalloc<double>((size_t)chunk * 3 * pe, owned);
            int *msk = dalloc<int>((size_t)chunk * pe, owned);
            for (int r0 = 0; r0 < count; r0 += chunk) {
                launch_em_batch_tiled(0, G, p_pad, bvec, p, pe, dr, dl, r0,
                                      std::min(chunk, count - r0), alpha, tol, max_iter, scr, vec,
                                      msk, db, ds);
                HIPCHECK(hipGetLastError());
            }
        }
        HIPCHECK(hipMemcpy(beta, db, (size_t)count * p * sizeof(double), hipMemcpyDeviceToHost));
        HIPCHECK(hipMemcpy(solves, ds, count * sizeof(int), hipMemcpyDeviceToHost));
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        rc = -1;
    }
    for (void *q : owned) (void)hipFree(q);
    return rc;
}

// ---------------------------------------------------------------------------
// Reference .C entry points
// ---------------------------------------------------------------------------
// BridgeWrapper.cpp:738-756: flags NaN / +Inf / -Inf / NA in x[0] and sets x[0] = NA when
// it is 0 (a marshalling test of R's special values; host only).
void mytest(int *out, double *x) {
    const uint64_t na_bits = 0x7FF00000000007A2ull;  // R's NA_REAL
    uint64_t bits;
    memcpy(&bits, x, sizeof(bits));
    out[0] = 0;
    if (std::isnan(x[0])) out[0] = 1;
    if (x[0] == HUGE_VAL) out[0] = 2;
    if (x[0] == -HUGE_VAL) out[0] = 3;
    if (std::isnan(x[0]) && (uint32_t)bits == 1954u) out[0] = 4;
    if (x[0] == 0.0) memcpy(x, &na_bits, sizeof(na_bits));
}

static void trunc_call(int mode, int num, double *x, const double *p0, const double *p1,
                       const double *p2, const double *p3, const char *name) {
    uint64_t k0, k1;
    next_call_key(&k0, &k1);
    if (bb_trunc_batch(mode, num, x, p0, p1, p2, p3, k0, k1) != 0)
        fprintf(stderr, "Error: %s: %s\n", name, g_last_error.c_str());
}

// BridgeWrapper.cpp:843-935 (decl. BridgeWrapper.h:236-242)
void rtnorm_left(double *x, double *left, double *mu, double *sig, int *num) {
    trunc_call(0, *num, x, left, mu, sig, nullptr, "rtnorm_left");
}
void rtnorm_both(double *x, double *left, double *right, double *mu, double *sig, int *num) {
    trunc_call(1, *num, x, left, right, mu, sig, "rtnorm_both");
}
void rtnorm(double *x, double *left, double *right, double *mu, double *sig, int *num) {
    trunc_call(2, *num, x, left, right, mu, sig, "rtnorm");
}
// BridgeWrapper.cpp:762-830 (decl. BridgeWrapper.h:230-234)
void rtexpon_rate_left(double *x, double *left, double *rate, int *num) {
    trunc_call(3, *num, x, left, rate, nullptr, nullptr, "rtexpon_rate_left");
}
void rtexpon_rate_both(double *x, double *left, double *right, double *rate, int *num) {
    trunc_call(4, *num, x, left, right, rate, nullptr, "rtexpon_rate_both");
}
void rtexpon_rate(double *x, double *left, double *right, double *rate, int *num) {
    trunc_call(5, *num, x, left, right, rate, nullptr, "rtexpon_rate");
}

// BridgeWrapper.cpp:944-962 (decl. BridgeWrapper.h:242); `scale` carries the shape, as
// rrtgamma (BridgeWrapper.R:482-509) passes it.
void rrtgamma_rate(double *x, double *scale, double *rate, double *right_t, int *num) {
    uint64_t k0, k1;
    next_call_key(&k0, &k1);
    if (bb_rrtgamma_batch(*num, x, scale, rate, right_t, k0, k1) != 0)
        fprintf(stderr, "Error: rrtgamma_rate: %s\n", g_last_error.c_str());
}

void retstable_LD(double *x, double *alpha, double *V0, double *h, int *num) {
    uint64_t k0, k1;
    next_call_key(&k0, &k1);
    int rc = bb_retstable_batch(x, alpha, V0, h, *num, k0, k1, 0, 0);
    if (rc != 0) fprintf(stderr, "Error: retstable_LD: %s\n", g_last_error.c_str());
}

// BridgeWrapper.cpp:544-568 (decl. BridgeWrapper.h:166-176); R passes use.cg through
// as.integer, so it is read as int (BridgeWrapper.R:116-123).  max_iter returns the number
// of solves; errors print as the reference's EM wrapper does (BridgeWrapper.cpp:64-70).
void bridge_EM(double *betap, const double *yp, const double *Xp, const double *ratio,
               const double *alpha, const int *P, const int *N, const double *lambda_max,
               const double *tol, int *max_iter, const int *use_cg) {
    if (*use_cg && g_verbose) printf("Using conjugate gradient method.\n");
    const int it = bb_bridge_em(betap, yp, Xp, *N, *P, *ratio, *alpha, *lambda_max, *tol,
                                *max_iter, *use_cg);
    if (it < 0) {
        printf("Error: %s\n", g_last_error.c_str());
        printf("Aborting EM.\n");
    }
    *max_iter = it;
}

}  // extern "C"

namespace {

// ---------------------------------------------------------------------------
// .C drivers: device selection, trace ring with chunked copy-out, interrupt polling.
// ---------------------------------------------------------------------------
// bb_set_device_count: devices a .C chain may shard over (0: every visible device).  The
// default is 1: a sharded chain sums its Gram in a different fp64 order than one device, and
// p > n chains amplify such roundoff, so traces depend on the device count and
// multi-device sharding is opt-in.
int g_max_devices = 1;
size_t g_trace_budget = size_t(1) << 30;   // device bytes of trace ring per engine
std::atomic<int> g_debug_interrupt{-1};     // bb_debug_interrupt_after (test hook)
int g_last_devices = 0, g_last_interrupted = 0, g_last_capacity = 0;

// R's interrupt machinery, resolved at run time (absent outside R).  The reference polls
// R_CheckUserInterrupt every 10 sweeps (BridgeWrapper.cpp:273-275, 295-297), which longjmps
// out of the sampler; here the check runs under R_ToplevelExec, so a pending interrupt is
// caught without unwinding through frames that own device memory or communicators, the
// chain stops, the device is released, and the interrupt is re-raised from the .C frame.
struct RInterrupt {
    int (*toplevel)(void (*)(void *), void *) = nullptr;  // R_ToplevelExec (Rboolean)
    void (*check)(void) = nullptr;                        // R_CheckUserInterrupt
    void (*onintr)(void) = nullptr;                       // Rf_onintr
    bool tried = false;
    bool ok() {
        if (!tried) {
            tried = true;
            toplevel = (int (*)(void (*)(void *), void *))dlsym(RTLD_DEFAULT, "R_ToplevelExec");
            check = (void (*)(void))dlsym(RTLD_DEFAULT, "R_CheckUserInterrupt");
            onintr = (void (*)(void))dlsym(RTLD_DEFAULT, "Rf_onintr");
        }
        return toplevel && check;
    }
} g_rint;

void r_check_cb(void *) { g_rint.check(); }

bool poll_interrupt() {
    int d = g_debug_interrupt.load();
    while (d >= 0) {  // test hook: the d-th poll from now reports an interrupt
        if (g_debug_interrupt.compare_exchange_weak(d, d == 0 ? -1 : d - 1)) {
            if (d == 0) return true;
            break;
        }
    }
    if (g_rint.ok()) return g_rint.toplevel(r_check_cb, nullptr) == 0;
    return false;
}

// From a .C frame with no live C++ objects: hand the caught interrupt back to R.
void reraise_interrupt() {
    if (g_rint.ok() && g_rint.onintr) g_rint.onintr();
}

// bb_config of a .C bridge_reg_stable call (BridgeWrapper.cpp:659-693)
bb_config stable_call_config(const double *sig2_shape, const double *sig2_scale,
                             const double *nu_shape, const double *nu_rate, const double *alpha_a,
                             const double *alpha_b, const double *true_sig2,
                             const double *true_tau, const double *true_alpha, int p, int n,
                             int m, const int *ortho) {
    bb_config c;
    bb_config_default(&c);
    c.n = n;
    c.p = p;
    c.p_local = p;
    c.sig2_shape = *sig2_shape;
    c.sig2_scale = *sig2_scale;
    c.nu_shape = *nu_shape;
    c.nu_rate = *nu_rate;
    c.alpha_a = *alpha_a;
    c.alpha_b = *alpha_b;
    c.true_sig2 = *true_sig2;
    c.true_tau = *true_tau;
    c.true_alpha = *true_alpha;
    c.ortho = *ortho != 0;
    c.trace_capacity = m < 1 ? 1 : m;
    c.device = g_device;
    next_call_key(&c.seed, &c.stream);
    return c;
}

// Trace ring slots for M samples of p_local coefficients (`ntr` p-long traces per slot):
// the whole run if it fits the per-engine budget, else a ring copied out in chunks.
int ring_capacity(int m, int p_local, int ntr) {
    const size_t per = (size_t)ntr * p_local * sizeof(double) + 3 * sizeof(double);
    size_t cap = g_trace_budget / (per ? per : 1);
    if (cap < 16) cap = 16;
    return (int)std::min<size_t>(cap, (size_t)(m < 1 ? 1 : m));
}

// Devices for a column-sharded chain: 1 unless p > n (the Woodbury path, or the orthogonal
// design; alpha known or unknown) and sharding was enabled (bb_set_device_count); at least
// 4096 columns per device.
int chain_devices(const bb_config &c, int nvis = -1) {
    if (nvis < 0) nvis = bb_device_count();
    int k = g_max_devices > 0 ? std::min(g_max_devices, nvis) : nvis;
    if (c.p <= c.n || (c.method != 0 && c.method != 2 && c.method != 3)) return 1;
    k = std::min(k, std::max(1, c.p / 4096));
    return std::max(1, k);
}

// One chain: a single engine, or the column shards of a multi-device RCCL group.
struct Chain {
    std::vector<bb_engine *> eng;
    std::vector<int> j0s;
    bb_group *grp = nullptr;
    int p = 0, cap = 1;
    hipEvent_t evring[3] = {nullptr, nullptr, nullptr};
    long nmarks = 0;

    ~Chain() {
        for (auto e : evring)
            if (e) (void)hipEventDestroy(e);
        if (grp) bb_group_destroy(grp);
        for (auto *e : eng) bb_engine_destroy(e);
    }
    int init() { return grp ? bb_group_init_state(grp) : bb_engine_init_state(eng[0]); }
    bool fused() const { return !grp && eng.size() == 1 && eng[0]->fused; }
    int run(uint64_t t0, int count, int slot, int step, int mcmc) {
        return grp ? bb_group_run(grp, t0, count, slot, step, mcmc)
                   : bb_engine_run(eng[0], t0, count, slot, step, mcmc);
    }
    int sync() { return grp ? bb_group_sync(grp) : bb_engine_sync(eng[0]); }
    uint32_t flags() {
        uint32_t all = 0;
        for (auto *e : eng) {
            uint32_t f = 0;
            (void)hipSetDevice(e->cfg.device);
            if (bb_engine_error_flags(e, &f) == 0) all |= f;
        }
        return all;
    }
    // Marks the work enqueued so far (member 0's stream: members advance in lockstep through
    // the exchanges) and waits until at most two marked blocks are ahead of the device.
    void throttle() {
        HIPCHECK(hipSetDevice(eng[0]->cfg.device));
        hipEvent_t &e = evring[nmarks % 3];
        if (!e) HIPCHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        HIPCHECK(hipEventRecord(e, eng[0]->stream));
        if (nmarks >= 2) HIPCHECK(hipEventSynchronize(evring[(nmarks - 2) % 3]));
        ++nmarks;
    }
    // trace slots [slot0, slot0 + count) -> samples [s0, s0 + count) of the P x M outputs
    int copy_out(int slot0, int count, int s0, double *beta, double *lam, double *sig2,
                 double *tau, double *alpha, double *u = nullptr, double *shape = nullptr) {
        if (count <= 0) return 0;
        const size_t P = (size_t)p;
        if (eng.size() == 1) {
            int rc = bb_engine_get_trace(eng[0], slot0, count, beta + s0 * P, lam + s0 * P,
                                         sig2 ? sig2 + s0 : nullptr, tau + s0, alpha + s0);
            if (rc == 0 && (u || shape))
                rc = bb_engine_get_tri_trace(eng[0], slot0, count, u ? u + s0 * P : nullptr,
                                             shape ? shape + s0 * P : nullptr);
            return rc;
        }
        for (size_t r = 0; r < eng.size(); ++r) {
            bb_engine *e = eng[r];
            const size_t pl = (size_t)e->p_loc;
            std::vector<double> b(pl * count), l(pl * count);
            (void)hipSetDevice(e->cfg.device);
            if (bb_engine_get_trace(e, slot0, count, b.data(), l.data(),
                                    r == 0 && sig2 ? sig2 + s0 : nullptr,
                                    r == 0 ? tau + s0 : nullptr, r == 0 ? alpha + s0 : nullptr))
                return -1;
            for (int k = 0; k < count; ++k) {
                memcpy(beta + (s0 + k) * P + j0s[r], &b[k * pl], pl * sizeof(double));
                memcpy(lam + (s0 + k) * P + j0s[r], &l[k * pl], pl * sizeof(double));
            }
        }
        return 0;
    }
};

// Builds the chain: `create(cfg, j0, j1, &engine)` makes the engine of columns [j0, j1).
template <class Create>
int chain_build(Chain &ch, bb_config c, int ntr, Create create) {
    const int ndev = chain_devices(c);
    const int nvis = std::max(1, bb_device_count());
    ch.p = c.p;
    if (ndev <= 1) {
        c.trace_capacity = ring_capacity(c.trace_capacity, c.p, ntr);
        ch.cap = c.trace_capacity;
        bb_engine *e = nullptr;
        if (create(&c, 0, c.p, &e) != 0) return -1;
        ch.eng.push_back(e);
        ch.j0s.push_back(0);
        return 0;
    }
    const int per = (c.p + ndev - 1) / ndev;
    const int cap = ring_capacity(c.trace_capacity, per, ntr);
    ch.cap = cap;
    for (int r = 0; r < ndev; ++r) {
        bb_config cr = c;
        const int j0 = r * per, j1 = std::min(c.p, j0 + per);
        cr.p_local = j1 - j0;
        cr.j0 = j0;
        cr.rank = r;
        cr.world = ndev;
        cr.device = (g_device + r) % nvis;
        cr.trace_capacity = cap;
        bb_engine *e = nullptr;
        if (create(&cr, j0, j1, &e) != 0) return -1;
        ch.eng.push_back(e);
        ch.j0s.push_back(j0);
    }
    ch.grp = group_create(ch.eng.data(), ndev, true);
    return ch.grp ? 0 : -1;
}

enum Outcome { OUT_OK = 0, OUT_ERROR = 1, OUT_INTERRUPTED = 2 };

// Burn-in then the MCMC samples, in blocks of 10 sweeps between interrupt polls (at most two
// blocks queued ahead of the device), the trace ring copied out whenever it is full.
// Sample s >= 1 runs at t = t_base + s; burn-in is `nburn` sweeps in slot 0 from t = 1.
Outcome drive_chain(Chain &ch, int nburn, uint64_t t_base, int m, int b, double *betap,
                    double *lambdap, double *sig2p, double *taup, double *alphap,
                    double *runtime, double *up = nullptr, double *shapep = nullptr) {
    // BridgeWrapper.cpp:273-275, 295-297 poll every 10 sweeps.  A fused engine runs a
    // whole block in one launch at ~15-30 us per sweep, so it polls every 50 (< 2 ms) and
    // pays the launch and LDS-staging prologue once per 50 sweeps instead of per 10.
    const int kBlock = ch.fused() ? 50 : 10;
    *runtime = 0.0;
    if (ch.init() != 0) return OUT_ERROR;
    bool interrupted = false;
    try {
        auto t0 = std::chrono::steady_clock::now();
        for (int k = 0; k < nburn && !interrupted; k += kBlock) {
            if (ch.run(1 + (uint64_t)k, std::min(kBlock, nburn - k), 0, 0, 0) != 0)
                return OUT_ERROR;
            ch.throttle();
            interrupted = poll_interrupt();
        }
        if (ch.sync() != 0) return OUT_ERROR;
        auto t1 = std::chrono::steady_clock::now();
        if (g_verbose && !interrupted) {
            const double bt = std::chrono::duration<double>(t1 - t0).count();
            printf("Burn-in complete: %g sec. for %i iterations.\n", bt, b);
            if (b > 0) printf("Expect approx. %g sec. for %i samples.\n", bt * m / b, m);
        }
        int copied = 0, next = 1;  // samples copied out / next sample to compute
        while (copied < m && !interrupted) {
            const int hi = std::min(m, copied + ch.cap);
            for (int s = next; s < hi && !interrupted; s += kBlock) {
                const int cnt = std::min(kBlock, hi - s);
                if (ch.run(t_base + (uint64_t)s, cnt, s % ch.cap, 1, 1) != 0) return OUT_ERROR;
                ch.throttle();
                interrupted = poll_interrupt();
                next = s + cnt;
            }
            if (ch.sync() != 0) return OUT_ERROR;
            if (ch.copy_out(copied % ch.cap, next - copied, copied, betap, lambdap, sig2p, taup,
                            alphap, up, shapep) != 0)
                return OUT_ERROR;
            copied = next;
        }
        if (interrupted && copied == 0 && ch.sync() == 0)
            (void)ch.copy_out(0, 1, 0, betap, lambdap, sig2p, taup, alphap, up, shapep);
        *runtime = std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
        if (interrupted) {
            printf("Interrupted: %i of %i samples returned.\n", std::max(copied, 1), m);
            return OUT_INTERRUPTED;
        }
        const uint32_t f = ch.flags();
        if (f & ~4u) {
            printf("Error: numerical failure in the device sampler (flags %u)\n", f);
            printf("Aborting Gibbs sampler.\n");
            fflush(stdout);
        }
    } catch (std::exception &ex) {
        set_error("%s", ex.what());
        return OUT_ERROR;
    }
    return OUT_OK;
}

void print_banner(const char *title, const bb_config &c, int b, int m) {
    if (!g_verbose) return;  // BridgeWrapper.cpp:235-240 (stable), :112-117 (triangles)
    printf("%s", title);
    if (c.true_alpha > 0) printf(" known alpha=%g", c.true_alpha);
    if (c.true_sig2 > 0 && c.method != 6) printf(", sig2=%g", c.true_sig2);
    if (c.true_tau > 0) printf(", tau=%g", c.true_tau);
    if (c.ortho) printf("\nAssuming orthogonal design matrix!");
    printf("\nBurn-in: %i, Num. Samples: %i\n", b, m);
}

// The stable-family .C driver (BridgeWrapper.cpp:207-313 / :434-537): B + 1 burn-in sweeps
// in slot 0, MCMC sample i at t = B + 1 + i.  Errors print and return partial traces.
template <class Create>
Outcome stable_call(const bb_config &c, Create create, int b, double *betap, double *lambdap,
                    double *sig2p, double *taup, double *alphap, double *runtime,
                    const char *title) {
    const int m = c.trace_capacity;
    print_banner(title, c, b, m);
    g_last_interrupted = 0;
    Outcome o;
    {
        Chain ch;
        if (chain_build(ch, c, 2, create) != 0) {
            printf("Error: %s\n", g_last_error.c_str());
            printf("Aborting Gibbs sampler.\n");
            fflush(stdout);
            *runtime = 0.0;
            return OUT_ERROR;
        }
        g_last_devices = (int)ch.eng.size();
        g_last_capacity = ch.cap;
        o = drive_chain(ch, b + 1, (uint64_t)b + 1, m, b, betap, lambdap, sig2p, taup, alphap,
                        runtime);
        if (o == OUT_ERROR) {
            printf("Error: %s\n", g_last_error.c_str());
            printf("Aborting Gibbs sampler.\n");
            fflush(stdout);
        }
    }
    if (g_verbose && o == OUT_OK) printf("Sampling complete: %g sec. for %i iterations.\n", *runtime, m);
    g_last_interrupted = o == OUT_INTERRUPTED;
    return o;
}

Outcome stable_dense(const bb_config &c, const double *yp, const double *Xp, int b,
                     double *betap, double *lambdap, double *sig2p, double *taup, double *alphap,
                     double *runtime, const char *title) {
    const int n = c.n;
    return stable_call(
        c,
        [&](const bb_config *cc, int j0, int, bb_engine **e) {
            return bb_engine_create(cc, Xp + (size_t)j0 * n, yp, e);
        },
        b, betap, lambdap, sig2p, taup, alphap, runtime, title);
}

}  // namespace

extern "C" {

void bb_set_device_count(int count) { g_max_devices = count < 0 ? 0 : count; }

// .C-callable forms of the controls (R's .C passes every argument as a pointer,
// BridgeWrapper.h:164-245; the by-value forms above are for C / ctypes hosts)
void bb_set_device_count_C(const int *count) { bb_set_device_count(*count); }
void bb_get_device_count_C(int *count) { *count = g_max_devices; }
void bb_plan_devices_C(const int *n, const int *p, const int *ortho, const int *nvisible,
                       int *devices) {
    bb_config c;
    bb_config_default(&c);
    c.n = *n;
    c.p = *p;
    c.ortho = *ortho != 0;
    *devices = chain_devices(c, *nvisible >= 0 ? *nvisible : -1);
}
void bb_set_device_C(const int *device, int *status) {
    const int rc = bb_set_device(*device);
    if (status) *status = rc;
}
void bb_set_verbose_C(const int *verbose) { bb_set_verbose(*verbose); }
void bb_use_r_rng_C(const int *enable) { bb_use_r_rng(*enable); }
// R passes numbers as doubles; converting a negative, NaN or out-of-range double to an
// integer type is undefined behaviour, so such a value is refused (the state is kept, the
// reason goes to bb_last_error and stderr) instead of being cast
static bool r_count_ok(const char *what, double v) {
    if (std::isfinite(v) && v >= 0.0 && v <= 9007199254740992.0 && v == std::floor(v)) return true;
    set_error("%s: %g is not an integer in [0, 2^53]; ignored", what, v);
    fprintf(stderr, "BayesBridge: %s: %g is not an integer in [0, 2^53]; ignored\n", what, v);
    return false;
}
void bb_set_seed_C(const double *seed) {
    if (r_count_ok("bb_set_seed_C seed", *seed)) bb_set_seed((uint64_t)*seed);
}
void bb_set_rng_state_C(const double *seed, const double *stream) {
    if (r_count_ok("bb_set_rng_state_C seed", *seed) &&
        r_count_ok("bb_set_rng_state_C stream", *stream))
        bb_set_rng_state((uint64_t)*seed, (uint64_t)*stream);
}
void bb_get_rng_state_C(double *seed, double *stream) {
    uint64_t s = 0, t = 0;
    bb_get_rng_state(&s, &t);
    *seed = (double)s;
    *stream = (double)t;
}
void bb_set_trace_budget_C(const double *bytes) {
    if (r_count_ok("bb_set_trace_budget_C bytes", *bytes)) bb_set_trace_budget((long long)*bytes);
}
void bb_last_call_info_C(int *devices, int *trace_capacity, int *interrupted) {
    (void)bb_last_call_info(devices, trace_capacity, interrupted);
}
void bb_debug_fail_member(int member, int sweep) {
    g_debug_fail_sweep = sweep;
    g_debug_fail_member = member;
}

int bb_set_chol_version(int version) {
    if (version == 0) return g_chol_version;  // query
    if (version < 1 || version > 4) return -1;
    g_chol_version = version;
    return 0;
}
int bb_set_tuning(int key, int value) {
    switch (key) {
        case 1: {
            const int old = g_oz_res_nt;
            if (value >= 0) g_oz_res_nt = value > 2 ? 2 : value;
            return old;
        }
        case 2: {
            const int old = g_bxb_nt;
            if (value >= 0) g_bxb_nt = value ? 1 : 0;
            return old;
        }
        case 3: {
            const int old = g_sp_nt;
            if (value >= 0) g_sp_nt = value > 3 ? 3 : value;
            return old;
        }
        case 4: {
            const int old = g_lam_occ;
            if (value >= 0) g_lam_occ = value & 15;
            return old;
        }
        case 5: {
            const int old = g_lam_lanes;
            if (value == 0 || value == 4 || value == 8 || value == 16 || value == 32 || value == 64)
                g_lam_lanes = value;
            return old;
        }
        case 6: {
            const int old = g_nid_kmax;
            if (value >= 0) g_nid_kmax = value > 64 ? 64 : value;
            return old;
        }
        case 7: {
            const int old = g_lam_xu;
            if (value >= 0) g_lam_xu = value > 3 ? 3 : value;
            return old;
        }
        case 8: {
            const int old = g_nid_sync;
            if (value >= 0) g_nid_sync = value > 2 ? 2 : value;
            return old;
        }
        case 10: {
            const int old = g_nid_mixed;
            if (value >= 0) g_nid_mixed = value ? 1 : 0;
            return old;
        }
        case 9: {
            const int old = g_shard_proto;
            if (value >= 0) g_shard_proto = value ? 1 : 0;
            return old;
        }
        case 11: {
            const int old = g_nid_poll;
            if (value >= 0) g_nid_poll = value ? 1 : 0;
            return old;
        }
        case 16: {  // forced Chebyshev iterate count (benchmarking only; bb_nid.hip)
            const int old = g_nid_force_k;
            if (value >= 0) nid_set_force_k(value > 64 ? 64 : value);
            return old;
        }
        case 12: {
            const int old = g_rs_xcd;
            if (value >= 0) g_rs_xcd = value ? 1 : 0;
            return old;
        }
        case 13: {
            const int old = g_lam_wave;
            if (value >= 0) g_lam_wave = value ? 1 : 0;
            return old;
        }
        case 20: {
            const int old = g_bsolve_ll;
            if (value >= 0) g_bsolve_ll = value ? 1 : 0;
            return old;
        }
        case 17: {
            const int old = g_nid_fold;
            if (value >= 0) g_nid_fold = value > 2 ? 2 : value;
            return old;
        }
        case 15: {
            const int old = g_lam_lend;
            if (value >= 0) g_lam_lend = value ? 1 : 0;
            return old;
        }
        default: return -1;
    }
}
void bb_set_trace_budget(long long bytes) {
    g_trace_budget = bytes > 0 ? (size_t)bytes : (size_t(1) << 30);
}
void bb_debug_interrupt_after(int polls) { g_debug_interrupt = polls; }
int bb_last_call_info(int *devices, int *trace_capacity, int *interrupted) {
    if (devices) *devices = g_last_devices;
    if (trace_capacity) *trace_capacity = g_last_capacity;
    if (interrupted) *interrupted = g_last_interrupted;
    return 0;
}

void bridge_reg_stable(double *betap, double *lambdap, double *sig2p, double *taup,
                       double *alphap, const double *yp, const double *Xp,
                       const double *sig2_shape, const double *sig2_scale,
                       const double *nu_shape, const double *nu_rate, const double *alpha_a,
                       const double *alpha_b, const double *true_sig2, const double *true_tau,
                       const double *true_alpha, const int *P, const int *N, const int *M,
                       const int *burn, double *runtime, const int *ortho) {
    const bb_config c = stable_call_config(sig2_shape, sig2_scale, nu_shape, nu_rate, alpha_a,
                                           alpha_b, true_sig2, true_tau, true_alpha, *P, *N, *M,
                                           ortho);
    if (stable_dense(c, yp, Xp, *burn, betap, lambdap, sig2p, taup, alphap, runtime,
                     "Bridge Regression (mix. of normals):") == OUT_INTERRUPTED)
        reraise_interrupt();
}

}  // extern "C"

namespace {

Outcome stable_csc(const bb_config &c, const double *yp, const int *Xcolptr, const int *Xrowidx,
                   const double *Xval, int b, double *betap, double *lambdap, double *sig2p,
                   double *taup, double *alphap, double *runtime) {
    const int p = c.p, n = c.n;
    const char *title = "Bridge Regression (mix. of normals):";
    if (p > n && !c.ortho) {
        return stable_call(
            c,
            [&](const bb_config *cc, int j0, int j1, bb_engine **e) {
                // the shard's columns: colptr rebased to its first entry
                std::vector<int> cp(j1 - j0 + 1);
                for (int j = j0; j <= j1; ++j) cp[j - j0] = Xcolptr[j] - Xcolptr[j0];
                return bb_engine_create_csc(cc, cp.data(), Xrowidx + Xcolptr[j0],
                                            Xval + Xcolptr[j0], yp, e);
            },
            b, betap, lambdap, sig2p, taup, alphap, runtime, title);
    }
    // p <= n or the orthogonal design: the dense paths of bridge_reg_stable (least-squares
    // start, p x p Cholesky or ortho draw) on the densified X, after the same validation as
    // the sparse engine's
    try {
        csc_validate(n, p, Xcolptr, Xrowidx);
    } catch (std::exception &ex) {
        printf("Error: %s\n", ex.what());
        printf("Aborting Gibbs sampler.\n");
        fflush(stdout);
        *runtime = 0.0;
        return OUT_ERROR;
    }
    std::vector<double> Xd((size_t)n * p, 0.0);
    for (int j = 0; j < p; ++j)
        for (int q = Xcolptr[j]; q < Xcolptr[j + 1]; ++q) Xd[(size_t)j * n + Xrowidx[q]] = Xval[q];
    return stable_dense(c, yp, Xd.data(), b, betap, lambdap, sig2p, taup, alphap, runtime, title);
}

Outcome logit_call(bb_config c, const double *yp, const double *Xp, int b, double *betap,
                   double *lambdap, double *taup, double *alphap, double *runtime) {
    c.method = 6;
    for (int i = 0; i < c.n; ++i)
        if (!(yp[i] == 0.0 || yp[i] == 1.0)) {
            printf("Error: logistic bridge needs y in {0, 1} (y[%d] = %g)\n", i, yp[i]);
            printf("Aborting Gibbs sampler.\n");
            fflush(stdout);
            *runtime = 0.0;
            return OUT_ERROR;
        }
    std::vector<double> sig2(c.trace_capacity);
    return stable_dense(c, yp, Xp, b, betap, lambdap, sig2.data(), taup, alphap, runtime,
                        "Bridge Regression (logistic, Polya-Gamma mix. of normals):");
}

// The triangle-mixture driver (BridgeWrapper.cpp:80-204 / :320-432): `burn` sweeps in slot
// 0, MCMC sample i at t = burn + i.
Outcome tri_call(const bb_config &c, const double *yp, const double *Xp, int b, double *betap,
                 double *up, double *omegap, double *shapep, double *sig2p, double *taup,
                 double *alphap, double *runtime) {
    const int m = c.trace_capacity;
    print_banner("Bridge Regression (mix. of triangles):", c, b, m);
    g_last_interrupted = 0;
    Outcome o;
    {
        Chain ch;
        if (chain_build(ch, c, 4, [&](const bb_config *cc, int, int, bb_engine **e) {
                return bb_engine_create(cc, Xp, yp, e);
            }) != 0) {
            printf("Error: %s\n", g_last_error.c_str());
            printf("Aborting Gibbs sampler.\n");
            fflush(stdout);
            *runtime = 0.0;
            return OUT_ERROR;
        }
        g_last_devices = 1;
        g_last_capacity = ch.cap;
        o = drive_chain(ch, b, (uint64_t)b, m, b, betap, omegap, sig2p, taup, alphap, runtime, up,
                        shapep);
        if (o == OUT_ERROR) {
            printf("Error: %s\n", g_last_error.c_str());
            printf("Aborting Gibbs sampler.\n");
            fflush(stdout);
        }
    }
    if (g_verbose && o == OUT_OK) printf("Sampling complete: %g sec. for %i iterations.\n", *runtime, m);
    g_last_interrupted = o == OUT_INTERRUPTED;
    return o;
}

}  // namespace

extern "C" {

void bridge_reg_stable_csc(double *betap, double *lambdap, double *sig2p, double *taup,
                           double *alphap, const double *yp, const int *Xcolptr,
                           const int *Xrowidx, const double *Xval, const double *sig2_shape,
                           const double *sig2_scale, const double *nu_shape,
                           const double *nu_rate, const double *alpha_a, const double *alpha_b,
                           const double *true_sig2, const double *true_tau,
                           const double *true_alpha, const int *P, const int *N, const int *M,
                           const int *burn, double *runtime, const int *ortho) {
    const bb_config c = stable_call_config(sig2_shape, sig2_scale, nu_shape, nu_rate, alpha_a,
                                           alpha_b, true_sig2, true_tau, true_alpha, *P, *N, *M,
                                           ortho);
    if (stable_csc(c, yp, Xcolptr, Xrowidx, Xval, *burn, betap, lambdap, sig2p, taup, alphap,
                   runtime) == OUT_INTERRUPTED)
        reraise_interrupt();
}

void bridge_reg_logit(double *betap, double *lambdap, double *taup, double *alphap,
                      const double *yp, const double *Xp, const double *nu_shape,
                      const double *nu_rate, const double *alpha_a, const double *alpha_b,
                      const double *true_tau, const double *true_alpha, const int *P,
                      const int *N, const int *M, const int *burn, double *runtime) {
    const double zero = 0.0, one = 1.0;
    const int no = 0;
    const bb_config c = stable_call_config(&zero, &zero, nu_shape, nu_rate, alpha_a, alpha_b,
                                           &one, true_tau, true_alpha, *P, *N, *M, &no);
    if (logit_call(c, yp, Xp, *burn, betap, lambdap, taup, alphap, runtime) == OUT_INTERRUPTED)
        reraise_interrupt();
}

void bridge_regression(double *betap, double *up, double *omegap, double *shapep,
                       double *sig2p, double *taup, double *alphap, const double *yp,
                       const double *Xp, const double *sig2_shape, const double *sig2_scale,
                       const double *nu_shape, const double *nu_rate, const double *alpha_a,
                       const double *alpha_b, const double *true_sig2, const double *true_tau,
                       const double *true_alpha, const int *P, const int *N, const int *M,
                       const int *burn, double *runtime, const int *ortho,
                       const int *betaburn, const int *use_hmc) {
    (void)use_hmc;  // BridgeRegression.cpp:418 forces use_hmc = false
    const int no = 0;
    bb_config c = stable_call_config(sig2_shape, sig2_scale, nu_shape, nu_rate, alpha_a, alpha_b,
                                     true_sig2, true_tau, true_alpha, *P, *N, *M, &no);
    c.method = 4;
    c.ortho = *ortho != 0;                       // bridge_regression_ortho, :320-432
    c.betaburn = *betaburn > 0 ? *betaburn : 0;  // BridgeRegression.cpp:407
    if (tri_call(c, yp, Xp, *burn, betap, up, omegap, shapep, sig2p, taup, alphap, runtime) ==
        OUT_INTERRUPTED)
        reraise_interrupt();
}

}  // extern "C"
