"""GPU parity of the sparse-design (CSC) Woodbury path -- BASELINE config C5 -- against the
oracle's scipy restatement (oracle/gibbs.py beta_step_woodbury on a sparse X), through the
C ABI (bb_sparse_gram, bb_engine_create_csc, .C bridge_reg_stable_csc).

There is no reference implementation of a sparse design; the conditional is
the reference's beta | rest (BridgeRegression.cpp:552-575) in Woodbury form, so the bar is
the dense Woodbury path's: per teacher-forced sweep beta to 1e-10 relative L2, lambda /
tau / sig2 to 1e-11 with no rejection-decision flips.
"""
import numpy as np
import pytest
import scipy.sparse as sps

import oracle
from oracle import gibbs
from tests.test_gpu_parity import flips, rel_err

pytestmark = pytest.mark.gpu

SEED = 0xB4E5B41D6E


def rand_csc(n, p, density, seed, dense_cols=(), empty_rows=()):
    rng = np.random.default_rng(seed)
    X = sps.random(n, p, density=density, random_state=seed, format="lil",
                   data_rvs=rng.standard_normal)
    for j in dense_cols:  # a column with far more than 64 non-zeros
        X[:, j] = rng.standard_normal((n, 1))
    for r in empty_rows:
        X[r, :] = 0.0
    X = sps.csc_matrix(X)
    X.eliminate_zeros()
    return X


@pytest.fixture(params=[0, 2, 3], ids=["lanes", "flat8", "flat16"])
def sp_variant(request, gpu_lib):
    """The by-column sparse Gram kernels: lanes per entry (0) and the flat chunked pair
    stream with 8 or 16 pairs per lane (2, 3 = the production default), bb_set_tuning key 3."""
    old = gpu_lib.set_tuning(3, request.param)
    yield request.param
    gpu_lib.set_tuning(3, old)


@pytest.mark.parametrize("n,p,density,extra", [
    (100, 500, 0.05, {}),
    (130, 2000, 0.02, dict(dense_cols=(0, 777), empty_rows=(5, 129))),  # ragged n, edges
    (257, 4000, 0.01, {}),
    (64, 3, 0.5, {}),                                                    # p < 64, tiny
])
def test_sparse_gram_matches_scipy(gpu_lib, sp_variant, n, p, density, extra):
    bb = gpu_lib
    X = rand_csc(n, p, density, n + p, **extra)
    rng = np.random.default_rng(3)
    D = 10.0 ** rng.uniform(-8, 2, p)  # prior variances over 10 decades
    u = rng.standard_normal(p)
    C, xu = bb.sparse_gram(X, D, u)
    Xl = X.toarray().astype(np.longdouble)
    ref = (Xl * D.astype(np.longdouble)) @ Xl.T
    scale = (np.abs(X.toarray()) * D) @ np.abs(X.toarray()).T
    mask = scale > 0
    assert np.all(C[~mask] == 0)
    assert np.max(np.abs(C - ref)[mask] / scale[mask]) < 1e-14
    assert np.allclose(xu, X @ u, rtol=1e-13, atol=1e-13 * np.abs(X) @ np.abs(u))
    assert np.array_equal(C, C.T)


def test_sparse_gram_general_kernel_dense_row(gpu_lib):
    """A row with more than 8192 non-zeros sends the design to the general pair-list kernel
    (32-bit column indices, D gathered from HBM/L2) instead of the by-column one."""
    bb = gpu_lib
    n, p = 90, 9000
    X = rand_csc(n, p, 0.01, 61).tolil()
    rng = np.random.default_rng(62)
    X[7, :] = rng.standard_normal((1, p))
    X = sps.csc_matrix(X)
    D = 10.0 ** rng.uniform(-4, 1, p)
    u = rng.standard_normal(p)
    e = bb.Engine(bb.EngineConfig(n=n, p=p), X, np.zeros(n))
    info = e.sparse_info()
    e.close()
    assert not info["col_mode"] and info["max_row"] == p
    C, xu = bb.sparse_gram(X, D, u)
    ref = (X.toarray() * D) @ X.toarray().T
    scale = (np.abs(X.toarray()) * D) @ np.abs(X.toarray()).T
    m = scale > 0
    assert np.max(np.abs(C - ref)[m] / scale[m]) < 1e-14
    assert np.allclose(xu, X @ u, rtol=1e-12, atol=1e-12)


def test_sparse_gram_exact_on_integers(gpu_lib, sp_variant):
    """Integer X and D: every partial sum is an exact integer, so the pair-list Gram must
    equal the int64 product bit for bit (pins the pair placement and segment starts)."""
    bb = gpu_lib
    rng = np.random.default_rng(8)
    n, p = 300, 3000
    X = rand_csc(n, p, 0.03, 9, dense_cols=(17,))
    X.data = rng.integers(-50, 51, size=X.data.size).astype(np.float64)
    D = rng.integers(0, 7, size=p).astype(np.float64)
    C, _ = bb.sparse_gram(X, D)
    Xi = X.toarray().astype(np.int64)
    ref = (Xi * D.astype(np.int64)) @ Xi.T
    assert np.array_equal(C, ref.astype(np.float64))


def test_sparse_gram_flat_long_entries(gpu_lib, sp_variant):
    """Entries with thousands of pairs (two dense-ish rows over many columns) run across
    several of the flat kernel's 2048-pair chunks, carrying their partial sums; empty
    entries sit between them.  Integer data: bit-exact."""
    bb = gpu_lib
    rng = np.random.default_rng(21)
    n, p = 200, 12000
    X = rand_csc(n, p, 0.002, 22).tolil()
    for r in (3, 150, 151):
        cols = rng.choice(p, 5000, replace=False)
        X[r, cols] = rng.integers(1, 9, size=(1, 5000)).astype(np.float64)
    X = sps.csc_matrix(X)
    X.data = np.round(X.data * 4)
    X.eliminate_zeros()
    D = rng.integers(0, 4, size=p).astype(np.float64)
    C, _ = bb.sparse_gram(X, D)
    Xi = X.toarray().astype(np.int64)
    ref = (Xi * D.astype(np.int64)) @ Xi.T
    assert np.array_equal(C, ref.astype(np.float64))


def test_sparse_gram_rejects_noncanonical_csc(gpu_lib):
    bb = gpu_lib
    L = bb.library()
    import ctypes
    colptr = np.array([0, 2], dtype=np.int32)
    rowidx = np.array([3, 1], dtype=np.int32)  # unsorted rows
    val = np.ones(2)
    D = np.ones(1)
    C = np.zeros((4, 4))
    ip = ctypes.POINTER(ctypes.c_int)
    rc = L.bb_sparse_gram(bb._p(C), None, colptr.ctypes.data_as(ip), rowidx.ctypes.data_as(ip),
                          bb._p(val), bb._p(D), None, 4, 1)
    assert rc != 0 and b"strictly increasing" in L.bb_last_error()


def _teacher_forced(bb, X, y, sweeps, seed, stream, true_sig2=0.0, alpha=0.5):
    n, p = X.shape
    o = gibbs.bridge_regression_stable(y, X, sweeps, burn=0, alpha=alpha, seed=seed,
                                       stream=stream, method="woodbury", record_state=True,
                                       true_sig2=true_sig2)
    cfg = bb.EngineConfig(n=n, p=p, seed=seed, stream=stream, trace_capacity=1,
                          true_sig2=true_sig2, true_alpha=alpha)
    e = bb.Engine(cfg, X, y)
    assert e.method() == 5 and e.sparse_pairs() >= 0
    e.init_state()
    st = o["states"]
    for k in range(1, len(st)):
        t, tau, sig2, lam, beta, _ = st[k]
        _, tau0, sig20, _, beta0, alpha0 = st[k - 1]
        e.set_state(beta0, tau0, sig20, alpha0)
        e.run(t, 1, first_slot=-1)
        s = e.state()
        assert abs(s["tau"] - tau) <= 1e-12 * tau, (t, s["tau"], tau)
        assert abs(s["sig2"] - sig2) <= 1e-12 * sig2, (t, s["sig2"], sig2)
        assert flips(s["lambda"], lam) == 0, t
        assert np.max(np.abs(s["lambda"] - lam) / lam) < 1e-11, t
        D = tau * tau / lam
        assert rel_err(s["beta"], beta) < 1e-10, (t, rel_err(s["beta"], beta))
        assert np.max(np.abs(s["beta"] - beta) / (np.abs(beta) + np.sqrt(D))) < 1e-10, t
    assert e.error_flags() == 0
    e.close()


@pytest.mark.parametrize("n,p,density,kw", [
    (60, 800, 0.05, {}),
    (150, 3000, 0.03, dict(true_sig2=1.0)),
    (200, 5000, 0.01, dict(alpha=0.3)),
])
def test_sparse_chain_teacher_forced(gpu_lib, n, p, density, kw):
    bb = gpu_lib
    X = rand_csc(n, p, density, 11 + n)
    rng = np.random.default_rng(12)
    b = np.zeros(p)
    b[:5] = [2.0, -1.5, 1.0, 2.5, -2.0]
    y = X @ b + rng.standard_normal(n)
    _teacher_forced(bb, X, y, 25, SEED + 21, 0, **kw)


@pytest.mark.parametrize("world", [2, 3])
def test_sparse_shard_group_matches_single_engine(gpu_lib, world):
    """Column shards of a CSC design (each builds its own pair list) exchanging the partial
    Gram through the group's sums, against the unsharded sparse engine."""
    bb = gpu_lib
    n, p = 180, 2600
    X = rand_csc(n, p, 0.03, 23)
    rng = np.random.default_rng(24)
    b = np.zeros(p)
    b[:4] = [1.5, -2.0, 2.0, 1.0]
    y = X @ b + rng.standard_normal(n)
    seed = SEED + 25
    single = bb.Engine(bb.EngineConfig(n=n, p=p, seed=seed), X, y)
    single.init_state()
    per = (p + world - 1) // world
    shards = []
    for r in range(world):
        j0, j1 = r * per, min(p, (r + 1) * per)
        cfg = bb.EngineConfig(n=n, p=p, p_local=j1 - j0, j0=j0, rank=r, world=world, seed=seed)
        shards.append(bb.Engine(cfg, X[:, j0:j1], y))
    grp = bb.ShardGroup(shards)
    grp.init_state()
    beta = b + 0.05 * rng.standard_normal(p)
    tau, sig2 = 0.9, 1.1
    for t in range(1, 6):
        single.set_state(beta, tau, sig2, 0.5)
        for r, e in enumerate(shards):
            e.set_state(beta[r * per:min(p, (r + 1) * per)], tau, sig2, 0.5)
        single.run(t, 1)
        grp.run(t, 1)
        grp.sync()
        s1 = single.state()
        parts = [e.state() for e in shards]
        bg = np.concatenate([q["beta"] for q in parts])
        lg = np.concatenate([q["lambda"] for q in parts])
        assert flips(lg, s1["lambda"]) == 0
        assert rel_err(bg, s1["beta"]) < 1e-10, (t, rel_err(bg, s1["beta"]))
        beta, tau, sig2 = s1["beta"], s1["tau"], s1["sig2"]
    grp.close()
    single.close()


def test_sparse_engine_matches_dense_engine(gpu_lib):
    """Same design, CSC vs dense (fp64 Gram) Woodbury engines: one sweep from one state."""
    bb = gpu_lib
    n, p = 250, 4000
    X = rand_csc(n, p, 0.02, 31)
    rng = np.random.default_rng(32)
    y = X[:, :6] @ rng.standard_normal(6) + rng.standard_normal(n)
    beta0 = 0.1 * rng.standard_normal(p)
    out = []
    for Xin, gm in ((X, None), (X.toarray(), bb.GRAM_FP64)):
        e = bb.Engine(bb.EngineConfig(n=n, p=p, seed=SEED, stream=4, gram_mode=gm), Xin, y)
        e.init_state()
        e.set_state(beta0, 0.8, 1.2, 0.5)
        e.run(7, 1)
        out.append(e.state())
        e.close()
    assert flips(out[0]["lambda"], out[1]["lambda"]) == 0
    assert rel_err(out[0]["beta"], out[1]["beta"]) < 1e-10


def test_csc_entry_point_chain(gpu_lib):
    """.C("bridge_reg_stable_csc") free-running: the first sweeps agree with the oracle's
    sparse chain before roundoff compounds (p > n chains are chaotic)."""
    bb = gpu_lib
    n, p = 70, 900
    X = rand_csc(n, p, 0.05, 41)
    rng = np.random.default_rng(42)
    y = X[:, :5] @ np.array([2.0, -1.0, 1.5, 2.5, -2.0]) + rng.standard_normal(n)
    bb.set_seed(SEED + 5)
    g = bb.bridge_reg_stb(y, X, nsamp=8, burn=3)
    o = gibbs.bridge_regression_stable(y, X, 8, burn=3, seed=SEED + 5, stream=0,
                                       method="woodbury")
    for k in ("sig2", "tau"):
        assert np.max(np.abs(g[k] - o[k]) / o[k]) < 1e-8, k
    assert np.max(np.abs(g["beta"].T - o["beta"]) / np.maximum(np.abs(o["beta"]), 1e-8)) < 1e-6


def test_csc_entry_point_small_p_is_dense_path(gpu_lib):
    """p <= n through the CSC entry densifies and runs bridge_reg_stable's Cholesky path:
    bit-identical to the dense entry under the same key."""
    bb = gpu_lib
    X = rand_csc(120, 15, 0.4, 51)
    y = X @ np.linspace(-1, 1, 15) + np.random.default_rng(52).standard_normal(120)
    bb.set_seed(SEED + 6)
    a = bb.bridge_reg_stb(y, X, nsamp=50, burn=10)
    bb.set_seed(SEED + 6)
    b = bb.bridge_reg_stb(y, X.toarray(), nsamp=50, burn=10)
    for k in ("beta", "lambda", "sig2", "tau"):
        assert np.array_equal(a[k], b[k]), k


def test_teacher_forced_c5_workload(gpu_lib):
    """The C5 bench workload itself (n = 5000, p = 200000, 1 % density, alpha = 0.3; bench.py's
    X, y and key), two sweeps teacher-forced from the oracle's state (~6 s of scipy each)."""
    import bench
    bb = gpu_lib
    n, p, alpha = 5000, 200000, 0.3
    X = bench.make_sparse_columns(n, 0, p)
    y, btrue = bench.make_sparse_problem_y(n, p)
    e = bb.Engine(bb.EngineConfig(n=n, p=p, seed=SEED, stream=0, trace_capacity=2,
                                  true_alpha=alpha), X, y)
    assert e.method() == 5
    e.init_state()
    rng = np.random.default_rng(2)
    beta, tau, sig2 = btrue + 0.01 * rng.standard_normal(p), 1.0, 1.0
    for t in (101, 102):
        e.set_state(beta, tau, sig2, alpha)
        e.run(t, 1, first_slot=0, slot_step=0)
        s = e.state()
        tau = oracle.tau_from_sum(oracle.sum_abs_pow(beta, alpha), p, alpha, 2.0, 2.0, SEED, 0, t)
        r = y - X @ beta
        sig2 = oracle.sig2_from_rss(float(r @ r), n, 0.0, 0.0, SEED, 0, t)
        lam = oracle.sample_lambda(beta, alpha, tau, SEED, 0, t)
        z = oracle.normals(p, SEED, 0, t, oracle.KIND_BETA_Z)
        d = oracle.normals(n, SEED, 0, t, oracle.KIND_DELTA)
        b = gibbs.beta_step_woodbury(X, y, lam, sig2, tau, z, d)
        assert abs(s["tau"] - tau) / tau < 1e-12, t
        assert abs(s["sig2"] - sig2) / sig2 < 1e-12, t
        assert flips(s["lambda"], lam) == 0, t
        assert np.max(np.abs(s["lambda"] - lam) / lam) < 1e-11, t
        assert rel_err(s["beta"], b) < 1e-9, (t, rel_err(s["beta"], b))
        beta = b
    assert e.error_flags() == 0
    e.close()


@pytest.mark.parametrize("n,p", [(40, 12), (12, 40)])
@pytest.mark.parametrize("defect", ["unsorted", "duplicate", "out_of_range"])
def test_csc_entry_rejects_malformed_on_both_paths(gpu_lib, capfd, n, p, defect):
    """.C("bridge_reg_stable_csc") refuses a non-canonical dgCMatrix the same way whether the
    shape selects the densified dense path (p <= n) or the sparse engine (p > n): the usual
    'Error: ... Aborting Gibbs sampler.' and no samples."""
    import ctypes
    bb = gpu_lib
    L = bb.library()
    rng = np.random.default_rng(4)
    colptr = np.arange(0, 2 * p + 1, 2, dtype=np.int32)
    rowidx = np.concatenate([[0, 1 + (j % (n - 1))] for j in range(p)]).astype(np.int32)
    if defect == "unsorted":
        rowidx[2], rowidx[3] = rowidx[3], 0
    elif defect == "duplicate":
        rowidx[3] = rowidx[2]
    else:
        rowidx[5] = n
    val = rng.standard_normal(2 * p)
    y = rng.standard_normal(n)
    M = 4
    beta, lam = np.zeros((p, M), order="F"), np.zeros((p, M), order="F")
    sig2, tau, alph = np.zeros(M), np.zeros(M), np.zeros(M)
    d = lambda v: ctypes.byref(ctypes.c_double(float(v)))  # noqa: E731
    i = lambda v: ctypes.byref(ctypes.c_int(int(v)))  # noqa: E731
    rt = ctypes.c_double(0.0)
    ip = ctypes.POINTER(ctypes.c_int)
    capfd.readouterr()
    L.bridge_reg_stable_csc(bb._p(beta), bb._p(lam), bb._p(sig2), bb._p(tau), bb._p(alph),
                            bb._p(y), colptr.ctypes.data_as(ip), rowidx.ctypes.data_as(ip),
                            bb._p(val), d(0), d(0), d(2), d(2), d(1), d(1), d(0), d(0), d(0.5),
                            i(p), i(n), i(M), i(2), ctypes.byref(rt), i(0))
    out = capfd.readouterr().out
    assert "CSC:" in out and "Aborting Gibbs sampler." in out, out
    assert not beta.any() and not sig2.any()
