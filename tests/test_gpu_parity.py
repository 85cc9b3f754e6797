"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle on the
same Philox counters.

Tolerances (north star: posterior-mean beta within 1e-8 relative L2 of the CPU path):
  * per-draw tilted-stable / lambda values: relative 1e-11 (libm vs ocml last-ulp
    differences in pow/exp/log/sin), with accept/reject decision flips counted;
  * Gram / Cholesky kernels: relative 1e-11 of the problem scale;
  * whole chains: posterior mean relative L2 <= 1e-8, every trace <= 1e-6 elementwise.
"""
import math

import numpy as np
import pytest

import oracle
from oracle import gibbs
from tests.conftest import synthetic_problem

pytestmark = pytest.mark.gpu

SEED = 0xB4E5B41D6E


def rel_err(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def flips(a, b, tol=1e-6):
    a, b = np.asarray(a), np.asarray(b)
    return int(np.sum(np.abs(a - b) > tol * np.maximum(np.abs(b), 1e-300)))


GRID_A = [0.05, 0.15, 0.25, 0.45, 0.75, 1.0]
GRID_H = [0.0, 1e-4, 1e-2, 1.0, 1e2, 1e4, 1e6]


def grid_inputs(reps=120):
    a, h, v = [], [], []
    for aa in GRID_A:
        for hh in GRID_H:
            for V0 in (1.0, 2.5):
                a += [aa] * reps
                h += [hh] * reps
                v += [V0] * reps
    return np.array(a), np.array(v), np.array(h)


def test_retstable_batch_matches_oracle(gpu_lib):
    bb = gpu_lib
    a, v, h = grid_inputs()
    g = bb.retstable_batch(a, v, h, seed=SEED, stream=3, t=17)
    o = oracle.retstable_batch(a, v, h, seed=SEED, stream=3, t=17)
    assert np.all(np.isfinite(g)) and np.all(g > 0)
    nf = flips(g, o)
    assert nf == 0, f"{nf} decision flips out of {len(g)}"
    assert np.max(np.abs(g - o) / np.abs(o)) < 1e-11


@pytest.mark.parametrize("group", [1, 2, 8, 64])
def test_retstable_group_invariance(gpu_lib, group):
    """G lanes per coefficient evaluate attempts speculatively; the first accepted attempt
    in counter order wins, so every G gives the sequential result bit for bit."""
    bb = gpu_lib
    a, v, h = grid_inputs(reps=20)
    ref = bb.retstable_batch(a, v, h, seed=SEED, stream=4, t=0, group=1)
    got = bb.retstable_batch(a, v, h, seed=SEED, stream=4, t=0, group=group)
    assert np.array_equal(ref, got)


def test_retstable_c_entry_point(gpu_lib):
    bb = gpu_lib
    bb.set_seed(77)
    x = bb.retstable_ld(5000, alpha=0.25, V0=1.0, h=1.0)
    o = oracle.retstable_batch(np.full(5000, 0.25), np.ones(5000), np.ones(5000), seed=77,
                               stream=0, t=0)
    assert rel_err(x, o) < 1e-12
    assert bb.get_rng_state() == (77, 1)
    assert np.isnan(bb.retstable_ld(3, alpha=1.5))
    assert np.isnan(bb.retstable_ld(3, h=-1.0))


def test_sample_lambda_matches_oracle(gpu_lib):
    bb = gpu_lib
    rng = np.random.default_rng(0)
    beta = rng.standard_normal(3000) * rng.choice([1e-4, 1e-1, 1, 10], size=3000)
    for alpha, tau, j0 in ((0.5, 0.7, 0), (0.3, 2.0, 12345)):
        g = bb.sample_lambda(beta, alpha, tau, SEED, 1, 9, j0=j0)
        o = oracle.sample_lambda(beta, alpha, tau, SEED, 1, 9, j0=j0)
        assert flips(g, o) == 0
        assert np.max(np.abs(g - o) / o) < 1e-11


@pytest.mark.parametrize("n,k", [(100, 50), (128, 1000), (300, 5000), (1000, 257)])
def test_gram_matches_numpy(gpu_lib, n, k):
    bb = gpu_lib
    rng = np.random.default_rng(n + k)
    Y = rng.standard_normal((n, k))
    w = rng.uniform(0.0, 3.0, k)
    C = bb.gram(Y, w)
    ref = (Y * w) @ Y.T
    scale = np.abs(Y) ** 2 @ w
    assert np.max(np.abs(C - ref) / np.sqrt(np.outer(scale, scale))) < 1e-13 * max(k, 64)


def test_gram_mfma_layout_asymmetric(gpu_lib):
    """Exact integer data, asymmetric Y: catches a transposed or mis-rowed MFMA C/D map."""
    bb = gpu_lib
    rng = np.random.default_rng(5)
    Y = rng.integers(-3, 4, size=(256, 64)).astype(np.float64)
    w = rng.integers(0, 3, size=64).astype(np.float64)
    assert np.array_equal(bb.gram(Y, w), (Y * w) @ Y.T)


def test_gram_ozaki_exact_on_integers(gpu_lib):
    """Integer Y, square-integer w: the Ozaki-II Gram is exact (every scaled input
    sqrt(w_j) Y_ij is an integer times a power of two, the CRT recovers the exact integer product), so it must equal the int64
    product bit for bit -- this also pins the int8 MFMA operand and C/D lane maps, the tile
    decode and the split-K / XCD grouping (n not a multiple of the 256 tile, ragged k).
    (1500, 700) and (1100, 2500) have more virtual blocks than the persistent GEMM's grid
    with a unit's tiles straddling its rounds (18 and 13 workgroups per unit, 32 per XCD)."""
    bb = gpu_lib
    rng = np.random.default_rng(17)
    for n, k in [(300, 1000), (77, 5000), (600, 333), (1500, 700), (1100, 2500)]:
        Yi = rng.integers(-60, 61, size=(n, k))
        wi = rng.choice([0, 1, 4, 9], size=k)  # perfect squares: sqrt(w) Y stays integral
        # every partial sum is an integer below 2^53, so the fp64 BLAS product is exact
        ref = (Yi * wi).astype(np.float64) @ Yi.T.astype(np.float64)
        C = bb.gram(Yi.astype(np.float64), wi.astype(np.float64), mode=bb.GRAM_OZAKI)
        assert np.array_equal(C, ref.astype(np.float64)), (n, k)


@pytest.mark.parametrize("n,k", [(200, 3000), (450, 700)])
def test_gram_ozaki_fp64_accuracy(gpu_lib, n, k):
    """Random Y and weights over 10 decades (like D = tau^2/lambda): the Ozaki Gram's error
    against an 80-bit long-double reference, relative to (|Y| w |Y|')_ik, is at fp64 level and
    no worse than 4x the fp64 MFMA Gram's."""
    bb = gpu_lib
    rng = np.random.default_rng(n * 7 + k)
    Y = rng.standard_normal((n, k))
    w = 10.0 ** rng.uniform(-8, 2, k)
    Yl = Y.astype(np.longdouble)
    ref = (Yl * w.astype(np.longdouble)) @ Yl.T
    scale = (np.abs(Y) * w) @ np.abs(Y).T
    e_oz = np.max(np.abs(bb.gram(Y, w, mode=bb.GRAM_OZAKI) - ref) / scale)
    e_64 = np.max(np.abs(bb.gram(Y, w) - ref) / scale)
    assert e_oz < 2e-15, (e_oz, e_64)
    assert e_oz < 4 * max(e_64, 1e-16), (e_oz, e_64)


@pytest.mark.parametrize("m,nrhs", [(20, 1), (64, 2), (130, 1), (700, 2), (3500, 2)])
def test_chol_solve_matches_numpy(gpu_lib, m, nrhs):
    bb = gpu_lib
    rng = np.random.default_rng(m)
    B = rng.standard_normal((m, m + 5))
    A = B @ B.T + 0.1 * np.eye(m)
    b = rng.standard_normal((m, nrhs))
    x = bb.chol_solve(A, b)
    ref = np.linalg.solve(A, b)
    assert rel_err(x, ref) < 1e-10 * np.linalg.cond(A) ** 0.5


@pytest.mark.parametrize("version", [1, 2, 3, 4])
@pytest.mark.parametrize("m", [40, 64, 128, 200, 1000, 2048, 5000])
def test_chol_chain_versions_match_numpy(gpu_lib, m, version):
    """Every chain variant of k_chol_persistent (1: the round-2 chain; 2, 3: pipelined; 4: the
    16-column leaf pipeline), from one block (m <= 64) to 79 block steps, on an
    ill-conditioned SPD system.  The variant in use before the test is restored afterwards."""
    bb = gpu_lib
    rng = np.random.default_rng(m + 7)
    B = rng.standard_normal((m, m)) * np.exp(rng.uniform(-6, 6, m))
    A = B @ B.T + 1e-3 * np.eye(m)
    b = rng.standard_normal((m, 1))
    default = bb.chol_version()
    bb.set_chol_version(version)
    try:
        x = bb.chol_solve(A, b)
    finally:
        bb.set_chol_version(default)
    ref = np.linalg.solve(A, b)
    cond = np.linalg.cond(A)
    # backward error of the solve against A (normwise), and the forward error
    res = np.linalg.norm(A @ x - b) / (np.linalg.norm(A, 2) * np.linalg.norm(x))
    assert res < 1e-13, res
    assert rel_err(x, ref) < 1e-12 * cond, (rel_err(x, ref), cond)


def test_chol_solve_detects_non_spd(gpu_lib):
    bb = gpu_lib
    A = np.array([[1.0, 2.0], [2.0, 1.0]])
    with pytest.raises(RuntimeError):
        bb.chol_solve(A, np.ones(2))


def compare_chain(g, o, tol_mean=1e-8, tol_elem=1e-6):
    for key in ("beta", "lambda", "sig2", "tau", "alpha"):
        gv = np.asarray(g[key])
        ov = np.asarray(o[key])
        if key in ("beta", "lambda"):
            gv = gv.T  # R-style M x P  ->  P x M
        assert gv.shape == ov.shape, (key, gv.shape, ov.shape)
        assert np.all(np.isfinite(gv)), key
        e = np.max(np.abs(gv - ov) / np.maximum(np.abs(ov), 1e-8))
        assert e < tol_elem, (key, e)
    pm_g = np.asarray(g["beta"]).mean(axis=0)
    pm_o = np.asarray(o["beta"]).mean(axis=1)
    assert rel_err(pm_g, pm_o) < tol_mean


@pytest.mark.parametrize("kw", [
    dict(),                                   # C1 defaults: sig2, tau unknown, alpha = 0.5
    dict(sig2_true=1.5),
    dict(tau_true=0.8),
    dict(alpha=0.3, nu_shape=0.5, nu_rate=0.5),
])
@pytest.mark.parametrize("n,p", [(100, 20), (120, 40), (50, 6), (200, 16), (100, 13),
                                 (3000, 8), (150, 32), (90, 17)])
def test_chain_small_p_matches_oracle(gpu_lib, kw, n, p):
    """C1 (n=100, p=20): reference-literal p x p Cholesky draw, full chain -- through the
    fused single-launch kernel (p <= 32, bb_small.hip: 64 lanes per lambda draw at p = 6, 8;
    32 at p = 13, 16; 16 at p = 17, 20, 32, where 16 threads own two Cholesky entries; X from
    HBM instead of LDS at n = 3000) and the general path (p = 40)."""
    bb = gpu_lib
    X, y, _ = synthetic_problem(n, p)
    bb.set_seed(SEED)
    g = bb.bridge_reg_stb(y, X, nsamp=300, burn=100, **kw)
    o = gibbs.bridge_regression_stable(
        y, X, 300, burn=100, alpha=kw.get("alpha", 0.5), nu_shape=kw.get("nu_shape", 2.0),
        nu_rate=kw.get("nu_rate", 2.0), true_sig2=kw.get("sig2_true", 0.0),
        true_tau=kw.get("tau_true", 0.0), seed=SEED, stream=0, method="chol")
    compare_chain(g, o)


def test_chain_unknown_alpha_matches_oracle(gpu_lib):
    bb = gpu_lib
    X, y, _ = synthetic_problem(80, 12, seed=3)
    bb.set_seed(SEED + 1)
    g = bb.bridge_reg_stb(y, X, nsamp=200, burn=50, alpha=0.0)
    o = gibbs.bridge_regression_stable(y, X, 200, burn=50, alpha=0.0, seed=SEED + 1, stream=0,
                                       method="chol")
    compare_chain(g, o)


def test_chain_ortho_matches_oracle(gpu_lib):
    bb = gpu_lib
    rng = np.random.default_rng(9)
    Q, _ = np.linalg.qr(rng.standard_normal((120, 15)))
    X = Q * 4.0
    y = X @ np.r_[np.ones(3), np.zeros(12)] + rng.standard_normal(120)
    bb.set_seed(SEED + 2)
    g = bb.bridge_reg_stb(y, X, nsamp=200, burn=50, ortho=True)
    o = gibbs.bridge_regression_stable(y, X, 200, burn=50, ortho=True, seed=SEED + 2, stream=0)
    compare_chain(g, o)


@pytest.mark.parametrize("gram_mode", [0, 1], ids=["fp64", "ozaki"])
@pytest.mark.parametrize("n,p,kw", [(60, 250, {}), (100, 160, dict(true_sig2=1.0)),
                                     (200, 1000, {})])
def test_chain_wide_p_woodbury_teacher_forced(gpu_lib, n, p, kw, gram_mode):
    """p > n: every GPU sweep starts from the oracle's previous state (teacher forcing).

    Free-running p > n chains are chaotic under fp64 roundoff -- the CPU oracle decouples
    from ITSELF within ~100 sweeps when only the Gram summation order changes (coefficients
    with tiny lambda_j get prior variance D_j = tau^2/lambda_j and the Woodbury update
    cancels two O(sqrt(D_j)) terms) -- so the parity bar for p > n is per sweep.
    """
    bb = gpu_lib
    X, y, _ = synthetic_problem(n, p, seed=11)
    seed, stream = SEED + 3, 0
    o = gibbs.bridge_regression_stable(y, X, 40, burn=0, seed=seed, stream=stream,
                                       method="woodbury", record_state=True, **kw)
    cfg = bb.EngineConfig(n=n, p=p, seed=seed, stream=stream, method=2, trace_capacity=1,
                          true_sig2=kw.get("true_sig2", 0.0), gram_mode=gram_mode)
    e = bb.Engine(cfg, X, y)
    e.init_state()
    st = o["states"]
    for k in range(1, len(st)):
        t, tau, sig2, lam, beta, alpha = st[k]
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


def test_chain_wide_p_free_running_short(gpu_lib):
    """The first sweeps of a free-running wide-p chain agree before roundoff compounds."""
    bb = gpu_lib
    X, y, _ = synthetic_problem(60, 250, seed=11)
    bb.set_seed(SEED + 3)
    g = bb.bridge_reg_stb(y, X, nsamp=10, burn=5)
    o = gibbs.bridge_regression_stable(y, X, 10, burn=5, seed=SEED + 3, stream=0,
                                       method="woodbury")
    compare_chain(g, o, tol_mean=1e-8, tol_elem=1e-6)


def test_diabetes_end_to_end(gpu_lib):
    """442 x 10 diabetes design (Efron et al.; the reference's man/diabetes.Rd data)."""
    sk = pytest.importorskip("sklearn.datasets")
    d = sk.load_diabetes(scaled=False)
    X = d.data - d.data.mean(axis=0)
    y = d.target - d.target.mean()
    bb = gpu_lib
    bb.set_seed(SEED + 4)
    g = bb.bridge_reg_stb(y, X, nsamp=500, burn=100)
    o = gibbs.bridge_regression_stable(y, X, 500, burn=100, seed=SEED + 4, stream=0,
                                       method="chol")
    compare_chain(g, o)
    # posterior means close to least squares for this well-determined design
    ls = np.linalg.lstsq(X, y, rcond=None)[0]
    pm = g["beta"].mean(axis=0)
    assert np.corrcoef(pm, ls)[0, 1] > 0.9


def teacher_forced_sweep(X, y, beta, tau, sig2, alpha, t, seed, stream, hyper):
    """One oracle sweep (tau, sig2, lambda, beta) from a given state, Woodbury form."""
    n, p = X.shape
    tau = oracle.tau_from_sum(oracle.sum_abs_pow(beta, alpha), p, alpha, hyper["nu_shape"],
                              hyper["nu_rate"], seed, stream, t)
    r = y - X @ beta
    sig2 = oracle.sig2_from_rss(float(r @ r), n, hyper["sig2_shape"], hyper["sig2_scale"], seed,
                                stream, t)
    lam = oracle.sample_lambda(beta, alpha, tau, seed, stream, t)
    z = oracle.normals(p, seed, stream, t, oracle.KIND_BETA_Z)
    d = oracle.normals(n, seed, stream, t, oracle.KIND_DELTA)
    b = gibbs.beta_step_woodbury(X, y, lam, sig2, tau, z, d)
    return b, lam, tau, sig2


@pytest.mark.parametrize("gram_mode", [0, 1], ids=["fp64", "ozaki"])
@pytest.mark.parametrize("n,p", [(1000, 5000), (2000, 6000)])
def test_teacher_forced_sweep_large(gpu_lib, n, p, gram_mode):
    """C2-scale and C3-height sweeps from an identical state (one sweep each)."""
    bb = gpu_lib
    X, y, btrue = synthetic_problem(n, p, seed=n + p)
    cfg = bb.EngineConfig(n=n, p=p, seed=SEED, stream=7, trace_capacity=2, gram_mode=gram_mode)
    e = bb.Engine(cfg, X, y)
    assert e.method() == 2
    e.init_state()
    rng = np.random.default_rng(1)
    beta0 = btrue + 0.05 * rng.standard_normal(p)
    e.set_state(beta0, 1.0, 1.0, 0.5)
    t = 5
    e.run(t, 1, first_slot=0, slot_step=0)
    s = e.state()
    hyper = dict(nu_shape=2.0, nu_rate=2.0, sig2_shape=0.0, sig2_scale=0.0)
    b, lam, tau, sig2 = teacher_forced_sweep(X, y, beta0, 1.0, 1.0, 0.5, t, SEED, 7, hyper)
    assert abs(s["tau"] - tau) / tau < 1e-12
    assert abs(s["sig2"] - sig2) / sig2 < 1e-12
    assert flips(s["lambda"], lam) == 0
    assert np.max(np.abs(s["lambda"] - lam) / lam) < 1e-11
    assert rel_err(s["beta"], b) < 1e-9
    assert e.error_flags() == 0
    e.close()


def test_teacher_forced_bench_workload(gpu_lib):
    """The benchmarked workload itself -- C3 (n = 2000, p = 50000) with bench.py's synthetic
    X, y and sampler key, Ozaki-II Gram -- three sweeps, each teacher-forced from the oracle
    state of the previous one (SURVEY 8(d) inputs; one oracle sweep is ~1 s of numpy)."""
    import bench
    bb = gpu_lib
    n, p = 2000, 50000
    X = bench.make_columns(n, 0, p)
    y, btrue = bench.make_problem_y(n, p)
    cfg = bb.EngineConfig(n=n, p=p, seed=SEED, stream=0, trace_capacity=2,
                          gram_mode=bb.GRAM_OZAKI)
    e = bb.Engine(cfg, X, y)
    assert e.method() == 2
    e.init_state()
    rng = np.random.default_rng(2)
    beta, tau, sig2 = btrue + 0.01 * rng.standard_normal(p), 1.0, 1.0
    hyper = dict(nu_shape=2.0, nu_rate=2.0, sig2_shape=0.0, sig2_scale=0.0)
    for t in (101, 102, 103):
        e.set_state(beta, tau, sig2, 0.5)
        e.run(t, 1, first_slot=0, slot_step=0)
        s = e.state()
        b, lam, tau, sig2 = teacher_forced_sweep(X, y, beta, tau, sig2, 0.5, t, SEED, 0, hyper)
        assert abs(s["tau"] - tau) / tau < 1e-12, t
        assert abs(s["sig2"] - sig2) / sig2 < 1e-12, t
        assert flips(s["lambda"], lam) == 0, t
        assert np.max(np.abs(s["lambda"] - lam) / lam) < 1e-11, t
        assert rel_err(s["beta"], b) < 1e-9, t
        beta = b
    assert e.error_flags() == 0
    e.close()


@pytest.mark.parametrize("world,kind", [(2, "known"), (3, "known"), (2, "alpha"), (3, "alpha"),
                                        (2, "alpha_accept"), (2, "ortho")])
def test_shard_group_matches_single_engine(gpu_lib, world, kind):
    """The column-sharded sweep (two exchanges per sweep; a third, of the two alpha MH sums,
    when alpha is unknown) on one GPU vs the unsharded engine, teacher-forced from identical
    states for several sweeps.  "ortho": the orthogonal-design draw for p > n, sharded.
    "alpha_accept" starts alpha at 0.9, from where the MH step accepts (the oracle chain of
    this state accepts at sweeps 5 and 8), so the split step's decide kernel is compared on
    its accepting branch too; the test requires at least one acceptance."""
    bb = gpu_lib
    n, p = 200, 1100
    X, y, btrue = synthetic_problem(n, p, seed=21)
    seed, stream = SEED + 9, 0
    ta = 0.0 if kind.startswith("alpha") else 0.5
    ortho = kind == "ortho"
    single = bb.Engine(bb.EngineConfig(n=n, p=p, seed=seed, stream=stream, true_alpha=ta,
                                       ortho=ortho), X, y)
    single.init_state()
    assert single.method() == (3 if ortho else 2)
    per = (p + world - 1) // world
    shards = []
    for r in range(world):
        j0, j1 = r * per, min(p, (r + 1) * per)
        cfg = bb.EngineConfig(n=n, p=p, p_local=j1 - j0, j0=j0, rank=r, world=world, seed=seed,
                              stream=stream, true_alpha=ta, ortho=ortho)
        shards.append(bb.Engine(cfg, np.asfortranarray(X[:, j0:j1]), y))
    grp = bb.ShardGroup(shards)
    grp.init_state()
    rng = np.random.default_rng(3)
    beta = btrue + 0.05 * rng.standard_normal(p)
    tau, sig2, alpha = 0.9, 1.1, (0.9 if kind == "alpha_accept" else 0.5)
    accepts = 0
    for t in range(1, 9):
        single.set_state(beta, tau, sig2, alpha)
        for r, e in enumerate(shards):
            e.set_state(beta[r * per:min(p, (r + 1) * per)], tau, sig2, alpha)
        single.run(t, 1)
        grp.run(t, 1)
        grp.sync()
        s1 = single.state()
        parts = [e.state() for e in shards]
        bg = np.concatenate([q["beta"] for q in parts])
        lg = np.concatenate([q["lambda"] for q in parts])
        for q in parts:
            assert abs(q["tau"] - s1["tau"]) <= 1e-13 * s1["tau"]
            assert abs(q["sig2"] - s1["sig2"]) <= 1e-12 * s1["sig2"]
            assert abs(q["alpha"] - s1["alpha"]) <= 1e-14, (t, q["alpha"], s1["alpha"])
        # same counters; tau differs only by the summation order of S_alpha
        assert flips(lg, s1["lambda"]) == 0
        assert np.max(np.abs(lg - s1["lambda"]) / s1["lambda"]) < 1e-11
        assert rel_err(bg, s1["beta"]) < 1e-10, (t, rel_err(bg, s1["beta"]))
        accepts += int(s1["alpha"] != alpha)
        beta, tau, sig2, alpha = s1["beta"], s1["tau"], s1["sig2"], s1["alpha"]
    # (from alpha = 0.5 the MH step mostly rejects; "alpha_accept" must see the accepting
    # branch -- also covered on the CPU by tests/test_sharded_cpu.py)
    if kind == "alpha_accept":
        assert accepts >= 1, "the MH step never accepted: the accepting branch is untested"
    grp.close()
    single.close()


def test_shard_group_cu_filling_system(gpu_lib):
    """An on-device shard group whose n x n system fills every CU with its persistent
    Cholesky (n = 1600: 25 block rows, 350 tiles > CUs): the members' factorisations must
    run one after another (bb_group_run chains their phase c; overlapped, each held part of
    the CUs while waiting on tiles owned by workgroups that could not start).  Two
    teacher-forced sweeps against the unsharded engine, no error flags."""
    bb = gpu_lib
    n, p, world = 1600, 4000, 2
    X, y, btrue = synthetic_problem(n, p, seed=23)
    seed, stream = SEED + 11, 0
    single = bb.Engine(bb.EngineConfig(n=n, p=p, seed=seed, stream=stream, true_alpha=0.5), X, y)
    single.init_state()
    per = p // world
    shards = [bb.Engine(bb.EngineConfig(n=n, p=p, p_local=per, j0=r * per, rank=r, world=world,
                                        seed=seed, stream=stream, true_alpha=0.5),
                        np.asfortranarray(X[:, r * per:(r + 1) * per]), y) for r in range(world)]
    grp = bb.ShardGroup(shards)
    grp.init_state()
    beta = btrue + 0.05 * np.random.default_rng(5).standard_normal(p)
    tau, sig2 = 0.9, 1.1
    for t in (1, 2):
        single.set_state(beta, tau, sig2, 0.5)
        for r, e in enumerate(shards):
            e.set_state(beta[r * per:(r + 1) * per], tau, sig2, 0.5)
        single.run(t, 1)
        grp.run(t, 1)
        grp.sync()
        s1 = single.state()
        bg = np.concatenate([e.state()["beta"] for e in shards])
        assert rel_err(bg, s1["beta"]) < 1e-9, (t, rel_err(bg, s1["beta"]))
        beta, tau, sig2 = s1["beta"], s1["tau"], s1["sig2"]
    assert single.error_flags() == 0
    assert all(e.error_flags() == 0 for e in shards)
    grp.close()
    single.close()
    for e in shards:
        e.close()


def test_shard_group_c3_full_size(gpu_lib):
    """The sharded decomposition at the size it exists for: the C3 workload itself (n = 2000,
    p = 50000, bench.py's X, y and key, Ozaki-II Gram) as a 2-member on-device shard group,
    25 000 columns per member -- the shard a 2-GPU .C call holds -- three sweeps
    teacher-forced against the unsharded engine, no error flags.  The members' Grams are
    rounded to fp64 separately and summed, so only the summation order differs."""
    import bench
    bb = gpu_lib
    n, p, world = 2000, 50000, 2
    X = bench.make_columns(n, 0, p)
    y, btrue = bench.make_problem_y(n, p)
    single = bb.Engine(bb.EngineConfig(n=n, p=p, seed=SEED, stream=0, true_alpha=0.5,
                                       gram_mode=bb.GRAM_OZAKI), X, y)
    single.init_state()
    per = p // world
    shards = [bb.Engine(bb.EngineConfig(n=n, p=p, p_local=per, j0=r * per, rank=r, world=world,
                                        seed=SEED, stream=0, true_alpha=0.5,
                                        gram_mode=bb.GRAM_OZAKI),
                        np.asfortranarray(X[:, r * per:(r + 1) * per]), y) for r in range(world)]
    del X
    grp = bb.ShardGroup(shards)
    grp.init_state()
    beta = btrue + 0.01 * np.random.default_rng(6).standard_normal(p)
    tau, sig2 = 1.0, 1.0
    for t in (201, 202, 203):
        single.set_state(beta, tau, sig2, 0.5)
        for r, e in enumerate(shards):
            e.set_state(beta[r * per:(r + 1) * per], tau, sig2, 0.5)
        single.run(t, 1)
        grp.run(t, 1)
        grp.sync()
        s1 = single.state()
        parts = [e.state() for e in shards]
        bg = np.concatenate([q["beta"] for q in parts])
        lg = np.concatenate([q["lambda"] for q in parts])
        for q in parts:
            assert abs(q["tau"] - s1["tau"]) <= 1e-12 * s1["tau"], t
            assert abs(q["sig2"] - s1["sig2"]) <= 1e-11 * s1["sig2"], t
        assert flips(lg, s1["lambda"]) == 0, t
        assert np.max(np.abs(lg - s1["lambda"]) / s1["lambda"]) < 1e-10, t
        assert rel_err(bg, s1["beta"]) < 1e-9, (t, rel_err(bg, s1["beta"]))
        beta, tau, sig2 = s1["beta"], s1["tau"], s1["sig2"]
    assert single.error_flags() == 0
    assert all(e.error_flags() == 0 for e in shards)
    grp.close()
    single.close()
    for e in shards:
        e.close()


def test_gpu_matches_golden_vectors(gpu_lib):
    """The HIP path against the committed fixtures (tests/golden/oracle_vectors.npz)."""
    import os

    bb = gpu_lib
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "oracle_vectors.npz"))
    x = bb.retstable_batch(g["rs_alpha"], g["rs_V0"], g["rs_h"], seed=SEED, stream=0, t=0)
    assert flips(x, g["rs_x"]) == 0
    assert np.max(np.abs(x - g["rs_x"]) / g["rs_x"]) < 1e-11
    bb.set_seed(SEED)
    ch = bb.bridge_reg_stb(g["chain_y"], g["chain_X"], nsamp=20, burn=5)
    compare_chain(ch, {k: g["chain_" + k] for k in ("beta", "lambda", "sig2", "tau", "alpha")})


def test_rccl_one_rank_communicator_is_identity(gpu_lib):
    """The RCCL exchange path (ncclCommInitRank + ncclAllReduce on the engine stream) with a
    1-rank communicator must reproduce the communicator-free engine bit for bit."""
    bb = gpu_lib
    n, p = 150, 700
    X, y, _ = synthetic_problem(n, p, seed=31)
    outs = []
    for use_comm in (False, True):
        e = bb.Engine(bb.EngineConfig(n=n, p=p, seed=SEED, stream=11, method=2,
                                      trace_capacity=8), X, y)
        if use_comm:
            e.comm_init(bb.Engine.comm_unique_id())
        e.init_state()
        e.run(1, 8, first_slot=0, slot_step=1)
        outs.append(e.trace(0, 8))
        e.close()
    for k in ("beta", "lambda", "sig2", "tau"):
        assert np.array_equal(outs[0][k], outs[1][k]), k


# ---------------------------------------------------------------------------------------
# Bridge EM (.C bridge_EM, BridgeRegression.cpp:600-708) against oracle/em.py
# ---------------------------------------------------------------------------------------
def _em_case(n, p, seed):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, p))
    b = np.zeros(p)
    k = max(3, p // 10)
    b[:k] = rng.choice([-1.0, 1.0], k) * rng.uniform(0.5, 3, k)
    y = X @ b + rng.standard_normal(n)
    return X, y


@pytest.mark.parametrize("n,p,ratio", [(200, 12, 0.3), (300, 150, 0.05), (442, 10, 2.0)])
def test_bridge_em_direct_matches_oracle(gpu_lib, n, p, ratio):
    """Direct (Cholesky) maximisation steps: same active sets, same solve count, estimates
    within 1e-9 relative (the device Cholesky's summation order differs from LAPACK's)."""
    from oracle import em
    bb = gpu_lib
    X, y = _em_case(n, p, n + p)
    tol = 1e-9
    g = bb.bridge_em(y, X, alpha=0.5, ratio=ratio, lambda_max=ratio / tol, tol=tol,
                     max_iter=30, ret_solves=True)
    o, solves = em.bridge_em(y, X, ratio, 0.5, ratio / tol, tol, 30)
    assert g["num.solves"] == solves
    assert np.array_equal(g["beta"] == 0, o == 0)
    scale = np.max(np.abs(o))
    assert np.max(np.abs(g["beta"] - o)) <= 1e-9 * scale


def test_bridge_em_cg_matches_oracle(gpu_lib):
    """CG maximisation steps (parity unpinned: the reference's cg is un-vendored; both sides
    run the textbook iteration), to the CG tolerance."""
    from oracle import em
    bb = gpu_lib
    X, y = _em_case(250, 40, 3)
    g = bb.bridge_em(y, X, alpha=0.5, ratio=0.2, lambda_max=0.2 / 1e-9, tol=1e-10,
                     max_iter=60, use_cg=True, ret_solves=True)
    o, solves = em.bridge_em(y, X, 0.2, 0.5, 0.2 / 1e-9, 1e-10, 60, use_cg=True)
    assert np.array_equal(g["beta"] == 0, o == 0)
    assert np.max(np.abs(g["beta"] - o)) <= 1e-6 * np.max(np.abs(o))
    assert abs(g["num.solves"] - solves) <= 0.1 * solves + 5


def test_bridge_em_all_dropped_and_trace(gpu_lib):
    bb = gpu_lib
    X, y = _em_case(120, 8, 5)
    g = bb.bridge_em(y, X, alpha=0.5, ratio=1.0, lambda_max=1e-300, ret_solves=True)
    assert g["num.solves"] == 0 and not g["beta"].any()
    tr = bb.trace_beta(y, X, ratio_grid=np.exp(np.arange(-4.0, 4.01, 2.0)))
    assert tr["beta"].shape == (5, 8)
    # more shrinkage at smaller ratio: the L1 norm grows along the grid
    l1 = np.abs(tr["beta"]).sum(axis=1)
    assert np.all(np.diff(l1) >= -1e-9 * l1.max())


@pytest.mark.parametrize("n,p", [(442, 10), (300, 64), (506, 103), (400, 128)])
def test_bridge_em_batch_matches_oracle(gpu_lib, n, p):
    """trace.beta's grid in one launch (a workgroup per ratio, p <= 128) against the EM
    oracle ratio by ratio: same active sets and solve counts, estimates to 1e-9."""
    from oracle import em
    bb = gpu_lib
    X, y = _em_case(n, p, 7 * p)
    tol = 1e-9
    grid = np.exp(np.arange(-6.0, 6.01, 0.5))
    beta, solves = bb.bridge_em_batch(y, X, grid, alpha=0.5, lambda_max=grid / tol, tol=tol,
                                      max_iter=30)
    for r, ratio in enumerate(grid):
        o, s = em.bridge_em(y, X, ratio, 0.5, ratio / tol, tol, 30)
        assert solves[r] == s, (ratio, solves[r], s)
        assert np.array_equal(beta[r] == 0, o == 0), ratio
        scale = max(np.max(np.abs(o)), 1e-300)
        assert np.max(np.abs(beta[r] - o)) <= 1e-9 * scale, ratio
    tr = bb.trace_beta(y, X, ratio_grid=grid)
    assert np.array_equal(tr["beta"], beta)


@pytest.mark.parametrize("n,p", [(400, 129), (500, 200), (700, 300)])
def test_bridge_em_batch_tiled_matches_oracle(gpu_lib, n, p):
    """trace.beta's grid for p > 128 (a workgroup per ratio, the p x p system in global
    memory, tiled Cholesky over LDS tiles) against the EM oracle ratio by ratio: same
    active sets and solve counts, estimates to 1e-9; trace_beta takes the batched path."""
    from oracle import em
    bb = gpu_lib
    X, y = _em_case(n, p, 11 * p)
    tol = 1e-9
    grid = np.exp(np.arange(-6.0, 6.01, 1.0))
    beta, solves = bb.bridge_em_batch(y, X, grid, alpha=0.5, lambda_max=grid / tol, tol=tol,
                                      max_iter=30)
    for r, ratio in enumerate(grid):
        o, s = em.bridge_em(y, X, ratio, 0.5, ratio / tol, tol, 30)
        assert solves[r] == s, (ratio, solves[r], s)
        assert np.array_equal(beta[r] == 0, o == 0), ratio
        scale = max(np.max(np.abs(o)), 1e-300)
        assert np.max(np.abs(beta[r] - o)) <= 1e-9 * scale, ratio
    tr = bb.trace_beta(y, X, ratio_grid=grid)
    assert np.array_equal(tr["beta"], beta)
    # a ratio's result does not depend on the batch it runs in
    b1, s1 = bb.bridge_em_batch(y, X, grid[3:4], alpha=0.5, lambda_max=grid[3:4] / tol,
                                tol=tol, max_iter=30)
    assert np.array_equal(b1[0], beta[3]) and s1[0] == solves[3]


# ---------------------------------------------------------------------------------------
# The Ozaki-II Gram on the prior variances the chain actually produces, and a long
# free-running p > n chain against an independent oracle chain (statistical parity).
# ---------------------------------------------------------------------------------------
def _gram_errors(bb, Y, w, rows):
    """Max error of the Ozaki and fp64 Grams over the rows x rows block against an 80-bit
    reference, relative to (|Y| w |Y|')_ik."""
    Cz = bb.gram(Y, w, mode=bb.GRAM_OZAKI)[np.ix_(rows, rows)]
    C6 = bb.gram(Y, w)[np.ix_(rows, rows)]
    Yl = Y[rows].astype(np.longdouble)
    ref = (Yl * w.astype(np.longdouble)) @ Yl.T
    scale = (np.abs(Y[rows]) * w) @ np.abs(Y[rows]).T
    return (float(np.max(np.abs(Cz - ref) / scale)), float(np.max(np.abs(C6 - ref) / scale)))


def test_gram_ozaki_on_c3_chain_prior_variances(gpu_lib):
    """D = tau^2 / lambda after 120 sweeps of the C3 bench chain (beta_j ~ 0 for most j, so
    lambda comes from the h = 0 stable law and D spans many decades): the Ozaki Gram keeps
    the 2e-15 / 4x-fp64 bounds of test_gram_ozaki_fp64_accuracy on that D."""
    import bench
    bb = gpu_lib
    n, p = 2000, 50000
    X = bench.make_columns(n, 0, p)
    y, _ = bench.make_problem_y(n, p)
    e = bb.Engine(bb.EngineConfig(n=n, p=p, seed=SEED, stream=0, gram_mode=bb.GRAM_OZAKI), X, y)
    e.init_state()
    e.run(1, 120)
    s = e.state()
    e.close()
    D = s["tau"] ** 2 / s["lambda"]
    span = np.log10(D.max() / D.min())
    assert span > 10, span
    rows = np.sort(np.random.default_rng(4).choice(n, 48, replace=False))
    e_oz, e_64 = _gram_errors(bb, np.asfortranarray(X), D, rows)
    assert e_oz < 2e-15, (e_oz, e_64, span)
    assert e_oz < 4 * max(e_64, 1e-16), (e_oz, e_64)


def test_gram_ozaki_thirty_decades(gpu_lib):
    bb = gpu_lib
    rng = np.random.default_rng(30)
    Y = rng.standard_normal((300, 3000))
    w = 10.0 ** rng.uniform(-25, 5, 3000)
    e_oz, e_64 = _gram_errors(bb, Y, w, np.arange(300))
    assert e_oz < 2e-15, (e_oz, e_64)
    assert e_oz < 4 * max(e_64, 1e-16), (e_oz, e_64)


def test_long_free_running_wide_chain_statistics(gpu_lib):
    """A free-running p > n chain (60 x 250, 5000 samples) decouples from any same-seed
    oracle chain within ~100 sweeps, so its parity is statistical: posterior
    means and sds against an independent long oracle chain (another key), within
    Monte-Carlo error from coda-style effective sample sizes."""
    from bayesbridge_amd.diagnostics import effective_size
    bb = gpu_lib
    X, y, _ = synthetic_problem(60, 250, seed=11)
    M, B = 5000, 500
    # sig2 known: with p > n and the Jeffreys sig2 prior the posterior has a degenerate mode
    # at sig2 -> 0 (an exact fit); the oracle chain itself falls into it near sweep 1860
    # (sig2 ~ 5e-15, I + X D X'/sig2 numerically singular)
    bb.set_seed(SEED + 40)
    g = bb.bridge_reg_stb(y, X, nsamp=M, burn=B, sig2_true=1.0)["beta"]
    o = gibbs.bridge_regression_stable(y, X, M, burn=B, seed=SEED + 41, stream=0,
                                       method="woodbury", true_sig2=1.0)["beta"].T
    for tr in (g, o):
        assert np.all(np.isfinite(tr))
    mg, mo = g.mean(axis=0), o.mean(axis=0)
    sg, so = g.std(axis=0), o.std(axis=0)
    eg = np.maximum(effective_size(g), 20.0)
    eo = np.maximum(effective_size(o), 20.0)
    z = (mg - mo) / np.sqrt(sg ** 2 / eg + so ** 2 / eo)
    assert np.max(np.abs(z)) < 5.0, float(np.max(np.abs(z)))
    assert 0.3 < np.sqrt(np.mean(z ** 2)) < 1.6, float(np.sqrt(np.mean(z ** 2)))
    # posterior sds of the larger half agree to 30 % (two oracle chains with different keys:
    # max deviation 18 %, max |z| 3.7, rms z 1.16)
    big = sg > np.median(sg)
    assert np.max(np.abs(sg[big] / so[big] - 1)) < 0.3
