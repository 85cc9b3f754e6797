"""CPU tests: pin the oracle (tests' checker) before trusting it.

The reference ships no golden vectors for this path and cannot be built or run here
(DESIGN.md "Oracle"), so the oracle is pinned by
  * Philox4x64-10 known-answer vectors (Random123 kat_vectors) and numpy's
    independent Philox implementation,
  * analytic properties of the tilted stable law (mean, Laplace transform),
  * the exact Gaussian conditional of beta | rest (both draw maps),
  * quadrature of the exact bridge posterior on 1-D problems (whole Gibbs chain).
"""
import math

import numpy as np
import pytest
import scipy.integrate as si
import scipy.stats as ss

import oracle
from oracle import gibbs

M64 = 0xFFFFFFFFFFFFFFFF


def test_philox_random123_kat():
    # Random123 kat_vectors, philox4x64_10
    assert oracle.philox4x64([0, 0, 0, 0], [0, 0]) == [
        0x16554D9ECA36314C, 0xDB20FE9D672D0FDC, 0xD7E772CEE186176B, 0x7E68B68AEC7BA23B]
    assert oracle.philox4x64([M64] * 4, [M64, M64]) == [
        0x87B092C3013FE90B, 0x438C3C67BE8D0224, 0x9CC7D7C69CD777B6, 0xA09CAEBF594F0BA0]
    assert oracle.philox4x64(
        [0x243F6A8885A308D3, 0x13198A2E03707344, 0xA4093822299F31D0, 0x082EFA98EC4E6C89],
        [0x452821E638D01377, 0xBE5466CF34E90C6C]) == [
        0xA528F45403E61D95, 0x38C72DBD566E9788, 0xA5A1610E72FD18B5, 0x57BD43B5E52B7FE6]


def test_philox_matches_numpy():
    rng = np.random.default_rng(7)
    for _ in range(50):
        key = [int(x) for x in rng.integers(0, 2**63, size=2)]
        ctr = [int(x) for x in rng.integers(0, 2**63, size=4)]
        # numpy increments the counter before generating
        pre = list(ctr)
        pre[0] = (pre[0] - 1) & M64
        bg = np.random.Philox(key=np.array(key, dtype=np.uint64),
                              counter=np.array(pre, dtype=np.uint64))
        assert [int(x) for x in bg.random_raw(4)] == oracle.philox4x64(ctr, key)


def test_uniforms_open_interval_and_layout():
    u = oracle.uniforms(1, 2, 3, oracle.KIND_BETA_Z, 5, 0, 0)
    assert np.all((u > 0) & (u < 1))
    raw = oracle.philox4x64([3, (oracle.KIND_BETA_Z << 56) | 5, 0, 0], [1, 2])
    expect = [((x >> 11) + 0.5) * 2.0**-53 for x in raw]
    assert np.array_equal(u, np.array(expect))


def test_normals_moments():
    z = oracle.normals(200000, 11, 0, 1, oracle.KIND_BETA_Z)
    assert abs(z.mean()) < 5 / math.sqrt(len(z))
    assert abs(z.var() - 1) < 5 * math.sqrt(2 / len(z))
    assert ss.kstest(z, "norm").pvalue > 1e-4


@pytest.mark.parametrize("a", [0.05, 0.15, 0.25, 0.45, 0.75])
@pytest.mark.parametrize("h", [0.0, 1e-4, 1e-2, 1.0, 1e2, 1e4])
def test_retstable_laplace_transform(a, h):
    """E[exp(-s S)] = exp(-((h+s)^a - h^a)) (retstable.cpp:79-93 doc)."""
    N = 40000
    x = oracle.retstable_batch(np.full(N, a), np.ones(N), np.full(N, h), seed=3, stream=1, t=0)
    assert np.all(x > 0) and np.all(np.isfinite(x))
    scale = 1.0 / max(a * max(h, 1e-300) ** (a - 1), 1e-300) if h > 0 else 1.0
    for s in (0.1 / scale, 1.0 / scale, 5.0 / scale):
        est = np.mean(np.exp(-s * x))
        exact = math.exp(-((h + s) ** a - h ** a))
        assert abs(est - exact) < 5 * 0.5 / math.sqrt(N) + 1e-12, (s, est, exact)


@pytest.mark.parametrize("a,h", [(0.25, 1.0), (0.25, 100.0), (0.45, 1.0), (0.45, 0.01),
                                 (0.15, 1e4), (0.75, 3.0)])
def test_retstable_mean(a, h):
    """E[S] = a h^(a-1) for h > 0."""
    N = 100000
    x = oracle.retstable_batch(np.full(N, a), np.ones(N), np.full(N, h), seed=5, stream=2, t=0)
    mean = a * h ** (a - 1)
    # variance a(1-a) h^(a-2)
    se = math.sqrt(a * (1 - a) * h ** (a - 2) / N)
    assert abs(x.mean() - mean) < 6 * se, (x.mean(), mean, se)


def test_retstable_alpha_one_and_V0():
    x = oracle.retstable_batch(np.ones(10), np.full(10, 2.5), np.full(10, 3.0), seed=1)
    assert np.all(x == 2.5)
    # V0 scaling: LST exp(-V0((h+t)^a - h^a)) at h = 0 -> S = V0^(1/a) S_1
    N = 40000
    a, V0 = 0.4, 2.0
    x = oracle.retstable_batch(np.full(N, a), np.full(N, V0), np.zeros(N), seed=9)
    for s in (0.3, 1.0, 3.0):
        est = np.mean(np.exp(-s * x))
        assert abs(est - math.exp(-V0 * s ** a)) < 5 * 0.5 / math.sqrt(N)


def test_gamma_moments():
    for shape in (0.3, 1.0, 2.5, 50.0, 5000.5):
        g = np.array([oracle.gamma1(shape, 13, 0, t, oracle.KIND_TAU) for t in range(20000)])
        assert abs(g.mean() - shape) < 6 * math.sqrt(shape / len(g))
        assert ss.kstest(g, "gamma", args=(shape,)).pvalue > 1e-4


def test_beta_step_maps_agree_in_distribution():
    """Woodbury (p > n) and reference Cholesky maps sample the same N(m, sig2 A^-1)."""
    rng = np.random.default_rng(0)
    n, p = 7, 12
    X = rng.standard_normal((n, p))
    y = rng.standard_normal(n)
    lam = rng.uniform(0.1, 5, p)
    sig2, tau = 0.7, 1.3
    G, c = X.T @ X, X.T @ y
    A = G + np.diag(lam * sig2 / tau ** 2)
    m_exact = np.linalg.solve(A, c)
    cov_exact = sig2 * np.linalg.inv(A)
    # affine maps in the standard-normal inputs
    b0c = gibbs.beta_step_chol(G, c, lam, sig2, tau, np.zeros(p))
    b0w = gibbs.beta_step_woodbury(X, y, lam, sig2, tau, np.zeros(p), np.zeros(n))
    np.testing.assert_allclose(b0c, m_exact, rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(b0w, m_exact, rtol=1e-10, atol=1e-12)
    Bc = np.column_stack([gibbs.beta_step_chol(G, c, lam, sig2, tau, e) - b0c for e in np.eye(p)])
    Bw = np.column_stack(
        [gibbs.beta_step_woodbury(X, y, lam, sig2, tau, e[:p], e[p:]) - b0w
         for e in np.eye(p + n)])
    np.testing.assert_allclose(Bc @ Bc.T, cov_exact, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(Bw @ Bw.T, cov_exact, rtol=1e-9, atol=1e-12)


def _posterior_mean_1d(x, y, sig2, tau, alpha, nu=None):
    """Exact posterior mean of beta for p = 1 by quadrature.

    Known tau: prior exp(-|b/tau|^a).  Unknown tau with nu = tau^-a ~ Ga(a0, b0):
    marginal prior (b0 + |b|^a)^-(a0 + 1/a)   (BridgeRegression.cpp:453-465 model).
    """
    xx, xy = float(x @ x), float(x @ y)
    bhat = xy / xx
    sd = math.sqrt(sig2 / xx)

    def logpost(b):
        ll = -0.5 * (xx * b * b - 2 * xy * b) / sig2
        if nu is None:
            lp = -abs(b / tau) ** alpha
        else:
            a0, b0 = nu
            lp = -(a0 + 1.0 / alpha) * math.log(b0 + abs(b) ** alpha)
        return ll + lp

    lo, hi = bhat - 12 * sd - 1, bhat + 12 * sd + 1
    grid = np.linspace(lo, hi, 40001)
    lv = np.array([logpost(b) for b in grid])
    wv = np.exp(lv - lv.max())
    Z = si.simpson(wv, x=grid)
    return si.simpson(wv * grid, x=grid) / Z


def _batch_means_se(x, nb=40):
    bm = np.array([c.mean() for c in np.array_split(x, nb)])
    return bm.std(ddof=1) / math.sqrt(nb)


@pytest.mark.parametrize("know_tau", [True, False])
def test_gibbs_chain_matches_exact_posterior(know_tau):
    rng = np.random.default_rng(42)
    n = 6
    x = rng.standard_normal(n)
    y = 0.4 * x + rng.standard_normal(n)
    sig2, tau, alpha = 1.0, 0.5, 0.5
    out = gibbs.bridge_regression_stable(y, x[:, None], nsamp=20000, burn=200, alpha=alpha,
                                         true_sig2=sig2, true_tau=tau if know_tau else 0.0,
                                         nu_shape=2.0, nu_rate=2.0, seed=99, stream=0)
    draws = out["beta"][0]
    exact = _posterior_mean_1d(x, y, sig2, tau, alpha, None if know_tau else (2.0, 2.0))
    se = _batch_means_se(draws)
    assert abs(draws.mean() - exact) < 5 * se + 1e-3, (draws.mean(), exact, se)


def test_gibbs_driver_slot_semantics():
    """Trace layout and known-parameter fills (BridgeWrapper.cpp:242-250, 266-298)."""
    rng = np.random.default_rng(1)
    X = rng.standard_normal((30, 4))
    y = X @ np.array([1.0, 0, -2, 0]) + rng.standard_normal(30)
    out = gibbs.bridge_regression_stable(y, X, nsamp=5, burn=3, alpha=0.5, true_sig2=2.0,
                                         seed=1)
    assert out["beta"].shape == (4, 5) and out["lambda"].shape == (4, 5)
    assert np.all(out["sig2"] == 2.0) and np.all(out["alpha"] == 0.5)
    assert np.all(out["tau"] > 0) and np.all(out["lambda"] > 0)
    # deterministic given the key
    out2 = gibbs.bridge_regression_stable(y, X, nsamp=5, burn=3, alpha=0.5, true_sig2=2.0,
                                          seed=1)
    assert np.array_equal(out["beta"], out2["beta"])
    out3 = gibbs.bridge_regression_stable(y, X, nsamp=5, burn=3, alpha=0.5, true_sig2=2.0,
                                          seed=1, stream=1)
    assert not np.array_equal(out["beta"], out3["beta"])


def test_unknown_alpha_chain_runs():
    rng = np.random.default_rng(2)
    X = rng.standard_normal((40, 5))
    y = X @ np.array([2.0, 0, -1, 0, 0]) + rng.standard_normal(40)
    out = gibbs.bridge_regression_stable(y, X, nsamp=300, burn=50, alpha=0.0, seed=3)
    a = out["alpha"]
    assert np.all((a > 0) & (a < 1))
    assert len(np.unique(a)) > 10  # MH moves


def test_ortho_chain_matches_dense_on_orthogonal_design():
    """For orthogonal X the ortho step's law equals the dense step's law."""
    rng = np.random.default_rng(3)
    Q, _ = np.linalg.qr(rng.standard_normal((50, 4)))
    X = Q * 3.0
    y = X @ np.array([0.5, 0, -0.7, 0]) + 0.3 * rng.standard_normal(50)
    o1 = gibbs.bridge_regression_stable(y, X, nsamp=6000, burn=100, alpha=0.5, true_sig2=0.09,
                                        true_tau=1.0, ortho=True, seed=4)
    o2 = gibbs.bridge_regression_stable(y, X, nsamp=6000, burn=100, alpha=0.5, true_sig2=0.09,
                                        true_tau=1.0, seed=5)
    for j in range(4):
        se = math.hypot(_batch_means_se(o1["beta"][j]), _batch_means_se(o2["beta"][j]))
        assert abs(o1["beta"][j].mean() - o2["beta"][j].mean()) < 5 * se + 1e-3


# ---------------------------------------------------------------------------------------
# Bridge EM oracle (oracle/em.py, restating BridgeRegression.cpp:600-708)
# ---------------------------------------------------------------------------------------
def _em_problem(n=200, p=12, seed=11):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, p))
    b = np.zeros(p)
    b[:4] = [3.0, -2.0, 1.5, 0.02]
    y = X @ b + rng.standard_normal(n)
    return X, y


def test_em_large_ratio_is_least_squares():
    """tau large against O(1) coefficients: the penalty c2 lambda_j = alpha tau^-alpha
    |beta_j|^(alpha-2) is ~5e-5 against X'X's ~200 diagonal, so EM stops next to OLS."""
    from oracle import em
    rng = np.random.default_rng(12)
    X = rng.standard_normal((200, 12))
    b = rng.choice([-1.0, 1.0], 12) * rng.uniform(1, 3, 12)
    y = X @ b + rng.standard_normal(200)
    beta, solves = em.bridge_em(y, X, ratio=1e8, alpha=0.5, lambda_max=1e300, tol=1e-12,
                                max_iter=50)
    ls = np.linalg.lstsq(X, y, rcond=None)[0]
    assert np.allclose(beta, ls, rtol=1e-5, atol=0)
    assert solves >= 2 * X.shape[1]


def test_em_fixed_point_is_stationary():
    """At convergence the active set satisfies (X'X + c2 diag(lambda(beta))) beta = X'y."""
    from oracle import em
    X, y = _em_problem()
    ratio, alpha = 0.05, 0.5
    beta, _ = em.bridge_em(y, X, ratio, alpha, lambda_max=ratio / 1e-9, tol=1e-13,
                           max_iter=500)
    act = beta != 0
    assert 0 < act.sum() < X.shape[1]  # shrinkage drops the null coordinates
    c1 = alpha * ratio ** (2 - alpha)
    c2 = ratio ** -2
    lam = c1 * np.abs(beta[act]) ** (alpha - 2)
    Xa = X[:, act]
    r = (Xa.T @ Xa + np.diag(c2 * lam)) @ beta[act] - Xa.T @ y
    assert np.max(np.abs(r)) < 1e-6 * np.max(np.abs(Xa.T @ y))


def test_em_cg_matches_direct():
    from oracle import em
    X, y = _em_problem()
    bd, _ = em.bridge_em(y, X, 0.3, 0.5, 0.3 / 1e-9, 1e-10, 100)
    bc, _ = em.bridge_em(y, X, 0.3, 0.5, 0.3 / 1e-9, 1e-10, 100, use_cg=True)
    assert np.allclose(bc, bd, rtol=1e-6, atol=1e-8)


def test_em_all_dropped_returns_iteration_count():
    """lambda_max below every lambda: beta = 0 and the EM iteration count (0) is returned
    (the reference's early `return iter`, BridgeRegression.cpp:654-657)."""
    from oracle import em
    X, y = _em_problem()
    beta, it = em.bridge_em(y, X, 1.0, 0.5, lambda_max=1e-300, tol=1e-9, max_iter=30)
    assert it == 0 and not beta.any()
