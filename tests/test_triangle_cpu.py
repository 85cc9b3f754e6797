"""CPU tests of the triangle-mixture restatement (bridge.reg.tri): the truncated-normal
draw r.tnorm (restated from Robert 1995 -- the reference's RNG library is un-vendored, so
this is pinned distributionally against scipy's truncnorm), the omega/u/beta update
(BridgeRegression.cpp:97-147, 235-286, 405-433) and the driver
(BridgeWrapper.cpp:80-204) against the exact 1-D bridge posterior and against the
normal-mixture chain, which targets the same posterior."""
import math

import numpy as np
import pytest
import scipy.stats as ss

import oracle
from oracle import gibbs
from tests.test_oracle_cpu import _batch_means_se, _posterior_mean_1d


@pytest.mark.parametrize("lo,hi,mu,sd", [
    (-1.0, 1.0, 0.0, 1.0),        # holds 0, narrow: uniform rejection
    (-3.0, 4.0, 0.5, 1.0),        # holds 0, wide: normal rejection
    (-np.inf, 0.3, 0.0, 2.0),     # one-sided, holds the mean
    (2.0, 2.5, 0.0, 1.0),         # positive, narrow: uniform with rho = e^{(a^2-x^2)/2}
    (4.0, np.inf, 0.0, 1.0),      # far tail: translated exponential
    (-7.0, -5.0, 1.0, 1.0),       # negative side (mirror)
    (0.1, 0.1000001, 3.0, 0.5),   # extremely narrow
])
def test_tnorm_matches_scipy_truncnorm(lo, hi, mu, sd):
    x = np.array([oracle.tnorm(lo, hi, mu, sd, seed=7, stream=0, t=3, i=i) for i in range(4000)])
    assert np.all(x >= lo) and np.all(x <= hi)
    a, b = (lo - mu) / sd, (hi - mu) / sd
    ks = ss.kstest(x, ss.truncnorm(a, b, loc=mu, scale=sd).cdf)
    assert ks.pvalue > 1e-3, ks


def _basis(X, y):
    G = X.T @ X
    ev, V = np.linalg.eigh(G)
    o = np.argsort(ev)[::-1]
    tV = V[:, o].T.copy()
    return tV, tV @ (X.T @ y), np.sqrt(np.maximum(ev[o], 0.0))


def test_tri_update_respects_box_and_is_deterministic():
    rng = np.random.default_rng(3)
    n, p = 40, 6
    X = rng.standard_normal((n, p))
    y = X @ np.array([1.5, 0, 0, -2.0, 0, 0.5]) + rng.standard_normal(n)
    tV, a, d = _basis(X, y)
    beta0 = np.linalg.solve(X.T @ X, X.T @ y)
    for betaburn in (0, 2):
        beta, u = beta0.copy(), np.full(p, 0.5)
        om, sh = oracle.tri_update(beta, u, tV, a, d, 1.3, 1.1, 0.5, betaburn, 5, 0, 1)
        b = (1 - u) * om ** (1 / 0.5) * 1.3
        assert np.all(np.abs(beta) <= b * (1 + 1e-12))
        assert set(np.unique(sh)) <= {1.0, 2.0}
        right = 1 - np.abs(beta0) / 1.3 * om ** (-1 / 0.5)
        assert np.all((u >= 0) & (u <= right))
        beta2, u2 = beta0.copy(), np.full(p, 0.5)
        oracle.tri_update(beta2, u2, tV, a, d, 1.3, 1.1, 0.5, betaburn, 5, 0, 1)
        assert np.array_equal(beta, beta2) and np.array_equal(u, u2)


@pytest.mark.parametrize("know_tau,ortho", [(True, False), (False, False), (False, True)])
def test_tri_chain_matches_exact_posterior(know_tau, ortho):
    rng = np.random.default_rng(42)
    n = 6
    x = rng.standard_normal(n)
    y = 0.4 * x + rng.standard_normal(n)
    sig2, tau, alpha = 1.0, 0.5, 0.5
    X = x[:, None]
    out = gibbs.bridge_regression_tri(y, X, nsamp=20000, basis=_basis(X, y), burn=200,
                                      alpha=alpha, true_sig2=sig2,
                                      true_tau=tau if know_tau else 0.0, nu_shape=2.0,
                                      nu_rate=2.0, seed=99, stream=0, ortho=ortho)
    draws = out["beta"][:, 0]
    exact = _posterior_mean_1d(x, y, sig2, tau, alpha, None if know_tau else (2.0, 2.0))
    se = _batch_means_se(draws)
    # the triangle chain mixes more slowly than the normal mixture: wider batch margin
    assert abs(draws.mean() - exact) < 6 * se + 2e-3, (draws.mean(), exact, se)


def test_tri_and_stable_chains_agree_in_mean():
    """Both samplers target the same bridge posterior (Notes/bbnotes.tex)."""
    rng = np.random.default_rng(11)
    n, p = 50, 3
    X = rng.standard_normal((n, p))
    y = X @ np.array([1.0, 0.0, -0.5]) + rng.standard_normal(n)
    tri = gibbs.bridge_regression_tri(y, X, nsamp=6000, basis=_basis(X, y), burn=200,
                                      alpha=0.5, seed=4)
    stb = gibbs.bridge_regression_stable(y, X, nsamp=6000, burn=200, alpha=0.5, seed=4)
    for j in range(p):
        bt, bs = tri["beta"][:, j], stb["beta"][j]
        se = math.hypot(_batch_means_se(bt), _batch_means_se(bs))
        assert abs(bt.mean() - bs.mean()) < 6 * se + 2e-3, (j, bt.mean(), bs.mean(), se)


def test_tri_driver_slot_semantics():
    rng = np.random.default_rng(1)
    X = rng.standard_normal((30, 4))
    y = X @ np.array([1.0, 0, -2, 0]) + rng.standard_normal(30)
    out = gibbs.bridge_regression_tri(y, X, nsamp=5, basis=_basis(X, y), burn=0, alpha=0.5,
                                      true_sig2=2.0, seed=1)
    assert out["beta"].shape == (5, 4) and out["shape"].shape == (5, 4)
    # burn = 0: slot 0 holds the starting values (least squares, u = 0.5, omega = 1)
    assert np.allclose(out["beta"][0], np.linalg.solve(X.T @ X, X.T @ y))
    assert np.all(out["u"][0] == 0.5) and np.all(out["w"][0] == 1.0)
    assert np.all(out["shape"][0] == 0.0) and np.all(out["sig2"] == 2.0)
    assert set(np.unique(out["shape"][1:])) <= {1.0, 2.0}


def test_tri_ortho_chain_matches_dense_on_orthogonal_design():
    """On an orthogonal design the coordinate-wise beta update (sample_beta_ortho) and
    the svd-basis rtnorm_gibbs target the same posterior."""
    rng = np.random.default_rng(8)
    n, p = 40, 3
    Q, _ = np.linalg.qr(rng.standard_normal((n, p)))
    X = Q * np.array([3.0, 2.0, 1.5])
    y = X @ np.array([0.8, 0.0, -0.6]) + rng.standard_normal(n)
    kw = dict(nsamp=6000, basis=_basis(X, y), burn=200, alpha=0.5, seed=12)
    a = gibbs.bridge_regression_tri(y, X, ortho=True, **kw)
    b = gibbs.bridge_regression_tri(y, X, ortho=False, **kw)
    for j in range(p):
        se = math.hypot(_batch_means_se(a["beta"][:, j]), _batch_means_se(b["beta"][:, j]))
        assert abs(a["beta"][:, j].mean() - b["beta"][:, j].mean()) < 6 * se + 2e-3, j


def test_tri_golden_fixture_invariants():
    """The committed triangle fixture (tests/golden) respects the box constraint it was
    drawn under (b = (1 - u) omega^(1/alpha) tau, tau = 1.1, alpha = 0.5)."""
    import os

    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "oracle_vectors.npz"))
    b = (1 - g["tri_u"]) * g["tri_omega"] ** 2.0 * 1.1
    assert np.all(np.abs(g["tri_beta"]) <= b * (1 + 1e-12))
    assert np.allclose(g["tri_tV"] @ g["tri_tV"].T, np.eye(4), atol=1e-12)
