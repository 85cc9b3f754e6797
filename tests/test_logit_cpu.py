"""CPU checks of the logistic-bridge oracle (BASELINE config C4).  The reference has no
logistic model, so the oracle's Polya-Gamma sampler (Polson, Scott & Windle 2013, restated
in oracle/bb_oracle.c) is pinned by the PG law itself -- exact moments, the Laplace
transform, and a two-sample KS test against the infinite-convolution definition -- and
the whole chain by the exact 1-D posterior (quadrature).  Parity unpinned against any
reference implementation."""
import numpy as np
import pytest
from scipy import integrate, stats

import oracle
from oracle import gibbs


def pg_mean_var(c):
    if c == 0:
        return 0.25, 1.0 / 24.0
    return np.tanh(c / 2) / (2 * c), (np.sinh(c) - c) / (4 * c ** 3 * np.cosh(c / 2) ** 2)


@pytest.mark.parametrize("c", [0.0, 0.3, 2.0, 8.0, 40.0, -5.0])
def test_pg_moments(c):
    w = oracle.pg_batch(np.full(200000, c), 11, 0, 3)
    m, v = pg_mean_var(abs(c))
    assert abs(w.mean() - m) < 5 * np.sqrt(v / w.size)
    assert abs(w.var() / v - 1) < 0.03
    assert np.all(w > 0)


@pytest.mark.parametrize("c", [0.0, 1.0, 6.0])
def test_pg_laplace_transform(c):
    w = oracle.pg_batch(np.full(200000, c), 12, 1, 0)
    for s in (0.5, 2.0, 10.0, 50.0):
        e = np.exp(-s * w)
        exact = np.cosh(c / 2) / np.cosh(np.sqrt((c * c / 2 + s) / 2))
        assert abs(e.mean() - exact) < 5 * e.std() / np.sqrt(w.size) + 1e-12, (c, s)


@pytest.mark.parametrize("c", [0.0, 1.5, 10.0])
def test_pg_matches_series_definition(c):
    """PG(1, c) = (1 / 2 pi^2) sum_k g_k / ((k - 1/2)^2 + c^2 / (4 pi^2)), g_k ~ Exp(1)."""
    rng = np.random.default_rng(5)
    K, N = 300, 20000
    k = np.arange(1, K + 1)
    d = (k - 0.5) ** 2 + c * c / (4 * np.pi ** 2)
    kk = np.arange(K + 1, 400000)
    tail = (1.0 / ((kk - 0.5) ** 2 + c * c / (4 * np.pi ** 2))).sum()
    ref = ((rng.exponential(size=(N, K)) / d).sum(axis=1) + tail) / (2 * np.pi ** 2)
    w = oracle.pg_batch(np.full(N, c), 13, 0, 0)
    assert stats.ks_2samp(w, ref).pvalue > 1e-3


def test_pg_counter_determinism():
    psi = np.linspace(-20, 20, 1001)
    a = oracle.pg_batch(psi, 1, 2, 3)
    b = oracle.pg_batch(psi, 1, 2, 3)
    c = oracle.pg_batch(psi, 1, 2, 4)
    assert np.array_equal(a, b) and not np.array_equal(a, c)
    # omega depends on |psi| only through the same counters
    assert np.array_equal(oracle.pg_batch(-psi, 1, 2, 3), a)


def test_logit_chain_matches_exact_posterior():
    """p = 1, tau known: the chain's posterior mean of beta against 1-D quadrature of
    prod_i sigma((2 y_i - 1) x_i beta) exp(-|beta / tau|^alpha)."""
    rng = np.random.default_rng(21)
    n, tau, alpha = 60, 0.8, 0.5
    x = rng.standard_normal(n)
    y = (rng.random(n) < 1 / (1 + np.exp(-1.2 * x))).astype(float)
    s = 2 * y - 1

    def logpost(b):
        return -np.sum(np.logaddexp(0.0, -s * x * b)) - abs(b / tau) ** alpha

    lo, hi = -6.0, 8.0
    bm = integrate.quad(lambda b: np.exp(logpost(b) + 30), lo, hi, limit=400, points=[0.0])[0]
    m1 = integrate.quad(lambda b: b * np.exp(logpost(b) + 30), lo, hi, limit=400, points=[0.0])[0]
    exact = m1 / bm
    o = gibbs.bridge_regression_logit(y, x[:, None], 6000, burn=300, alpha=alpha, true_tau=tau,
                                      seed=77)
    tr = o["beta"][0]
    # batch-means standard error
    bmeans = tr.reshape(60, -1).mean(axis=1)
    se = bmeans.std(ddof=1) / np.sqrt(bmeans.size)
    assert abs(tr.mean() - exact) < 5 * se + 1e-3, (tr.mean(), exact, se)
    assert np.all(o["tau"] == tau)
