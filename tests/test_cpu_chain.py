"""The compiled CPU-baseline chain (oracle/bb_cpu_chain.c, scipy's OpenBLAS) against the
Python oracle (oracle/gibbs.py) on the same Philox counters: it restates the same driver,
so it must draw the same chain up to LAPACK rounding.  This is what makes its timing a
baseline for the same computation the GPU runs."""
import numpy as np
import pytest

import oracle
from oracle import gibbs
from tests.conftest import synthetic_problem

SEED = 0xB4E5B41D6E


def _close(c, o, tol_elem, tol_mean):
    for k in ("tau", "sig2"):
        assert np.max(np.abs(c[k] - o[k]) / np.abs(o[k])) < tol_elem, k
    b, ob = c["beta"], o["beta"]
    assert np.max(np.abs(b - ob) / np.maximum(np.abs(ob), 1e-8)) < tol_elem
    assert np.linalg.norm(b.mean(1) - ob.mean(1)) / np.linalg.norm(ob.mean(1)) < tol_mean


@pytest.mark.parametrize("method,n,p", [("chol", 100, 20), ("chol", 442, 64),
                                        ("ortho", 120, 10)])
def test_cpu_chain_matches_oracle_narrow(method, n, p):
    X, y, _ = synthetic_problem(n, p, seed=n + p)
    c = oracle.cpu_chain(y, X, 200, burn=20, method=method, seed=SEED, stream=3)
    o = gibbs.bridge_regression_stable(y, X, 200, burn=20, method=method, seed=SEED, stream=3)
    _close(c, o, 1e-6, 1e-8)


def test_cpu_chain_matches_oracle_wide_first_sweeps():
    """p > n chains are chaotic under roundoff: compare the first sweeps."""
    X, y, _ = synthetic_problem(60, 250, seed=11)
    c = oracle.cpu_chain(y, X, 6, burn=2, seed=SEED, stream=0)
    o = gibbs.bridge_regression_stable(y, X, 6, burn=2, seed=SEED, stream=0, method="woodbury")
    assert c["method"] == "woodbury"
    _close(c, o, 1e-8, 1e-9)


def test_cpu_chain_threads_do_not_change_draws():
    X, y, _ = synthetic_problem(200, 40, seed=5)
    a = oracle.cpu_chain(y, X, 50, burn=5, seed=SEED, stream=1, threads=1)
    b = oracle.cpu_chain(y, X, 50, burn=5, seed=SEED, stream=1, threads=4)
    # lambda draws are counter-based; only BLAS summation order may differ with threads
    assert np.max(np.abs(a["beta"] - b["beta"]) / np.maximum(np.abs(a["beta"]), 1e-8)) < 1e-9


def test_cpu_logit_chain_matches_oracle():
    """The compiled logistic (Polya-Gamma) chain against gibbs.bridge_regression_logit."""
    rng = np.random.default_rng(9)
    n, p = 400, 30
    X = rng.standard_normal((n, p))
    b = np.zeros(p)
    b[:4] = [1.5, -1.0, 0.8, -2.0]
    y = (rng.random(n) < 1 / (1 + np.exp(-(X @ b)))).astype(np.float64)
    c = oracle.cpu_logit_chain(y, X, 40, burn=5, seed=SEED, stream=2)
    o = gibbs.bridge_regression_logit(y, X, 40, burn=5, seed=SEED, stream=2)
    assert np.max(np.abs(c["tau"] - o["tau"]) / o["tau"]) < 1e-8
    assert np.max(np.abs(c["beta"] - o["beta"]) / np.maximum(np.abs(o["beta"]), 1e-8)) < 1e-7


def test_cpu_sparse_chain_matches_oracle_first_sweeps():
    """The compiled sparse (CSC) Woodbury chain against gibbs on the same sparse design."""
    import bench
    X = bench.make_sparse_columns(150, 0, 900, density=0.05, seed=3)
    y = np.asarray(X[:, :6] @ np.array([2.0, -1.5, 1.0, 2.5, -2.0, 1.2])).ravel()
    y = y + np.random.default_rng(4).standard_normal(150)
    y -= y.mean()
    c = oracle.cpu_sparse_chain(y, X, 6, burn=2, seed=SEED, stream=0)
    o = gibbs.bridge_regression_stable(y, X, 6, burn=2, seed=SEED, stream=0, method="woodbury")
    _close(c, o, 1e-8, 1e-9)
    c4 = oracle.cpu_sparse_chain(y, X, 6, burn=2, seed=SEED, stream=0, threads=4)
    assert np.max(np.abs(c4["beta"] - c["beta"]) / np.maximum(np.abs(c["beta"]), 1e-8)) < 1e-9
