"""CPU checks of the sparse-design (BASELINE config C5) pieces that need no GPU: the
synthetic CSC generator, and the oracle's sparse Woodbury step against its dense form."""
import numpy as np
import scipy.sparse as sps

import bench
import oracle
from oracle import gibbs

SEED = 0xB4E5B41D6E


def test_sparse_generator_is_shard_independent():
    n, p = 300, 2500
    full = bench.make_sparse_columns(n, 0, p, density=0.02)
    for j0, j1 in ((0, 700), (700, 1999), (1999, 2500), (123, 124)):
        part = bench.make_sparse_columns(n, j0, j1, density=0.02)
        assert (part != full[:, j0:j1]).nnz == 0
    dens = full.nnz / (n * p)
    assert abs(dens - 0.02) < 5 * np.sqrt(0.02 / (n * p))
    # canonical CSC (what the C ABI requires): sorted, unique rows per column
    assert full.has_canonical_format


def test_sparse_problem_matches_its_design():
    n, p = 200, 3000
    y, b = bench.make_sparse_problem_y(n, p, density=0.05)
    assert y.shape == (n,) and abs(y.mean()) < 1e-12
    assert np.count_nonzero(b) == max(5, p // 100)


def test_sparse_woodbury_step_equals_dense():
    """The oracle's sparse (scipy SpGEMM) Woodbury draw is the dense one on the same X."""
    rng = np.random.default_rng(4)
    n, p = 80, 900
    X = sps.random(n, p, density=0.05, random_state=5, format="csc",
                   data_rvs=rng.standard_normal)
    y = rng.standard_normal(n)
    lam = rng.exponential(1.0, p) + 1e-3
    z, d = rng.standard_normal(p), rng.standard_normal(n)
    bs = gibbs.beta_step_woodbury(X, y, lam, 1.3, 0.7, z, d)
    bd = gibbs.beta_step_woodbury(X.toarray(), y, lam, 1.3, 0.7, z, d)
    assert np.linalg.norm(bs - bd) <= 1e-12 * np.linalg.norm(bd)


def test_sparse_oracle_chain_equals_dense_chain_first_sweeps():
    rng = np.random.default_rng(6)
    n, p = 60, 400
    X = sps.random(n, p, density=0.08, random_state=7, format="csc",
                   data_rvs=rng.standard_normal)
    y = X[:, :5] @ np.array([2.0, -1.0, 1.5, 2.5, -2.0]) + rng.standard_normal(n)
    a = gibbs.bridge_regression_stable(y, X, 6, burn=2, seed=SEED, method="woodbury")
    b = gibbs.bridge_regression_stable(y, X.toarray(), 6, burn=2, seed=SEED, method="woodbury")
    for k in ("tau", "sig2"):
        assert np.allclose(a[k], b[k], rtol=1e-9, atol=0)
    assert np.allclose(a["beta"], b["beta"], rtol=1e-7, atol=1e-9)
    assert oracle.sum_abs_pow(a["beta"][:, -1], 0.5) > 0
