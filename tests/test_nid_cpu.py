"""The near-identity (Chebyshev) solve of the Woodbury system, restated on
the CPU (oracle/gibbs.py woodbury_solve_cheb / beta_step_woodbury_nid): its certified bound
holds and its draw equals the Cholesky draw of beta_step_woodbury (BridgeRegression.cpp:
552-575 in Woodbury form) to rounding across the regimes where it is taken."""
import numpy as np
import pytest

from oracle import gibbs
from tests.conftest import synthetic_problem


def test_iteration_rule():
    # tiny eps: two iterates (one product); the count grows with eps; beyond kmax: 0
    assert gibbs.cheb_iterations(0.0, 16) == 1
    assert gibbs.cheb_iterations(1e-12, 16) == 2
    assert gibbs.cheb_iterations(1e-6, 16) == 3
    ks = [gibbs.cheb_iterations(e, 64) for e in (1e-9, 1e-6, 1e-3, 1e-2, 0.1, 1.0)]
    assert ks == sorted(ks) and ks[-1] > ks[0]
    assert gibbs.cheb_iterations(10.0, 16) == 0
    assert gibbs.cheb_iterations(float("nan"), 16) == 0


@pytest.mark.parametrize("eps_target", [1e-12, 1e-8, 1e-5, 1e-3, 1e-1, 1.0])
def test_certified_bound_holds(eps_target):
    """Random PSD E scaled so tr(E) = eps: the K-iterate solve is within the bound of the
    exact solve (and within 2^-56 relative, the decision tolerance)."""
    rng = np.random.default_rng(int(-np.log10(eps_target)) + 3)
    n = 120
    B = rng.standard_normal((n, 300)) * rng.uniform(0, 1, 300)
    E = B @ B.T
    E *= eps_target / np.trace(E)
    rhs = rng.standard_normal(n)
    K = gibbs.cheb_iterations(eps_target, 64)
    assert K > 0
    x = gibbs.woodbury_solve_cheb(lambda t: E @ t, rhs, eps_target, K)
    w = np.linalg.solve(np.eye(n) + E, rhs)
    err = np.linalg.norm(x - w) / np.linalg.norm(w)
    assert err < 1e-15 + 4e-16 * np.sqrt(n), (K, err)


@pytest.mark.parametrize("certified", [False, True])
@pytest.mark.parametrize("tau", [1e-7, 1e-4, 1e-3, 3e-3])
def test_nid_draw_matches_cholesky_draw(tau, certified):
    """Woodbury beta draws (n = 80, p = 400) at prior scales from the near-null regime up to
    where the path hands over to the Cholesky factor: same draw to rounding, with the trace
    bound alone or the thresholded bound (Lambda = 1.02 lambda_max(X X'))."""
    X, y, b = synthetic_problem(80, 400, seed=9)
    rng = np.random.default_rng(1)
    lam = rng.exponential(1.0, 400) * 2.0
    z, d = rng.standard_normal(400), rng.standard_normal(80)
    sig2 = float(np.var(y))
    lam_x = 1.02 * np.linalg.eigvalsh(X @ X.T)[-1] if certified else 0.0
    bn, K = gibbs.beta_step_woodbury_nid(X, y, lam, sig2, tau, z, d, lam_x=lam_x)
    bc = gibbs.beta_step_woodbury(X, y, lam, sig2, tau, z, d)
    assert np.linalg.norm(bn - bc) / np.linalg.norm(bc) < 1e-13, K
    if tau <= 1e-4:
        assert 1 <= K <= 4


def test_nid_draw_sparse():
    import bench
    X = bench.make_sparse_columns(300, 0, 3000, density=0.02, seed=4)
    y = np.asarray(X[:, :5] @ np.ones(5)).ravel() + np.random.default_rng(2).standard_normal(300)
    rng = np.random.default_rng(3)
    lam = rng.exponential(1.0, 3000) * 2.0
    z, d = rng.standard_normal(3000), rng.standard_normal(300)
    bn, K = gibbs.beta_step_woodbury_nid(X, y, lam, 50.0, 1e-4, z, d)
    bc = gibbs.beta_step_woodbury(X, y, lam, 50.0, 1e-4, z, d)
    assert K > 0 and np.linalg.norm(bn - bc) / np.linalg.norm(bc) < 1e-13


@pytest.mark.parametrize("world", [1, 2, 4])
@pytest.mark.parametrize("log_tau", [-6.0, -3.0, -1.0])
def test_shard_bound_is_certified(world, log_tau):
    """The column-sharded decision (bb_nid.hip k_nid_sums / k_nid_decide_from): the bound
    from the summed shard sums and the summed shard certificates Lambda_r is an upper bound of
    lambda_max(E), E = X D X' / sig2, and never above the trace bound."""
    rng = np.random.default_rng(world * 10 + int(-log_tau))
    n, p = 60, 400
    X = rng.standard_normal((n, p)) * rng.uniform(0.2, 2.0, p)
    tau, sig2 = 10.0 ** log_tau, 0.7
    lam = rng.exponential(1.0, p) ** 3 + 1e-12  # heavy-tailed 1 / lambda
    D = tau * tau / lam
    E = (X * D) @ X.T / sig2
    lmax = np.linalg.eigvalsh(E)[-1]
    per = (p + world - 1) // world
    red = np.zeros(gibbs.NID_TS + 2)
    for r in range(world):
        Xr = X[:, r * per:(r + 1) * per]
        lam_r = 1.02 * np.linalg.eigvalsh(Xr @ Xr.T)[-1]
        red += gibbs.nid_shard_partials(D[r * per:(r + 1) * per], (Xr * Xr).sum(axis=0), tau,
                                        lam_r)
    eps, K = gibbs.nid_decide_from(red, tau, sig2)
    trace = float(np.sum(D * (X * X).sum(axis=0))) / sig2
    assert lmax <= eps <= trace * (1 + 2e-6)
    # an uncertified shard leaves the trace bound
    red[gibbs.NID_TS + 1] = np.inf
    eps_t, _ = gibbs.nid_decide_from(red, tau, sig2)
    assert abs(eps_t - trace * (1 + 1e-6)) <= 1e-12 * trace


# ---------------------------------------------------------------------------------------
# The mixed-precision plan (bb_nid.hip nid_plan_mixed, bb_engine
# nidx_mixed_tail) restated in oracle/gibbs.py
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("seed,n,p,spread", [(1, 80, 400, 2.0), (2, 120, 900, 6.0),
                                             (3, 60, 200, 0.5), (4, 100, 600, 10.0)])
def test_mixed_eta_bounds_fp32_rounding_of_E(seed, n, p, spread):
    """eta = 2 u32 sqrt(tr(E) eps) + u32^2 tr(E) bounds |E - E~|_2 for E~ = X32 D X32' / sig2
    with X32 = fl32(X) and eps >= lambda_max(E) -- the certificate the mixed plan rests on --
    on random designs with D over `spread` decades."""
    from oracle import gibbs
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, p)) * 10.0 ** rng.uniform(-3, 3, size=p)
    D = 10.0 ** rng.uniform(-spread, 0, size=p) * 1e-3
    sig2 = 1.7
    X32 = X.astype(np.float32).astype(np.float64)
    E = (X * D) @ X.T / sig2
    E32 = (X32 * D) @ X32.T / sig2
    lmax = np.linalg.eigvalsh(E)[-1]
    tr = np.trace(E)
    for eps in (lmax, 3 * lmax, tr):
        _, _, eta, _ = gibbs.nid_plan_mixed(eps, tr, 16, np.inf)
        err = np.abs(np.linalg.eigvalsh(E - E32)).max()
        assert err <= eta, (eps, err, eta)
        assert eta < 64 * gibbs.U32 * np.sqrt(tr * eps) + 1e-300


@pytest.mark.parametrize("eps_scale", [1e-12, 1e-8, 1e-5, 1e-3, 3e-2])
def test_mixed_solve_meets_certified_bound(eps_scale):
    """The mixed plan chosen for a state solves (I + E) w = b to the fp64 plan's accuracy: the
    certified product (eta + t2)(eta + t1) <= 2^-56, and the computed w agrees with the exact
    solve to rounding; it is chosen only when cheaper than the fp64 plan."""
    from oracle import gibbs
    rng = np.random.default_rng(7)
    n, p = 150, 1200
    X = rng.standard_normal((n, p))
    lam_true = np.linalg.eigvalsh(X @ X.T)[-1]
    D = rng.exponential(size=p) * eps_scale / lam_true * 3
    sig2 = 1.0
    X32 = X.astype(np.float32).astype(np.float64)
    E = (X * D) @ X.T / sig2
    tr = np.trace(E)
    eps = 3.0 * np.linalg.eigvalsh(E)[-1]  # a certified bound (as the device's thresholded sums)
    K64 = gibbs.cheb_iterations(eps, 16)
    cost64 = (K64 - 1) * (1.0 + gibbs.COST_STEP) if K64 else np.inf
    K1, K2, eta, e2 = gibbs.nid_plan_mixed(eps, tr, 16, cost64)
    b = rng.standard_normal(n)
    w_exact = np.linalg.solve(np.eye(n) + E, b)
    if K2:
        t = gibbs.cheb_bounds(e2, 64)  # the recurrence form: the closed form's margin holds
        assert (eta + t[K2] * (1 + eta)) * (eta + t[K1] * (1 + eta)) <= gibbs.NID_TOL * (1 + 1e-9)
        step32 = gibbs.COST32 + gibbs.COST_STEP
        cost = (K1 + K2 - 2) * step32 + 1.0 + gibbs.COST_STEP
        assert cost < cost64
        w = gibbs.woodbury_solve_mixed(lambda v: (X @ (D * (X.T @ v))) / sig2,
                                       lambda v: (X32 @ (D * (X32.T @ v))) / sig2, b, e2, K1, K2)
    elif K64 == 0:
        return  # neither Chebyshev plan within the cap: the sweep takes the factor
    else:
        w = gibbs.woodbury_solve_cheb(lambda v: (X @ (D * (X.T @ v))) / sig2, b, eps, K64)
    err = np.linalg.norm(w - w_exact) / np.linalg.norm(w_exact)
    print(f"\n[eps ~ {eps:.2e}] K64 {K64}, mixed ({K1}, {K2}), eta {eta:.2e}, rel err {err:.2e}")
    assert err < 1e-14
    if 1e-8 <= eps_scale <= 1e-5:
        assert K2 > 0  # the plan is taken where the fp64 plan needs several products
    if eta * eta > gibbs.NID_TOL:
        assert K2 == 0  # beyond a single refinement's reach: the fp64 plan
