"""GPU parity of the triangle-mixture sampler (bridge.reg.tri, .C("bridge_regression"))
against the CPU oracle on the same Philox counters.

The engine computes the design basis X = U diag(d) V' at setup (host Householder QR of X,
then one-sided Jacobi on R -- X'X is never formed, so the small singular values keep fp64
accuracy relative to themselves up to cond(X)); the basis is checked on its own (orthonormal, reconstructs X'X, a = V'X'y) and then
handed to the oracle, so the chain comparison covers everything downstream of it.
Finding: free-running triangle chains are chaotic under fp64 roundoff.  A 3e-14 difference
in the least-squares start grows about 3x per sweep (measured with tools/tri_diag.py:
beta 1e-9 relative by sweep 9, first omega-shape flip at sweep 21), with no decision flip
needed -- the truncated-normal bounds move with beta.  So, as for the Woodbury path
(DESIGN.md s6), the bar is per sweep: every sweep teacher-forced from the oracle's state
must agree to 1e-10 (relative L2 for beta, u, omega; tau, sig2, alpha) with identical mixture shapes, and
the free-running chains must agree over their first four sweeps to 1e-9."""
import numpy as np
import pytest

import bayesbridge_amd as bb
from oracle import gibbs
from tests.conftest import synthetic_problem

pytestmark = pytest.mark.gpu


def engine_basis(X, y, **kw):
    n, p = X.shape
    cfg = bb.EngineConfig(n=n, p=p, method=4)
    for k, v in kw.items():
        setattr(cfg, k, v)
    e = bb.Engine(cfg, X, y)
    return e, e.tri_basis()


def rel(a, b):
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-12)))


def rel_l2(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


@pytest.mark.parametrize("n,p", [(100, 20), (442, 10), (300, 129)])
def test_engine_basis_is_the_svd_of_x(gpu_lib, n, p):
    X, y, _ = synthetic_problem(n, p, seed=n + p)
    e, (tV, a, d) = engine_basis(X, y)
    assert np.allclose(tV @ tV.T, np.eye(p), atol=1e-12)
    G = X.T @ X
    assert np.allclose(tV.T @ np.diag(d * d) @ tV, G, atol=1e-10 * np.abs(G).max())
    assert np.all(np.diff(d) <= 0)
    sv = np.linalg.svd(X, compute_uv=False)
    assert np.allclose(d, sv, rtol=1e-10)
    assert np.allclose(a, tV @ (X.T @ y), rtol=1e-10, atol=1e-10 * np.abs(a).max())


def test_engine_basis_ill_conditioned(gpu_lib):
    """Singular values spanning 7 decades (near-collinear columns): the engine's basis keeps
    the smallest ones to ~1e-9 relative, where an eigendecomposition of X'X loses ~1e-3."""
    rng = np.random.default_rng(8)
    n, p = 200, 30
    U, _ = np.linalg.qr(rng.standard_normal((n, p)))
    W, _ = np.linalg.qr(rng.standard_normal((p, p)))
    s = np.logspace(0, -7, p)
    X = np.asfortranarray(U @ np.diag(s) @ W.T)
    y = rng.standard_normal(n)
    _, (tV, a, d) = engine_basis(X, y)
    assert np.max(np.abs(d - s) / s) < 1e-8
    assert np.allclose(tV @ tV.T, np.eye(p), atol=1e-12)
    # right singular vectors: |V' W| is a permutation-free identity (distinct values)
    assert np.allclose(np.abs(tV @ W), np.eye(p), atol=1e-6)


# (n, p, betaburn).  Designs with alpha known and p <= 32 run the fused single-launch chain
# (bb_tri.hip k_tri_chain; "ortho" its orthogonal-design coordinate pass, round 3);
# "betaburn" (p = 33), "unknown_alpha" and ("ortho", 800, 600) the general per-sweep path.
# "x_in_hbm": n p 8 bytes above the fused kernel's LDS staging limit, so X is read from HBM.
SHAPES = {"c1": (100, 20, 0), "unknown_alpha": (100, 20, 0), "betaburn": (80, 33, 2),
          "betaburn_fused": (80, 24, 2), "x_in_hbm": (400, 32, 0),
          "known_tau_sig2": (100, 20, 0), "ortho": (100, 20, 0)}
CASES = list(SHAPES)


@pytest.mark.parametrize("case,n,p", [(c, None, None) for c in CASES] + [("ortho", 800, 600)])
def test_tri_sweeps_teacher_forced(gpu_lib, case, n, p):
    betaburn = SHAPES[case][2]
    if n is None:
        n, p = SHAPES[case][:2]
    X, y, _ = synthetic_problem(n, p, seed=5)
    alpha = 0.0 if case == "unknown_alpha" else 0.5
    tk = dict(true_sig2=1.5, true_tau=0.8) if case == "known_tau_sig2" else {}
    seed, M = 777, (40 if p < 100 else 12)
    tol = 1e-10
    ortho = case == "ortho"
    e, basis = engine_basis(X, y, seed=seed, stream=0, true_alpha=alpha, betaburn=betaburn,
                            trace_capacity=1, ortho=ortho, **tk)
    e.init_state()
    o = gibbs.bridge_regression_tri(y, X, M, basis, burn=0, betaburn=betaburn, seed=seed,
                                    stream=0, true_alpha=alpha, ortho=ortho, **tk)
    for i in range(1, M):
        a_prev = o["alpha"][i - 1] if alpha <= 0 else alpha
        e.set_state(o["beta"][i - 1], o["tau"][i - 1], o["sig2"][i - 1], a_prev)
        e.set_tri_state(o["u"][i - 1])
        e.run(i, 1, first_slot=0, slot_step=0, mcmc_phase=1)
        g, gt = e.trace(0, 1), e.tri_trace(0, 1)
        assert np.array_equal(gt["shape"][:, 0], o["shape"][i]), i
        err = rel_l2(g["beta"][:, 0], o["beta"][i])
        assert err < tol, (i, err)
        assert rel_l2(gt["u"][:, 0], o["u"][i]) < tol, i
        assert rel_l2(g["lambda"][:, 0], o["w"][i]) < tol, i
        for k in ("tau", "sig2", "alpha"):
            assert rel(g[k][0], o[k][i]) < 1e-10, (i, k)
    assert e.error_flags() == 0


# Wide p: all four waves of the 256-thread workgroup, strided ownership (e >= 1 for p > 256,
# e = 2 for p > 512), the cross-wave max/min exchange, p not a multiple of 64.
# Finding (tools/tri_wide_diag.py): one rtnorm_gibbs pass is a chain of p truncated-normal
# draws whose bounds (b_j -+ r_ji) / |v_ji| divide by the smallest entries of V (1e-7 .. 1e-8
# here), so an ulp of difference early in the chain is amplified along it -- the ORACLE
# against ITSELF with beta perturbed by 1e-15 relative diverges by 1e-7 .. 4e-2 after one
# sweep at these shapes, the same as the GPU against the oracle.  So the bar is: omega, u
# and the mixture shapes (parallel per-coefficient draws over every ownership slot) to
# 1e-12, the first coordinates of z (whose bounds reduce over all p constraints) to 1e-10,
# and beta within 20x the oracle's own sensitivity.
WIDE = [(700, 300, 0), (900, 517, 0), (900, 517, 2), (1200, 1000, 0)]


@pytest.mark.parametrize("n,p,betaburn", WIDE)
def test_tri_wide_p_sweep(gpu_lib, n, p, betaburn):
    import oracle
    X, y, _ = synthetic_problem(n, p, seed=5)
    e, (tV, a, d) = engine_basis(X, y, seed=777, stream=0, betaburn=betaburn, trace_capacity=1)
    e.init_state()
    o = gibbs.bridge_regression_tri(y, X, 2, (tV, a, d), burn=0, betaburn=betaburn, seed=777,
                                    stream=0)
    e.set_state(o["beta"][0], o["tau"][1], o["sig2"][1], 0.5)
    e.set_tri_state(o["u"][0])
    e.run(1, 1, first_slot=0, slot_step=0, mcmc_phase=1)
    g, gt = e.trace(0, 1), e.tri_trace(0, 1)
    assert e.error_flags() == 0
    assert np.array_equal(gt["shape"][:, 0], o["shape"][1])
    assert rel(gt["u"][:, 0], o["u"][1]) < 1e-12
    assert rel(g["lambda"][:, 0], o["w"][1]) < 1e-12
    bg, bo = g["beta"][:, 0], o["beta"][1]
    if betaburn == 0:
        zg, zo = tV @ bg, tV @ bo
        assert np.max(np.abs(zg[:8] - zo[:8]) / np.abs(zo[:8])) < 1e-10
    # the oracle's own sensitivity: the same sweep from beta perturbed by 1e-15 relative
    bp = o["beta"][0] * (1 + 1e-15 * np.random.default_rng(1).standard_normal(p))
    up = o["u"][0].copy()
    oracle.tri_update(bp, up, tV, a, d, o["tau"][1], o["sig2"][1], 0.5, betaburn, 777, 0, 1)
    sens = rel_l2(bp, bo)
    assert rel_l2(bg, bo) < 20 * sens + 1e-10, (rel_l2(bg, bo), sens)
    e.close()


@pytest.mark.parametrize("case", CASES)
def test_tri_chain_matches_oracle(gpu_lib, case):
    n, p, betaburn = SHAPES[case]
    X, y, _ = synthetic_problem(n, p, seed=5)
    kw = dict(alpha=0.5, nu_shape=2.0, nu_rate=2.0)
    if case == "unknown_alpha":
        kw["alpha"] = 0.0
    tk = dict(true_sig2=1.5, true_tau=0.8) if case == "known_tau_sig2" else {}
    _, basis = engine_basis(X, y)
    bb.set_seed(4321)
    ortho = case == "ortho"
    g = bb.bridge_reg_tri(y, X, nsamp=8, burn=0, betaburn=betaburn, extras=True, ortho=ortho,
                          sig2_true=tk.get("true_sig2", 0.0), tau_true=tk.get("true_tau", 0.0),
                          **kw)
    o = gibbs.bridge_regression_tri(y, X, 8, basis, burn=0, betaburn=betaburn, seed=4321,
                                    ortho=ortho,
                                    stream=0, true_alpha=kw["alpha"],
                                    true_sig2=tk.get("true_sig2", 0.0),
                                    true_tau=tk.get("true_tau", 0.0),
                                    nu_shape=2.0, nu_rate=2.0)
    # free-running: the first sweeps only (chaotic divergence, see the module docstring)
    assert np.array_equal(g["shape"], o["shape"])
    for s in range(4):
        l2 = np.linalg.norm(g["beta"][s] - o["beta"][s]) / np.linalg.norm(o["beta"][s])
        assert l2 < 1e-9, (s, l2)
    for k in ("sig2", "tau", "alpha"):
        assert rel(g[k][1:4], o[k][1:4]) < 1e-9, k


def test_tri_rejects_wide_p(gpu_lib, capfd):
    X, y, _ = synthetic_problem(20, 40, seed=2)
    g = bb.bridge_reg_tri(y, X, nsamp=3, burn=1, extras=True)
    assert np.all(g["beta"] == 0.0)
    assert "Aborting Gibbs sampler" in capfd.readouterr().out


def test_bridge_reg_triangle_dispatch(gpu_lib):
    X, y, _ = synthetic_problem(100, 8, seed=9)
    out = bb.bridge_reg(y, X, 50, method="triangle")
    assert out["beta"].shape == (50, 8) and np.all(np.isfinite(out["beta"]))
    assert np.all(out["tau"] > 0) and np.all(out["sig2"] > 0)
