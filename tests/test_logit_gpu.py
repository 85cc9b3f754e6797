"""GPU parity of the logistic bridge (Polya-Gamma Gibbs, BASELINE config C4) against the
oracle (oracle/gibbs.py logit_sweep / bridge_regression_logit, bb_oracle.c bbo_pg1) on the
same Philox counters, through the C ABI (bb_pg_batch, the engine, .C bridge_reg_logit).
No reference implementation exists: parity unpinned against a reference; the
oracle itself is pinned by tests/test_logit_cpu.py.

Tolerances: per-draw PG values relative 1e-12 with no decision flips (the same expression
trees on both sides; libm vs ocml last-ulp differences only); teacher-forced sweeps beta
relative L2 1e-10, tau / lambda / omega 1e-11; p <= n chains are stable, so whole chains
agree to the north star's 1e-8 posterior-mean tolerance.
"""
import numpy as np
import pytest

from oracle import gibbs
import oracle
from tests.test_gpu_parity import flips, rel_err

pytestmark = pytest.mark.gpu

SEED = 0xB4E5B41D6E


def logit_problem(n, p, seed, scale=1.0):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, p)) * scale
    b = np.zeros(p)
    k = max(3, p // 20)
    b[:k] = rng.uniform(0.5, 1.5, k) * rng.choice([-1.0, 1.0], k)
    y = (rng.random(n) < 1.0 / (1.0 + np.exp(-X @ b))).astype(np.float64)
    return np.asfortranarray(X), y, b


def test_pg_batch_matches_oracle(gpu_lib):
    bb = gpu_lib
    rng = np.random.default_rng(1)
    psi = np.concatenate([np.zeros(1000), rng.standard_normal(5000) * 3,
                          rng.uniform(-200, 200, 2000), [1e-300, -1e-12, 1.5625 * 2, 700.0]])
    g = bb.pg_batch(psi, SEED, 3, 17)
    o = oracle.pg_batch(psi, SEED, 3, 17)
    assert np.all(np.isfinite(g)) and np.all(g > 0)
    assert flips(g, o, 1e-9) == 0
    assert np.max(np.abs(g - o) / o) < 1e-12


@pytest.mark.parametrize("n,p,kw", [(500, 40, {}), (1500, 300, dict(alpha=0.3)),
                                    (300, 25, dict(true_tau=0.7)),
                                    (1500, 300, dict(gram_mode=0)),
                                    (3000, 2000, dict(sweeps=6))])
def test_logit_teacher_forced(gpu_lib, n, p, kw):
    """25 teacher-forced sweeps; X'Omega X on the Ozaki-II int8 Gram (the default) and on the
    fp64 MFMA Gram (gram_mode=0).  p = 2000 > 1024 runs the 16-lane speculative lambda
    kernel with the Polya-Gamma draws as its trailing workgroups."""
    bb = gpu_lib
    X, y, _ = logit_problem(n, p, n + p)
    alpha = kw.get("alpha", 0.5)
    true_tau = kw.get("true_tau", 0.0)
    seed, stream = SEED + 31, 2
    o = gibbs.bridge_regression_logit(y, X, kw.get("sweeps", 25), burn=0, alpha=alpha,
                                      true_tau=true_tau,
                                      seed=seed, stream=stream, record_state=True)
    e = bb.Engine(bb.EngineConfig(n=n, p=p, method=6, seed=seed, stream=stream,
                                  true_alpha=alpha, true_tau=true_tau,
                                  gram_mode=kw.get("gram_mode")), X, y)
    assert e.method() == 6
    assert e.gram_mode() == kw.get("gram_mode", bb.GRAM_OZAKI)
    e.init_state()
    st = o["states"]
    for k in range(1, len(st)):
        t, tau, lam, om, beta, _ = st[k]
        _, tau0, _, _, beta0, alpha0 = st[k - 1]
        e.set_state(beta0, tau0, 1.0, alpha0)
        e.run(t, 1, first_slot=-1)
        s = e.state()
        assert abs(s["tau"] - tau) <= 1e-12 * tau, (t, s["tau"], tau)
        assert s["sig2"] == 1.0
        assert flips(s["lambda"], lam) == 0, t
        assert np.max(np.abs(s["lambda"] - lam) / lam) < 1e-11, t
        og = e.omega()
        assert np.max(np.abs(og - om) / om) < 1e-11, t
        assert rel_err(s["beta"], beta) < 1e-10, (t, rel_err(s["beta"], beta))
    assert e.error_flags() == 0
    e.close()


def test_logit_c_entry_point_chain(gpu_lib):
    """.C("bridge_reg_logit") whole chain (burn-in, MCMC slots) against the oracle driver."""
    bb = gpu_lib
    X, y, _ = logit_problem(400, 12, 5)
    bb.set_seed(SEED + 7)
    g = bb.bridge_reg_logit(y, X, nsamp=300, burn=50)
    o = gibbs.bridge_regression_logit(y, X, 300, burn=50, seed=SEED + 7, stream=0)
    for k in ("tau", "alpha"):
        assert np.max(np.abs(g[k] - o[k]) / o[k]) < 1e-8, k
    assert np.max(np.abs(g["beta"].T - o["beta"]) / np.maximum(np.abs(o["beta"]), 1e-8)) < 1e-6
    assert rel_err(g["beta"].mean(axis=0), o["beta"].mean(axis=1)) < 1e-8


def test_logit_unknown_alpha_chain(gpu_lib):
    bb = gpu_lib
    X, y, _ = logit_problem(300, 8, 9)
    bb.set_seed(SEED + 8)
    g = bb.bridge_reg_logit(y, X, nsamp=150, burn=20, alpha=0.0)
    o = gibbs.bridge_regression_logit(y, X, 150, burn=20, alpha=0.0, seed=SEED + 8, stream=0)
    assert np.max(np.abs(g["alpha"] - o["alpha"])) < 1e-9
    assert rel_err(g["beta"].mean(axis=0), o["beta"].mean(axis=1)) < 1e-8


def test_logit_rejects_non_binary_y(gpu_lib):
    bb = gpu_lib
    X, y, _ = logit_problem(50, 3, 1)
    y[3] = 0.5
    with pytest.raises(ValueError):
        bb.bridge_reg_logit(y, X, nsamp=5, burn=1)


def test_teacher_forced_c4_workload(gpu_lib):
    """The C4 bench workload itself (n = 10000, p = 1000; bench.py's X, y and key), two
    sweeps teacher-forced from the oracle's state."""
    import bench
    bb = gpu_lib
    n, p = 10000, 1000
    X, y, btrue = bench.make_logit_problem(n, p)
    e = bb.Engine(bb.EngineConfig(n=n, p=p, method=6, seed=SEED, stream=0), X, y)
    e.init_state()
    rng = np.random.default_rng(3)
    beta, tau = btrue + 0.05 * rng.standard_normal(p), 0.5
    for t in (101, 102):
        e.set_state(beta, tau, 1.0, 0.5)
        e.run(t, 1, first_slot=-1)
        s = e.state()
        b, lam, tau, om = gibbs.logit_sweep(X, y, beta, tau, 0.5, t, SEED, 0)
        assert abs(s["tau"] - tau) / tau < 1e-12, t
        assert flips(s["lambda"], lam) == 0, t
        assert np.max(np.abs(e.omega() - om) / om) < 1e-11, t
        assert rel_err(s["beta"], b) < 1e-10, (t, rel_err(s["beta"], b))
        beta = b
    assert e.error_flags() == 0
    e.close()
