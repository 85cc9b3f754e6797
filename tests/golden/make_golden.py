"""Generate tests/golden/oracle_vectors.npz from the CPU oracle (test infrastructure).

The reference ships no fixtures for this path and cannot be run here, so
these vectors pin the oracle against silent drift: tests/test_golden.py regenerates them
and requires bit-identical results; the GPU tests compare the HIP path against them.
Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import oracle  # noqa: E402
from oracle import gibbs  # noqa: E402

SEED = 0xB4E5B41D6E


def vectors():
    out = {}
    # tilted-stable draws on the SURVEY 8(c) grid
    A = [0.05, 0.15, 0.25, 0.45]
    H = [0.0, 1e-4, 1e-2, 1.0, 1e2, 1e4, 1e6]
    a = np.repeat(A, len(H) * 8)
    h = np.tile(np.repeat(H, 8), len(A))
    v0 = np.ones_like(a)
    out["rs_alpha"], out["rs_h"], out["rs_V0"] = a, h, v0
    out["rs_x"] = oracle.retstable_batch(a, v0, h, seed=SEED, stream=0, t=0)
    # gamma / normal streams
    out["gamma_shape"] = np.array([0.5, 2.0, 50.0, 1000.5])
    out["gamma_x"] = np.array([oracle.gamma1(s, SEED, 0, 1, oracle.KIND_TAU)
                               for s in out["gamma_shape"]])
    out["normals"] = oracle.normals(64, SEED, 0, 3, oracle.KIND_BETA_Z)
    # a small chain (p <= n, reference-literal Cholesky map)
    rng = np.random.default_rng(20240501)
    X = rng.standard_normal((30, 5))
    X -= X.mean(axis=0)
    y = X @ np.array([2.0, 0.0, -1.5, 0.0, 0.5]) + rng.standard_normal(30)
    y -= y.mean()
    ch = gibbs.bridge_regression_stable(y, X, 20, burn=5, seed=SEED, stream=0, method="chol")
    out["chain_X"], out["chain_y"] = X, y
    for k in ("beta", "lambda", "sig2", "tau", "alpha"):
        out["chain_" + k] = ch[k]
    # one Woodbury step (p > n) from a fixed state
    Xw = rng.standard_normal((12, 40))
    yw = rng.standard_normal(12)
    lam = rng.uniform(0.1, 10.0, 40)
    z = oracle.normals(40, SEED, 0, 7, oracle.KIND_BETA_Z)
    d = oracle.normals(12, SEED, 0, 7, oracle.KIND_DELTA)
    out["wb_X"], out["wb_y"], out["wb_lambda"] = Xw, yw, lam
    out["wb_beta"] = gibbs.beta_step_woodbury(Xw, yw, lam, 0.8, 1.3, z, d)
    # truncated-distribution .C utilities (restated r.tnorm / texpon / rtgamma)
    lo = np.array([-np.inf, -1.0, 0.5, 2.0, 4.0, -7.0, -0.3, 1.0])
    hi = np.array([np.inf, 1.0, np.inf, 2.5, np.inf, -5.0, 0.2, 1.5])
    mu = np.array([0.0, 0.5, 1.0, 0.0, 0.0, 1.0, 0.0, 3.0])
    sg = np.array([1.0, 2.0, 2.0, 1.0, 1.0, 1.0, 0.1, 0.5])
    out["tn_lo"], out["tn_hi"], out["tn_mu"], out["tn_sig"] = lo, hi, mu, sg
    out["tn_rtnorm"] = oracle.trunc_batch("rtnorm", [lo, hi, mu, sg], SEED, 1)
    le, re_, rate = np.array([0.0, 1.0, -2.0, 3.0]), np.array([1.0, np.inf, 10.0, 3.5]), \
        np.array([2.0, 0.5, 5.0, 0.1])
    out["te_left"], out["te_right"], out["te_rate"] = le, re_, rate
    out["te_rtexpon"] = oracle.trunc_batch("rtexpon_rate", [le, re_, rate], SEED, 2)
    ga, gb, gt = np.array([0.5, 0.5, 3.0, 50.0, 1.5]), np.array([1.0, 1.0, 2.0, 1.0, 3.0]), \
        np.array([0.3, 5.0, 0.2, 40.0, 0.2])
    out["rg_shape"], out["rg_rate"], out["rg_right"] = ga, gb, gt
    out["rg_x"] = oracle.rrtgamma_batch(ga, gb, gt, SEED, 3)
    # one triangle-mixture update (omega, u, rtnorm_gibbs) from a fixed state
    Xt = rng.standard_normal((25, 4))
    yt = Xt @ np.array([1.0, 0.0, -1.0, 0.2]) + rng.standard_normal(25)
    G = Xt.T @ Xt
    ev, V = np.linalg.eigh(G)
    o = np.argsort(ev)[::-1]
    tV = np.asfortranarray(V[:, o].T)
    at, dt = tV @ (Xt.T @ yt), np.sqrt(ev[o])
    bt, ut = np.linalg.solve(G, Xt.T @ yt), np.full(4, 0.5)
    out["tri_tV"], out["tri_a"], out["tri_d"], out["tri_beta0"] = tV, at, dt, bt.copy()
    om, sh = oracle.tri_update(bt, ut, tV, at, dt, 1.1, 0.9, 0.5, 1, SEED, 0, 4)
    out["tri_beta"], out["tri_u"], out["tri_omega"], out["tri_shape"] = bt, ut, om, sh
    return out


if __name__ == "__main__":
    np.savez(os.path.join(HERE, "oracle_vectors.npz"), **vectors())
    print("wrote", os.path.join(HERE, "oracle_vectors.npz"))
