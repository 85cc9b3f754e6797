"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the reference stable Gibbs driver.

Restates ``bridge_regression_stable`` (Code/C/BridgeWrapper.cpp:207-313), its
orthogonal-design twin (:434-537) and the conditional samplers of
Code/C/BridgeRegression.cpp (:436-465 tau/sig2, :469-503 alpha, :506-510 lambda,
:514-521 beta ortho, :552-575 beta).  Scalar draws and the tilted-stable
sampler come from the C oracle (``oracle/bb_oracle.c``); dense linear algebra
from numpy/scipy LAPACK.

Used only as the checker (tests, smoke) and as bench.py's ``cpu_baseline``.
PARITY UNPINNED against reference outputs -- see oracle/__init__.py.

RNG counter layout (shared with the HIP path):
    key = (seed, stream); ctr = (t, kind << 56 | j, a, b)
    t = 0 is the pre-burn tau draw (BridgeWrapper.cpp:262), burn-in sweep i
    (0..burn) is t = 1 + i, MCMC sweep i (1..M-1) is t = burn + 1 + i.
"""
from __future__ import annotations

import time

import numpy as np
import scipy.linalg as sla
import scipy.sparse as sps

from . import (KIND_BETA_Z, KIND_DELTA, alpha_mh, normals, sample_lambda, sig2_from_rss,
               sum_abs_pow, tau_from_sum)


def least_squares(G, c, n):
    """BridgeRegression.cpp:79-91: symsolve(XX, Xy); singular X'X -> 0 with a warning.

    p > n is singular by construction and returns 0 without factorising.
    """
    p = G.shape[0]
    if p > n:
        return np.zeros(p), False
    try:
        L = np.linalg.cholesky(G)
    except np.linalg.LinAlgError:
        return np.zeros(p), False
    y = sla.solve_triangular(L, c, lower=True)
    return sla.solve_triangular(L.T, y, lower=False), True


def beta_step_chol(G, c, lam, sig2, tau, z):
    """BridgeRegression.cpp:552-575 (reference-literal p x p Cholesky)."""
    A = G.copy()
    A[np.diag_indices_from(A)] += lam * sig2 / (tau * tau)
    U = sla.cholesky(A, lower=False)  # A = U'U  (chol(U, VInv, 'U'))
    b = sla.solve_triangular(U, c, trans="T", lower=False)
    b = sla.solve_triangular(U, b, lower=False)
    x = sla.solve_triangular(U, z, lower=False)
    return b + np.sqrt(sig2) * x


def beta_step_woodbury(X, y, lam, sig2, tau, z, delta):
    """Exact draw of the same conditional for p > n (Bhattacharya et al. 2016).

    Delta = tau^2/lambda, u = sqrt(Delta) z, v = X u / sig + delta,
    M = I + X diag(Delta) X' / sig2, w = M^-1 (y/sig - v), beta = u + Delta X'w / sig.
    """
    sig = np.sqrt(sig2)
    D = (tau * tau) / lam
    u = np.sqrt(D) * z
    v = (X @ u) / sig + delta
    if sps.issparse(X):  # sparse design (BASELINE config C5): scipy SpGEMM
        Xc = sps.csc_matrix(X)
        M = np.asarray((Xc @ sps.diags(D) @ Xc.T).toarray()) / sig2
    else:
        M = (X * D) @ X.T / sig2
    M[np.diag_indices_from(M)] += 1.0
    Lm = np.linalg.cholesky(M)
    w = sla.solve_triangular(Lm, y / sig - v, lower=True)
    w = sla.solve_triangular(Lm.T, w, lower=False)
    return u + D * (X.T @ w) / sig


NID_TOL = 2.0 ** -56  # bb_kernels.h kNidTol


def cheb_iterations(eps, kmax, tol=NID_TOL):
    """Restates bb_kernels.h cheb_iterations: the smallest K <= kmax with
    sqrt(1 + eps) / T_K(sigma1) <= tol on the spectrum interval [1, 1 + eps], else 0."""
    if not (eps >= 0.0) or not (eps < 1e300):
        return 0
    if eps == 0.0:
        return 1 if kmax >= 1 else 0
    theta, delta = 1.0 + 0.5 * eps, 0.5 * eps
    sigma1 = theta / delta
    lim = np.sqrt(1.0 + eps) / tol
    tm1, tk = 1.0, sigma1
    for k in range(1, kmax + 1):
        if tk >= lim:
            return k
        tm1, tk = tk, 2.0 * sigma1 * tk - tm1
    return 0


def woodbury_solve_cheb(apply_E, rhs, eps, K):
    """Chebyshev iteration (Saad, Iterative Methods, Alg. 12.1; x_0 = 0) for (I + E) w = rhs
    with the spectrum of I + E in [1, 1 + eps] -- the device's near-identity solve
    (bb_nid.hip: k_cheb_init, then K - 1 steps of k_eapply + k_cheb_step)."""
    theta, delta = 1.0 + 0.5 * eps, 0.5 * eps
    sigma1 = theta / delta if delta > 0 else 0.0
    r = rhs.copy()
    d = r / theta
    x = d.copy()
    rho = 1.0 / sigma1 if sigma1 else 0.0
    for _ in range(1, K):
        q = d + apply_E(d)
        r = r - q
        rho1 = 1.0 / (2.0 * sigma1 - rho)
        d = rho1 * rho * d + (2.0 * rho1 / delta) * r
        x = x + d
        rho = rho1
    return x


def beta_step_woodbury_nid(X, y, lam, sig2, tau, z, delta, kmax=16, lam_x=0.0):
    """The same conditional draw as beta_step_woodbury, with w = M^-1 (y/sig - v) solved by
    the certified Chebyshev iteration when the bound eps >= lambda_max(X D X') / sig2 admits
    K <= kmax iterates, else by the Cholesky factor.  eps: the trace, or
    with lam_x >= lambda_max(X X') the least thresholded bound (nid_decide_from).  Returns
    (beta, K) (K = 0: the Cholesky path)."""
    sig = np.sqrt(sig2)
    D = (tau * tau) / lam
    u = np.sqrt(D) * z
    v = (X @ u) / sig + delta
    if sps.issparse(X):
        cn = np.asarray(X.multiply(X).sum(axis=0)).ravel()
    else:
        cn = (X * X).sum(axis=0)
    eps, K = nid_decide_from(nid_shard_partials(D, cn, tau, lam_x), tau, sig2, kmax)
    if K == 0:
        return beta_step_woodbury(X, y, lam, sig2, tau, z, delta), 0
    w = woodbury_solve_cheb(lambda t: (X @ (D * (X.T @ t))) / sig2, y / sig - v, eps, K)
    return u + D * (X.T @ w) / sig, K


U32 = 2.0 ** -24  # bb_kernels.h kU32
COST32, COST_STEP = 0.55, 0.05  # bb_nid.hip kCost32, kCostStep


def cheb_bounds(eps, kmax):
    """b[K] = sqrt(1 + eps) / T_K(sigma1), K = 1..kmax (b[0] unused): the relative error bound
    of K Chebyshev iterates on [1, 1 + eps]."""
    theta, delta = 1.0 + 0.5 * eps, 0.5 * eps
    sigma1 = theta / delta
    out = [np.inf]
    tm1, tk = 1.0, sigma1
    for _ in range(1, kmax + 1):
        out.append(np.sqrt(1.0 + eps) / tk)
        # T_K grows without bound: once it overflows every later bound is 0
        tm1, tk = tk, (2.0 * sigma1 * tk - tm1 if tk < 1e300 else np.inf)
    return out


def nid_plan_mixed(eps, tr, kcap, cost_fp64, c64=1.0, c32=COST32, cstep=COST_STEP,
                   tol=NID_TOL):
    """Restates bb_nid.hip nid_plan_mixed: eta >= |E - E~|_2 for E~ built from
    X rounded to fp32, and the cheapest (K1, K2) with
    (eta + t_K2 (1 + eta)) (eta + t_K1 (1 + eta)) <= tol on [1, 1 + eps + eta], t_K =
    sqrt(1 + e2) / cosh(K acosh sigma1) (1 + 1e-12); costs (K1 - 1 + K2 - 1)(c32 + cstep) +
    c64 + cstep against the fp64 plan's cost_fp64 and the cap (kcap - 1)(c64 + cstep); (0, 0)
    when neither is beaten.  Returns (K1, K2, eta, e2)."""
    eta = (2.0 * U32 * np.sqrt(tr * eps) + U32 * U32 * tr) * (1.0 + 1e-6)
    e2 = eps + eta
    if not e2 < 1e300 or kcap < 1:
        return 0, 0, eta, e2
    kmax = min(kcap, 64)
    sigma1 = (1.0 + 0.5 * e2) / (0.5 * e2)
    ac = np.arccosh(sigma1)
    with np.errstate(over="ignore"):
        t = [np.inf] + [np.sqrt(1.0 + e2) / np.cosh(k * ac) * (1.0 + 1e-12)
                        for k in range(1, kmax + 1)]
    step32, step64 = c32 + cstep, c64 + cstep
    cap = min(cost_fp64, (kcap - 1) * step64)
    best, K1, K2 = np.inf, 0, 0
    for k1 in range(1, kmax + 1):
        err1 = eta + t[k1] * (1.0 + eta)
        if not err1 < 1.0:
            continue
        need = tol / err1
        k2 = next((k for k in range(1, kmax + 1) if eta + t[k] * (1.0 + eta) <= need), 0)
        if not k2:
            continue
        cost = (k1 - 1) * step32 + step64 + (k2 - 1) * step32
        if cost < cap * (1.0 - 1e-9) and cost < best:
            best, K1, K2 = cost, k1, k2
    return K1, K2, eta, e2


def woodbury_solve_mixed(apply_E, apply_E32, rhs, e2, K1, K2):
    """The mixed plan's solve (bb_engine nidx_mixed_tail): K1 Chebyshev iterates on M~ (apply_E32
    = the product over X rounded to fp32), the fp64 residual r = rhs - M x0, then K2 iterates on
    M~ from r added to x0; the interval [1, 1 + e2] for both."""
    x0 = woodbury_solve_cheb(apply_E32, rhs, e2, K1)
    r = rhs - (x0 + apply_E(x0))
    return x0 + woodbury_solve_cheb(apply_E32, r, e2, K2)


NID_TS = 32  # bb_kernels.h kNidTS


def nid_shard_partials(D, cn, tau, lam_shard):
    """Restates bb_nid.hip k_nid_partials: a column shard's bound sums
    [S_0 .. S_31, trace, Lambda_shard], S_k = sum_{D_j > T_k} D_j |x_j|^2 with the thresholds
    T_k = tau^2 2^(40 - 2k) every rank knows; Lambda_shard >= lambda_max(X_r X_r') (+inf when
    the shard has no certificate).  Summed over ranks by the exchange."""
    t2 = tau * tau
    v = D * cn
    out = np.empty(NID_TS + 2)
    for k in range(NID_TS):
        out[k] = v[D > np.ldexp(t2, 40 - 2 * k)].sum()
    out[NID_TS] = v.sum()
    out[NID_TS + 1] = lam_shard if lam_shard > 0 else np.inf
    return out


def nid_decide_from(red, tau, sig2, kmax=16):
    """Restates k_nid_decide_from: eps = min(trace, min_k S_k + T_k sum_r Lambda_r) / sig2
    (times 1 + 1e-6), valid because sum_r lambda_max(X_r X_r') >= lambda_max(X X') (Weyl) and
    E <= [sum_{D_j > T} D_j x_j x_j' + T X X'] / sig2; returns (eps, K)."""
    t2 = tau * tau
    lam = red[NID_TS + 1]
    best = red[NID_TS]
    if 0 < lam < np.inf:
        for k in range(NID_TS):
            best = min(best, red[k] + np.ldexp(t2, 40 - 2 * k) * lam)
    eps = best / sig2 * (1.0 + 1e-6)
    return eps, cheb_iterations(eps, kmax)


def beta_step_ortho(Gdiag, c, lam, sig2, tau, z):
    """BridgeRegression.cpp:514-521."""
    u = Gdiag + lam * sig2 / (tau * tau)
    s = np.sqrt(sig2 / u)
    m = c / u
    return m + s * z


def bridge_regression_stable(y, X, nsamp, burn=500, alpha=0.5, sig2_shape=0.0, sig2_scale=0.0,
                             nu_shape=2.0, nu_rate=2.0, alpha_a=1.0, alpha_b=1.0,
                             true_sig2=0.0, true_tau=0.0, true_alpha=None, ortho=False,
                             seed=0, stream=0, method="auto", record_state=False):
    """Restatement of bridge_reg_stable / bridge_regression_stable[_ortho].

    ``alpha`` plays the role of bridge.reg.stb's ``alpha`` (= true_alpha).  Returns a
    dict with traces beta (P x M), lambda (P x M), sig2, tau, alpha (M), runtime.
    ``method``: "chol" (reference-literal), "woodbury" (p > n draw), "auto" (chol if
    p <= n else woodbury -- the HIP path's choice).
    """
    y = np.ascontiguousarray(y, dtype=np.float64)
    if sps.issparse(X):
        X = sps.csc_matrix(X, dtype=np.float64)
        if method == "auto" and X.shape[1] <= X.shape[0]:
            X = X.toarray()
    if not sps.issparse(X):
        X = np.asfortranarray(X, dtype=np.float64)
    n, p = X.shape
    M = int(nsamp)
    if true_alpha is None:
        true_alpha = alpha
    know_sig2 = true_sig2 > 0
    know_tau = true_tau > 0
    know_alpha = true_alpha > 0
    if method == "auto":
        method = "chol" if p <= n else "woodbury"
    if ortho:
        method = "ortho"

    need_G = method in ("chol", "ortho") or p <= n
    G = X.T @ X if need_G else None
    c = X.T @ y
    if G is not None:
        b0, _ = least_squares(G, c, n)
    else:
        b0 = np.zeros(p)

    beta = np.zeros((p, M))
    lam = np.ones((p, M))
    sig2 = np.zeros(M)
    tau = np.zeros(M)
    alph = np.zeros(M)
    beta[:, 0] = b0
    alph[0] = 0.5
    if know_sig2:
        sig2[:] = true_sig2
    if know_tau:
        tau[:] = true_tau
    if know_alpha:
        alph[:] = true_alpha

    def draw_tau(b, a, t):
        return tau_from_sum(sum_abs_pow(b, a), p, a, nu_shape, nu_rate, seed, stream, t)

    def draw_sig2(b, t):
        r = y - X @ b
        return sig2_from_rss(float(r @ r), n, sig2_shape, sig2_scale, seed, stream, t)

    def draw_beta(lmb, s2, tu, t):
        z = normals(p, seed, stream, t, KIND_BETA_Z)
        if method == "chol":
            return beta_step_chol(G, c, lmb, s2, tu, z)
        if method == "ortho":
            return beta_step_ortho(np.diag(G).copy(), c, lmb, s2, tu, z)
        d = normals(n, seed, stream, t, KIND_DELTA)
        return beta_step_woodbury(X, y, lmb, s2, tu, z, d)

    states = []
    if not know_tau and not ortho:  # BridgeWrapper.cpp:262 (the non-ortho driver only)
        tau[0] = draw_tau(beta[:, 0], alph[0], 0)
    # Burn-in (:266-276 / ortho :493-503), all in slot 0.
    for i in range(burn + 1):
        t = 1 + i
        if not know_tau:
            tau[0] = draw_tau(beta[:, 0], alph[0], t)
        if not know_sig2:
            sig2[0] = draw_sig2(beta[:, 0], t)
        lam[:, 0] = sample_lambda(beta[:, 0], alph[0], tau[0], seed, stream, t)
        beta[:, 0] = draw_beta(lam[:, 0], sig2[0], tau[0], t)
        if not know_alpha:
            alph[0] = alpha_mh(alph[0], beta[:, 0], tau[0], alpha_a, alpha_b, seed, stream, t)
        if record_state:
            states.append((t, tau[0], sig2[0], lam[:, 0].copy(), beta[:, 0].copy(), alph[0]))
    t0 = time.perf_counter()
    # MCMC (:287-298 / ortho :513-523).  Quirk kept: non-ortho passes (alpha_b, alpha_b).
    pa = alpha_a if ortho else alpha_b
    for i in range(1, M):
        t = burn + 1 + i
        if not know_tau:
            tau[i] = draw_tau(beta[:, i - 1], alph[i - 1], t)
        if not know_sig2:
            sig2[i] = draw_sig2(beta[:, i - 1], t)
        lam[:, i] = sample_lambda(beta[:, i - 1], alph[i - 1], tau[i], seed, stream, t)
        beta[:, i] = draw_beta(lam[:, i], sig2[i], tau[i], t)
        if not know_alpha:
            alph[i] = alpha_mh(alph[i - 1], beta[:, i], tau[i], pa, alpha_b, seed, stream, t)
        if record_state:
            states.append((t, tau[i], sig2[i], lam[:, i].copy(), beta[:, i].copy(), alph[i]))
    runtime = time.perf_counter() - t0
    out = dict(beta=beta, **{"lambda": lam}, sig2=sig2, tau=tau, alpha=alph, runtime=runtime,
               method=method)
    if record_state:
        out["states"] = states
    return out


def woodbury_sweep_sharded(Xk, y, beta_k, j0, p, alpha, tau, sig2, t, seed, stream,
                           allreduce, hyper, know_tau=False, know_sig2=False, nid_lam=None,
                           kmax=16, info=None):
    """One Gibbs sweep (tau, sig2, lambda, beta) on a column shard of X.

    The multi-GPU decomposition of SURVEY.md 8(e) restated on the CPU:
    ``allreduce`` sums a float64 vector over ranks.  Shard k holds columns
    [j0, j0 + p_k); variates are indexed by the GLOBAL column j so the result is
    independent of the shard count (up to Gram summation order).
    Returns (beta_k_new, lambda_k, tau, sig2).
    """
    n = Xk.shape[0]
    # 1. partial sum |b|^a and X_k b_k  -> one all-reduce
    buf = np.concatenate([[sum_abs_pow(beta_k, alpha)], Xk @ beta_k])
    buf = allreduce(buf)
    S, Xb = buf[0], buf[1:]
    if not know_tau:
        tau = tau_from_sum(S, p, alpha, hyper["nu_shape"], hyper["nu_rate"], seed, stream, t)
    if not know_sig2:
        r = y - Xb
        sig2 = sig2_from_rss(float(r @ r), n, hyper["sig2_shape"], hyper["sig2_scale"], seed,
                             stream, t)
    # 2. local latent draws and the partial Gram / X u  -> one all-reduce
    lam = sample_lambda(beta_k, alpha, tau, seed, stream, t, j0=j0)
    z = normals(beta_k.shape[0], seed, stream, t, KIND_BETA_Z, j0=j0)
    D = (tau * tau) / lam
    u = np.sqrt(D) * z
    sig = np.sqrt(sig2)
    delta = normals(n, seed, stream, t, KIND_DELTA)
    if nid_lam is not None:
        # the near-identity decision from the exchanged bound sums (bb_engine.cpp
        # shard_solve), then either the Chebyshev solve with one exchange of X_k u_k and one
        # per product, or the Gram exchange below
        cn = (Xk * Xk).sum(axis=0)
        eps, K = nid_decide_from(allreduce(nid_shard_partials(D, cn, tau, nid_lam)), tau, sig2,
                                 kmax)
        if info is not None:
            info.append((eps, K))
        if K > 0:
            Xu = allreduce(Xk @ u)
            rhs = y / sig - (Xu / sig + delta)
            w = woodbury_solve_cheb(lambda d: allreduce(Xk @ (D * (Xk.T @ d))) / sig2, rhs, eps,
                                    K)
            return u + D * (Xk.T @ w) / sig, lam, tau, sig2
    Gk = (Xk * D) @ Xk.T
    buf = allreduce(np.concatenate([Gk.ravel(), Xk @ u]))
    G = buf[: n * n].reshape(n, n)
    Xu = buf[n * n:]
    # 3. replicated n x n solve, then the local beta update
    v = Xu / sig + delta
    Mm = G / sig2
    Mm[np.diag_indices_from(Mm)] += 1.0
    Lm = np.linalg.cholesky(Mm)
    w = sla.solve_triangular(Lm, y / sig - v, lower=True)
    w = sla.solve_triangular(Lm.T, w, lower=False)
    return u + D * (Xk.T @ w) / sig, lam, tau, sig2


def alpha_mh_sharded(a_old, beta_k, p, tau, pr_a, pr_b, seed, stream, t, allreduce, ep=0.1):
    """The alpha MH step (BridgeRegression.cpp:469-503) on a column shard: every shard draws
    the same proposal from the shared counter, sums exp(a log|beta_j / tau|) over its own
    columns for a_new and a_old, the two sums are all-reduced, and the decision uses the
    GLOBAL p -- the engine's k_alpha_sums / exchange / k_alpha_decide."""
    from . import KIND_ALPHA, uniforms

    u = uniforms(seed, stream, t, KIND_ALPHA, 0)
    l_new, r_new = max(0.0, a_old - ep), min(1.0, a_old + ep)
    d_new = r_new - l_new
    a_new = l_new + d_new * u[0]
    sl = np.log(np.abs(beta_k / tau))
    S = allreduce(np.array([np.exp(a_new * sl).sum(), np.exp(a_old * sl).sum()]))
    lg = __import__("math").lgamma

    def llh(a, Sa):
        return p * np.log(a) - p * lg(1.0 / a) - Sa

    def ldb(x):
        return (pr_a - 1.0) * np.log(x) + (pr_b - 1.0) * np.log(1.0 - x) - (
            lg(pr_a) + lg(pr_b) - lg(pr_a + pr_b))

    d_old = min(1.0, a_new + ep) - max(0.0, a_new - ep)
    log_accept = (llh(a_new, S[0]) - llh(a_old, S[1]) + ldb(a_new) - ldb(a_old) +
                  np.log(d_old) - np.log(d_new))
    return a_old if u[1] > np.exp(log_accept) else a_new


def bridge_regression_tri(y, X, nsamp, basis, burn=500, alpha=0.5, sig2_shape=0.0,
                          sig2_scale=0.0, nu_shape=2.0, nu_rate=2.0, alpha_a=1.0, alpha_b=1.0,
                          true_sig2=0.0, true_tau=0.0, true_alpha=None, betaburn=0, seed=0,
                          stream=0, ortho=False):
    """Restatement of bridge_regression (triangle mixture), BridgeWrapper.cpp:80-204.

    ``basis`` = (tV, a, d) with X = U diag(d) V', tV = V', a = V'X'y
    (BridgeRegression.cpp:47-57).  Sweep order per :136-168: tau, sig2, omega, u,
    beta (rtnorm_gibbs x (betaburn + 1)), alpha.  Burn-in runs ``burn`` sweeps in slot 0
    (:141); the MCMC loop fills slots 1..M-1.  Sweep counters: t = 0 extra tau draw,
    1..burn burn-in, burn + i MCMC slot i.  ``ortho``: bridge_regression_ortho
    (:320-432): beta by sample_beta_ortho, and sig2 is also drawn before burn-in (:374).
    The ortho driver draws sig2 after omega and u, which does not change any variate here
    (sig2 depends on beta only and every draw has its own counter).
    """
    from . import tri_update

    y = np.ascontiguousarray(y, dtype=np.float64)
    X = np.asfortranarray(X, dtype=np.float64)
    n, p = X.shape
    M = int(nsamp)
    tV, av, dv = basis
    if true_alpha is None:
        true_alpha = alpha
    know_sig2, know_tau, know_alpha = true_sig2 > 0, true_tau > 0, true_alpha > 0
    G = X.T @ X
    c = X.T @ y
    b0, _ = least_squares(G, c, n)
    tr = {k: np.zeros((p, M)) for k in ("beta", "u", "w", "shape")}
    tr["w"][:] = 1.0  # BridgeWrapper.cpp:604
    sig2, tau, alph = np.zeros(M), np.zeros(M), np.zeros(M)
    beta = b0.copy()
    u = np.full(p, 0.5)  # :123
    tr["beta"][:, 0] = beta
    tr["u"][:, 0] = u
    alph[0] = 0.5
    if know_sig2:
        sig2[:] = true_sig2
    if know_tau:
        tau[:] = true_tau
    if know_alpha:
        alph[:] = true_alpha

    def draw_tau(b, a, t):
        return tau_from_sum(sum_abs_pow(b, a), p, a, nu_shape, nu_rate, seed, stream, t)

    def draw_sig2(b, t):
        r = y - X @ b
        return sig2_from_rss(float(r @ r), n, sig2_shape, sig2_scale, seed, stream, t)

    def sweep(slot, prev, t):
        nonlocal beta
        if not know_tau:
            tau[slot] = draw_tau(beta, alph[prev], t)
        if not know_sig2:
            sig2[slot] = draw_sig2(beta, t)
        om, sh = tri_update(beta, u, tV, av, dv, tau[slot], sig2[slot], alph[prev], betaburn,
                            seed, stream, t, *((G, c) if ortho else ()))
        tr["w"][:, slot], tr["shape"][:, slot] = om, sh
        tr["u"][:, slot], tr["beta"][:, slot] = u, beta
        if not know_alpha:
            alph[slot] = alpha_mh(alph[prev], beta, tau[slot], alpha_a, alpha_b, seed, stream, t)

    if ortho and not know_sig2:
        sig2[0] = draw_sig2(beta, 0)  # :374
    if not know_tau:
        tau[0] = draw_tau(beta, alph[0], 0)  # :139, ortho :375
    for i in range(burn):
        sweep(0, 0, 1 + i)
    t0 = time.perf_counter()
    for i in range(1, M):
        sweep(i, i - 1, burn + i)
    out = {k: v.T.copy() for k, v in tr.items()}
    out.update(sig2=sig2, tau=tau, alpha=alph, runtime=time.perf_counter() - t0)
    return out


def logit_sweep(X, y, beta, tau, alpha, t, seed, stream, nu_shape=2.0, nu_rate=2.0,
                know_tau=False):
    """One logistic-bridge sweep (BASELINE config C4; no reference counterpart) in the
    order tau | beta, lambda | beta, tau, omega | beta, beta | omega, lambda, tau.

    tau and lambda are the reference's conditionals (BridgeRegression.cpp:453-465, 506-510);
    omega_i ~ PG(1, x_i'beta) (Polson, Scott & Windle 2013; bb_oracle.c bbo_pg1); beta is
    the reference's sample_beta_stable map (:552-575) with sig2 = 1, X'X -> X'Omega X and
    X'y -> X'(y - 1/2).  Returns (beta, lambda, tau, omega)."""
    from . import pg_batch

    n, p = X.shape
    if not know_tau:
        tau = tau_from_sum(sum_abs_pow(beta, alpha), p, alpha, nu_shape, nu_rate, seed, stream, t)
    lam = sample_lambda(beta, alpha, tau, seed, stream, t)
    omega = pg_batch(X @ beta, seed, stream, t)
    G = (X.T * omega) @ X
    c = X.T @ (y - 0.5)
    z = normals(p, seed, stream, t, KIND_BETA_Z)
    return beta_step_chol(G, c, lam, 1.0, tau, z), lam, tau, omega


def bridge_regression_logit(y, X, nsamp, burn=500, alpha=0.5, nu_shape=2.0, nu_rate=2.0,
                            alpha_a=1.0, alpha_b=1.0, true_tau=0.0, seed=0, stream=0,
                            record_state=False):
    """Restatement of .C("bridge_reg_logit"): the stable driver's slots and counters
    (pre-burn tau draw at t = 0, B + 1 burn-in sweeps in slot 0 at t = 1 + i, MCMC slot i at
    t = B + 1 + i; BridgeWrapper.cpp:262-298), beta starting at 0, alpha MH (if alpha <= 0)
    with the (alpha_a, alpha_b) prior.  Returns traces beta, lambda (P x M), tau, alpha (M)."""
    y = np.ascontiguousarray(y, dtype=np.float64)
    X = np.asfortranarray(X, dtype=np.float64)
    n, p = X.shape
    M = int(nsamp)
    know_tau, know_alpha = true_tau > 0, alpha > 0
    beta = np.zeros((p, M))
    lam = np.ones((p, M))
    tau = np.full(M, true_tau if know_tau else 0.0)
    alph = np.full(M, alpha if know_alpha else 0.5)
    states = []
    if not know_tau:
        tau[0] = tau_from_sum(sum_abs_pow(beta[:, 0], alph[0]), p, alph[0], nu_shape, nu_rate,
                              seed, stream, 0)

    def step(slot, prev, t):
        b, lam[:, slot], tau[slot], om = logit_sweep(X, y, beta[:, prev], tau[prev], alph[prev],
                                                     t, seed, stream, nu_shape, nu_rate, know_tau)
        beta[:, slot] = b
        if not know_alpha:
            alph[slot] = alpha_mh(alph[prev], b, tau[slot], alpha_a, alpha_b, seed, stream, t)
        else:
            alph[slot] = alph[prev]
        if record_state:
            states.append((t, tau[slot], lam[:, slot].copy(), om, b.copy(), alph[slot]))

    for i in range(burn + 1):
        step(0, 0, 1 + i)
    for i in range(1, M):
        step(i, i - 1, burn + 1 + i)
    out = dict(beta=beta, **{"lambda": lam}, tau=tau, alpha=alph)
    if record_state:
        out["states"] = states
    return out
