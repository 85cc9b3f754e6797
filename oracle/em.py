"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the reference bridge EM.

Restates ``BR::EM`` (Code/C/BridgeRegression.cpp:600-708) as the EM wrapper calls it
(Code/C/BridgeWrapper.cpp:57-73: sig = 1, tau = ratio) behind ``.C("bridge_EM")``
(BridgeWrapper.cpp:544-568).  Direct maximisation steps solve with a Cholesky
factorisation (the reference's ``symsolve``, LAPACK dposv through the un-vendored Matrix
library).  The conjugate-gradient option restates textbook CG with an absolute residual
tolerance and at most p iterations from the previous estimate; the reference's ``cg``
lives in that un-vendored library, so the CG variant is PARITY UNPINNED.

Used only by tests/ as the checker.
"""
from __future__ import annotations

import numpy as np
import scipy.linalg as sla


def _symsolve(A, b):
    """symsolve (Cholesky solve); raises LinAlgError when A is not positive definite."""
    c = sla.cho_factor(A, lower=False, check_finite=True)
    return sla.cho_solve(c, b)


def _cg(x, A, b, tol, max_it):
    """CG from x: returns (x, iterations); stops at |r| <= tol or after max_it steps."""
    x = x.copy()
    r = b - A @ x
    d = r.copy()
    rr = float(r @ r)
    it = 0
    while it < max_it and np.sqrt(rr) > tol:
        ad = A @ d
        a = rr / float(d @ ad)
        x += a * d
        r -= a * ad
        rn = float(r @ r)
        d = r + (rn / rr) * d
        rr = rn
        it += 1
    return x, it


def bridge_em(y, X, ratio, alpha, lambda_max, tol, max_iter, use_cg=False):
    """Returns (beta (P), solves) exactly as bridge_EM fills betap / max_iter:
    solves = total_iter, or the EM iteration count when every coefficient was dropped
    (BridgeRegression.cpp:639-643)."""
    X = np.asarray(X, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    P = X.shape[1]
    XX = X.T @ X                       # BridgeRegression.cpp:24 (the ctor's X'X)
    b = X.T @ y                        # :607
    sig, tau = 1.0, float(ratio)
    c1 = alpha * np.exp((2 - alpha) * (np.log(tau) - np.log(sig)))   # :620
    c2 = np.exp(-2 * (np.log(tau) - np.log(sig)))                      # :621
    ss = np.arange(P)
    total_iter = P
    new_beta = _symsolve(XX, b)        # :630-632, one maximisation step
    dist, it = tol + 1.0, 0
    while dist > tol and it < max_iter:
        with np.errstate(divide="ignore", over="ignore"):
            lam = c1 * np.exp((alpha - 2) * np.log(np.fabs(new_beta)))  # :639
        keep = lam < lambda_max
        if not keep.all():
            if not keep.any():
                return np.zeros(P), it                                  # :654-657
            ss = ss[keep]
            lam = lam[keep]
            new_beta = new_beta[keep]
        old_beta = new_beta.copy()
        A = XX[np.ix_(ss, ss)] + np.diag(c2 * lam)                      # :666-668
        bs = b[ss]
        if not use_cg:
            new_beta = _symsolve(A, bs)
            total_iter += ss.size
        else:
            new_beta, k = _cg(old_beta, A, bs, tol, ss.size)
            total_iter += k
        diff = new_beta - old_beta
        dist = np.sqrt(diff @ diff)                                     # :700-701
        it += 1
    beta = np.zeros(P)
    beta[ss] = new_beta
    return beta, total_iter
