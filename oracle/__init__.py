"""TEST INFRASTRUCTURE ONLY -- CPU oracle for the BayesBridge stable Gibbs sweep.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg import this package, and only as the checker.  The product
(``bayesbridge_amd`` / ``BayesBridge.so``) never imports, links or calls it.

PARITY UNPINNED against reference outputs (no reference fixtures exist and the
reference cannot be built or run here -- see ``bb_oracle.c`` header and
DESIGN.md); pinned instead by Philox KATs, numpy's Philox, analytic moments of
the tilted stable law and exact-posterior quadrature (tests/test_oracle_cpu.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libbboracle.so")
_lib = None

KIND_LAMBDA_INNER = 1
KIND_LAMBDA_OUTER = 2
KIND_TAU = 3
KIND_SIG2 = 4
KIND_BETA_Z = 5
KIND_DELTA = 6
KIND_ALPHA = 7
KIND_TRI_OMEGA = 8
KIND_TRI_U = 9
KIND_TRI_Z = 10
KIND_PG = 11
KIND_PG_IG = 12

_u64p = ctypes.POINTER(ctypes.c_uint64)
_dp = ctypes.POINTER(ctypes.c_double)
_lp = ctypes.POINTER(ctypes.c_long)


def build() -> str:
    src = os.path.join(_HERE, "bb_oracle.c")
    if (not os.path.exists(_LIB_PATH)) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        L.bbo_philox4x64.argtypes = [_u64p, _u64p, _u64p]
        L.bbo_uniforms.argtypes = [_u64p, ctypes.c_uint64, ctypes.c_uint, ctypes.c_uint64,
                                   ctypes.c_uint64, ctypes.c_uint64, _dp]
        L.bbo_normals.argtypes = [_dp, ctypes.c_long, _u64p, ctypes.c_uint64, ctypes.c_uint,
                                  ctypes.c_uint64]
        L.bbo_retstable.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_double, _u64p,
                                    ctypes.c_uint64, ctypes.c_uint64, _lp, _lp]
        L.bbo_retstable.restype = ctypes.c_double
        L.bbo_retstable_batch.argtypes = [_dp, _dp, _dp, _dp, ctypes.c_long, _u64p,
                                          ctypes.c_uint64]
        L.bbo_sample_lambda.argtypes = [_dp, _dp, ctypes.c_long, ctypes.c_double,
                                        ctypes.c_double, _u64p, ctypes.c_uint64,
                                        ctypes.c_uint64, _lp]
        L.bbo_gamma1.argtypes = [ctypes.c_double, _u64p, ctypes.c_uint64, ctypes.c_uint]
        L.bbo_gamma1.restype = ctypes.c_double
        L.bbo_tau_from_sum.argtypes = [ctypes.c_double, ctypes.c_long, ctypes.c_double,
                                       ctypes.c_double, ctypes.c_double, _u64p, ctypes.c_uint64]
        L.bbo_tau_from_sum.restype = ctypes.c_double
        L.bbo_sum_abs_pow.argtypes = [_dp, ctypes.c_long, ctypes.c_double]
        L.bbo_sum_abs_pow.restype = ctypes.c_double
        L.bbo_sig2_from_rss.argtypes = [ctypes.c_double, ctypes.c_long, ctypes.c_double,
                                        ctypes.c_double, _u64p, ctypes.c_uint64]
        L.bbo_sig2_from_rss.restype = ctypes.c_double
        L.bbo_alpha_mh.argtypes = [ctypes.c_double, _dp, ctypes.c_long, ctypes.c_double,
                                   ctypes.c_double, ctypes.c_double, ctypes.c_double, _dp,
                                   _u64p, ctypes.c_uint64]
        L.bbo_alpha_mh.restype = ctypes.c_double
        L.bbo_tnorm.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                ctypes.c_double, _u64p, ctypes.c_uint64, ctypes.c_uint64,
                                ctypes.c_uint64, ctypes.POINTER(ctypes.c_int)]
        L.bbo_tnorm.restype = ctypes.c_double
        L.bbo_tri_update.argtypes = [_dp, _dp, _dp, _dp, ctypes.c_long, _dp, _dp, _dp, _dp,
                                     _dp, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                     ctypes.c_int, _u64p, ctypes.c_uint64, _dp, _dp, _dp]
        L.bbo_tri_update.restype = ctypes.c_long
        L.bbo_trunc_batch.argtypes = [ctypes.c_int, ctypes.c_long, _dp, _dp, _dp, _dp, _dp,
                                      _u64p]
        L.bbo_trunc_batch.restype = ctypes.c_long
        L.bbo_rrtgamma_batch.argtypes = [ctypes.c_long, _dp, _dp, _dp, _dp, _u64p]
        L.bbo_rrtgamma_batch.restype = ctypes.c_long
        L.bbo_pg_batch.argtypes = [_dp, _dp, ctypes.c_long, _u64p, ctypes.c_uint64]
        L.bbo_pg_batch.restype = ctypes.c_long
        _lib = L
    return _lib


def _key(seed: int, stream: int):
    return (ctypes.c_uint64 * 2)(seed & 0xFFFFFFFFFFFFFFFF, stream & 0xFFFFFFFFFFFFFFFF)


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(_dp)


def philox4x64(ctr, key):
    c = (ctypes.c_uint64 * 4)(*[int(x) for x in ctr])
    k = (ctypes.c_uint64 * 2)(*[int(x) for x in key])
    o = (ctypes.c_uint64 * 4)()
    lib().bbo_philox4x64(c, k, o)
    return [int(x) for x in o]


def uniforms(seed, stream, t, kind, j, a=0, b=0):
    out = (ctypes.c_double * 4)()
    lib().bbo_uniforms(_key(seed, stream), t, kind, j, a, b, out)
    return np.array(out[:])


def normals(count, seed, stream, t, kind, j0=0):
    out = np.empty(count, dtype=np.float64)
    lib().bbo_normals(_ptr(out), count, _key(seed, stream), t, kind, j0)
    return out


def retstable(h, alpha, V0=1.0, seed=0, stream=0, t=0, j=0, counts=False):
    no, ni = ctypes.c_long(0), ctypes.c_long(0)
    x = lib().bbo_retstable(float(h), float(alpha), float(V0), _key(seed, stream), t, j,
                            ctypes.byref(no), ctypes.byref(ni))
    if counts:
        return x, no.value, ni.value
    return x


def retstable_batch(alpha, V0, h, seed=0, stream=0, t=0):
    """Mirror of ``.C("retstable_LD", x, alpha, V0, h, num)`` (BridgeWrapper.cpp:965-984)."""
    alpha = np.ascontiguousarray(alpha, dtype=np.float64)
    V0 = np.ascontiguousarray(V0, dtype=np.float64)
    h = np.ascontiguousarray(h, dtype=np.float64)
    x = np.zeros(h.shape[0], dtype=np.float64)
    lib().bbo_retstable_batch(_ptr(x), _ptr(alpha), _ptr(V0), _ptr(h), h.shape[0],
                              _key(seed, stream), t)
    return x


def sample_lambda(beta, alpha, tau, seed, stream, t, j0=0):
    beta = np.ascontiguousarray(beta, dtype=np.float64)
    lam = np.empty_like(beta)
    att = ctypes.c_long(0)
    lib().bbo_sample_lambda(_ptr(lam), _ptr(beta), beta.shape[0], alpha, tau,
                            _key(seed, stream), t, j0, ctypes.byref(att))
    return lam


def gamma1(shape, seed, stream, t, kind):
    return lib().bbo_gamma1(shape, _key(seed, stream), t, kind)


def sum_abs_pow(beta, alpha):
    beta = np.ascontiguousarray(beta, dtype=np.float64)
    return lib().bbo_sum_abs_pow(_ptr(beta), beta.shape[0], alpha)


def tau_from_sum(s, p, alpha, nu_shape, nu_rate, seed, stream, t):
    return lib().bbo_tau_from_sum(s, p, alpha, nu_shape, nu_rate, _key(seed, stream), t)


def sig2_from_rss(rss, n, sig2_shape, sig2_scale, seed, stream, t):
    return lib().bbo_sig2_from_rss(rss, n, sig2_shape, sig2_scale, _key(seed, stream), t)


def alpha_mh(a_old, beta, tau, pr_a, pr_b, seed, stream, t, ep=0.1):
    beta = np.ascontiguousarray(beta, dtype=np.float64)
    s = np.empty_like(beta)
    return lib().bbo_alpha_mh(a_old, _ptr(beta), beta.shape[0], tau, pr_a, pr_b, ep, _ptr(s),
                              _key(seed, stream), t)


def tnorm(lo, hi, mu, sd, seed, stream, t, i, it=0):
    """r.tnorm(lo, hi, mu, sd) restated (Robert 1995); see bb_oracle.c bbo_tnorm."""
    f = ctypes.c_int(0)
    x = lib().bbo_tnorm(lo, hi, mu, sd, _key(seed, stream), t, i, it, ctypes.byref(f))
    if f.value:
        raise ValueError(f"tnorm failed (code {f.value})")
    return x


def tri_update(beta, u, tV, a, d, tau, sig2, alpha, betaburn, seed, stream, t, G=None, c=None):
    """One sweep's omega, u, beta updates of the triangle sampler (bb_oracle.c
    bbo_tri_update).  beta and u are updated in place; returns (omega, shape).
    With G = X'X and c = X'y given, beta is drawn by the orthogonal-design variant."""
    p = beta.shape[0]
    ortho = G is not None
    G = np.ascontiguousarray(G if ortho else np.zeros((1, 1)), dtype=np.float64)
    c = np.ascontiguousarray(c if ortho else np.zeros(1), dtype=np.float64)
    tV = np.asfortranarray(tV, dtype=np.float64)
    a = np.ascontiguousarray(a, dtype=np.float64)
    d = np.ascontiguousarray(d, dtype=np.float64)
    omega, shape = np.empty(p), np.empty(p)
    z, bcur, b = np.empty(p), np.empty(p), np.empty(p)
    fails = lib().bbo_tri_update(_ptr(beta), _ptr(u), _ptr(omega), _ptr(shape), p, _ptr(tV),
                                 _ptr(a), _ptr(d), _ptr(G), _ptr(c), int(ortho), tau, sig2,
                                 alpha, betaburn,
                                 _key(seed, stream), t, _ptr(z), _ptr(bcur), _ptr(b))
    if fails:
        raise ValueError(f"tri_update: {fails} failed truncated-normal draws")
    return omega, shape


TRUNC_MODES = {"rtnorm_left": (0, 3), "rtnorm_both": (1, 4), "rtnorm": (2, 4),
               "rtexpon_rate_left": (3, 2), "rtexpon_rate_both": (4, 3), "rtexpon_rate": (5, 3)}


def rrtgamma_batch(shape, rate, right_t, seed, stream=0):
    """Oracle of .C("rrtgamma_rate"): Ga(shape, rate) truncated to (0, right_t]."""
    ps = [np.ascontiguousarray(q, dtype=np.float64) for q in (shape, rate, right_t)]
    x = np.zeros(ps[0].shape[0])
    fails = lib().bbo_rrtgamma_batch(x.shape[0], _ptr(x), *[_ptr(q) for q in ps],
                                     _key(seed, stream))
    if fails:
        raise ValueError(f"rrtgamma: {fails} failed draws")
    return x


def trunc_batch(name, params, seed, stream=0):
    """Oracle of the truncated-distribution .C utilities (bb_oracle.c bbo_trunc_batch);
    ``params`` are the .C arguments after x, as equal-length arrays."""
    mode, npar = TRUNC_MODES[name]
    assert len(params) == npar
    ps = [np.ascontiguousarray(q, dtype=np.float64) for q in params]
    num = ps[0].shape[0]
    ps += [np.zeros(1)] * (4 - npar)
    x = np.zeros(num)
    fails = lib().bbo_trunc_batch(mode, num, _ptr(x), *[_ptr(q) for q in ps],
                                  _key(seed, stream))
    if fails:
        raise ValueError(f"{name}: {fails} failed draws")
    return x


def pg_batch(psi, seed, stream, t):
    """omega_i ~ PG(1, psi_i) (Polson, Scott & Windle 2013; bb_oracle.c bbo_pg1), counters
    (t, kind 11/12, i, attempt, sub-attempt)."""
    psi = np.ascontiguousarray(psi, dtype=np.float64)
    om = np.empty_like(psi)
    fails = lib().bbo_pg_batch(_ptr(om), _ptr(psi), psi.shape[0], _key(seed, stream), t)
    if fails:
        raise ValueError(f"pg_batch: {fails} failed draws")
    return om


# ---------------------------------------------------------------------------
# Compiled reference-literal CPU chain (bb_cpu_chain.c + scipy's OpenBLAS): bench.py's
# cpu_baseline.  Test infrastructure only, like the rest of this package.
# ---------------------------------------------------------------------------
_CPU_LIB_PATH = os.path.join(_HERE, "build", "libbbcpu.so")
_cpu = None
CPU_METHODS = {"chol": 0, "woodbury": 1, "ortho": 2}


def cpu_lib():
    global _cpu
    if _cpu is None:
        srcs = [os.path.join(_HERE, f) for f in ("bb_cpu_chain.c", "bb_oracle.c", "Makefile")]
        if (not os.path.exists(_CPU_LIB_PATH)) or any(
                os.path.getmtime(_CPU_LIB_PATH) < os.path.getmtime(s) for s in srcs):
            subprocess.check_call(["make", "-s", "-C", _HERE])
        L = ctypes.CDLL(_CPU_LIB_PATH)
        d, i = ctypes.c_double, ctypes.c_int
        L.bbc_stable_chain.argtypes = [i, _dp, _dp, i, i, d, d, d, d, d, d, i, i,
                                       ctypes.c_uint64, ctypes.c_uint64, i, _dp, _dp, _dp]
        L.bbc_stable_chain.restype = d
        _cpu = L
    return _cpu


def cpu_chain(y, X, nsamp, burn=500, alpha=0.5, method="auto", sig2_shape=0.0, sig2_scale=0.0,
              nu_shape=2.0, nu_rate=2.0, true_sig2=0.0, seed=0, stream=0, threads=1,
              record=True):
    """The stable chain (alpha known) in compiled C: bridge_regression_stable's driver with
    the reference-literal p x p Cholesky ("chol"), the exact Woodbury form ("woodbury") or
    the orthogonal design ("ortho"); "auto" = chol if p <= n else woodbury.  Same counters
    as oracle/gibbs.py.  Returns dict(beta P x M, tau, sig2, runtime = post-burn seconds)."""
    X = np.asfortranarray(X, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    n, p = X.shape
    if method == "auto":
        method = "chol" if p <= n else "woodbury"
    M = int(nsamp)
    beta = np.zeros((p, M), order="F") if record else None
    tau, sig2 = np.zeros(M), np.zeros(M)
    rt = cpu_lib().bbc_stable_chain(CPU_METHODS[method], _ptr(X), _ptr(y), n, p, alpha,
                                    nu_shape, nu_rate, sig2_shape, sig2_scale, true_sig2,
                                    int(burn), M, seed, stream, int(threads),
                                    _ptr(beta) if record else None, _ptr(tau), _ptr(sig2))
    if rt < 0:
        raise RuntimeError(f"bbc_stable_chain failed ({rt})")
    return dict(beta=beta, tau=tau, sig2=sig2, runtime=rt, method=method)


def _cpu_lib_ext():
    L = cpu_lib()
    if not getattr(L, "_ext", False):
        d, i, u64 = ctypes.c_double, ctypes.c_int, ctypes.c_uint64
        L.bbc_logit_chain.argtypes = [_dp, _dp, i, i, d, d, d, i, i, u64, u64, i, _dp, _dp]
        L.bbc_logit_chain.restype = d
        ip = ctypes.POINTER(ctypes.c_int)
        L.bbc_sparse_chain.argtypes = [ip, ip, _dp, _dp, i, i, d, d, d, d, d, i, i, u64, u64, i,
                                       _dp, _dp, _dp]
        L.bbc_sparse_chain.restype = d
        L._ext = True
    return L


def cpu_logit_chain(y, X, nsamp, burn=500, alpha=0.5, nu_shape=2.0, nu_rate=2.0, seed=0,
                    stream=0, threads=1, record=True):
    """The logistic (Polya-Gamma) bridge chain in compiled C (bb_cpu_chain.c
    bbc_logit_chain): gibbs.bridge_regression_logit with alpha known, on the same counters.
    Returns dict(beta P x M, tau, runtime = post-burn seconds)."""
    X = np.asfortranarray(X, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    n, p = X.shape
    M = int(nsamp)
    beta = np.zeros((p, M), order="F") if record else None
    tau = np.zeros(M)
    rt = _cpu_lib_ext().bbc_logit_chain(_ptr(X), _ptr(y), n, p, alpha, nu_shape, nu_rate,
                                        int(burn), M, seed, stream, int(threads),
                                        _ptr(beta) if record else None, _ptr(tau))
    if rt < 0:
        raise RuntimeError(f"bbc_logit_chain failed ({rt})")
    return dict(beta=beta, tau=tau, runtime=rt)


def cpu_sparse_chain(y, X, nsamp, burn=500, alpha=0.5, nu_shape=2.0, nu_rate=2.0,
                     sig2_shape=0.0, sig2_scale=0.0, seed=0, stream=0, threads=1, record=True):
    """The stable chain on a sparse CSC design (p > n, Woodbury form) in compiled C
    (bb_cpu_chain.c bbc_sparse_chain: CSR/CSC passes, OpenMP sparse Gram, LAPACK dpotrf).
    Same driver and counters as gibbs.bridge_regression_stable(method="woodbury").
    Returns dict(beta P x M, tau, sig2, runtime = post-burn seconds)."""
    import scipy.sparse as sps

    Xc = sps.csc_matrix(X, dtype=np.float64)
    Xc.sort_indices()
    n, p = Xc.shape
    colptr = np.ascontiguousarray(Xc.indptr, dtype=np.int32)
    rowidx = np.ascontiguousarray(Xc.indices, dtype=np.int32)
    val = np.ascontiguousarray(Xc.data, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    M = int(nsamp)
    beta = np.zeros((p, M), order="F") if record else None
    tau, sig2 = np.zeros(M), np.zeros(M)
    ip = ctypes.POINTER(ctypes.c_int)
    rt = _cpu_lib_ext().bbc_sparse_chain(colptr.ctypes.data_as(ip), rowidx.ctypes.data_as(ip),
                                         _ptr(val), _ptr(y), n, p, alpha, nu_shape, nu_rate,
                                         sig2_shape, sig2_scale, int(burn), M, seed, stream,
                                         int(threads), _ptr(beta) if record else None,
                                         _ptr(tau), _ptr(sig2))
    if rt < 0:
        raise RuntimeError(f"bbc_sparse_chain failed ({rt})")
    return dict(beta=beta, tau=tau, sig2=sig2, runtime=rt)
