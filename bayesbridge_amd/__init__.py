"""bayesbridge_amd -- MI355X-native Bayesian bridge regression (normal-mixture Gibbs sweep).

Python mirror of the reference package's R front end for the stable path
(Code/C/BridgeWrapper.R): ``bridge_reg_stb`` (bridge.reg.stb, :194-234),
``bridge_reg`` (bridge.reg, :240-276, method="stable") and ``retstable_ld``
(retstable.ld, :511-537).  Each call goes through the same C ABI that R's ``.C``
would bind (``include/bayesbridge.h``), with R's marshalling emulated here:
column-major doubles, integer scalars, caller-allocated outputs, P x M traces
transposed to M x P on return.

All compute runs in the gfx950 HIP kernels of ``BayesBridge.so``; there is no
CPU fallback -- the functions raise if the library or a GPU is unavailable.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _build

__all__ = ["bridge_reg_stb", "bridge_reg", "retstable_ld", "set_seed", "get_rng_state",
           "set_rng_state", "Engine", "EngineConfig", "library", "device_count",
           "sample_lambda", "retstable_batch", "gram", "chol_solve"]

_lib: Optional[ctypes.CDLL] = None
_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int)


class bb_config(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("p", ctypes.c_int), ("p_local", ctypes.c_int),
                ("j0", ctypes.c_int), ("rank", ctypes.c_int), ("world", ctypes.c_int),
                ("sig2_shape", ctypes.c_double), ("sig2_scale", ctypes.c_double),
                ("nu_shape", ctypes.c_double), ("nu_rate", ctypes.c_double),
                ("alpha_a", ctypes.c_double), ("alpha_b", ctypes.c_double),
                ("true_sig2", ctypes.c_double), ("true_tau", ctypes.c_double),
                ("true_alpha", ctypes.c_double), ("ortho", ctypes.c_int),
                ("method", ctypes.c_int), ("trace_capacity", ctypes.c_int),
                ("seed", ctypes.c_uint64), ("stream", ctypes.c_uint64), ("device", ctypes.c_int),
                ("gram_mode", ctypes.c_int), ("betaburn", ctypes.c_int)]

GRAM_FP64, GRAM_OZAKI = 0, 1


EXPORTED_SYMBOLS = [
    "bridge_reg_stable", "retstable_LD", "bb_version", "bb_last_error", "bb_device_count",
    "bb_set_seed", "bb_get_rng_state", "bb_set_rng_state", "bb_use_r_rng", "bb_set_device",
    "bb_set_verbose", "bb_config_default", "bb_engine_create", "bb_engine_destroy",
    "bb_comm_id_size", "bb_comm_unique_id", "bb_engine_comm_init", "bb_engine_init_state",
    "bb_engine_run", "bb_engine_sync", "bb_engine_get_trace", "bb_engine_get_state",
    "bb_engine_set_state", "bb_engine_method", "bb_engine_enable_timing",
    "bb_engine_kernel_times", "bb_engine_reset_timing", "bb_engine_error_flags",
    "bb_retstable_batch", "bb_sample_lambda", "bb_gram", "bb_chol_solve",
    "bb_engine_phase_times", "bb_phase_count", "bb_phase_name", "bb_bench_lambda",
    "bb_group_create", "bb_group_destroy", "bb_group_init_state", "bb_group_run",
    "bb_bench_chol", "bb_gram_ozaki", "bb_engine_gram_mode", "bb_bench_ozaki",
    "bridge_EM", "bb_bridge_em", "bb_bridge_em_batch", "bridge_regression",
    "bb_engine_get_tri_trace", "bb_engine_get_tri_basis", "bb_engine_set_tri_state",
    "rtnorm_left", "rtnorm_both", "rtnorm", "rtexpon_rate_left", "rtexpon_rate_both",
    "rtexpon_rate", "mytest", "bb_trunc_batch", "rrtgamma_rate", "bb_rrtgamma_batch",
    "bridge_reg_stable_csc", "bb_engine_create_csc", "bb_engine_sparse_pairs", "bb_sparse_gram",
    "bb_bench_sparse_gram", "bb_engine_sparse_info", "bridge_reg_logit", "bb_engine_get_omega",
    "bb_pg_batch", "bb_group_create_rccl", "bb_group_sync", "bb_set_device_count",
    "bb_set_trace_budget", "bb_debug_interrupt_after", "bb_last_call_info",
    "bb_engine_set_timed_phase", "bb_engine_set_timing_stride", "bb_set_chol_version",
    "bb_set_tuning",
]


def library(build: bool = True) -> ctypes.CDLL:
    """Load BayesBridge.so (building it in-tree first if stale and hipcc is present)."""
    global _lib
    if _lib is not None:
        return _lib
    path = _build.SO_PATH
    if build:
        try:
            path = _build.build()
        except Exception:
            if not os.path.exists(_build.SO_PATH):
                raise
    if not os.path.exists(path):
        raise RuntimeError(f"BayesBridge.so not found at {path}; run bayesbridge_amd._build")
    L = ctypes.CDLL(path)
    c = ctypes
    L.bb_version.restype = c.c_char_p
    L.bb_last_error.restype = c.c_char_p
    L.bb_device_count.restype = c.c_int
    L.bb_set_seed.argtypes = [c.c_uint64]
    L.bb_get_rng_state.argtypes = [c.POINTER(c.c_uint64), c.POINTER(c.c_uint64)]
    L.bb_set_rng_state.argtypes = [c.c_uint64, c.c_uint64]
    L.bb_use_r_rng.argtypes = [c.c_int]
    L.bb_set_device.argtypes = [c.c_int]
    L.bb_set_verbose.argtypes = [c.c_int]
    L.bb_config_default.argtypes = [c.POINTER(bb_config)]
    L.bb_engine_create.argtypes = [c.POINTER(bb_config), _dp, _dp, c.POINTER(c.c_void_p)]
    L.bb_engine_destroy.argtypes = [c.c_void_p]
    L.bb_comm_id_size.restype = c.c_int
    L.bb_comm_unique_id.argtypes = [c.c_void_p]
    L.bb_engine_comm_init.argtypes = [c.c_void_p, c.c_void_p]
    L.bb_engine_init_state.argtypes = [c.c_void_p]
    L.bb_engine_run.argtypes = [c.c_void_p, c.c_uint64, c.c_int, c.c_int, c.c_int, c.c_int]
    L.bb_engine_sync.argtypes = [c.c_void_p]
    L.bb_engine_get_trace.argtypes = [c.c_void_p, c.c_int, c.c_int, _dp, _dp, _dp, _dp, _dp]
    L.bb_engine_get_state.argtypes = [c.c_void_p, _dp, _dp, _dp, _dp, _dp]
    L.bb_engine_set_state.argtypes = [c.c_void_p, _dp, c.c_double, c.c_double, c.c_double]
    L.bb_engine_method.argtypes = [c.c_void_p]
    L.bb_engine_gram_mode.argtypes = [c.c_void_p]
    L.bb_engine_enable_timing.argtypes = [c.c_void_p, c.c_int]
    L.bb_engine_reset_timing.argtypes = [c.c_void_p]
    L.bb_engine_set_timed_phase.argtypes = [c.c_void_p, c.c_int]
    L.bb_engine_set_timing_stride.argtypes = [c.c_void_p, c.c_int]
    L.bb_engine_kernel_times.argtypes = [c.c_void_p, _dp, _dp, _ip]
    L.bb_engine_error_flags.argtypes = [c.c_void_p, c.POINTER(c.c_uint32)]
    L.bb_retstable_batch.argtypes = [_dp, _dp, _dp, _dp, c.c_int, c.c_uint64, c.c_uint64,
                                     c.c_uint64, c.c_int]
    L.bb_sample_lambda.argtypes = [_dp, _dp, c.c_int, c.c_double, c.c_double, c.c_uint64,
                                   c.c_uint64, c.c_uint64, c.c_uint64, c.c_int]
    L.bb_gram.argtypes = [_dp, _dp, _dp, c.c_int, c.c_int]
    L.bb_gram_ozaki.argtypes = [_dp, _dp, _dp, c.c_int, c.c_int]
    L.bb_bench_ozaki.argtypes = [c.c_int, c.c_int, c.c_int, c.c_int, c.c_int, _dp]
    L.bb_chol_solve.argtypes = [_dp, _dp, _dp, c.c_int, c.c_int]
    L.bb_group_create.argtypes = [c.POINTER(c.c_void_p), c.c_int, c.POINTER(c.c_void_p)]
    L.bb_group_create_rccl.argtypes = [c.POINTER(c.c_void_p), c.c_int, c.POINTER(c.c_void_p)]
    L.bb_group_sync.argtypes = [c.c_void_p]
    L.bb_set_device_count.argtypes = [c.c_int]
    L.bb_set_chol_version.argtypes = [c.c_int]
    L.bb_set_tuning.argtypes = [c.c_int, c.c_int]
    L.bb_set_trace_budget.argtypes = [c.c_longlong]
    L.bb_debug_interrupt_after.argtypes = [c.c_int]
    L.bb_last_call_info.argtypes = [_ip, _ip, _ip]
    L.bb_debug_fail_member.argtypes = [c.c_int, c.c_int]
    u64p = c.POINTER(c.c_ulonglong)
    L.bb_engine_nid_stats.argtypes = [c.c_void_p, u64p, u64p, u64p, _dp, _ip]
    L.bb_engine_timed_brackets.argtypes = [c.c_void_p, _ip]
    L.bb_engine_nid_bound.argtypes = [c.c_void_p, _dp, _ip]
    L.bb_engine_launch_counts.argtypes = [c.c_void_p, u64p, u64p]
    L.bb_kernel_instance.argtypes = [c.c_char_p, c.c_char_p, c.c_int]
    L.bb_engine_nid_mixed.argtypes = [c.c_void_p, u64p, u64p, _dp, _ip, _ip]
    L.bb_group_destroy.argtypes = [c.c_void_p]
    L.bb_group_init_state.argtypes = [c.c_void_p]
    L.bb_group_run.argtypes = [c.c_void_p, c.c_uint64, c.c_int, c.c_int, c.c_int, c.c_int]
    L.bb_bench_chol.argtypes = [c.c_int, c.c_int, _dp, _dp, c.c_void_p]
    L.bb_bench_lambda.argtypes = [_dp, c.c_int, c.c_double, c.c_double, c.c_int, c.c_int,
                                  c.c_int, _dp, _dp]
    L.bb_engine_phase_times.argtypes = [c.c_void_p, _dp, c.c_int, _ip]
    L.bb_phase_count.restype = c.c_int
    L.bb_phase_name.argtypes = [c.c_int]
    L.bb_phase_name.restype = c.c_char_p
    L.retstable_LD.argtypes = [_dp, _dp, _dp, _dp, _ip]
    L.bridge_reg_stable.argtypes = [_dp] * 7 + [_dp] * 9 + [_ip] * 4 + [_dp, _ip]
    L.bridge_reg_stable_csc.argtypes = ([_dp] * 6 + [_ip, _ip, _dp] + [_dp] * 9 + [_ip] * 4 +
                                        [_dp, _ip])
    L.bb_engine_create_csc.argtypes = [c.POINTER(bb_config), _ip, _ip, _dp, _dp,
                                       c.POINTER(c.c_void_p)]
    L.bb_engine_sparse_pairs.argtypes = [c.c_void_p]
    L.bb_engine_sparse_pairs.restype = c.c_longlong
    L.bridge_reg_logit.argtypes = [_dp] * 6 + [_dp] * 6 + [_ip] * 4 + [_dp]
    L.bb_engine_get_omega.argtypes = [c.c_void_p, _dp]
    L.bb_pg_batch.argtypes = [_dp, _dp, c.c_int, c.c_uint64, c.c_uint64, c.c_uint64]
    L.bb_engine_sparse_info.argtypes = [c.c_void_p, c.POINTER(c.c_longlong),
                                        c.POINTER(c.c_longlong), _ip, _ip]
    L.bb_sparse_gram.argtypes = [_dp, _dp, _ip, _ip, _dp, _dp, _dp, c.c_int, c.c_int]
    L.bb_bench_sparse_gram.argtypes = [_ip, _ip, _dp, _dp, c.c_int, c.c_int, c.c_int, _dp, _dp,
                                       c.POINTER(c.c_longlong)]
    L.bridge_regression.argtypes = [_dp] * 9 + [_dp] * 9 + [_ip] * 4 + [_dp] + [_ip] * 3
    for name, npar in (("rtnorm_left", 3), ("rtnorm_both", 4), ("rtnorm", 4),
                       ("rtexpon_rate_left", 2), ("rtexpon_rate_both", 3), ("rtexpon_rate", 3)):
        getattr(L, name).argtypes = [_dp] * (1 + npar) + [_ip]
    L.mytest.argtypes = [_ip, _dp]
    L.rrtgamma_rate.argtypes = [_dp] * 4 + [_ip]
    L.bb_rrtgamma_batch.argtypes = [c.c_int, _dp, _dp, _dp, _dp, c.c_uint64, c.c_uint64]
    L.bb_trunc_batch.argtypes = [c.c_int, c.c_int, _dp, _dp, _dp, _dp, _dp, c.c_uint64,
                                 c.c_uint64]
    L.bb_engine_get_tri_trace.argtypes = [c.c_void_p, c.c_int, c.c_int, _dp, _dp]
    L.bb_engine_get_tri_basis.argtypes = [c.c_void_p, _dp, _dp, _dp]
    L.bb_engine_set_tri_state.argtypes = [c.c_void_p, _dp]
    L.bridge_EM.argtypes = [_dp, _dp, _dp, _dp, _dp, _ip, _ip, _dp, _dp, _ip, _ip]
    L.bb_bridge_em.argtypes = [_dp, _dp, _dp, c.c_int, c.c_int, c.c_double, c.c_double,
                               c.c_double, c.c_double, c.c_int, c.c_int]
    L.bb_bridge_em_batch.argtypes = [_dp, _ip, _dp, _dp, c.c_int, c.c_int, _dp, _dp, c.c_int,
                                     c.c_double, c.c_double, c.c_int]
    _lib = L
    return L


def device_count() -> int:
    return int(library().bb_device_count())


def _require_gpu():
    if device_count() < 1:
        raise RuntimeError("bayesbridge_amd: no HIP device visible (the sampler has no CPU path)")


def kernel_instance(phase: str):
    """The kernel instance this process last launched for a roofline phase (exact name as in
    the rocprofv3 summaries, e.g. "bb::k_eapply<8, false>"), or None."""
    buf = ctypes.create_string_buffer(512)
    if library().bb_kernel_instance(phase.encode(), buf, 512) != 0:
        return None
    return buf.value.decode()


def _err() -> str:
    return library().bb_last_error().decode()


def _check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc}): {_err()}")


def _p(a: np.ndarray):
    return a.ctypes.data_as(_dp)


def set_seed(seed: int) -> None:
    """Seed the Philox key for subsequent calls (stream counter reset to 0)."""
    library().bb_set_seed(int(seed) & 0xFFFFFFFFFFFFFFFF)


def get_rng_state():
    s, t = ctypes.c_uint64(), ctypes.c_uint64()
    library().bb_get_rng_state(ctypes.byref(s), ctypes.byref(t))
    return int(s.value), int(t.value)


def set_rng_state(seed: int, stream: int) -> None:
    library().bb_set_rng_state(int(seed), int(stream))


def set_verbose(v: int) -> None:
    library().bb_set_verbose(int(v))


def set_device_count(k: int) -> None:
    """Cap the devices a .C sampler call may shard over (0: every visible device)."""
    library().bb_set_device_count(int(k))


def set_chol_version(version: int) -> None:
    """Device Cholesky chain variant: 1 (default) or the pipelined 2 / 3 (A/B only)."""
    _check(library().bb_set_chol_version(int(version)), "bb_set_chol_version")


def set_tuning(key: int, value: int) -> int:
    """A/B tuning knob (bb_set_tuning): key 1 = non-temporal Ozaki residue stores.  Returns
    the previous value."""
    return int(library().bb_set_tuning(int(key), int(value)))


def chol_version() -> int:
    """The device Cholesky chain variant in use (bb_set_chol_version(0) reports it)."""
    return int(library().bb_set_chol_version(0))


def set_trace_budget(nbytes: int) -> None:
    """Device bytes of the trace ring per engine (<= 0 restores the 1 GiB default)."""
    library().bb_set_trace_budget(int(nbytes))


def debug_interrupt_after(polls: int) -> None:
    """Test hook: the polls-th interrupt poll from now reports an interrupt (-1 clears)."""
    library().bb_debug_interrupt_after(int(polls))


def last_call_info():
    """dict(devices, trace_capacity, interrupted) of the last .C sampler call."""
    d, c, i = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    library().bb_last_call_info(ctypes.byref(d), ctypes.byref(c), ctypes.byref(i))
    return dict(devices=d.value, trace_capacity=c.value, interrupted=bool(i.value))


def debug_fail_member(member: int, sweep: int) -> None:
    """Test hook: member `member` of the next RCCL shard-group run fails before its sweep
    `sweep` (the group then aborts its communicators and refuses further runs)."""
    library().bb_debug_fail_member(int(member), int(sweep))


def dot_c(name, *args):
    """R's ``.C(name, ...)`` calling convention, for symbols with no ctypes prototype: each
    argument is an int or float scalar / sequence (R integer or double vector), passed as a
    pointer to a fresh copy (int -> int32, float -> float64, as R's as.integer / as.double);
    the copies come back as numpy arrays, like .C's returned list."""
    fn = getattr(library(), name)
    bufs, ptrs = [], []
    for a in args:
        arr = np.atleast_1d(np.asarray(a))
        arr = np.ascontiguousarray(arr, dtype=np.int32 if arr.dtype.kind in "biu" else np.float64)
        bufs.append(arr)
        ptrs.append(arr.ctypes.data_as(ctypes.c_void_p))
    fn.argtypes = [ctypes.c_void_p] * len(ptrs)
    fn.restype = None
    fn(*ptrs)
    return bufs


# ---------------------------------------------------------------------------
# R front-end mirror (Code/C/BridgeWrapper.R)
# ---------------------------------------------------------------------------
def _is_above(param, val, name):
    """BridgeWrapper.R:31-47 (is.above): TRUE iff param >= val and numeric."""
    above = True
    if not np.issubdtype(np.asarray(param).dtype, np.number):
        print(f"Error: {name} is not numeric.")
        return False
    if np.any(np.asarray(param) < val):
        print(f"Error: {name}<{val}")
        above = False
    return above


def check_parameters(N, R, M, sig2_shape, sig2_scale, nu_shape, nu_rate, alpha_a, alpha_b):
    """BridgeWrapper.R:50-69 (check.parameters)."""
    ok = True
    if N != R:
        print("Error: y and X do not conform.")
        ok = False
    checks = [_is_above(M, 1, "niter"), _is_above(sig2_shape, 0, "sig2.shape"),
              _is_above(sig2_scale, 0, "sig2.scale"), _is_above(nu_shape, 0, "nu.shape"),
              _is_above(nu_rate, 0, "nu.rate"), _is_above(alpha_a, -1, "alpha.a"),
              _is_above(alpha_b, -1, "alpha.b")]
    return ok and all(checks)


def _is_sparse(X) -> bool:
    try:
        import scipy.sparse as sp
    except ImportError:  # pragma: no cover
        return False
    return sp.issparse(X)


def csc_arrays(X):
    """(colptr, rowidx, val, shape) of a scipy.sparse matrix in canonical CSC form -- the
    layout of R's dgCMatrix (X@p, X@i, X@x): int32 indices, rows sorted and unique within
    each column."""
    import scipy.sparse as sp

    Xc = sp.csc_matrix(X, dtype=np.float64, copy=True)
    Xc.sum_duplicates()
    Xc.sort_indices()
    colptr = np.ascontiguousarray(Xc.indptr, dtype=np.int32)
    rowidx = np.ascontiguousarray(Xc.indices, dtype=np.int32)
    val = np.ascontiguousarray(Xc.data, dtype=np.float64)
    if rowidx.size == 0:  # keep valid pointers for the C ABI
        rowidx = np.zeros(1, dtype=np.int32)
        val = np.zeros(1)
    return colptr, rowidx, val, Xc.shape


def bridge_reg_stb(y, X, nsamp, alpha=0.5, sig2_shape=0.0, sig2_scale=0.0, nu_shape=2.0,
                   nu_rate=2.0, alpha_a=1.0, alpha_b=1.0, sig2_true=0.0, tau_true=0.0,
                   burn=500, ortho=False, colnames=None):
    """bridge.reg.stb (BridgeWrapper.R:194-234) through ``.C("bridge_reg_stable", ...)``.

    Returns a dict: beta (M x P), lambda (M x P), sig2, tau, alpha (M), runtime.
    ``alpha`` is alpha.true (> 0 fixes alpha; <= 0 samples it by MH).  A scipy.sparse X
    goes through ``.C("bridge_reg_stable_csc", ...)`` (the dgCMatrix layout; the sparse
    Woodbury draw for P > N).
    """
    L = library()
    _require_gpu()
    y = np.asarray(y, dtype=np.float64).ravel()
    sparse = _is_sparse(X)
    if sparse:
        colptr, rowidx, val, (R, P) = csc_arrays(X)
    else:
        X = np.asarray(X, dtype=np.float64)
        if X.ndim == 1:
            X = X[:, None]
        R, P = X.shape
    N = y.shape[0]
    M = int(nsamp)
    if not check_parameters(N, R, M, sig2_shape, sig2_scale, nu_shape, nu_rate, alpha_a,
                            alpha_b):
        # the R wrapper halts here (`break` outside a loop, BridgeWrapper.R:212)
        raise ValueError("bridge_reg_stb: invalid parameters")
    beta = np.zeros((P, M), order="F")
    lam = np.zeros((P, M), order="F")
    sig2 = np.zeros(M)
    tau = np.zeros(M)
    alph = np.zeros(M)
    d = lambda v: ctypes.byref(ctypes.c_double(float(v)))  # noqa: E731
    i = lambda v: ctypes.byref(ctypes.c_int(int(v)))  # noqa: E731
    rt = ctypes.c_double(0.0)
    hyper = (d(sig2_shape), d(sig2_scale), d(nu_shape), d(nu_rate), d(alpha_a), d(alpha_b),
             d(sig2_true), d(tau_true), d(alpha), i(P), i(N), i(M), i(burn), ctypes.byref(rt),
             i(1 if ortho else 0))
    if sparse:
        # .C("bridge_reg_stable_csc", ..., X@p, X@i, X@x, ...) for a dgCMatrix
        L.bridge_reg_stable_csc(_p(beta), _p(lam), _p(sig2), _p(tau), _p(alph), _p(y),
                                colptr.ctypes.data_as(_ip), rowidx.ctypes.data_as(_ip), _p(val),
                                *hyper)
    else:
        Xf = np.asfortranarray(X)
        L.bridge_reg_stable(_p(beta), _p(lam), _p(sig2), _p(tau), _p(alph), _p(y), _p(Xf),
                            *hyper)
    out = {"beta": beta.T.copy(), "lambda": lam.T.copy(), "sig2": sig2, "tau": tau,
           "alpha": alph, "runtime": rt.value}
    if colnames is not None:
        out["colnames"] = list(colnames)
    return out


def bridge_reg_tri(y, X, nsamp, alpha=0.5, sig2_shape=0.0, sig2_scale=0.0, nu_shape=2.0,
                   nu_rate=2.0, alpha_a=1.0, alpha_b=1.0, sig2_true=0.0, tau_true=0.0,
                   burn=500, ortho=False, betaburn=0, extras=False):
    """bridge.reg.tri (BridgeWrapper.R:139-186) through ``.C("bridge_regression", ...)``.

    Returns a dict: beta, u, w (omega), shape (M x P), sig2, tau, alpha (M), runtime.
    Needs P <= N (the reference's svd-based rtnorm_gibbs indexes d[0..P-1]).
    """
    L = library()
    _require_gpu()
    y = np.asarray(y, dtype=np.float64).ravel()
    X = np.asarray(X, dtype=np.float64)
    if X.ndim == 1:
        X = X[:, None]
    N = y.shape[0]
    R, P = X.shape
    M = int(nsamp)
    if not check_parameters(N, R, M, sig2_shape, sig2_scale, nu_shape, nu_rate, alpha_a,
                            alpha_b):
        raise ValueError("bridge_reg_tri: invalid parameters")
    if not extras:
        print("Variable extras only for Package testing.")
    tr = {k: np.zeros((P, M), order="F") for k in ("beta", "u", "w", "shape")}
    sig2 = np.zeros(M)
    tau = np.zeros(M)
    alph = np.zeros(M)
    Xf = np.asfortranarray(X)
    d = lambda v: ctypes.byref(ctypes.c_double(float(v)))  # noqa: E731
    i = lambda v: ctypes.byref(ctypes.c_int(int(v)))  # noqa: E731
    rt = ctypes.c_double(0.0)
    L.bridge_regression(_p(tr["beta"]), _p(tr["u"]), _p(tr["w"]), _p(tr["shape"]), _p(sig2),
                        _p(tau), _p(alph), _p(y), _p(Xf), d(sig2_shape), d(sig2_scale),
                        d(nu_shape), d(nu_rate), d(alpha_a), d(alpha_b), d(sig2_true),
                        d(tau_true), d(alpha), i(P), i(N), i(M), i(burn), ctypes.byref(rt),
                        i(1 if ortho else 0), i(betaburn), i(0))
    out = {k: v.T.copy() for k, v in tr.items()}
    out.update(sig2=sig2, tau=tau, alpha=alph, runtime=rt.value)
    return out


def bridge_reg_logit(y, X, nsamp, alpha=0.5, nu_shape=2.0, nu_rate=2.0, alpha_a=1.0,
                     alpha_b=1.0, tau_true=0.0, burn=500):
    """Logistic bridge regression (Polya-Gamma Gibbs, BASELINE config C4) through
    ``.C("bridge_reg_logit", ...)``; y in {0, 1}.  No reference counterpart: the R-style
    front end mirrors bridge.reg.stb (same checks, same trace layout, no sig2).

    Returns a dict: beta (M x P), lambda (M x P), tau, alpha (M), runtime.
    """
    L = library()
    _require_gpu()
    y = np.asarray(y, dtype=np.float64).ravel()
    X = np.asarray(X, dtype=np.float64)
    if X.ndim == 1:
        X = X[:, None]
    N = y.shape[0]
    R, P = X.shape
    M = int(nsamp)
    if not check_parameters(N, R, M, 0.0, 0.0, nu_shape, nu_rate, alpha_a, alpha_b):
        raise ValueError("bridge_reg_logit: invalid parameters")
    if not np.all((y == 0) | (y == 1)):
        raise ValueError("bridge_reg_logit: y must be 0/1")
    beta = np.zeros((P, M), order="F")
    lam = np.zeros((P, M), order="F")
    tau = np.zeros(M)
    alph = np.zeros(M)
    Xf = np.asfortranarray(X)
    d = lambda v: ctypes.byref(ctypes.c_double(float(v)))  # noqa: E731
    i = lambda v: ctypes.byref(ctypes.c_int(int(v)))  # noqa: E731
    rt = ctypes.c_double(0.0)
    L.bridge_reg_logit(_p(beta), _p(lam), _p(tau), _p(alph), _p(y), _p(Xf), d(nu_shape),
                       d(nu_rate), d(alpha_a), d(alpha_b), d(tau_true), d(alpha), i(P), i(N),
                       i(M), i(burn), ctypes.byref(rt))
    return {"beta": beta.T.copy(), "lambda": lam.T.copy(), "tau": tau, "alpha": alph,
            "runtime": rt.value}


def pg_batch(psi, seed, stream=0, t=0):
    """omega_i ~ PG(1, psi_i) on the device under an explicit key (tests)."""
    L = library()
    _require_gpu()
    psi = np.ascontiguousarray(psi, dtype=np.float64)
    om = np.zeros_like(psi)
    _check(L.bb_pg_batch(_p(om), _p(psi), psi.shape[0], seed, stream, t), "bb_pg_batch")
    return om


def _dotC(name, num, *params):
    """``.C(name, x, params..., as.integer(num))`` with R's recycling (array(v, num))."""
    L = library()
    _require_gpu()
    ps = [np.ascontiguousarray(np.resize(np.asarray(v, dtype=np.float64), num)) for v in params]
    x = np.zeros(num)
    getattr(L, name)(_p(x), *[_p(q) for q in ps], ctypes.byref(ctypes.c_int(num)))
    return x


def rtexp_left(num=1, left=0.0, rate=1.0):
    """rtexp.left (BridgeWrapper.R:295-315)."""
    if np.any(np.asarray(rate) <= 0):
        print("rate must be >= 0.")
        return None
    if not num > 0:
        print("num must be greater than zero.")
        return None
    return _dotC("rtexpon_rate_left", num, left, rate)


def rtexp_both(num=1, left=0.0, right=1.0, rate=1.0):
    """rtexp.both (BridgeWrapper.R:317-344); like R it only warns on bad bounds."""
    if np.any(np.asarray(rate) <= 0):
        print("rate must be >= 0.")
        return None
    if not num > 0:
        print("num must be greater than zero.")
        return None
    if np.any(np.asarray(left) > np.asarray(right)):
        print("left must be <= right.")
    if np.any(np.asarray(right) == np.inf):
        print("right must be < infinity.")
    return _dotC("rtexpon_rate_both", num, left, right, rate)


def rtexp(num=1, left=0.0, right=np.inf, rate=1.0):
    """rtexp (BridgeWrapper.R:346-375)."""
    if np.any(np.asarray(rate) <= 0):
        print("rate must be > 0.")
        return None
    if not num > 0:
        print("num must be greater than zero.")
        return None
    if np.any(np.asarray(left) > np.asarray(right)):
        print("left must be <= right.")
        return None
    return _dotC("rtexpon_rate", num, left, right, rate)


def rtnorm_left(num=1, left=0.0, mu=0.0, sig=1.0):
    """rtnorm.left (BridgeWrapper.R:380-402)."""
    if np.any(np.asarray(sig) <= 0):
        print("sig must be greater than zero.")
        return None
    if not num > 0:
        print("num must be greater than zero.")
        return None
    return _dotC("rtnorm_left", num, left, mu, sig)


def rtnorm_right(num=1, right=0.0, mu=0.0, sig=1.0):
    """rtnorm.right (BridgeWrapper.R:404-407)."""
    x = rtnorm_left(num=num, left=-1.0 * np.asarray(right), mu=-1.0 * np.asarray(mu), sig=sig)
    return None if x is None else -1.0 * x


def rtnorm_both(num=1, left=-1.0, right=1.0, mu=0.0, sig=1.0):
    """rtnorm.both (BridgeWrapper.R:409-437)."""
    if np.any(np.asarray(sig) <= 0):
        print("sig must be greater than zero.")
        return None
    if np.any(np.asarray(left) >= np.asarray(right)):
        print("rtnorm: left must be less than right.")
        return None
    if not num > 0:
        print("rtnorm: num must be greater than zero.")
        return None
    return _dotC("rtnorm_both", num, left, right, mu, sig)


def rtruncated_norm(num=1, left=-np.inf, right=np.inf, mu=0.0, sig=1.0):
    """rtruncated.norm (BridgeWrapper.R:439-474); rtnorm (:477-480) calls it."""
    if np.any(np.asarray(sig) <= 0):
        print("sig must be greater than zero.")
        return None
    if np.any(np.asarray(left) > np.asarray(right)):
        print("left must be less than or equal to right.")
        return None
    if not num > 0:
        print("num must be greater than zero.")
        return None
    return _dotC("rtnorm", num, left, right, mu, sig)


def rtnorm(num=1, mu=0.0, sig=1.0, left=-np.inf, right=np.inf):
    return rtruncated_norm(num=num, left=left, right=right, mu=mu, sig=sig)


def rrtgamma(num=1, shape=1.0, rate=1.0, rtrunc=1.0, scale=None):
    """rrtgamma (BridgeWrapper.R:482-509): Ga(shape, rate) right-truncated at rtrunc."""
    rate = 1.0 / np.asarray(scale if scale is not None else 1.0 / np.asarray(rate, float), float)
    if not np.all(np.asarray(shape) > 0):
        print("shape must be greater than zero.")
        return None
    if not np.all(rate > 0):
        print("scale/rate must be greater than zero.")
        return None
    if not np.all(np.asarray(rtrunc) > 0):
        print("rtrunc must be greater than zero.")
        return None
    return _dotC("rrtgamma_rate", num, shape, rate, rtrunc)


def rrtgamma_batch(shape, rate, right_t, seed, stream=0):
    """Device batch behind rrtgamma_rate under an explicit key (tests)."""
    L = library()
    _require_gpu()
    ps = [np.ascontiguousarray(q, dtype=np.float64) for q in (shape, rate, right_t)]
    x = np.zeros(ps[0].shape[0])
    _check(L.bb_rrtgamma_batch(x.shape[0], _p(x), *[_p(q) for q in ps], seed, stream),
           "bb_rrtgamma_batch")
    return x


def trunc_batch(name, params, seed, stream=0):
    """Device batch behind the truncated .C utilities under an explicit key (tests)."""
    modes = {"rtnorm_left": 0, "rtnorm_both": 1, "rtnorm": 2, "rtexpon_rate_left": 3,
             "rtexpon_rate_both": 4, "rtexpon_rate": 5}
    L = library()
    _require_gpu()
    ps = [np.ascontiguousarray(q, dtype=np.float64) for q in params]
    num = ps[0].shape[0]
    ptrs = [_p(q) for q in ps] + [None] * (4 - len(ps))
    x = np.zeros(num)
    _check(L.bb_trunc_batch(modes[name], num, _p(x), *ptrs, seed, stream), "bb_trunc_batch")
    return x


def bridge_reg(y, X, nsamp, alpha=0.5, sig2_shape=0.0, sig2_scale=0.0, nu_shape=2.0,
               nu_rate=2.0, alpha_a=1.0, alpha_b=1.0, sig2_true=0.0, tau_true=0.0, burn=500,
               method="triangle", ortho=False):
    """bridge.reg (BridgeWrapper.R:240-276).

    Like the reference, the "stable" branch IGNORES the caller's hyper-parameters and
    calls bridge.reg.stb with alpha=0.5, nu.shape = nu.rate = 0.5, burn=500; the
    "triangle" branch likewise calls bridge.reg.tri with those constants.
    """
    if method == "stable":
        return bridge_reg_stb(y, X, nsamp, alpha=0.5, sig2_shape=0.0, sig2_scale=0.0,
                              nu_shape=0.5, nu_rate=0.5, alpha_a=1.0, alpha_b=1.0,
                              sig2_true=0.0, tau_true=0.0, burn=500, ortho=ortho)
    if method == "triangle":
        return bridge_reg_tri(y, X, nsamp, alpha=0.5, sig2_shape=0.0, sig2_scale=0.0,
                              nu_shape=0.5, nu_rate=0.5, alpha_a=1.0, alpha_b=1.0,
                              sig2_true=0.0, tau_true=0.0, burn=500, ortho=ortho)
    print('Unrecognized method.  Use "triangles" or "stable".')
    return None


def check_em(lambda_max, tol, max_iter):
    """BridgeWrapper.R:73-82 (check.EM)."""
    checks = [_is_above(lambda_max, 0.0, "lambda.max"), _is_above(tol, 0.0, "tolerance"),
              _is_above(max_iter, 1.0, "max.iter")]
    return all(checks)


def bridge_em(y, X, alpha=0.5, ratio=1.0, lambda_max=None, tol=1e-9, max_iter=30,
              use_cg=False, ret_solves=False):
    """bridge.EM (BridgeWrapper.R:89-133) through ``.C("bridge_EM", ...)``.

    Bridge posterior mode by EM with sig = 1 and tau = ratio; lambda.max defaults to
    1e9 * ratio.  Returns beta (P), or {"beta", "num.solves"} with ret_solves.
    """
    L = library()
    _require_gpu()
    if lambda_max is None:
        lambda_max = 1e9 * ratio
    y = np.asarray(y, dtype=np.float64).ravel()
    X = np.asarray(X, dtype=np.float64)
    if X.ndim == 1:
        X = X[:, None]
    N = y.shape[0]
    R, P = X.shape
    if ratio < 0:
        print("bridge.EM: ratio < 0")
        return 0
    if alpha < 0:
        print("bridge.EM: alpha < 0")
        return 0
    ok = check_parameters(N, R, 1, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0) and check_em(
        lambda_max, tol, max_iter)
    if not ok:
        raise ValueError("bridge_em: invalid parameters")
    beta = np.zeros(P)
    Xf = np.asfortranarray(X)
    d = lambda v: ctypes.byref(ctypes.c_double(float(v)))  # noqa: E731
    it = ctypes.c_int(int(max_iter))
    L.bridge_EM(_p(beta), _p(y), _p(Xf), d(ratio), d(alpha), ctypes.byref(ctypes.c_int(P)),
                ctypes.byref(ctypes.c_int(N)), d(lambda_max), d(tol), ctypes.byref(it),
                ctypes.byref(ctypes.c_int(1 if use_cg else 0)))
    if ret_solves:
        return {"beta": beta, "num.solves": it.value}
    return beta


# Above this p a single workgroup's p x p factorisations are slower than the per-ratio
# loop over the whole-device Cholesky (bridge_em), so trace_beta loops there.
EM_BATCH_MAX_P = 2048


def trace_beta(y, X, alpha=0.5, ratio_grid=None, tol=1e-9, max_iter=30, use_cg=False):
    """trace.beta (Code/R/bridge-trace.R:22-54) without the plot: bridge.EM over a grid of
    ratios with lambda.max = ratio / tol.  Returns {"beta" (L x P), "grid", "log.grid"}."""
    if ratio_grid is None:
        ratio_grid = np.exp(np.arange(-20.0, 20.0 + 1e-9, 0.1))
    ratio_grid = np.asarray(ratio_grid, dtype=np.float64)
    X = np.asarray(X, dtype=np.float64)
    if X.ndim == 1:
        X = X[:, None]
    P = X.shape[1]
    if 1 <= P <= EM_BATCH_MAX_P and not use_cg:
        # the whole grid in one device launch (a workgroup per ratio)
        beta, _ = bridge_em_batch(y, X, ratio_grid, alpha=alpha,
                                  lambda_max=ratio_grid / tol, tol=tol, max_iter=max_iter)
    else:
        beta = np.zeros((ratio_grid.size, P))
        for i, r in enumerate(ratio_grid):
            beta[i] = bridge_em(y, X, alpha, ratio=r, lambda_max=r / tol, tol=tol,
                                max_iter=max_iter, use_cg=use_cg)
    return {"beta": beta, "grid": ratio_grid, "log.grid": np.log(ratio_grid)}


def bridge_em_batch(y, X, ratios, alpha=0.5, lambda_max=None, tol=1e-9, max_iter=30):
    """bridge.EM (direct solves) for every ratio in one device launch (a workgroup per
    ratio; the system in LDS for p <= 128, a tiled Cholesky over global memory above).
    Returns (beta (len(ratios) x P), solves (len(ratios)))."""
    L = library()
    _require_gpu()
    y = np.ascontiguousarray(np.asarray(y, dtype=np.float64).ravel())
    X = np.asfortranarray(np.asarray(X, dtype=np.float64))
    ratios = np.ascontiguousarray(ratios, dtype=np.float64)
    if lambda_max is None:
        lambda_max = 1e9 * ratios
    lmax = np.ascontiguousarray(np.broadcast_to(lambda_max, ratios.shape), dtype=np.float64)
    N, P = X.shape
    beta = np.zeros((ratios.size, P))
    solves = np.zeros(ratios.size, dtype=np.int32)
    _check(L.bb_bridge_em_batch(_p(beta), solves.ctypes.data_as(_ip), _p(y), _p(X), N, P,
                                _p(ratios), _p(lmax), ratios.size, float(alpha), float(tol),
                                int(max_iter)), "bb_bridge_em_batch")
    return beta, solves


def retstable_ld(num=1, alpha=1.0, V0=1.0, h=1.0):
    """retstable.ld (BridgeWrapper.R:511-537) through ``.C("retstable_LD", ...)``.

    Draws from the exponentially tilted positive stable law with Laplace transform
    exp(-V0((h+t)^alpha - h^alpha)).  Invalid parameters print and return NaN, as
    the R function prints and returns NA.
    """
    if not np.all(np.asarray(V0) > 0):
        print("V0 must be > 0.")
        return np.nan
    if not np.all(np.asarray(h) >= 0):
        print("h must be >= 0")
        return np.nan
    a = np.asarray(alpha)
    if not (np.all(a > 0) and np.all(a <= 1)):
        print("alpha must be in (0,1].")
        return np.nan
    L = library()
    _require_gpu()
    num = int(num)
    # R's array(v, num) recycles
    alpha_a = np.resize(np.asarray(alpha, dtype=np.float64), num)
    h_a = np.resize(np.asarray(h, dtype=np.float64), num)
    V0_a = np.resize(np.asarray(V0, dtype=np.float64), num)
    x = np.zeros(num)
    L.retstable_LD(_p(x), _p(alpha_a), _p(V0_a), _p(h_a), ctypes.byref(ctypes.c_int(num)))
    return x


# ---------------------------------------------------------------------------
# Kernel-level helpers (tests / microbenchmarks)
# ---------------------------------------------------------------------------
def retstable_batch(alpha, V0, h, seed, stream=0, t=0, group=0):
    L = library()
    _require_gpu()
    alpha = np.ascontiguousarray(alpha, dtype=np.float64)
    V0 = np.ascontiguousarray(V0, dtype=np.float64)
    h = np.ascontiguousarray(h, dtype=np.float64)
    x = np.zeros(h.shape[0])
    _check(L.bb_retstable_batch(_p(x), _p(alpha), _p(V0), _p(h), h.shape[0], seed, stream, t,
                                group), "bb_retstable_batch")
    return x


def sample_lambda(beta, alpha, tau, seed, stream, t, j0=0, group=0):
    L = library()
    _require_gpu()
    beta = np.ascontiguousarray(beta, dtype=np.float64)
    lam = np.zeros_like(beta)
    _check(L.bb_sample_lambda(_p(lam), _p(beta), beta.shape[0], alpha, tau, seed, stream, t, j0,
                              group), "bb_sample_lambda")
    return lam


def bench_lambda(beta, alpha, tau, group, noinline=1, reps=20):
    """Average ms of one lambda-kernel launch (microbenchmark) and its last draws."""
    L = library()
    _require_gpu()
    beta = np.ascontiguousarray(beta, dtype=np.float64)
    lam = np.zeros_like(beta)
    ms = ctypes.c_double()
    _check(L.bb_bench_lambda(_p(beta), beta.shape[0], alpha, tau, group, noinline, reps,
                             ctypes.byref(ms), _p(lam)), "bb_bench_lambda")
    return ms.value, lam


def bench_chol(m, reps=10, trace=False):
    """(factor ms, solve ms[, stamps]) of the blocked device Cholesky on an m x m SPD test
    matrix; with trace=True also the (steps, 8) s_memrealtime stamps (100 MHz ticks) of one
    traced factorisation (see bb_bench_chol in include/bayesbridge.h), followed by the same
    points in shader clocks (s_memtime), then the elimination's 8 producer-group start and 8
    end stamps (100 MHz): shape (steps + 1, 32); the last row holds owner stamps."""
    L = library()
    _require_gpu()
    f, s = ctypes.c_double(), ctypes.c_double()
    ts = np.zeros((-(-m // 64) + 1, 32), dtype=np.uint64) if trace else None
    _check(L.bb_bench_chol(m, reps, ctypes.byref(f), ctypes.byref(s),
                           ts.ctypes.data if trace else None), "bb_bench_chol")
    return (f.value, s.value, ts) if trace else (f.value, s.value)


def bench_ozaki(n, k, nsplit=0, dbg=0, reps=10):
    """Average ms of the Ozaki int8 GEMM kernel alone (random residues)."""
    L = library()
    _require_gpu()
    ms = ctypes.c_double()
    _check(L.bb_bench_ozaki(n, k, nsplit, dbg, reps, ctypes.byref(ms)), "bb_bench_ozaki")
    return ms.value


def gram(Y, w, mode=GRAM_FP64):
    """C = Y diag(w) Y' on the device: fp64 MFMA (mode 0) or Ozaki-II int8 MFMA (mode 1,
    w >= 0)."""
    L = library()
    _require_gpu()
    Y = np.asfortranarray(Y, dtype=np.float64)
    w = np.ascontiguousarray(w, dtype=np.float64)
    n, k = Y.shape
    C = np.zeros((n, n), order="F")
    if mode == GRAM_OZAKI:
        if np.any(w < 0):
            raise ValueError("the Ozaki Gram needs w >= 0")
        _check(L.bb_gram_ozaki(_p(C), _p(Y), _p(w), n, k), "bb_gram_ozaki")
    else:
        _check(L.bb_gram(_p(C), _p(Y), _p(w), n, k), "bb_gram")
    return C


def sparse_gram(X, D, u=None):
    """(X diag(D) X', X u) for a sparse X through the pair-list kernels (full n x n)."""
    L = library()
    _require_gpu()
    colptr, rowidx, val, (n, p) = csc_arrays(X)
    D = np.ascontiguousarray(D, dtype=np.float64)
    C = np.zeros((n, n), order="F")
    xu = np.zeros(n)
    uu = None if u is None else np.ascontiguousarray(u, dtype=np.float64)
    _check(L.bb_sparse_gram(_p(C), _p(xu), colptr.ctypes.data_as(_ip), rowidx.ctypes.data_as(_ip),
                            _p(val), _p(D), None if uu is None else _p(uu), n, p),
           "bb_sparse_gram")
    return C, xu


def bench_sparse_gram(X, D, reps=10):
    """(pair-list Gram ms, CSR row pass ms, pair count) for a sparse X."""
    L = library()
    _require_gpu()
    colptr, rowidx, val, (n, p) = csc_arrays(X)
    D = np.ascontiguousarray(D, dtype=np.float64)
    g, r, k = ctypes.c_double(), ctypes.c_double(), ctypes.c_longlong()
    _check(L.bb_bench_sparse_gram(colptr.ctypes.data_as(_ip), rowidx.ctypes.data_as(_ip), _p(val),
                                  _p(D), n, p, reps, ctypes.byref(g), ctypes.byref(r),
                                  ctypes.byref(k)), "bb_bench_sparse_gram")
    return g.value, r.value, k.value


def chol_solve(A, b):
    L = library()
    _require_gpu()
    A = np.asfortranarray(A, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    nrhs = 1 if b.ndim == 1 else b.shape[1]
    bf = np.asfortranarray(b.reshape(A.shape[0], nrhs))
    x = np.zeros_like(bf, order="F")
    _check(L.bb_chol_solve(_p(x), _p(A), _p(bf), A.shape[0], nrhs), "bb_chol_solve")
    return x.ravel() if b.ndim == 1 else x


# ---------------------------------------------------------------------------
# Engine (benchmarks, multi-GPU, teacher-forced tests)
# ---------------------------------------------------------------------------
@dataclass
class EngineConfig:
    n: int
    p: int
    p_local: int = 0
    j0: int = 0
    rank: int = 0
    world: int = 1
    sig2_shape: float = 0.0
    sig2_scale: float = 0.0
    nu_shape: float = 2.0
    nu_rate: float = 2.0
    alpha_a: float = 1.0
    alpha_b: float = 1.0
    true_sig2: float = 0.0
    true_tau: float = 0.0
    true_alpha: float = 0.5
    ortho: bool = False
    method: int = 0
    trace_capacity: int = 1
    seed: int = 0xB4E5B41D6E
    stream: int = 0
    device: int = 0
    gram_mode: Optional[int] = None  # None: library default (Ozaki-II)
    betaburn: int = 0

    def to_c(self) -> bb_config:
        c = bb_config()
        library().bb_config_default(ctypes.byref(c))
        for name, _ in bb_config._fields_:
            v = getattr(self, name)
            if v is None:
                continue
            setattr(c, name, int(v) if isinstance(v, bool) else v)
        if c.p_local <= 0:
            c.p_local = c.p
        return c


class Engine:
    """One Gibbs chain (or one column shard of it) resident on one GPU."""

    def __init__(self, cfg: EngineConfig, X_local, y):
        """X_local: dense (n x p_local) or scipy.sparse (-> the sparse Woodbury engine)."""
        L = library()
        _require_gpu()
        self.cfg = cfg
        self._c = cfg.to_c()
        y = np.ascontiguousarray(y, dtype=np.float64)
        self.p_local = self._c.p_local
        h = ctypes.c_void_p()
        if _is_sparse(X_local):
            colptr, rowidx, val, shape = csc_arrays(X_local)
            assert shape == (cfg.n, self._c.p_local), shape
            _check(L.bb_engine_create_csc(ctypes.byref(self._c), colptr.ctypes.data_as(_ip),
                                          rowidx.ctypes.data_as(_ip), _p(val), _p(y),
                                          ctypes.byref(h)), "bb_engine_create_csc")
        else:
            X_local = np.asfortranarray(X_local, dtype=np.float64)
            assert X_local.shape == (cfg.n, self._c.p_local), X_local.shape
            _check(L.bb_engine_create(ctypes.byref(self._c), _p(X_local), _p(y),
                                      ctypes.byref(h)), "bb_engine_create")
        self._h = h

    def sparse_pairs(self) -> int:
        return int(library().bb_engine_sparse_pairs(self._h))

    def sparse_info(self):
        """dict(pairs, nnz, max_row, col_mode) of a sparse-design engine."""
        pr, nz, mr, cm = ctypes.c_longlong(), ctypes.c_longlong(), ctypes.c_int(), ctypes.c_int()
        _check(library().bb_engine_sparse_info(self._h, ctypes.byref(pr), ctypes.byref(nz),
                                               ctypes.byref(mr), ctypes.byref(cm)),
               "bb_engine_sparse_info")
        return dict(pairs=pr.value, nnz=nz.value, max_row=mr.value, col_mode=bool(cm.value))

    def comm_init(self, id_bytes: bytes):
        _check(library().bb_engine_comm_init(self._h, ctypes.c_char_p(id_bytes)),
               "bb_engine_comm_init")

    @staticmethod
    def comm_unique_id() -> bytes:
        L = library()
        buf = ctypes.create_string_buffer(L.bb_comm_id_size())
        _check(L.bb_comm_unique_id(buf), "bb_comm_unique_id")
        return buf.raw

    def init_state(self):
        _check(library().bb_engine_init_state(self._h), "bb_engine_init_state")

    def run(self, t0: int, count: int, first_slot: int = -1, slot_step: int = 1,
            mcmc_phase: int = 1):
        _check(library().bb_engine_run(self._h, int(t0), int(count), int(first_slot),
                                       int(slot_step), int(mcmc_phase)), "bb_engine_run")

    def sync(self):
        _check(library().bb_engine_sync(self._h), "bb_engine_sync")

    def method(self) -> int:
        return int(library().bb_engine_method(self._h))

    def gram_mode(self) -> int:
        return int(library().bb_engine_gram_mode(self._h))

    def trace(self, slot0: int, count: int):
        pl = self.p_local
        beta = np.zeros((pl, count), order="F")
        lam = np.zeros((pl, count), order="F")
        sig2, tau, alpha = np.zeros(count), np.zeros(count), np.zeros(count)
        _check(library().bb_engine_get_trace(self._h, slot0, count, _p(beta), _p(lam), _p(sig2),
                                             _p(tau), _p(alpha)), "bb_engine_get_trace")
        return dict(beta=beta, **{"lambda": lam}, sig2=sig2, tau=tau, alpha=alpha)

    def omega(self):
        """Logistic engine: the current Polya-Gamma latents (n)."""
        om = np.zeros(self.cfg.n)
        _check(library().bb_engine_get_omega(self._h, _p(om)), "bb_engine_get_omega")
        return om

    def tri_trace(self, slot0: int, count: int):
        """Triangle method: u and shape traces (omega is ``trace()['lambda']``)."""
        pl = self.p_local
        u = np.zeros((pl, count), order="F")
        shape = np.zeros((pl, count), order="F")
        _check(library().bb_engine_get_tri_trace(self._h, slot0, count, _p(u), _p(shape)),
               "bb_engine_get_tri_trace")
        return dict(u=u, shape=shape)

    def set_tri_state(self, u):
        u = np.ascontiguousarray(u, dtype=np.float64)
        _check(library().bb_engine_set_tri_state(self._h, _p(u)), "bb_engine_set_tri_state")

    def tri_basis(self):
        """Triangle method: (tV, a, d) with X = U diag(d) V', tV = V' (P x P), a = V'X'y."""
        p = self.p_local
        tV = np.zeros((p, p), order="F")
        a, d = np.zeros(p), np.zeros(p)
        _check(library().bb_engine_get_tri_basis(self._h, _p(tV), _p(a), _p(d)),
               "bb_engine_get_tri_basis")
        return tV, a, d

    def state(self):
        pl = self.p_local
        beta, lam = np.zeros(pl), np.zeros(pl)
        tau, sig2, alpha = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        _check(library().bb_engine_get_state(self._h, _p(beta), _p(lam), ctypes.byref(tau),
                                             ctypes.byref(sig2), ctypes.byref(alpha)),
               "bb_engine_get_state")
        return dict(beta=beta, **{"lambda": lam}, tau=tau.value, sig2=sig2.value,
                    alpha=alpha.value)

    def set_state(self, beta, tau, sig2, alpha):
        beta = np.ascontiguousarray(beta, dtype=np.float64)
        _check(library().bb_engine_set_state(self._h, _p(beta), tau, sig2, alpha),
               "bb_engine_set_state")

    def enable_timing(self, on: bool = True, phases: bool = True, timed_phase: str = "gram",
                      stride: int = 1):
        """HIP-event timing on the engine stream: every phase start (phases=True) or only
        the bracket of `timed_phase` (a bb_phase_name, two events per bracketed sweep, used
        inside timed loops; kernel_times()[0] is its average) in every `stride`-th sweep."""
        L = library()
        names = [L.bb_phase_name(i).decode() for i in range(L.bb_phase_count())]
        _check(L.bb_engine_set_timed_phase(self._h, names.index(timed_phase)),
               "bb_engine_set_timed_phase")
        _check(L.bb_engine_set_timing_stride(self._h, int(stride)),
               "bb_engine_set_timing_stride")
        L.bb_engine_enable_timing(self._h, (2 if phases else 1) if on else 0)

    def reset_timing(self):
        library().bb_engine_reset_timing(self._h)

    def kernel_times(self):
        g, s, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
        _check(library().bb_engine_kernel_times(self._h, ctypes.byref(g), ctypes.byref(s),
                                                ctypes.byref(n)), "bb_engine_kernel_times")
        return g.value, s.value, n.value

    def phase_times(self):
        """Average ms per sweep per phase (HIP events on the engine stream)."""
        L = library()
        k = L.bb_phase_count()
        ms = np.zeros(k)
        n = ctypes.c_int()
        _check(L.bb_engine_phase_times(self._h, _p(ms), k, ctypes.byref(n)),
               "bb_engine_phase_times")
        return {L.bb_phase_name(i).decode(): float(ms[i]) for i in range(k) if ms[i] > 0}

    def timed_brackets(self) -> int:
        """Launches of the timed phase bracketed since the last reset_timing()."""
        k = ctypes.c_int()
        _check(library().bb_engine_timed_brackets(self._h, ctypes.byref(k)),
               "bb_engine_timed_brackets")
        return int(k.value)

    def nid_stats(self):
        """Near-identity (Chebyshev) solve counters: dict(cheb_sweeps,
        products, chol_sweeps, eps, mode) -- mode/eps of the latest sweep, -1 when the engine
        has no near-identity path."""
        a, b, c = ctypes.c_ulonglong(), ctypes.c_ulonglong(), ctypes.c_ulonglong()
        eps, mode = ctypes.c_double(), ctypes.c_int()
        _check(library().bb_engine_nid_stats(self._h, ctypes.byref(a), ctypes.byref(b),
                                             ctypes.byref(c), ctypes.byref(eps),
                                             ctypes.byref(mode)), "bb_engine_nid_stats")
        lam, kmax = ctypes.c_double(), ctypes.c_int()
        library().bb_engine_nid_bound(self._h, ctypes.byref(lam), ctypes.byref(kmax))
        return dict(cheb_sweeps=a.value, products=b.value, chol_sweeps=c.value, eps=eps.value,
                    mode=mode.value, lambda_x=lam.value, kmax=kmax.value)

    def nid_mixed(self):
        """The mixed-precision plan: dict(mixed_sweeps, products32 (fp32
        E-apply passes), eta and k2 of the latest sweep, holds_x32)."""
        a, b = ctypes.c_ulonglong(), ctypes.c_ulonglong()
        eta, k2, hx = ctypes.c_double(), ctypes.c_int(), ctypes.c_int()
        _check(library().bb_engine_nid_mixed(self._h, ctypes.byref(a), ctypes.byref(b),
                                             ctypes.byref(eta), ctypes.byref(k2),
                                             ctypes.byref(hx)), "bb_engine_nid_mixed")
        return dict(mixed_sweeps=a.value, products32=b.value, eta=eta.value, k2=k2.value,
                    holds_x32=bool(hx.value))

    def launch_counts(self):
        """Woodbury lambda launches since creation: dict(lambda_xu = fused with the X u stream
        of the near-identity solve (k_lambda_xu), lambda_alone = a launch of their own)."""
        a, b = ctypes.c_ulonglong(), ctypes.c_ulonglong()
        library().bb_engine_launch_counts(self._h, ctypes.byref(a), ctypes.byref(b))
        return dict(lambda_xu=a.value, lambda_alone=b.value)

    def error_flags(self) -> int:
        f = ctypes.c_uint32()
        _check(library().bb_engine_error_flags(self._h, ctypes.byref(f)), "bb_engine_error_flags")
        return int(f.value)

    def close(self):
        if getattr(self, "_h", None):
            library().bb_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ShardGroup:
    """Column shards of one chain driven from one process.  rccl=False: engines on ONE
    device, one host thread, exchanges through on-device sums (the sharded decomposition on
    a single GPU); rccl=True: engines on distinct devices exchanging with RCCL
    (ncclCommInitAll), each member's sweeps enqueued by its own host thread -- the
    single-process multi-GPU path of the .C entry points."""

    def __init__(self, engines, rccl=False):
        L = library()
        self.engines = list(engines)
        arr = (ctypes.c_void_p * len(self.engines))(*[e._h.value for e in self.engines])
        h = ctypes.c_void_p()
        fn = L.bb_group_create_rccl if rccl else L.bb_group_create
        _check(fn(arr, len(self.engines), ctypes.byref(h)), "bb_group_create")
        self._h = h

    def init_state(self):
        _check(library().bb_group_init_state(self._h), "bb_group_init_state")

    def run(self, t0, count, first_slot=-1, slot_step=1, mcmc_phase=1):
        _check(library().bb_group_run(self._h, int(t0), int(count), int(first_slot),
                                      int(slot_step), int(mcmc_phase)), "bb_group_run")

    def sync(self):
        _check(library().bb_group_sync(self._h), "bb_group_sync")

    def close(self):
        if getattr(self, "_h", None):
            library().bb_group_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
