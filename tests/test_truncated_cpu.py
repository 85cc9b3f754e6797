"""CPU tests of the truncated-distribution utilities (BridgeWrapper.cpp:738-935): the
oracle restatement against scipy (the reference's RNG library is un-vendored, so these
draws are pinned distributionally), the rtnorm / rtexpon_rate special-value rules, and
the host-only mytest marshalling check through the C ABI."""
import ctypes
import struct

import numpy as np
import pytest
import scipy.stats as ss

import bayesbridge_amd as bb
import oracle

N = 4000


def test_rtexpon_left_is_shifted_exponential():
    x = oracle.trunc_batch("rtexpon_rate_left", [np.full(N, 1.5), np.full(N, 2.0)], seed=1)
    assert np.all(x >= 1.5)
    assert ss.kstest(x - 1.5, ss.expon(scale=0.5).cdf).pvalue > 1e-3


@pytest.mark.parametrize("l,r,rate", [(0.0, 1.0, 2.0), (3.0, 3.5, 0.1), (-2.0, 10.0, 5.0)])
def test_rtexpon_both_matches_truncexpon(l, r, rate):
    x = oracle.trunc_batch("rtexpon_rate_both", [np.full(N, l), np.full(N, r), np.full(N, rate)],
                           seed=2)
    assert np.all((x >= l) & (x <= r))
    dist = ss.truncexpon(b=(r - l) * rate, loc=l, scale=1.0 / rate)
    assert ss.kstest(x, dist.cdf).pvalue > 1e-3


@pytest.mark.parametrize("name,params,dist", [
    ("rtnorm_left", [0.5, 1.0, 2.0], ss.truncnorm(-0.25, np.inf, loc=1.0, scale=2.0)),
    ("rtnorm_both", [-1.0, 0.5, 0.0, 1.0], ss.truncnorm(-1.0, 0.5)),
    ("rtnorm", [-np.inf, -2.0, 0.0, 1.0], ss.truncnorm(-np.inf, -2.0)),
    ("rtnorm", [-np.inf, np.inf, 3.0, 0.5], ss.norm(3.0, 0.5)),
    ("rtnorm", [1.0, np.inf, 0.0, 1.0], ss.truncnorm(1.0, np.inf)),
])
def test_rtnorm_family_matches_scipy(name, params, dist):
    x = oracle.trunc_batch(name, [np.full(N, v) for v in params], seed=3)
    assert ss.kstest(x, dist.cdf).pvalue > 1e-3


def test_special_values():
    x = oracle.trunc_batch("rtnorm", [np.array([np.nan, 0.0]), np.array([1.0, 1.0]),
                                      np.array([0.0, np.nan]), np.ones(2)], seed=4)
    assert np.all(np.isnan(x))
    # rtexpon_rate (BridgeWrapper.cpp:816-828): the NaN the reference assigns for a
    # non-finite input is overwritten by the draw that follows (no else), and a non-finite
    # right bound means left truncation only -- reproduced, not replaced by NaN
    x = oracle.trunc_batch("rtexpon_rate", [np.array([-np.inf, 0.0, 0.0, 1.0, np.nan, np.inf]),
                                            np.array([1.0, np.inf, 2.0, np.nan, 2.0, np.inf]),
                                            np.ones(6)], seed=4)
    assert x[0] == -np.inf and x[1] >= 0 and 0 <= x[2] <= 2
    assert x[3] >= 1.0 and np.isfinite(x[3])  # right = NaN: left-truncated draw
    assert np.isnan(x[4]) and x[5] == np.inf


def test_mytest_flags_r_special_values():
    """Host-only entry: no device needed."""
    L = bb.library()
    NA = struct.unpack("<d", struct.pack("<Q", 0x7FF00000000007A2))[0]
    for v, code in [(1.0, 0), (float("nan"), 1), (float("inf"), 2), (float("-inf"), 3), (NA, 4)]:
        out = ctypes.c_int(-1)
        x = ctypes.c_double(v)
        L.mytest(ctypes.byref(out), ctypes.byref(x))
        assert out.value == code, (v, out.value)
    out, x = ctypes.c_int(-1), ctypes.c_double(0.0)
    L.mytest(ctypes.byref(out), ctypes.byref(x))
    assert out.value == 0
    assert struct.unpack("<Q", struct.pack("<d", x.value))[0] == 0x7FF00000000007A2


@pytest.mark.parametrize("a,b,t", [(0.5, 1.0, 0.3), (0.5, 1.0, 5.0), (3.0, 2.0, 0.2),
                                   (3.0, 1.0, 2.5), (50.0, 1.0, 40.0), (50.0, 1.0, 49.5),
                                   (2.0, 0.5, 100.0), (1.0, 1.0, 0.001), (1.5, 3.0, 0.2)])
def test_rrtgamma_matches_truncated_gamma(a, b, t):
    """All four rejection regimes of the restated r.rtgamma_rate (bbo_rtgamma_std)."""
    x = oracle.rrtgamma_batch(np.full(N, a), np.full(N, b), np.full(N, t), seed=5)
    assert np.all((x > 0) & (x <= t))
    g = ss.gamma(a, scale=1.0 / b)
    assert ss.kstest(x, lambda v: g.cdf(v) / g.cdf(t)).pvalue > 1e-3
