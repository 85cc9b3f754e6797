"""The stable sampler's own log and sin (bb_sampler.h bb_log, bb_sin_0pi) restated in numpy with
the constants read from the header, checked against 120-bit references (mpmath).

The device functions are straight-line IEEE double arithmetic (the library is compiled with
-ffp-contract=off, and the frexp / division steps are exact or correctly rounded), so this
float64 emulation computes the same bits; the GPU parity tests then compare the draws built on
them with the oracle's libm-based ones (retstable.cpp:18-29, 94-271)."""
import os
import re

import numpy as np
import pytest

mpmath = pytest.importorskip("mpmath")

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "bayesbridge_amd", "csrc", "bb_sampler.h")


def _consts(func):
    src = open(HDR).read()
    body = src[src.index(f"double {func}(double x)"):]
    body = body[:body.index("#endif")]
    return {k: float(v) for k, v in re.findall(r"(\w+) = (-?[0-9.]+(?:e[-+][0-9]+)?)", body)}


def bb_log(x):
    c = _consts("bb_log")
    x = np.asarray(x, dtype=np.float64)
    m, e = np.frexp(x)
    m = m * 2.0
    e = e - 1
    big = m > 1.41421356237309504880
    m = np.where(big, m * 0.5, m)
    e = np.where(big, e + 1, e)
    f = m - 1.0
    s = f / (2.0 + f)
    z = s * s
    w = z * z
    t1 = w * (c["Lg2"] + w * (c["Lg4"] + w * c["Lg6"]))
    t2 = z * (c["Lg1"] + w * (c["Lg3"] + w * (c["Lg5"] + w * c["Lg7"])))
    R = t2 + t1
    hfsq = 0.5 * f * f
    dk = e.astype(np.float64)
    with np.errstate(all="ignore"):
        r = dk * c["ln2_hi"] - ((hfsq - (s * (hfsq + R) + dk * c["ln2_lo"])) - f)
    return np.where(x == 0, -np.inf, np.where(x == np.inf, np.inf, np.where(x > 0, r, np.nan)))


def bb_sin_0pi(x):
    c = _consts("bb_sin_0pi")
    x = np.asarray(x, dtype=np.float64)
    y = np.where(x > 1.57079632679489661923, (c["pi_hi"] - x) + c["pi_lo"], x)
    z = y * y
    p = c["c23"]
    for k in (21, 19, 17, 15, 13, 11, 9, 7, 5, 3):
        p = p * z + c[f"c{k}"]
    return y + (y * z) * p


def _ulps(a, x, ref):
    mpmath.mp.prec = 120
    t = np.array([float(ref(mpmath.mpf(float(v)))) for v in x])
    return np.abs(a - t) / np.spacing(np.abs(t))


def test_bb_log_within_one_ulp():
    rng = np.random.default_rng(11)
    # uniforms (the attempts' -log U), the sinc and power arguments, the whole exponent range,
    # subnormals and the neighbourhood of 1
    x = np.concatenate([rng.uniform(0, 1, 3000), np.exp(rng.uniform(-700, 700, 3000)),
                        rng.uniform(0.5, 2, 2000), 1 + rng.uniform(-1e-7, 1e-7, 1000),
                        np.ldexp(rng.uniform(1, 2, 200), rng.integers(-1070, -1023, 200))])
    u = _ulps(bb_log(x), x, mpmath.log)
    assert u.max() <= 1.0, u.max()


def test_bb_log_special_values():
    r = bb_log(np.array([0.0, -0.0, np.inf, -1.0, np.nan, 1.0]))
    assert r[0] == -np.inf and r[1] == -np.inf and r[2] == np.inf
    assert np.isnan(r[3]) and np.isnan(r[4]) and r[5] == 0.0


def test_bb_sin_0pi_within_two_ulp():
    rng = np.random.default_rng(12)
    x = np.concatenate([rng.uniform(0, np.pi, 4000), np.pi - np.exp(rng.uniform(-40, 0, 1000)),
                        np.exp(rng.uniform(-20, 0, 1000)), [np.pi / 2, np.pi / 4, 1e-300]])
    x = x[(x > 0) & (x < np.pi)]
    u = _ulps(bb_sin_0pi(x), x, mpmath.sin)
    assert u.max() <= 2.0, u.max()
