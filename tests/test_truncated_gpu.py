"""GPU parity of the truncated-distribution .C utilities: the device batch (one lane per
draw) against the oracle on the same Philox counters, per draw to 1e-12 relative (libm vs
ocml last-ulp differences in exp/log/log1p), NaNs where the reference returns NaN."""
import numpy as np
import pytest

import bayesbridge_amd as bb
import oracle

pytestmark = pytest.mark.gpu

rng = np.random.default_rng(17)
M = 5000
CASES = {
    "rtnorm_left": [rng.normal(0, 3, M), rng.normal(0, 2, M), rng.uniform(0.1, 3, M)],
    "rtnorm_both": [np.full(M, -1.0), rng.uniform(-0.9, 8, M), rng.normal(0, 2, M),
                    rng.uniform(0.05, 2, M)],
    "rtnorm": [np.where(rng.random(M) < 0.3, -np.inf, -1.0), np.where(rng.random(M) < 0.3,
               np.inf, 2.0), rng.normal(0, 2, M), rng.uniform(0.1, 2, M)],
    "rtexpon_rate_left": [rng.normal(0, 3, M), rng.uniform(0.1, 5, M)],
    "rtexpon_rate_both": [np.zeros(M), rng.uniform(0.01, 4, M), rng.uniform(0.1, 5, M)],
    "rtexpon_rate": [np.where(rng.random(M) < 0.05, np.nan,
                              np.where(rng.random(M) < 0.05, np.inf, 1.0)),
                     np.where(rng.random(M) < 0.5, np.inf,
                              np.where(rng.random(M) < 0.05, np.nan, 3.0)),
                     rng.uniform(0.1, 5, M)],
}
CASES["rtnorm_both"][1] = np.maximum(CASES["rtnorm_both"][1], -0.5)


@pytest.mark.parametrize("name", sorted(CASES))
def test_trunc_batch_matches_oracle(gpu_lib, name):
    params = CASES[name]
    g = bb.trunc_batch(name, params, seed=123, stream=4)
    o = oracle.trunc_batch(name, params, seed=123, stream=4)
    assert np.array_equal(np.isnan(g), np.isnan(o))
    assert np.array_equal(np.isinf(g), np.isinf(o)) and np.array_equal(g[np.isinf(o)],
                                                                        o[np.isinf(o)])
    ok = np.isfinite(o)
    assert np.allclose(g[ok], o[ok], rtol=1e-12, atol=1e-300)


def test_dotC_wrappers_respect_bounds(gpu_lib):
    x = bb.rtnorm_both(2000, left=-0.5, right=0.25, mu=3.0, sig=0.1)
    assert np.all((x >= -0.5) & (x <= 0.25))
    x = bb.rtnorm_right(2000, right=-4.0)
    assert np.all(x <= -4.0)
    x = bb.rtnorm(2000, mu=1.0, sig=2.0)
    assert abs(x.mean() - 1.0) < 0.2
    x = bb.rtexp(2000, left=1.0, right=2.0, rate=3.0)
    assert np.all((x >= 1.0) & (x <= 2.0))
    assert bb.rtnorm_both(10, left=1.0, right=0.0) is None


def test_rrtgamma_matches_oracle(gpu_lib):
    shape = rng.uniform(0.2, 60, M)
    rate = rng.uniform(0.1, 4, M)
    right_t = shape / rate * rng.uniform(0.01, 2.0, M)  # below and above the mean
    g = bb.rrtgamma_batch(shape, rate, right_t, seed=9, stream=2)
    o = oracle.rrtgamma_batch(shape, rate, right_t, seed=9, stream=2)
    assert np.all((g > 0) & (g <= right_t))
    assert np.allclose(g, o, rtol=1e-12, atol=0)
    x = bb.rrtgamma(1000, shape=2.0, rate=1.0, rtrunc=0.5)
    assert np.all((x > 0) & (x <= 0.5))


def test_gpu_matches_golden_truncated_vectors(gpu_lib):
    """Device truncated draws against the committed fixtures (tests/golden/make_golden.py)."""
    import os

    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "oracle_vectors.npz"))
    seed = 0xB4E5B41D6E
    x = bb.trunc_batch("rtnorm", [g["tn_lo"], g["tn_hi"], g["tn_mu"], g["tn_sig"]], seed, 1)
    assert np.allclose(x, g["tn_rtnorm"], rtol=1e-12, atol=0)
    x = bb.trunc_batch("rtexpon_rate", [g["te_left"], g["te_right"], g["te_rate"]], seed, 2)
    assert np.allclose(x, g["te_rtexpon"], rtol=1e-12, atol=0)
    x = bb.rrtgamma_batch(g["rg_shape"], g["rg_rate"], g["rg_right"], seed, 3)
    assert np.allclose(x, g["rg_x"], rtol=1e-12, atol=0)
