"""coda::effectiveSize restatement (bayesbridge_amd.diagnostics) on processes with known
integrated autocorrelation: ESS ~ n (1 - phi) / (1 + phi) for an AR(1)."""
import numpy as np
import pytest

from bayesbridge_amd.diagnostics import effective_size, sum_stat


def ar1(phi, n, seed):
    rng = np.random.default_rng(seed)
    e = rng.standard_normal(n)
    x = np.empty(n)
    x[0] = e[0] / np.sqrt(1 - phi * phi)
    for i in range(1, n):
        x[i] = phi * x[i - 1] + e[i]
    return x


@pytest.mark.parametrize("phi", [0.0, 0.5, 0.9, -0.3])
def test_ess_ar1(phi):
    n = 40000
    ess = effective_size(ar1(phi, n, 3))[0]
    target = n * (1 - phi) / (1 + phi)
    assert abs(ess / target - 1) < 0.1, (ess, target)


def test_ess_columns_and_constant():
    x = np.column_stack([ar1(0.5, 5000, 1), np.ones(5000)])
    ess = effective_size(x)
    assert ess[1] == 0.0 and ess[0] > 1000


def test_sum_stat():
    x = np.column_stack([ar1(0.2, 4000, i) for i in range(3)])
    s = sum_stat(x, 2.0)
    assert np.allclose(s["esr"], s["ess"] / 2.0)
    assert s["ess_summary"][0] <= s["ess_summary"][1] <= s["ess_summary"][2]
