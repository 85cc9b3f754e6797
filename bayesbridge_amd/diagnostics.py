"""MCMC output diagnostics used by the reference's benchmark protocol.

The reference publishes effective sample size (ESS) and ESS per second (ESR) per
coefficient, computed by ``coda::effectiveSize`` (Code/R/PublicBenchmark.R:112-134,
``sum.stat``).  ``effective_size`` restates coda's estimator: the spectral density of each
trace at frequency 0 from an autoregressive fit (``spectrum0.ar``: ``ar()`` by Yule-Walker
with the order chosen by AIC up to ``10 log10(n)``), and ESS = n var(x) / spec0.
Pure numpy, host-side post-processing of the traces the sampler returns.
"""
from __future__ import annotations

import numpy as np

__all__ = ["effective_size", "sum_stat"]


def _acov(x: np.ndarray, maxlag: int) -> np.ndarray:
    """Biased autocovariances (divisor n) at lags 0..maxlag, as R's acf(type="covariance")."""
    n = x.shape[0]
    xc = x - x.mean()
    m = 1 << int(np.ceil(np.log2(2 * n)))
    f = np.fft.rfft(xc, m)
    ac = np.fft.irfft(f * np.conj(f), m)[: maxlag + 1] / n
    return ac


def _ar_yw_aic(x: np.ndarray, order_max: int | None = None):
    """R's ar.yw(x, aic = TRUE): Levinson-Durbin on the sample autocovariances, the order
    with the smallest AIC = n log(var_k) + 2 k, var.pred = var_k n / (n - (k + 1)).
    Returns (coefficients, var.pred)."""
    n = x.shape[0]
    if order_max is None:
        order_max = int(np.floor(min(n - 1, 10 * np.log10(n))))
    order_max = max(0, min(order_max, n - 1))
    r = _acov(x, order_max)
    if r[0] <= 0:
        return np.zeros(0), 0.0
    # Levinson-Durbin recursion
    best_k, best_aic = 0, n * np.log(r[0])
    phi = np.zeros(0)
    v = r[0]
    coefs = {0: (np.zeros(0), r[0])}
    for k in range(1, order_max + 1):
        acc = r[k] - (phi @ r[k - 1:0:-1] if k > 1 else 0.0)
        kappa = acc / v
        phi = np.concatenate([phi - kappa * phi[::-1], [kappa]])
        v = v * (1.0 - kappa * kappa)
        if v <= 0:
            break
        coefs[k] = (phi.copy(), v)
        aic = n * np.log(v) + 2 * k
        if aic < best_aic:
            best_aic, best_k = aic, k
    ar, v = coefs[best_k]
    var_pred = v * n / (n - (best_k + 1))
    return ar, var_pred


def effective_size(x) -> np.ndarray:
    """coda::effectiveSize of each column of x (samples x parameters; a 1-D trace is one
    parameter): n var(x) / spectrum0.ar(x), 0 where the spectral estimate is 0."""
    x = np.asarray(x, dtype=np.float64)
    if x.ndim == 1:
        x = x[:, None]
    n = x.shape[0]
    out = np.zeros(x.shape[1])
    for j in range(x.shape[1]):
        col = x[:, j]
        if np.all(col == col[0]):
            out[j] = 0.0
            continue
        ar, vp = _ar_yw_aic(col)
        spec = vp / (1.0 - ar.sum()) ** 2
        out[j] = 0.0 if spec == 0 else n * col.var(ddof=1) / spec
    return out


def sum_stat(beta, runtime: float):
    """PublicBenchmark.R:112-134 (sum.stat) without the posterior summaries' formatting:
    per-coefficient ESS and ESR (= ESS / runtime), with their min / median / max."""
    ess = effective_size(beta)
    esr = ess / runtime if runtime > 0 else np.full_like(ess, np.inf)
    return {"ess": ess, "esr": esr,
            "ess_summary": (float(ess.min()), float(np.median(ess)), float(ess.max())),
            "esr_summary": (float(esr.min()), float(np.median(esr)), float(esr.max())),
            "runtime": runtime}
