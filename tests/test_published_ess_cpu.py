"""The oracle pinned to the only numbers the reference itself published for this path.

Notes/bbnotes.tex:901-905 (general design) and :955-959 (orthogonal design) give, for the
stable (normal-mixture) sampler on the diabetes design (DB) and its quadratic expansion
(DBI: squares and pairwise interactions, 64 columns), the per-coefficient effective sample
size of beta under the benchmark protocol of Code/R/PublicBenchmark.R:140-310: 10
simulations x 100 000 samples after 10 000 burn-in, alpha = 0.5, sig2 Jeffreys,
nu = tau^-alpha ~ Ga(2, rate 2); per simulation coda::effectiveSize of every beta_j
(sum.stat :112-134), per coefficient the median over the simulations (table.info :276-305),
reported as min / median / max / sd over the 10 coefficients.

Here the compiled oracle chain (oracle/bb_cpu_chain.c: the reference-literal p x p dpotrf
path of BridgeRegression.cpp:552-575, and the orthogonal draw of :514-521) runs that exact
protocol on the reference's data (man/diabetes.Rd:22: unit-L2, zero-mean columns; sklearn's
copy of the same Efron et al. data, tools/published_ess.py) and the four summary statistics
must match the published ones within a band derived from the protocol's own Monte Carlo
spread: the relative standard error of a median over 10 simulations of a coefficient's ESS
(from this run's 10 simulations), times sqrt(2) (two independent runs: ours and the
published one), times 4, floored at 3 % -- i.e. a 4-sigma test.  Both runs are a different
realisation of the same sampler (R's RNG vs Philox), so this pins the sampler's statistical
behaviour, not individual draws: per-value parity with the reference stays unpinned (it
needs R's RNG stream, absent here).  The Boston Housing rows (bbnotes.tex:907-911) need
mlbench data that is not available offline and are not covered.
"""
import numpy as np
import pytest

import oracle
from bayesbridge_amd.diagnostics import effective_size
from tools.published_ess import PUBLISHED, designs, qr_q

NSIM, NSAMP, BURN = 10, 100000, 10000


def _sim_ess(args):
    X, y, method, s = args
    r = oracle.cpu_chain(y, X, NSAMP, burn=BURN, alpha=0.5, method=method, seed=1000 + s,
                         threads=1)
    return effective_size(r["beta"].T)


def ess_table(X, y, method):
    """The NSIM compiled chains (in parallel processes) -> the per-coefficient medians over
    simulations, and each coefficient's relative standard error of that median."""
    import concurrent.futures as cf
    import multiprocessing as mp
    import os

    workers = max(1, min(NSIM, os.cpu_count() or 1))
    with cf.ProcessPoolExecutor(workers, mp_context=mp.get_context("fork")) as ex:
        ess = np.array(list(ex.map(_sim_ess, [(X, y, method, s) for s in range(NSIM)])))
    med = np.median(ess, axis=0)
    # standard error of a median of NSIM draws ~ 1.2533 sd / sqrt(NSIM)
    rse = 1.2533 * ess.std(axis=0, ddof=1) / np.sqrt(NSIM) / med
    return med, rse


def check_against_published(med, rse, key, capsys=None):
    pub = dict(zip(("min", "median", "max", "sd"), PUBLISHED[key][1:]))
    got = {"min": med.min(), "median": np.median(med), "max": med.max(),
           "sd": np.std(med, ddof=1)}
    band = max(0.03, 4.0 * np.sqrt(2.0) * float(np.max(rse)))
    rel = {k: got[k] / pub[k] - 1.0 for k in pub}
    if capsys is not None:
        with capsys.disabled():
            print(f"\n[{key}] ESS min/median/max/sd {got['min']:.0f} / {got['median']:.0f} / "
                  f"{got['max']:.0f} / {got['sd']:.0f} against published {pub['min']:.0f} / "
                  f"{pub['median']:.0f} / {pub['max']:.0f} / {pub['sd']:.0f}; band "
                  f"+-{100 * band:.1f} %, worst {100 * max(abs(v) for v in rel.values()):.1f} %")
    for k in ("min", "median", "max"):
        assert abs(rel[k]) <= band, (key, k, got[k], pub[k], band)
    # the spread over coefficients is itself a statistic of 10 ESS values: twice the band
    assert abs(rel["sd"]) <= 2 * band, (key, "sd", got["sd"], pub["sd"], band)


@pytest.mark.parametrize("design,method", [("DB", "stable"), ("DB", "stable_orth"),
                                           ("DBI", "stable"), ("DBI", "stable_orth")])
def test_oracle_chain_reproduces_published_ess(design, method, capsys):
    """The four published rows reproducible offline (bbnotes.tex:901-905 DB / DBI general,
    :955-959 DB / DBI orthogonal; the Boston rows need mlbench data absent here)."""
    X, y = designs()[design]
    orth = method == "stable_orth"
    med, rse = ess_table(qr_q(X) if orth else X, y, "ortho" if orth else "chol")
    check_against_published(med, rse, (design, method), capsys)
