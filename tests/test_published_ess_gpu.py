"""The published ESS check of tests/test_published_ess_cpu.py through the product's .C
entry point on the GPU (bridge_reg_stable, DB design, stable and orthogonal-design stable)."""
import numpy as np
import pytest

from bayesbridge_amd.diagnostics import effective_size
from tests.test_published_ess_cpu import BURN, NSAMP, NSIM, check_against_published
from tools.published_ess import designs, qr_q

pytestmark = pytest.mark.gpu


def ess_table(run):
    """run(sim) -> beta trace (M x p) of one GPU chain; the per-coefficient medians of ESS over
    the NSIM simulations and each one's relative standard error (as the CPU test's table)."""
    ess = np.array([effective_size(run(s)) for s in range(NSIM)])  # NSIM x p
    med = np.median(ess, axis=0)
    rse = 1.2533 * ess.std(axis=0, ddof=1) / np.sqrt(NSIM) / med
    return med, rse


@pytest.mark.parametrize("method", ["stable", "stable_orth"])
def test_c_entry_reproduces_published_ess(gpu_lib, method, capsys):
    bb = gpu_lib
    X, y = designs()["DB"]
    orth = method == "stable_orth"
    Xm = qr_q(X) if orth else X

    def run(s):
        bb.set_seed(1000 + s)
        return bb.bridge_reg_stb(y, Xm, nsamp=NSAMP, burn=BURN, alpha=0.5, ortho=orth)["beta"]

    med, rse = ess_table(run)
    check_against_published(med, rse, ("DB", method), capsys)
