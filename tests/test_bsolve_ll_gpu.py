"""The persistent backward solve's tagged-word hand-off (bb_set_tuning key 20, bb_kernels.hip
k_bsolve_persist): each solved 64-row block travels to the next as 64-bit words holding 32 bits
of the value and the solve's epoch, polled directly, instead of a flag followed by a load of the
data.  The arithmetic is the same, so the chains are bit-identical with the hand-off on and
off: a p <= n chain (the p x p factor and solve, BridgeRegression.cpp:552-575) and a p > n chain
in the fitted regime (the Woodbury n x n factor, near-identity path off), several sweeps each,
so consecutive solves also exercise the epoch tags."""
import numpy as np
import pytest

from tests.conftest import synthetic_problem
from tests.test_nid_gpu import SEED, _engine

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,p,fitted", [(400, 300, False), (300, 1200, True), (700, 3000, True)])
def test_bsolve_ll_same_chain(gpu_lib, n, p, fitted):
    bb = gpu_lib
    X, y, btrue = synthetic_problem(n, p, seed=n + p)
    out = []
    for ll in (1, 0):
        o20, o6 = bb.set_tuning(20, ll), bb.set_tuning(6, 0)
        try:
            e = _engine(bb, X, y, n, p)
            e.init_state()
            if fitted:
                e.set_state(btrue, 1.0, 1.0, 0.5)
            e.run(3, 6)
            e.sync()
            out.append(e.state())
            assert e.error_flags() == 0
            e.close()
        finally:
            bb.set_tuning(20, o20)
            bb.set_tuning(6, o6)
    a, b = out
    for k in ("beta", "lambda"):
        assert np.array_equal(a[k], b[k]), (k, np.max(np.abs(a[k] - b[k])))
    assert a["tau"] == b["tau"] and a["sig2"] == b["sig2"]
    assert np.all(np.isfinite(a["beta"]))
