"""The benchmarking key 16 (forced Chebyshev iterate count, used to time a C3 rank's product
count on the per-rank proxy) runs exactly that many iterates per near-identity
sweep."""
import numpy as np
import pytest

from tests.conftest import synthetic_problem

pytestmark = pytest.mark.gpu


def test_forced_iterates_run_that_many(gpu_lib):
    bb = gpu_lib
    n, p = 300, 6000
    X, y, _ = synthetic_problem(n, p, seed=9, s=0)  # near-null: every sweep near identity
    old = bb.set_tuning(16, -1)
    try:
        for k in (2, 4):
            bb.set_tuning(16, k)
            e = bb.Engine(bb.EngineConfig(n=n, p=p, true_alpha=0.5, method=2, trace_capacity=4,
                                          seed=3, stream=0), X, y)
            e.init_state()
            s0 = e.nid_stats()
            e.run(1, 4, first_slot=0)
            e.sync()
            s1 = e.nid_stats()
            assert e.error_flags() == 0
            sweeps = s1["cheb_sweeps"] - s0["cheb_sweeps"]
            assert sweeps == 4, (s0, s1)
            assert s1["products"] - s0["products"] == sweeps * (k - 1), (k, s0, s1)
            e.close()
    finally:
        bb.set_tuning(16, old)
