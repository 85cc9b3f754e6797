"""The lambda launches' two occupancy instances (bb_set_tuning key 4) draw the same chain.

k_lambda_spec<16> (1024 < p <= 50000) and k_lambda_cb<8> (p > 50000) each exist at their
register-minimal 3 waves per SIMD and capped at 128 VGPRs for 4 waves per SIMD (and
k_lambda_cb with its sampler bodies inlined, key 4 bit 2); all run
the sequential retstable_LD loop of every coefficient on its own counters
(retstable.cpp:94-271, BridgeRegression.cpp:506-510), so the traces must be bit-identical."""
import numpy as np
import pytest

from tests.conftest import synthetic_problem

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,p", [(200, 3000), (50, 45000), (60, 60000)])
def test_lambda_occupancy_variants_same_chain(gpu_lib, n, p):
    bb = gpu_lib
    X, y, _ = synthetic_problem(n, p, seed=11, s=10)
    traces = []
    old = bb.set_tuning(4, -1)
    old6 = bb.set_tuning(6, 0)  # the separate lambda launch on every sweep (no fused X u)
    try:
        for occ in (0, 3, 4, 5, 12):
            bb.set_tuning(4, occ)
            e = bb.Engine(bb.EngineConfig(n=n, p=p, true_alpha=0.5, method=2, trace_capacity=6,
                                          seed=77, stream=0), X, y)
            e.init_state()
            e.run(1, 6, first_slot=0)
            e.sync()
            assert e.error_flags() == 0
            traces.append(e.trace(0, 6))
            e.close()
    finally:
        bb.set_tuning(4, old)
        bb.set_tuning(6, old6)
    for k in ("beta", "lambda", "tau", "sig2"):
        for tr in traces[1:]:
            assert np.array_equal(traces[0][k], tr[k]), k


def test_lambda_lane_counts_same_chain(gpu_lib):
    """p = 45000 runs k_lambda_spec<8> by default; forcing 4 (one outer attempt of 4 inner
    attempts per round), 16, 32 or 64 lanes per coefficient (bb_set_tuning key 5) must give
    the same chain bit for bit."""
    bb = gpu_lib
    n, p = 40, 45000
    X, y, _ = synthetic_problem(n, p, seed=12, s=8)
    traces = []
    old = bb.set_tuning(5, -1)
    old6 = bb.set_tuning(6, 0)  # the separate lambda launch on every sweep (no fused X u)
    try:
        for lanes in (0, 4, 16, 32, 64):
            bb.set_tuning(5, lanes)
            e = bb.Engine(bb.EngineConfig(n=n, p=p, true_alpha=0.5, method=2, trace_capacity=5,
                                          seed=78, stream=0), X, y)
            e.init_state()
            e.run(1, 5, first_slot=0)
            e.sync()
            assert e.error_flags() == 0
            traces.append(e.trace(0, 5))
            e.close()
    finally:
        bb.set_tuning(5, old)
        bb.set_tuning(6, old6)
    for tr in traces[1:]:
        for k in ("beta", "lambda", "tau", "sig2"):
            assert np.array_equal(traces[0][k], tr[k]), k


@pytest.mark.parametrize("n,p", [(60, 60000), (200, 90000)])
def test_lambda_tail_lending_same_chain(gpu_lib, n, p):
    """bb_set_tuning key 15: the inlined continuous-batching launch (k_lambda_cl) lends the
    lanes of a wave's idle groups to its unfinished draws once its range is used up
    (wave_draw_rounds); with the key off (k_lambda_cb_in) every group finishes its own draw.
    The same attempts in the same order: the chains are bit-identical."""
    bb = gpu_lib
    X, y, _ = synthetic_problem(n, p, seed=13, s=10)
    traces = []
    old = bb.set_tuning(15, -1)
    old6 = bb.set_tuning(6, 0)  # the separate lambda launch on every sweep (no fused X u)
    try:
        for lend in (1, 0):
            bb.set_tuning(15, lend)
            e = bb.Engine(bb.EngineConfig(n=n, p=p, true_alpha=0.5, method=2, trace_capacity=6,
                                          seed=79, stream=0), X, y)
            e.init_state()
            e.run(1, 6, first_slot=0)
            e.sync()
            assert e.error_flags() == 0
            traces.append(e.trace(0, 6))
            e.close()
    finally:
        bb.set_tuning(15, old)
        bb.set_tuning(6, old6)
    for k in ("beta", "lambda", "tau", "sig2"):
        assert np.array_equal(traces[0][k], traces[1][k]), k
