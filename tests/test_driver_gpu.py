"""The .C drivers' host machinery on the GPU: the device trace ring with chunked copy-out,
interrupt polling (simulated through bb_debug_interrupt_after), and the single-process
RCCL shard group that bridge_reg_stable uses across devices (exercised at one device, the
only count a one-GPU box can hold: RCCL cannot place two ranks on one device)."""
import numpy as np
import pytest

from tests.conftest import synthetic_problem

pytestmark = pytest.mark.gpu

SEED = 0xB4E5B41D6E


def _same(a, b, keys=("beta", "lambda", "sig2", "tau", "alpha")):
    for k in keys:
        assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("n,p", [(100, 20), (60, 700)])
def test_trace_ring_copy_out_is_exact(gpu_lib, n, p):
    """A 16-slot ring copied out every 16 samples gives the whole-run traces bit for bit."""
    bb = gpu_lib
    X, y, _ = synthetic_problem(n, p, seed=3)
    bb.set_seed(SEED)
    full = bb.bridge_reg_stb(y, X, nsamp=100, burn=15)
    assert bb.last_call_info()["trace_capacity"] == 100
    bb.set_trace_budget(1)
    try:
        bb.set_seed(SEED)
        ring = bb.bridge_reg_stb(y, X, nsamp=100, burn=15)
        assert bb.last_call_info()["trace_capacity"] == 16
    finally:
        bb.set_trace_budget(0)
    _same(full, ring)


def test_trace_ring_triangle(gpu_lib):
    bb = gpu_lib
    X, y, _ = synthetic_problem(80, 10, seed=4)
    bb.set_seed(SEED + 1)
    full = bb.bridge_reg_tri(y, X, nsamp=50, burn=5, extras=True)
    bb.set_trace_budget(1)
    try:
        bb.set_seed(SEED + 1)
        ring = bb.bridge_reg_tri(y, X, nsamp=50, burn=5, extras=True)
    finally:
        bb.set_trace_budget(0)
    _same(full, ring, ("beta", "u", "w", "shape", "sig2", "tau"))


@pytest.mark.parametrize("p,block", [(40, 10), (20, 50)])
def test_interrupt_returns_partial_traces_and_rerun_is_clean(gpu_lib, p, block):
    """An interrupt at the 4th poll (burn-in is 2 blocks, so it lands after 2 blocks of MCMC
    sweeps) stops the chain, returns the samples drawn so far -- identical to the same
    samples of an uninterrupted run -- and leaves the library ready for the next call.
    Blocks are 10 sweeps on the general path (p = 40) and 50 on the fused single-launch
    path (p = 20)."""
    bb = gpu_lib
    X, y, _ = synthetic_problem(100, p, seed=5)
    burn, nsamp = 2 * block - 1, 6 * block
    bb.set_seed(SEED + 2)
    full = bb.bridge_reg_stb(y, X, nsamp=nsamp, burn=burn)
    bb.set_seed(SEED + 2)
    bb.debug_interrupt_after(3)
    part = bb.bridge_reg_stb(y, X, nsamp=nsamp, burn=burn)
    info = bb.last_call_info()
    assert info["interrupted"]
    done = 1 + 2 * block  # sample 0 (after burn-in) + two blocks of MCMC sweeps
    for k in ("beta", "lambda"):
        assert np.array_equal(part[k][:done], full[k][:done]), k
        assert not part[k][done:].any(), k
    for k in ("sig2", "tau"):
        assert np.array_equal(part[k][:done], full[k][:done]), k
    bb.set_seed(SEED + 2)
    again = bb.bridge_reg_stb(y, X, nsamp=nsamp, burn=burn)
    assert not bb.last_call_info()["interrupted"]
    _same(full, again)


def test_interrupt_during_burn_in(gpu_lib):
    bb = gpu_lib
    X, y, _ = synthetic_problem(60, 400, seed=6)
    bb.debug_interrupt_after(0)
    out = bb.bridge_reg_stb(y, X, nsamp=30, burn=50)
    assert bb.last_call_info()["interrupted"]
    assert np.all(np.isfinite(out["beta"][0])) and not out["beta"][1:].any()


@pytest.mark.parametrize("mode", ["rccl", "ondevice"])
def test_one_member_group_equals_single_engine(gpu_lib, mode):
    """A one-member shard group (RCCL communicator from ncclCommInitAll, or the on-device
    sums) reproduces the communicator-free engine bit for bit.  Shard-group members decide the
    fp64 near-identity plan only, so the on-device member is compared with
    the engine run with the mixed-precision plan off (bb_set_tuning key 10 = 0)."""
    bb = gpu_lib
    n, p = 150, 2000
    X, y, _ = synthetic_problem(n, p, seed=31)
    outs = []
    for grouped in (False, True):
        e = bb.Engine(bb.EngineConfig(n=n, p=p, seed=SEED, stream=11, method=2,
                                      trace_capacity=8), X, y)
        if grouped:
            g = bb.ShardGroup([e], rccl=(mode == "rccl"))
            g.init_state()
            g.run(1, 8, first_slot=0, slot_step=1)
            g.sync()
        else:
            old = bb.set_tuning(10, 1 if mode == "rccl" else 0)
            try:
                e.init_state()
                e.run(1, 8, first_slot=0, slot_step=1)
                e.sync()
            finally:
                bb.set_tuning(10, old)
        outs.append(e.trace(0, 8))
        if grouped:
            g.close()
        e.close()
    for k in ("beta", "lambda", "sig2", "tau"):
        assert np.array_equal(outs[0][k], outs[1][k]), k


def test_c_entry_device_count_control(gpu_lib):
    """Sharding a .C chain over devices is opt-in: the default is one device;
    bb_set_device_count(0) allows every visible device (>= 4096 columns each)."""
    bb = gpu_lib
    X, y, _ = synthetic_problem(50, 9000, seed=7)
    bb.set_seed(SEED + 3)
    a = bb.bridge_reg_stb(y, X, nsamp=6, burn=2)
    assert bb.last_call_info()["devices"] == 1
    bb.set_device_count(0)
    try:
        bb.set_seed(SEED + 3)
        b = bb.bridge_reg_stb(y, X, nsamp=6, burn=2)
        assert bb.last_call_info()["devices"] == min(bb.device_count(), 9000 // 4096)
    finally:
        bb.set_device_count(1)
    if bb.device_count() == 1:
        _same(a, b)


def test_c_entry_device_count_control_dot_c(gpu_lib):
    """The same control through R's calling convention: .C("bb_set_device_count_C", k) with
    k = 0, 1 and 2, each followed by a .C sampler call and .C("bb_last_call_info_C", ...)."""
    bb = gpu_lib
    X, y, _ = synthetic_problem(50, 9000, seed=8)
    nvis = bb.device_count()
    try:
        for k in (0, 1, 2):
            bb.dot_c("bb_set_device_count_C", k)
            bb.dot_c("bb_set_seed_C", float(SEED + 4))
            out = bb.bridge_reg_stb(y, X, nsamp=4, burn=1)
            d, cap, intr = bb.dot_c("bb_last_call_info_C", 0, 0, 0)
            want = min(nvis if k == 0 else k, nvis, 9000 // 4096)
            assert int(d[0]) == want, (k, int(d[0]))
            assert int(cap[0]) == 4 and int(intr[0]) == 0
            assert np.all(np.isfinite(out["beta"]))
    finally:
        bb.set_device_count(1)


def test_rccl_group_member_failure_aborts_and_poisons(gpu_lib):
    """A member that fails part-way through a run (bb_debug_fail_member) makes the RCCL group
    abort its communicators, return an error instead of waiting on collectives that can never
    be matched, and refuse further runs; closing it does not hang, and a fresh group on the
    same device runs normally (one member: the only RCCL group a one-GPU box can hold)."""
    bb = gpu_lib
    n, p = 120, 1500
    X, y, _ = synthetic_problem(n, p, seed=32)
    e = bb.Engine(bb.EngineConfig(n=n, p=p, seed=SEED, stream=12, method=2, trace_capacity=4),
                  X, y)
    g = bb.ShardGroup([e], rccl=True)
    g.init_state()
    bb.debug_fail_member(0, 3)
    with pytest.raises(RuntimeError, match="injected failure"):
        g.run(1, 8, first_slot=-1)
    with pytest.raises(RuntimeError, match="unusable"):
        g.run(9, 1, first_slot=-1)
    g.close()
    e.close()
    # the hook is one-shot, and the device is usable again
    e2 = bb.Engine(bb.EngineConfig(n=n, p=p, seed=SEED, stream=12, method=2, trace_capacity=4),
                   X, y)
    g2 = bb.ShardGroup([e2], rccl=True)
    g2.init_state()
    g2.run(1, 4, first_slot=0)
    g2.sync()
    assert np.all(np.isfinite(e2.trace(0, 4)["beta"]))
    g2.close()
    e2.close()
