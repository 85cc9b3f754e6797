"""The column-sharded near-identity solve on the GPU (bb_engine.cpp shard_solve, bb_nid.hip
k_nid_partials / k_nid_decide_from).  Shards exchange their bound sums,
decide the path from the reduced sums (the same bits on every member), then either run the
Chebyshev iteration with one exchange of X_k u_k and one per product E d, or exchange the
partial Gram as before.  An on-device shard group (the group's reduce as the exchange; the
RCCL ranks of a multi-GPU job run the same stages through ncclAllReduce) against the
unsharded engine, teacher-forced from identical states across the regimes: near-null (the
Chebyshev path on every member), intermediate, fitted (the factor).  CPU restatement:
tests/test_sharded_cpu.py::test_sharded_near_identity_matches_unsharded."""
import numpy as np
import pytest

from tests.test_gpu_parity import flips, rel_err
from tests.test_nid_gpu import SEED, _design

pytestmark = pytest.mark.gpu


def _shards(bb, X, y, n, p, world, gram_mode):
    per = (p + world - 1) // world
    out = []
    for r in range(world):
        j0, j1 = r * per, min(p, (r + 1) * per)
        cfg = bb.EngineConfig(n=n, p=p, p_local=j1 - j0, j0=j0, rank=r, world=world, seed=SEED,
                              stream=0, true_alpha=0.5, trace_capacity=1, gram_mode=gram_mode)
        Xr = X[:, j0:j1]
        out.append(bb.Engine(cfg, Xr if not isinstance(Xr, np.ndarray) else
                             np.asfortranarray(Xr), y))
    return out, per


@pytest.mark.parametrize("kind,gram_mode,world", [("dense", 1, 2), ("dense", 0, 3),
                                                  ("sparse", 1, 2), ("dense", 1, 3)])
@pytest.mark.parametrize("scale", [1e-6, 1e-3, 3e-2, 1.0])
def test_shard_group_near_identity(gpu_lib, kind, gram_mode, world, scale):
    bb = gpu_lib
    n, p = 200, 2400
    X, y, btrue = _design(kind, n, p, 31)
    rng = np.random.default_rng(8)
    base = btrue if btrue is not None else np.zeros(p)
    beta = base * scale + scale * rng.standard_normal(p)
    # the unsharded reference with the near-identity path off: the Gram + Cholesky draw
    old = bb.set_tuning(6, 0)
    try:
        single = bb.Engine(bb.EngineConfig(n=n, p=p, seed=SEED, stream=0, true_alpha=0.5,
                                           trace_capacity=1, gram_mode=gram_mode), X, y)
        single.init_state()
    finally:
        bb.set_tuning(6, old)
    shards, per = _shards(bb, X, y, n, p, world, gram_mode)
    grp = bb.ShardGroup(shards)
    grp.init_state()
    modes = []
    for t in (3, 4, 5):
        single.set_state(beta, scale, 1.0, 0.5)
        for r, e in enumerate(shards):
            e.set_state(beta[r * per:min(p, (r + 1) * per)], scale, 1.0, 0.5)
        old = bb.set_tuning(6, 0)
        try:
            single.run(t, 1)
            single.sync()
        finally:
            bb.set_tuning(6, old)
        grp.run(t, 1)
        grp.sync()
        s1 = single.state()
        parts = [e.state() for e in shards]
        st = [e.nid_stats() for e in shards]
        assert len({q["mode"] for q in st}) == 1, st  # every member took the same path
        modes.append(st[0]["mode"])
        bg = np.concatenate([q["beta"] for q in parts])
        lg = np.concatenate([q["lambda"] for q in parts])
        for q in parts:
            assert abs(q["tau"] - s1["tau"]) <= 1e-12 * s1["tau"]
            assert abs(q["sig2"] - s1["sig2"]) <= 1e-11 * s1["sig2"]
        assert flips(lg, s1["lambda"]) == 0
        assert rel_err(bg, s1["beta"]) < 1e-10, (t, st[0], rel_err(bg, s1["beta"]))
        beta = s1["beta"]
    print(f"\n[{kind} gram_mode={gram_mode} world={world} scale={scale}] iterates {modes}")
    if scale <= 1e-6:
        assert all(m >= 1 for m in modes), modes
    if scale >= 1.0:
        assert all(m == 0 for m in modes), modes
    assert single.error_flags() == 0 and all(e.error_flags() == 0 for e in shards)
    grp.close()
    single.close()
    for e in shards:
        e.close()


def test_shard_group_free_run_agrees_with_single(gpu_lib):
    """From the reference start (beta0 = 0) a 2-member group and the unsharded engine
    (both with the near-identity path) free-run 12 sweeps of the near-null regime: the chains
    agree (the solves differ only below 2^-56 relative and in the Gram summation order)."""
    bb = gpu_lib
    n, p = 300, 4000
    X, y, _ = _design("dense", n, p, 33)
    single = bb.Engine(bb.EngineConfig(n=n, p=p, seed=SEED, stream=1, trace_capacity=16), X, y)
    single.init_state()
    shards, per = [], p // 2
    for r in range(2):
        cfg = bb.EngineConfig(n=n, p=p, p_local=per, j0=r * per, rank=r, world=2, seed=SEED,
                              stream=1, trace_capacity=16)
        shards.append(bb.Engine(cfg, np.asfortranarray(X[:, r * per:(r + 1) * per]), y))
    grp = bb.ShardGroup(shards)
    grp.init_state()
    single.run(1, 12)
    grp.run(1, 12)
    grp.sync()
    s1 = single.state()
    bg = np.concatenate([e.state()["beta"] for e in shards])
    st = [e.nid_stats() for e in shards]
    assert st[0]["cheb_sweeps"] >= 6, st
    assert rel_err(bg, s1["beta"]) < 1e-8, rel_err(bg, s1["beta"])
    grp.close()
    single.close()
    for e in shards:
        e.close()
