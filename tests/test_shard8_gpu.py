"""The C3 configuration's own decomposition on one GPU, and the shard protocol's exchange call
sites (VERDICT r4 "next" item 1).

- An 8-member on-device shard group at full C3 size (n = 2000, p = 50000, bench.py's X, y and
  key; 6250 columns per member -- the shard each rank of an 8-GPU job holds): free-running from
  the reference start every member must report the same path on every sweep, then sweeps are
  teacher-forced against the unsharded engine on the near-identity path and from a fitted
  state that must take the Gram + Cholesky path (bb_engine.cpp shard_solve and
  bb_group_run).
- bb_set_tuning key 9 makes a world-1 engine with a 1-rank RCCL communicator run the world > 1
  stage sequence (bound-sum exchange, k_nid_decide_from, the exchanged X u and products), so
  every ncclAllReduce call site of the sharded near-identity path executes; it must be
  bit-identical to the same stages with the on-device group's reduce as the exchange, and to
  a one-member RCCL group (its member thread polls the decision event, bb_engine::wait_event).
"""
import numpy as np
import pytest

from tests.test_gpu_parity import flips, rel_err

pytestmark = pytest.mark.gpu

SEED = 0xB4E5B41D6E  # bench.py's key


def _c3_shards(bb, X, y, n, p, world, cap=1):
    per = (p + world - 1) // world
    shards = []
    for r in range(world):
        j0, j1 = r * per, min(p, (r + 1) * per)
        cfg = bb.EngineConfig(n=n, p=p, p_local=j1 - j0, j0=j0, rank=r, world=world, seed=SEED,
                              stream=0, true_alpha=0.5, trace_capacity=cap,
                              gram_mode=bb.GRAM_OZAKI)
        shards.append(bb.Engine(cfg, np.asfortranarray(X[:, j0:j1]), y))
    return shards, per


def _compare(single, shards, label):
    s1 = single.state()
    parts = [e.state() for e in shards]
    bg = np.concatenate([q["beta"] for q in parts])
    lg = np.concatenate([q["lambda"] for q in parts])
    for q in parts:
        assert abs(q["tau"] - s1["tau"]) <= 1e-12 * s1["tau"], label
        assert abs(q["sig2"] - s1["sig2"]) <= 1e-11 * s1["sig2"], label
    assert flips(lg, s1["lambda"]) == 0, label
    assert np.max(np.abs(lg - s1["lambda"]) / s1["lambda"]) < 1e-10, label
    err = rel_err(bg, s1["beta"])
    assert err < 1e-9, (label, err)
    return s1, err


def test_shard_group_c3_eight_members(gpu_lib, capsys):
    import bench
    bb = gpu_lib
    n, p, world = 2000, 50000, 8
    X = bench.make_columns(n, 0, p)
    y, btrue = bench.make_problem_y(n, p)
    single = bb.Engine(bb.EngineConfig(n=n, p=p, seed=SEED, stream=0, true_alpha=0.5,
                                       gram_mode=bb.GRAM_OZAKI), X, y)
    single.init_state()
    shards, per = _c3_shards(bb, X, y, n, p, world)
    assert per == 6250 and all(e.p_local == 6250 for e in shards)
    del X
    grp = bb.ShardGroup(shards)
    grp.init_state()
    # every member caps the Chebyshev iterations alike (per-shard cost models)
    assert len({e.nid_stats()["kmax"] for e in shards}) == 1

    # free run from the reference start (beta0 = 0): 20 sweeps, the path of every member
    modes = []
    for t in range(1, 21):
        grp.run(t, 1)
        grp.sync()
        st = [e.nid_stats() for e in shards]
        assert len({q["mode"] for q in st}) == 1, (t, [q["mode"] for q in st])
        assert len({q["eps"] for q in st}) == 1, t  # decided from the same reduced sums
        modes.append(st[0]["mode"])
    cheb = sum(m > 0 for m in modes)
    with capsys.disabled():
        print(f"\n[C3 x8 free run] per-sweep iterates {modes}")
    assert cheb == 20, modes  # the near-null regime: every sweep on the Chebyshev path

    # teacher-forced from the group's state: 3 sweeps on the near-identity path
    parts = [e.state() for e in shards]
    beta = np.concatenate([q["beta"] for q in parts])
    tau, sig2 = parts[0]["tau"], parts[0]["sig2"]
    errs = []
    for t in (21, 22, 23):
        single.set_state(beta, tau, sig2, 0.5)
        for r, e in enumerate(shards):
            e.set_state(beta[r * per:(r + 1) * per], tau, sig2, 0.5)
        c0 = single.nid_stats()["cheb_sweeps"]
        g0 = [e.nid_stats()["cheb_sweeps"] for e in shards]
        single.run(t, 1)
        grp.run(t, 1)
        grp.sync()
        assert single.nid_stats()["cheb_sweeps"] == c0 + 1, t
        assert [e.nid_stats()["cheb_sweeps"] for e in shards] == [g + 1 for g in g0], t
        s1, err = _compare(single, shards, f"near-identity t={t}")
        errs.append(err)
        beta, tau, sig2 = s1["beta"], s1["tau"], s1["sig2"]

    # a fitted state: the bound is far above the cap, every member takes the factor
    beta = btrue + 0.01 * np.random.default_rng(6).standard_normal(p)
    single.set_state(beta, 1.0, 1.0, 0.5)
    for r, e in enumerate(shards):
        e.set_state(beta[r * per:(r + 1) * per], 1.0, 1.0, 0.5)
    h0 = single.nid_stats()["chol_sweeps"]
    g0 = [e.nid_stats()["chol_sweeps"] for e in shards]
    single.run(301, 1)
    grp.run(301, 1)
    grp.sync()
    assert single.nid_stats()["chol_sweeps"] == h0 + 1
    assert [e.nid_stats()["chol_sweeps"] for e in shards] == [g + 1 for g in g0]
    assert all(e.nid_stats()["mode"] == 0 for e in shards)
    _, ferr = _compare(single, shards, "fitted")
    with capsys.disabled():
        print(f"[C3 x8] teacher-forced beta rel L2 near-identity {errs}, fitted {ferr:.2e}")
    assert single.error_flags() == 0 and all(e.error_flags() == 0 for e in shards)
    grp.close()
    single.close()
    for e in shards:
        e.close()


def _traces(e, m):
    tr = e.trace(0, m)
    return {k: np.array(tr[k], copy=True) for k in ("beta", "lambda", "sig2", "tau")}


@pytest.mark.parametrize("n,p", [(300, 2400), (2000, 6250)])
def test_forced_shard_protocol_one_rank_rccl(gpu_lib, n, p, capsys):
    """The world > 1 near-identity stages over a 1-rank RCCL communicator (every exchange an
    ncclAllReduce) against the same stages with the on-device group's reduce and in a
    one-member RCCL group: bit-identical traces, both near-null sweeps (the Chebyshev path,
    X u and every product exchanged) and fitted sweeps (the packed Gram exchanged); against
    the unforced engine to rounding."""
    import bench
    bb = gpu_lib
    X = bench.make_columns(n, 0, p)
    y, btrue = bench.make_problem_y(n, p)
    m = 10

    def make():
        return bb.Engine(bb.EngineConfig(n=n, p=p, seed=SEED, stream=3, true_alpha=0.5,
                                         trace_capacity=2 * m, gram_mode=bb.GRAM_OZAKI), X, y)

    def drive(runner, eng):
        runner.init_state()
        runner.run(1, m, first_slot=0)
        runner.sync()
        st0 = eng.nid_stats()
        eng.set_state(btrue + 0.01 * np.random.default_rng(2).standard_normal(p), 1.0, 1.0, 0.5)
        runner.run(m + 1, m, first_slot=m)
        runner.sync()
        return _traces(eng, 2 * m), st0, eng.nid_stats()

    out = {}
    old = bb.set_tuning(9, 1)
    try:
        e = make()
        e.comm_init(bb.Engine.comm_unique_id())
        out["rccl_rank"] = drive(e, e)
        e.close()
        e = make()
        g = bb.ShardGroup([e])
        out["device_group"] = drive(g, e)
        g.close()
        e.close()
        e = make()
        g = bb.ShardGroup([e], rccl=True)
        out["rccl_group"] = drive(g, e)
        g.close()
        e.close()
    finally:
        bb.set_tuning(9, old)
    e = make()
    out["unforced"] = drive(e, e)
    e.close()
    ref, st0, st1 = out["rccl_rank"]
    with capsys.disabled():
        print(f"\n[forced shard protocol n={n} p={p}] near-null {st0}, after fitted {st1}")
    assert st0["cheb_sweeps"] == m and st0["products"] >= m, st0  # every sweep exchanged X u
    assert st1["chol_sweeps"] >= m - 2, st1  # the fitted sweeps exchanged the Gram
    for name in ("device_group", "rccl_group"):
        tr = out[name][0]
        for k in ref:
            assert np.array_equal(tr[k], ref[k]), (name, k)
        assert out[name][1]["cheb_sweeps"] == st0["cheb_sweeps"], name
    un = out["unforced"][0]
    # the unforced engine decides from its own sums with the same certificate and sums X u in
    # another order: the same chain to rounding over the near-null sweeps
    assert rel_err(un["beta"][:, :m], ref["beta"][:, :m]) < 1e-10
    assert np.max(np.abs(un["sig2"][:m] - ref["sig2"][:m]) / ref["sig2"][:m]) < 1e-11
