"""The near-identity decision's bound sums folded into the split lambda + X u launch
(bb_set_tuning key 17, bb_nid.hip k_lambda_xs): its stream workgroups add
D_j |x_j|^2 over the thresholds for the columns they stream, in place of k_nid_sums; k_nid_reduce
adds the partials and decides (key 17 = 1, the default) or, unsharded, the launch's last stream
workgroup does (2); 0 is the separate k_nid_sums + k_nid_reduce.  The
sums are added in another order, and the bound is rounded up to 12 significant bits before it
reaches the decision, so the fold changes no bit of the chain: the same path, the same
iterates, the same beta / lambda / tau / sig2 -- unsharded (C3's shape and a narrower one) and
in a 2-member shard group (each member's partials reduced by launch_nid_reduce, then
exchanged)."""
import numpy as np
import pytest

from tests.test_nid_gpu import SEED, _engine

pytestmark = pytest.mark.gpu


def _problem(n, p):
    import bench
    X = bench.make_columns(n, 0, p)
    y, _ = bench.make_problem_y(n, p)
    return X, y


@pytest.mark.parametrize("n,p", [(200, 45000), (2000, 50000)])
def test_fold_same_chain_unsharded(gpu_lib, n, p):
    bb = gpu_lib
    X, y = _problem(n, p)
    out = []
    for fold in (1, 2, 0):
        old = bb.set_tuning(17, fold)
        try:
            e = _engine(bb, X, y, n, p)
            e.init_state()
            e.run(1, 12)
            e.sync()
            out.append((e.state(), e.nid_stats()))
            assert e.error_flags() == 0
            e.close()
        finally:
            bb.set_tuning(17, old)
    b, sb = out[-1]
    assert sb["cheb_sweeps"] >= 10, sb
    for a, sa in out[:-1]:
        assert sa == sb, (sa, sb)
        for k in ("beta", "lambda"):
            assert np.array_equal(a[k], b[k]), (k, np.max(np.abs(a[k] - b[k])))
        assert a["tau"] == b["tau"] and a["sig2"] == b["sig2"]


def test_fold_same_chain_shard_group(gpu_lib):
    bb = gpu_lib
    n, p, world = 200, 90000, 2
    X, y = _problem(n, p)
    per = p // world
    out = []
    for fold in (1, 0):
        old = bb.set_tuning(17, fold)
        try:
            shards = []
            for r in range(world):
                cfg = bb.EngineConfig(n=n, p=p, p_local=per, j0=r * per, rank=r, world=world,
                                      seed=SEED, stream=0, trace_capacity=1)
                shards.append(bb.Engine(cfg, np.asfortranarray(X[:, r * per:(r + 1) * per]), y))
            grp = bb.ShardGroup(shards)
            grp.init_state()
            grp.run(1, 8)
            grp.sync()
            out.append(([e.state() for e in shards], [e.nid_stats() for e in shards]))
            assert all(e.error_flags() == 0 for e in shards)
            grp.close()
            for e in shards:
                e.close()
        finally:
            bb.set_tuning(17, old)
    (pa, sa), (pb, sb) = out
    assert sa == sb, (sa, sb)
    assert sa[0]["cheb_sweeps"] >= 6, sa
    for qa, qb in zip(pa, pb):
        for k in ("beta", "lambda"):
            assert np.array_equal(qa[k], qb[k]), k
        assert qa["tau"] == qb["tau"] and qa["sig2"] == qb["sig2"]
