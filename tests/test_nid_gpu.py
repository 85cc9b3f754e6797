"""The near-identity (Chebyshev) solve of the Woodbury system on the GPU (bb_nid.hip,
DESIGN.md s6.5).  Both paths of a Woodbury sweep -- Gram + Cholesky and the certified
Chebyshev iteration -- solve the same system exactly, so a sweep drawn through either gives
the same beta to rounding; the device decides per sweep from eps = tr(X D X') / sig2.
Checks: the decision (near-null states take the Chebyshev path, fitted states the factor),
per-sweep equality with the path disabled (bb_set_tuning key 6 = 0) for dense (Ozaki and
fp64 Gram) and sparse engines at iteration counts from 2 to ~12, and teacher-forced parity
with the oracle's Cholesky-based Woodbury draw (BridgeRegression.cpp:552-575)."""
import numpy as np
import pytest

import oracle
from oracle import gibbs
from tests.conftest import synthetic_problem
from tests.test_gpu_parity import flips, rel_err

pytestmark = pytest.mark.gpu

SEED = 0xB4E5B41D6E


def _design(kind, n, p, seed):
    if kind == "sparse":
        import bench
        X = bench.make_sparse_columns(n, 0, p, density=0.03, seed=seed)
        rng = np.random.default_rng(seed)
        y = np.asarray(X[:, :8] @ rng.uniform(1, 2, 8)).ravel() + rng.standard_normal(n)
        return X, y - y.mean(), None
    return synthetic_problem(n, p, seed=seed)


def _engine(bb, X, y, n, p, gram_mode=1, stream=0):
    return bb.Engine(bb.EngineConfig(n=n, p=p, seed=SEED, stream=stream, true_alpha=0.5,
                                     trace_capacity=1, gram_mode=gram_mode), X, y)


@pytest.mark.parametrize("kind,gram_mode", [("dense", 1), ("dense", 0), ("sparse", 1)])
@pytest.mark.parametrize("scale", [1e-6, 1e-3, 3e-2])
def test_nid_sweep_equals_cholesky_sweep(gpu_lib, kind, gram_mode, scale):
    """One sweep from the same state through the engine with the near-identity path (auto)
    and with it disabled: same beta to 1e-12 relative.  `scale` sets tau (and beta), so the
    sweeps span eps from ~1e-10 (2 iterates) to ~1e-1 (about 12) -- or the hand-over to the
    factor, reported by mode 0."""
    bb = gpu_lib
    n, p = 200, 2400
    X, y, btrue = _design(kind, n, p, 31)
    rng = np.random.default_rng(7)
    beta = (btrue if btrue is not None else np.zeros(p)) * scale + scale * rng.standard_normal(p)
    auto = _engine(bb, X, y, n, p, gram_mode)
    old = bb.set_tuning(6, 0)
    try:
        off = _engine(bb, X, y, n, p, gram_mode)
        off.init_state()
    finally:
        bb.set_tuning(6, old)
    auto.init_state()
    modes = []
    for t in (3, 4, 5):
        auto.set_state(beta, scale, 1.0, 0.5)
        off.set_state(beta, scale, 1.0, 0.5)
        auto.run(t, 1)
        old = bb.set_tuning(6, 0)
        try:
            off.run(t, 1)
            off.sync()
        finally:
            bb.set_tuning(6, old)
        a, o = auto.state(), off.state()
        st = auto.nid_stats()
        modes.append(st["mode"])
        assert a["tau"] == o["tau"] and a["sig2"] == o["sig2"]
        assert np.array_equal(a["lambda"], o["lambda"])
        assert rel_err(a["beta"], o["beta"]) < 1e-12, (t, st, rel_err(a["beta"], o["beta"]))
        beta = o["beta"]
    assert off.nid_stats()["cheb_sweeps"] == 0
    if scale <= 1e-6:
        assert all(m >= 1 for m in modes), modes  # the near-identity path was taken
    print(f"\n[{kind} gram_mode={gram_mode} scale={scale}] iterates per sweep {modes}")
    assert auto.error_flags() == 0 and off.error_flags() == 0
    auto.close()
    off.close()


@pytest.mark.parametrize("n,p", [(96, 700), (128, 1500)])
def test_nid_small_dense_partial_sums(gpu_lib, n, p):
    """Narrow dense designs whose E-apply / X u passes write fewer than 128 partial n-vectors
    (k_cheb_init / k_cheb_step then sum them in 64-row workgroups, the sparse engine's layout,
    instead of 8-row ones): sweeps with the near-identity path on and off agree to 1e-12."""
    bb = gpu_lib
    X, y, btrue = synthetic_problem(n, p, seed=61)
    rng = np.random.default_rng(9)
    auto = _engine(bb, X, y, n, p)
    old = bb.set_tuning(6, 0)
    try:
        off = _engine(bb, X, y, n, p)
        off.init_state()
    finally:
        bb.set_tuning(6, old)
    auto.init_state()
    modes = []
    for t, scale in ((3, 1e-6), (4, 1e-3)):
        beta = btrue * scale + scale * rng.standard_normal(p)
        auto.set_state(beta, scale, 1.0, 0.5)
        off.set_state(beta, scale, 1.0, 0.5)
        auto.run(t, 1)
        old = bb.set_tuning(6, 0)
        try:
            off.run(t, 1)
            off.sync()
        finally:
            bb.set_tuning(6, old)
        a, o = auto.state(), off.state()
        modes.append(auto.nid_stats()["mode"])
        assert np.array_equal(a["lambda"], o["lambda"])
        assert rel_err(a["beta"], o["beta"]) < 1e-12, (t, modes, rel_err(a["beta"], o["beta"]))
    assert modes[0] >= 1, modes  # the near-null state takes the near-identity path
    print(f"\n[dense n={n} p={p}] iterates per sweep {modes}")
    assert auto.error_flags() == 0 and off.error_flags() == 0
    auto.close()
    off.close()


@pytest.mark.parametrize("kind", ["dense", "sparse"])
def test_nid_teacher_forced_from_reference_start(gpu_lib, kind, capsys):
    """A chain from the reference start (beta0 = 0, BridgeRegression.cpp:85-89) sits in the
    near-null regime: 40 free sweeps, then 3 sweeps teacher-forced against the oracle's
    Cholesky-based Woodbury draw at the steady-state bars (beta 1e-10 relative L2; lambda,
    tau, sig2 1e-11; no flips), each taking the Chebyshev path."""
    bb = gpu_lib
    n, p = 400, 6000
    X, y, _ = _design(kind, n, p, 41)
    e = _engine(bb, X, y, n, p)
    e.init_state()
    e.run(1, 40)
    e.sync()
    s = e.state()
    beta, tau, sig2 = s["beta"], s["tau"], s["sig2"]
    hyper = dict(nu_shape=2.0, nu_rate=2.0, sig2_shape=0.0, sig2_scale=0.0)
    for t in (101, 102, 103):
        e.set_state(beta, tau, sig2, 0.5)
        e.run(t, 1)
        g = e.state()
        st = e.nid_stats()
        tau = oracle.tau_from_sum(oracle.sum_abs_pow(beta, 0.5), p, 0.5, 2.0, 2.0, SEED, 0, t)
        r = y - X @ beta
        sig2 = oracle.sig2_from_rss(float(r @ r), n, 0.0, 0.0, SEED, 0, t)
        lam = oracle.sample_lambda(beta, 0.5, tau, SEED, 0, t)
        z = oracle.normals(p, SEED, 0, t, oracle.KIND_BETA_Z)
        d = oracle.normals(n, SEED, 0, t, oracle.KIND_DELTA)
        b = gibbs.beta_step_woodbury(X, y, lam, sig2, tau, z, d)
        with capsys.disabled():
            print(f"\n[{kind} t={t}] eps={st['eps']:.3g} iterates={st['mode']} "
                  f"beta rel {rel_err(g['beta'], b):.2e}")
        assert st["mode"] >= 1, st
        assert abs(g["tau"] - tau) / tau < 1e-11 and abs(g["sig2"] - sig2) / sig2 < 1e-11
        assert flips(g["lambda"], lam) == 0
        assert np.max(np.abs(g["lambda"] - lam) / lam) < 1e-11
        assert rel_err(g["beta"], b) < 1e-10
        beta = b
    assert e.error_flags() == 0
    e.close()


def test_nid_fitted_state_takes_the_factor(gpu_lib):
    """A fitted state (beta at the truth, tau = 1): eps is far above the Chebyshev range, the
    device decides mode 0 and the sweep forms the Gram and factors it."""
    bb = gpu_lib
    n, p = 300, 3000
    X, y, btrue = synthetic_problem(n, p, seed=12)
    e = _engine(bb, X, y, n, p)
    e.init_state()
    before = e.nid_stats()
    e.set_state(btrue, 1.0, 1.0, 0.5)
    e.run(5, 3)
    e.sync()
    st = e.nid_stats()
    assert st["mode"] == 0 and st["eps"] > 1.0, st
    assert st["chol_sweeps"] - before["chol_sweeps"] == 3
    e.close()


@pytest.mark.parametrize("kind", ["dense", "sparse"])
def test_nid_lambda_bound_certified(gpu_lib, kind):
    """The setup's certified bound on lambda_max(X X') is an upper bound, and a tight one:
    numpy's eigenvalue lies in [bound / 1.6, bound]."""
    bb = gpu_lib
    n, p = 300, 3000
    X, y, _ = _design(kind, n, p, 51)
    e = _engine(bb, X, y, n, p)
    st = e.nid_stats()
    Xd = X.toarray() if hasattr(X, "toarray") else X
    lmax = float(np.linalg.eigvalsh(Xd @ Xd.T)[-1])
    assert st["lambda_x"] >= lmax * (1 - 1e-12), (st, lmax)
    assert st["lambda_x"] <= 1.6 * lmax, (st, lmax)
    assert st["kmax"] >= 2
    e.close()


def test_nid_shard_certifies_its_columns(gpu_lib):
    """A column shard (world > 1) holds the near-identity path (round 4; the sweeps are in
    tests/test_shard_nid_gpu.py): its Lambda certifies lambda_max(X_k X_k') of ITS columns
    from above (the decision sums the shards' certificates)."""
    bb = gpu_lib
    n, p = 100, 900
    X, y, _ = synthetic_problem(n, p, seed=13)
    Xk = np.asfortranarray(X[:, :450])
    e = bb.Engine(bb.EngineConfig(n=n, p=p, p_local=450, j0=0, rank=0, world=2, seed=SEED,
                                  stream=0), Xk, y)
    st = e.nid_stats()
    lmax = np.linalg.eigvalsh(Xk @ Xk.T)[-1]
    assert st["mode"] >= 0
    assert lmax <= st["lambda_x"] <= 2.0 * lmax, (st, lmax)
    e.close()


@pytest.mark.parametrize("n,p", [(200, 2400), (700, 6000), (2000, 50000)])
def test_lambda_xu_fused_equals_separate(gpu_lib, n, p):
    """The fused lambda + X u launch (k_lambda_xu, bb_set_tuning key 7 = 1, 7 = 2, one
    workgroup per chunk, and 7 = 3, the default: drawing and streaming workgroups of one grid,
    k_lambda_xs) against separate lambda and X u launches (key 7 = 0) on near-null states: the
    same
    lambda bits (the same draws), beta to rounding (X u summed in another order), both on
    the Chebyshev path.  (2000, 50000) is C3's shape."""
    import bench
    bb = gpu_lib
    if n == 2000:
        X = bench.make_columns(n, 0, p)
        y, _ = bench.make_problem_y(n, p)
    else:
        X, y, _ = synthetic_problem(n, p, seed=n)
    rng = np.random.default_rng(11)
    beta = 1e-6 * rng.standard_normal(p)
    out = []
    for fused in (1, 2, 3, 0):
        old = bb.set_tuning(7, fused)
        try:
            e = _engine(bb, X, y, n, p)
            e.init_state()
            e.set_state(beta, 1e-6, 1.0, 0.5)
            e.run(7, 2)
            e.sync()
            out.append((e.state(), e.nid_stats()))
            assert e.error_flags() == 0
            e.close()
        finally:
            bb.set_tuning(7, old)
    b, sb = out[-1]
    assert sb["cheb_sweeps"] == 2, sb
    assert np.array_equal(out[1][0]["lambda"], out[2][0]["lambda"])  # modes 2 and 3: same draws
    for a, sa in out[:-1]:  # modes 1 (loop over chunks), 2 (one chunk each), 3 (split roles)
        assert sa["cheb_sweeps"] == 2, (sa, sb)
        assert rel_err(a["beta"], b["beta"]) < 1e-12
        assert np.max(np.abs(a["lambda"] - b["lambda"]) / b["lambda"]) < 1e-12
        assert abs(a["tau"] - b["tau"]) <= 1e-12 * b["tau"]


@pytest.mark.parametrize("kind", ["dense", "sparse"])
def test_nid_synchronous_decision_same_chain(gpu_lib, kind):
    """bb_set_tuning key 8 = 1 (the default): the unsharded engine waits for each sweep's
    decision and launches that path only (the shards' protocol); key 8 = 0 launches both
    paths gated, with at most the iterations its lagged hint allows.  Both decide the same
    least K where the hint allows it; where it does not (eps grew more than 8x in three
    sweeps -- seen once in the first sweeps from the reference start) mode 0 takes the
    factor, the same draw to rounding.  From the reference start: the synchronous mode takes
    the Chebyshev path on every sweep mode 0 does, and the chains agree."""
    bb = gpu_lib
    n, p = 300, 4000
    X, y, _ = _design(kind, n, p, 51)
    out = []
    for mode in (0, 1):
        old = bb.set_tuning(8, mode)
        try:
            e = _engine(bb, X, y, n, p)
            e.init_state()
            e.run(1, 12)
            e.sync()
            out.append((e.state(), e.nid_stats()))
            assert e.error_flags() == 0
            e.close()
        finally:
            bb.set_tuning(8, old)
    (a, sa), (b, sb) = out
    assert sb["cheb_sweeps"] == 12 and sa["cheb_sweeps"] >= 10, (sa, sb)
    assert rel_err(a["beta"], b["beta"]) < 1e-9, rel_err(a["beta"], b["beta"])
    assert np.max(np.abs(a["lambda"] - b["lambda"]) / b["lambda"]) < 1e-9
    assert abs(a["tau"] - b["tau"]) <= 1e-9 * b["tau"]


@pytest.mark.parametrize("n,p,scale", [(200, 45000, 1e-6), (200, 45000, 1e-1),
                                        (2000, 50000, 1e-6), (2000, 50000, 1e-2)])
def test_lambda_wave_draw_same_bits(gpu_lib, n, p, scale):
    """bb_set_tuning key 13: the fused lambda + X u launch at 8 lanes per coefficient with the
    wave-adaptive sampler (stable_wave_draw: a wave's finished draws lend their lanes to the
    unfinished ones, up to 8 outer attempts per round) against fixed 8-lane groups
    (stable_spec_draw<8, 8>): the same attempts in the same order, so the same lambda bits and
    the same chain, from a near-null state and from one with sizeable coefficients (where the
    rejection loops run longer).  (2000, 50000) is C3's shape."""
    import bench
    bb = gpu_lib
    if n == 2000:
        X = bench.make_columns(n, 0, p)
        y, _ = bench.make_problem_y(n, p)
    else:
        X, y, _ = synthetic_problem(n, p, seed=n)
    rng = np.random.default_rng(17)
    beta = scale * rng.standard_normal(p)
    out = []
    for wave in (1, 0):
        old = bb.set_tuning(13, wave)
        try:
            e = _engine(bb, X, y, n, p)
            e.init_state()
            e.set_state(beta, 1e-3, 1.0, 0.5)
            e.run(5, 3)
            e.sync()
            out.append((e.state(), e.nid_stats()))
            assert e.error_flags() == 0
            e.close()
        finally:
            bb.set_tuning(13, old)
    (a, sa), (b, sb) = out
    assert sa == sb, (sa, sb)
    for k in ("lambda", "beta"):
        assert np.array_equal(a[k], b[k]), (k, np.max(np.abs(a[k] - b[k])))
    assert a["tau"] == b["tau"] and a["sig2"] == b["sig2"]
    assert np.all(np.isfinite(a["lambda"])) and np.all(a["lambda"] > 0)


@pytest.mark.parametrize("kind", ["dense", "sparse", "c3"])
def test_decision_poll_and_row_blocks_same_bits(gpu_lib, kind):
    """bb_set_tuning key 11 (the host polls the decision's tag word instead of waiting on an
    event) and key 12 (XCD-aware row blocks of the partial row sums) change neither the path
    nor a bit of the chain: 12 sweeps from the reference start, defaults against both off
    (C3's shape included: the fused lambda launch and the mixed plan's decision)."""
    bb = gpu_lib
    if kind == "c3":  # C3's shape: the fused lambda launch and the mixed plan's decision
        import bench
        n, p = 2000, 50000
        X = bench.make_columns(n, 0, p)
        y, _ = bench.make_problem_y(n, p)
    else:
        n, p = 300, 4000
        X, y, _ = _design(kind, n, p, 52)
    out = []
    for v in (1, 0):
        o11, o12 = bb.set_tuning(11, v), bb.set_tuning(12, v)
        try:
            e = _engine(bb, X, y, n, p)
            e.init_state()
            e.run(1, 12)
            e.sync()
            out.append((e.state(), e.nid_stats()))
            assert e.error_flags() == 0
            e.close()
        finally:
            bb.set_tuning(11, o11)
            bb.set_tuning(12, o12)
    (a, sa), (b, sb) = out
    assert sa["cheb_sweeps"] == sb["cheb_sweeps"] >= 10 and sa["products"] == sb["products"]
    for k in ("beta", "lambda"):
        assert np.array_equal(a[k], b[k]), k
    assert a["tau"] == b["tau"] and a["sig2"] == b["sig2"]


@pytest.mark.parametrize("stride", [1, 3])
def test_timed_phase_stride(gpu_lib, stride):
    """bench.py's live roofline timing: the timed phase is bracketed by an event pair in every
    stride-th sweep of a timed run (bb_engine_set_timing_stride), and its average is the
    bracketed launches' mean; a stride < 1 is refused."""
    bb = gpu_lib
    n, p = 200, 2400
    X, y, _ = synthetic_problem(n, p, seed=5)
    e = _engine(bb, X, y, n, p)
    e.init_state()
    e.run(1, 2, first_slot=-1)
    e.enable_timing(True, phases=False, timed_phase="lambda", stride=stride)
    e.reset_timing()
    e.run(3, 10, first_slot=-1)
    e.sync()
    ms, _, _ = e.kernel_times()
    assert e.timed_brackets() == len(range(0, 10, stride))
    assert 0.0 < ms < 50.0
    e.enable_timing(False)
    with pytest.raises(Exception):
        e.enable_timing(True, phases=False, timed_phase="lambda", stride=0)


# ---------------------------------------------------------------------------------------
# The mixed-precision plan: products over the fp32 copy of X, one fp64
# residual pass; the same certified bound as the fp64 plan
# ---------------------------------------------------------------------------------------
def test_mixed_plan_sweep_equals_fp64_plan(gpu_lib, capsys):
    """One sweep from the same state with the mixed plan allowed (bb_set_tuning key 10 = 1)
    and with fp64 products only (0): the same lambda, tau, sig2 bits and beta to 1e-12
    relative, over states from the near-null regime (2 iterates) to eps ~ 1e-2 (7, where the
    certificate's eta^2 exceeds the tolerance and the fp64 plan is kept); the device takes the
    mixed plan (nid_mixed counts it) in between.  C3's shape restricted to n = 2000,
    p = 6250 (the E-apply's rows in registers, n_pad = 2048)."""
    import bench
    bb = gpu_lib
    n, p = 2000, 6250
    X = bench.make_columns(n, 0, p)
    y, btrue = bench.make_problem_y(n, p)
    rng = np.random.default_rng(11)
    engs = {}
    for mixed in (1, 0):
        old = bb.set_tuning(10, mixed)
        try:
            e = _engine(bb, X, y, n, p)
            e.init_state()
            engs[mixed] = e
        finally:
            bb.set_tuning(10, old)
    assert engs[1].nid_mixed()["holds_x32"]
    # created with the plan off: no fp32 copy (it could never be used)
    assert not engs[0].nid_mixed()["holds_x32"]
    plans = []
    for scale in (1e-5, 1e-4, 3e-4, 1e-3, 1e-2):
        beta, tau = btrue * scale + scale * rng.standard_normal(p), scale
        for t in (3, 4):
            outs = {}
            for mixed, e in engs.items():
                old = bb.set_tuning(10, mixed)
                try:
                    e.set_state(beta, tau, 1.0, 0.5)
                    e.run(t, 1)
                    e.sync()
                    outs[mixed] = (e.state(), e.nid_stats(), e.nid_mixed())
                finally:
                    bb.set_tuning(10, old)
            (a, sa, ma), (o, so, _) = outs[1], outs[0]
            plans.append((scale, sa["mode"], ma["k2"], so["mode"], f"{ma['eta']:.1e}"))
            assert a["tau"] == o["tau"] and a["sig2"] == o["sig2"]
            assert np.array_equal(a["lambda"], o["lambda"])
            err = rel_err(a["beta"], o["beta"])
            assert err < 1e-12, (plans[-1], err)
            beta, tau = o["beta"], o["tau"]
    m = engs[1].nid_mixed()
    with capsys.disabled():
        print(f"\n[mixed] (scale, K1, K2, K fp64, eta) per sweep {plans}; {m}")
    assert engs[0].nid_mixed()["mixed_sweeps"] == 0
    assert m["mixed_sweeps"] >= 2 and m["products32"] >= 1, (plans, m)
    for e in engs.values():
        assert e.error_flags() == 0
        e.close()


def test_mixed_plan_refused_outside_fp32_range(gpu_lib):
    """A design with one column scaled to ~1e-39 (below fp32's normal range) gets no fp32
    copy: holds_x32 is false, no sweep takes the mixed plan, and the chain is bit-identical to
    an engine created with the plan off."""
    import bench
    bb = gpu_lib
    n, p = 2000, 6250
    X = bench.make_columns(n, 0, p)
    y, _ = bench.make_problem_y(n, p)
    X[:, 17] *= 1e-39
    outs = {}
    for mixed in (1, 0):
        old = bb.set_tuning(10, mixed)
        try:
            e = _engine(bb, X, y, n, p)
            e.init_state()
            e.run(1, 30, first_slot=-1)
            e.sync()
            outs[mixed] = (e.state(), e.nid_mixed())
            assert e.error_flags() == 0
            e.close()
        finally:
            bb.set_tuning(10, old)
    (a, ma), (o, mo) = outs[1], outs[0]
    assert not ma["holds_x32"] and not mo["holds_x32"]
    assert ma["mixed_sweeps"] == 0
    assert np.array_equal(a["beta"], o["beta"]) and np.array_equal(a["lambda"], o["lambda"])
    assert a["tau"] == o["tau"] and a["sig2"] == o["sig2"]


def test_mixed_plan_teacher_forced_against_oracle(gpu_lib, capsys):
    """The C3 workload itself (bench.py's X, y, key) run free from the reference start for
    600 sweeps -- eps ~ 2e-4, where the fp64 plan needs 4-5 products and the device takes the
    mixed plan -- then 3 sweeps teacher-forced against the oracle's Cholesky-based Woodbury draw
    (beta 1e-10 relative L2, lambda / tau / sig2 1e-11, no flips), asserting the plan each
    sweep took."""
    from tests.test_steady_state_gpu import oracle_sweep, workload
    bb = gpu_lib
    X, y, alpha = workload("c3")
    n, p = X.shape
    e = bb.Engine(bb.EngineConfig(n=n, p=p, seed=SEED, stream=0, true_alpha=alpha,
                                  trace_capacity=1), X, y)
    e.init_state()
    e.run(1, 600, first_slot=-1)
    e.sync()
    s0 = e.state()
    beta, tau, sig2 = s0["beta"], s0["tau"], s0["sig2"]
    taken = []
    for t in (1001, 1002, 1003):
        m0 = e.nid_mixed()["mixed_sweeps"]
        e.set_state(beta, tau, sig2, alpha)
        e.run(t, 1, first_slot=-1)
        g = e.state()
        st, m = e.nid_stats(), e.nid_mixed()
        b, lam, tau, sig2 = oracle_sweep(X, y, beta, tau, sig2, alpha, t, SEED, 0)
        taken.append(m["mixed_sweeps"] - m0)
        with capsys.disabled():
            print(f"\n[mixed c3 t={t}] eps={st['eps']:.3g} K1={st['mode']} K2={m['k2']} "
                  f"eta={m['eta']:.2e} beta rel {rel_err(g['beta'], b):.2e}")
        assert (m["k2"] >= 1) == (taken[-1] == 1), (st, m)
        assert abs(g["tau"] - tau) / tau < 1e-11 and abs(g["sig2"] - sig2) / sig2 < 1e-11
        assert flips(g["lambda"], lam) == 0
        assert np.max(np.abs(g["lambda"] - lam) / lam) < 1e-11
        assert rel_err(g["beta"], b) < 1e-10
        beta = b
    assert sum(taken) >= 2, taken  # the mixed plan was exercised
    assert e.error_flags() == 0
    e.close()
