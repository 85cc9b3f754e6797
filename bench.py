#!/usr/bin/env python3
"""Benchmark: Gibbs sweeps/s of the BayesBridge stable sampler on MI355X.

Default workload (BASELINE.json metric): Gaussian bridge regression, n=2000, p=50000,
alpha=0.5, synthetic design of SURVEY.md s8(d).  One step = one full Gibbs
sweep (tau, sig2, all p lambda_j, beta | rest) with X resident in HBM.  At N GPUs the p
columns are sharded across one process per GPU with one RCCL all-reduce per exchange step
(strong scaling: the total problem is fixed).

Other BASELINE configs, one JSON line each (``--workload``):
  c2  n=1000, p=5000, alpha=0.5, dense Woodbury
  c5  n=5000, p=200000, alpha=0.3, sparse CSC design at 1 % density (pair-list sparse Gram,
      the HBM-bound path)

Defaults follow SURVEY.md 8(d): M = 1000 timed sweeps after B = 100 burn-in sweeps, every
timed sweep recording beta / lambda / sig2 / tau into the device-resident trace.

Prints ONE JSON line (rank 0) with the driver's contract fields plus
  roofline     -- the dominant kernel: algorithmic work per launch / average launch duration
                  from HIP events on the engine stream
  cpu_baseline -- the oracle's sweep (numpy/scipy OpenBLAS + C latent sampler) timed on this
                  host on a bounded number of sweeps (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import re
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_MFMA_PEAK_TFLOPS = 78.6  # MI355X dense fp64 matrix peak (spec)
# dense int8 MFMA: 2048 ops/clk/SIMD (v_mfma_i32_16x16x64_i8 = 16 cycles) x 1024 SIMDs x 2.4 GHz
INT8_MFMA_PEAK_TOPS = 2048 * 1024 * 2.4e9 / 1e12
DATA_SEED = 20240501


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_columns(n, j0, j1, seed=DATA_SEED, block=1000):
    """Columns [j0, j1) of the synthetic X; column blocks are seeded independently so any
    shard can be generated without the rest.  X_ij ~ N(0,1), columns centred."""
    out = np.empty((n, j1 - j0), order="F")
    b0 = j0 // block
    b1 = (j1 + block - 1) // block
    for b in range(b0, b1):
        rng = np.random.default_rng([seed, b])
        cols = rng.standard_normal((block, n)).T  # n x block
        cols -= cols.mean(axis=0)
        lo, hi = max(j0, b * block), min(j1, (b + 1) * block)
        out[:, lo - j0:hi - j0] = cols[:, lo - b * block:hi - b * block]
    return out


def make_problem_y(n, p, seed=DATA_SEED):
    s = max(5, p // 100)
    rng = np.random.default_rng([seed, 999999])
    b = np.zeros(p)
    b[:s] = rng.uniform(1, 3, size=s) * rng.choice([-1.0, 1.0], size=s)
    Xs = make_columns(n, 0, s, seed)
    y = Xs @ b[:s] + rng.standard_normal(n)
    return y - y.mean(), b


SPARSE_DENSITY = 0.01  # C5: each X_ij non-zero independently with this probability

WORKLOADS = {
    # name: (n, p, alpha, kind)
    "c1": (100, 20, 0.5, "small"),
    "c2": (1000, 5000, 0.5, "dense"),
    "c3": (2000, 50000, 0.5, "dense"),
    "c4": (10000, 1000, 0.5, "logit"),
    "c5": (5000, 200000, 0.3, "sparse"),
}


def make_logit_problem(n, p, seed=DATA_SEED):
    """C4 synthetic logistic design: X_ij ~ N(0,1), beta's first max(5, p/100) entries
    +-U(1,3) and the rest 0, y_i ~ Bernoulli(1/(1 + exp(-x_i'beta))).
    Returns (X (F order), y in {0,1}, beta)."""
    rng = np.random.default_rng([seed, 4])
    X = np.asfortranarray(rng.standard_normal((n, p)))
    s = max(5, p // 100)
    b = np.zeros(p)
    b[:s] = rng.uniform(1, 3, size=s) * rng.choice([-1.0, 1.0], size=s)
    y = (rng.random(n) < 1.0 / (1.0 + np.exp(-(X @ b)))).astype(np.float64)
    return X, y, b


def cpu_baseline_logit(n, p, alpha, sweeps, threads=None):
    """The compiled logistic CPU chain (oracle/bb_cpu_chain.c bbc_logit_chain: dsyrk for
    X'Omega X + dpotrf + dtrsm on scipy's OpenBLAS, OpenMP Polya-Gamma and tilted-stable
    draws; checked against oracle/gibbs.py by tests/test_cpu_chain.py) from beta = 0.
    threads: BLAS / OpenMP threads (None: OMP_NUM_THREADS or every CPU).  Returns
    (s per sweep, threads)."""
    import oracle

    if threads is None:
        threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    X, y, _ = make_logit_problem(n, p)
    r = oracle.cpu_logit_chain(y, X, sweeps + 1, burn=0, alpha=alpha, seed=0xB4E5B41D6E,
                               threads=threads, record=False)
    log(f"[cpu_baseline] logistic threads={threads}: {sweeps} sweeps in {r['runtime']:.3f} s")
    return r["runtime"] / sweeps, threads


def make_sparse_columns(n, j0, j1, density=SPARSE_DENSITY, seed=DATA_SEED, block=1000):
    """Columns [j0, j1) of the synthetic sparse X of C5 as a scipy CSC matrix: every entry
    is non-zero independently with probability `density` (positions by geometric gaps over
    a column block, column-major), values N(0,1), columns NOT centred (centring would fill
    them in).  Column blocks are seeded independently, so any shard can be generated alone."""
    import scipy.sparse as sps

    rows, cols, vals = [], [], []
    for b in range(j0 // block, (j1 + block - 1) // block):
        rng = np.random.default_rng([seed, 7, b])
        N = n * block
        m = int(N * density + 12 * math.sqrt(N * density) + 64)
        pos = np.cumsum(rng.geometric(density, size=m)) - 1
        while pos[-1] < N:  # practically never: extend the gap sequence
            pos = np.concatenate([pos, pos[-1] + np.cumsum(rng.geometric(density, size=m))])
        pos = pos[pos < N]
        v = rng.standard_normal(pos.size)
        c = pos // n + b * block
        keep = (c >= j0) & (c < j1)
        rows.append(pos[keep] % n)
        cols.append(c[keep] - j0)
        vals.append(v[keep])
    r, c, v = np.concatenate(rows), np.concatenate(cols), np.concatenate(vals)
    return sps.csc_matrix((v, (r, c)), shape=(n, j1 - j0))


def make_sparse_problem_y(n, p, density=SPARSE_DENSITY, seed=DATA_SEED):
    """y = X b + e for the sparse design: b's first max(5, p/100) entries +-U(1,3), the rest
    0; e ~ N(0,1); y centred."""
    s = max(5, p // 100)
    rng = np.random.default_rng([seed, 999998])
    b = np.zeros(p)
    b[:s] = rng.uniform(1, 3, size=s) * rng.choice([-1.0, 1.0], size=s)
    Xs = make_sparse_columns(n, 0, s, density, seed)
    y = Xs @ b[:s] + rng.standard_normal(n)
    return y - y.mean(), b


def cpu_baseline_sparse(n, p, alpha, sweeps, threads=None):
    """The compiled sparse Woodbury CPU chain (oracle/bb_cpu_chain.c bbc_sparse_chain: CSR /
    CSC passes and the n x n sparse Gram by output column under OpenMP, LAPACK dpotrf on
    scipy's OpenBLAS, OpenMP tilted-stable draws; checked against oracle/gibbs.py by
    tests/test_cpu_chain.py) from beta = 0.  Returns (s per sweep, threads)."""
    import oracle

    if threads is None:
        threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    X = make_sparse_columns(n, 0, p)
    y, _ = make_sparse_problem_y(n, p)
    r = oracle.cpu_sparse_chain(y, X, sweeps + 1, burn=0, alpha=alpha, seed=0xB4E5B41D6E,
                                threads=threads, record=False)
    log(f"[cpu_baseline] sparse threads={threads}: {sweeps} sweeps in {r['runtime']:.3f} s")
    return r["runtime"] / sweeps, threads


def blas_threads(threads):
    """Context limiting the BLAS pools to `threads` (None: leave them as they are)."""
    import contextlib

    if threads is None:
        return contextlib.nullcontext()
    from threadpoolctl import threadpool_limits
    return threadpool_limits(limits=threads)


def cpu_baseline(n, p, alpha, sweeps, threads=None, literal=False):
    """The compiled CPU baseline (oracle/bb_cpu_chain.c + scipy's OpenBLAS, no Python in the
    loop): the stable chain from beta = 0 with the reference-literal p x p Cholesky
    (literal=True, BridgeRegression.cpp:552-575: X'X once, then dpotrf of
    X'X + diag(lambda sig2 / tau^2) and three triangular solves per sweep) or the exact
    Woodbury form the GPU runs (dsyrk + n x n dpotrf + dgemv).  threads: BLAS / OpenMP
    threads (None: OMP_NUM_THREADS or every CPU).  Returns (s per sweep, threads)."""
    import oracle

    if threads is None:
        threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    X = make_columns(n, 0, p)
    y, _ = make_problem_y(n, p)
    r = oracle.cpu_chain(y, X, sweeps + 1, burn=0, alpha=alpha,
                         method="chol" if literal else "woodbury", seed=0xB4E5B41D6E,
                         threads=threads, record=False)
    log(f"[cpu_baseline] {'literal' if literal else 'woodbury'} threads={threads}: "
        f"{sweeps} sweeps in {r['runtime']:.3f} s")
    return r["runtime"] / sweeps, threads


_SHA = None


def tree_sha():
    """source_sha of the library sources in this tree (bayesbridge_amd/_build.py)."""
    global _SHA
    if _SHA is None:
        from bayesbridge_amd import _build
        _SHA = _build.source_sha()
    return _SHA


def _profiles(pattern):
    """Committed profile summaries (newest round last) with their path."""
    import glob

    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", pattern))):
        try:
            yield json.load(open(f)), os.path.relpath(f, ROOT)
        except (OSError, ValueError):
            continue


def _stale_note(d, f, entry=None, instance=None):
    """None if the profile's entry for `instance` describes this build's kernel: the entry's
    recorded code identity (gfx950 code bytes + kernel descriptor, bayesbridge_amd/_kernel_code.py)
    equals this library's, or -- for an entry without one -- the profiled tree is this tree.
    Otherwise the reason it is not used."""
    cs = entry.get("code_sha") if isinstance(entry, dict) else None
    if cs is not None and instance:
        from bayesbridge_amd import _kernel_code

        cur = _kernel_code.code_sha(instance)
        if cur == cs:
            return None
        return (f"{f}: {instance} profiled as code {cs}, this build's is {cur}: not used "
                "(re-profile: tools/profile_round.sh / pmc_valu.sh / pmc_mfma.sh)")
    sha = d.get("source_sha")
    if sha == tree_sha():
        return None
    return (f"{f} profiled source {sha or 'unrecorded'}, this tree is {tree_sha()}: "
            "not used (re-profile: tools/profile_round.sh / pmc_valu.sh / pmc_mfma.sh)")


def pmc_traffic(n, p, world, instance, window=None):
    """HBM bytes per launch of the EXACT kernel instance (e.g. "bb::k_eapply<8, false>") from
    the newest committed PMC summary of this workload (profiles/rNN_pmc.json:
    tools/profile_round.sh + tools/profile_summary.py, separate FETCH_SIZE / WRITE_SIZE passes,
    gfx950 x2 read correction) whose source_sha is this tree's.  Returns (bytes, source, note);
    bytes None when there is no such profile (note says why)."""
    best, note = None, "no committed PMC summary of this workload"
    if instance is None or world != 1:
        return None, None, "no kernel instance / multi-rank"
    for d, f in _profiles("r*_pmc.json"):
        w = d.get("workload", {})
        if w.get("n") != n or w.get("p") != p:
            continue
        if window is not None and (d.get("window") or {}).get("steps") != window[0] or \
                window is not None and (d.get("window") or {}).get("warmup") != window[1]:
            continue  # a per-sweep kernel's average depends on the window's regime
        v = d.get("kernels", {}).get(instance)
        if not v or v.get("hbm_bytes") != v.get("hbm_bytes"):  # absent, or NaN (one pass lacks it)
            note = f"{f} has no entry for {instance}"
            continue
        stale = _stale_note(d, f, v, instance)
        if stale:
            best, note = None, stale
            continue
        best, note = (v["hbm_bytes"], f), None
    return (best[0], best[1], None) if best else (None, None, note)


def pmc_traffic_family(n, p, world, instances, window=None):
    """HBM bytes per launch averaged over several kernel instances that one timed phase
    launches (the E-apply phase of the mixed plan: k_eapply<NR, 0> fp32 or fp64 products,
    <NR, 2> the fp64 residual pass, <NR, 3> the fp32 correction products), weighted by their
    dispatch counts in the newest committed profile of this workload and window that has them
    all -- the same launches the live average over the phase's brackets covers.  Every
    instance's entry must describe this build's code.  Returns (bytes, source, note,
    {instance: {"dispatches", "hbm_bytes"}})."""
    best, note = None, "no committed PMC summary of this workload"
    if not instances or world != 1:
        return None, None, "no kernel instance / multi-rank", None
    for d, f in _profiles("r*_pmc.json"):
        w = d.get("workload", {})
        if w.get("n") != n or w.get("p") != p:
            continue
        if window is not None and ((d.get("window") or {}).get("steps"),
                                   (d.get("window") or {}).get("warmup")) != tuple(window):
            continue
        ks = d.get("kernels", {})
        ents = {i: ks.get(i) for i in instances if ks.get(i)}
        if not ents:
            note = f"{f} has none of {instances}"
            continue
        stale = [_stale_note(d, f, v, i) for i, v in ents.items()]
        stale = [x for x in stale if x]
        if stale:
            best, note = None, stale[0]
            continue
        cnt = sum(v.get("dispatches", 0) for v in ents.values())
        if not cnt or any(v.get("hbm_bytes") != v.get("hbm_bytes") for v in ents.values()):
            note = f"{f}: no dispatch counts / traffic for {sorted(ents)}"
            continue
        tot = sum(v["dispatches"] * v["hbm_bytes"] for v in ents.values())
        best = (tot / cnt, f, {i: {"dispatches": v["dispatches"], "hbm_bytes": v["hbm_bytes"]}
                               for i, v in ents.items()})
        note = None
    return (best[0], best[1], None, best[2]) if best else (None, None, note, None)


def pmc_mfma(n, p, world, instance, gram):
    """MFMA-busy evidence for the exact kernel instance at this workload from the newest
    committed profiles/rNN_pmc_mfma.json of this tree (tools/pmc_mfma.sh:
    SQ_VALU_MFMA_BUSY_CYCLES in its own rocprofv3 --pmc pass).  The busy fraction is taken
    against the NOMINAL clock: busy cycles / (1024 SIMDs x 2.4 GHz x the dispatch duration)
    (the GRBM_GUI_ACTIVE-derived clock read above 2.4 GHz on short dispatches)."""
    best = None
    for d, f in _profiles("r*_pmc_mfma.json"):
        for cfg in d.get("configs", {}).values():
            if cfg.get("n") != n or cfg.get("p") != p or world != 1 or cfg.get("gram") != gram:
                continue
            v = cfg.get("kernels", {}).get(instance)
            if v and "mfma_busy_frac_nominal_clock" in v and not _stale_note(d, f, v, instance):
                best = {"mfma_busy_frac": v["mfma_busy_frac_nominal_clock"], "source": f,
                        "definition": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x 2.4 GHz x the "
                                      "dispatch duration)"}
    return best


VALU_PEAK_GCYC = 1024 * 2.4  # SIMD issue cycles per ns: 1024 SIMDs at 2.4 GHz


def pmc_valu(n, p, world, instance, window=None):
    """VALU evidence for the exact kernel instance at this workload from the newest committed
    profiles/rNN_pmc_valu.json of this tree (tools/pmc_valu.sh: SQ_INSTS_VALU and the per-class
    SQ_INSTS_VALU_* counts, one counter per --pmc pass; tools/pmc_valu_summary.py prices them
    in SIMD issue cycles).  Returns (entry, note)."""
    best, note = None, "no committed VALU profile of this workload"
    for d, f in _profiles("r*_pmc_valu.json"):
        for cfg in d.get("configs", {}).values():
            if cfg.get("n") != n or cfg.get("p") != p or world != 1:
                continue
            cw = cfg.get("window") or {}
            if window is not None and (cw.get("steps"), cw.get("warmup")) != tuple(window):
                continue
            v = cfg.get("kernels", {}).get(instance)
            if not v or "SQ_INSTS_VALU" not in v:
                note = f"{f} has no entry for {instance}"
                continue
            stale = _stale_note(d, f, v, instance)
            if stale:
                best, note = None, stale
                continue
            best, note = dict(v, kernel=instance, source=f), None
    return best, note


def rel_l2(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


# Phases whose bracket (HIP events at phase starts) covers exactly one kernel launch, in the
# engine's per-sweep order (bb_engine.cpp phase_b / phase_c): the candidates for the
# `roofline` kernel.  "ozprep" (k_oz_bound + k_oz_finalize + k_oz_residues) is not a single
# kernel and is reported through phases_ms only.
SINGLE_KERNEL_PHASES = ("lambda", "gram", "reduce", "chol", "solve", "beta", "eapply")
CHOL_NB = 64  # k_chol_persistent block size (bb_kernels.hip kNB)


def roofline_for(phase, ms, ctx, traffic_world):
    """Roofline object of the kernel behind `phase`, given its average launch time `ms`.
    ctx: dict(n, p, p_loc, kind, gram_mode, eng, bb).  Formulas: DESIGN.md s5 / s8."""
    bb, eng, kind = ctx["bb"], ctx["eng"], ctx["kind"]
    n, p, p_loc = ctx["n"], ctx["p"], ctx["p_loc"]
    gram_mode = ctx["gram_mode"]
    logit, sparse = kind == "logit", kind == "sparse"
    # (a phase whose launches all returned at once can time as 0: no rate then)
    sec = max(ms, 1e-9) * 1e-3
    out = {"phase": phase, "kernel_ms_avg": ms}
    if phase == "gram":
        n_pad = -(-n // 128) * 128
        ntri = n_pad * (n_pad + 1) // 2
        if sparse:
            # pair-list Gram by output column, per launch: 8 B product + 2 B row position per
            # pair, 4 B segment start + 8 B packed entry per triangle entry, the CSR rows
            # (12 B per non-zero) and D, u (8 B each per column)
            si = eng.sparse_info()
            if si["col_mode"]:
                byts = 10.0 * si["pairs"] + 12.0 * ntri + 12.0 * si["nnz"] + 16.0 * p_loc
                if bb.set_tuning(3, -1) >= 2:  # the flat chunked stream (the default)
                    kname, kfull = ("k_sp_gram_flat (pair-list Gram by output column, flat "
                                    "stream)", "bb::k_sp_gram_flat")
                else:
                    kname, kfull = ("k_sp_gram_col (pair-list Gram by output column)",
                                    "bb::k_sp_gram_col")
            else:
                byts = 12.0 * si["pairs"] + 12.0 * ntri + 8.0 * p_loc
                kname, kfull = "k_sp_gram (pair-list Gram)", "bb::k_sp_gram"
            out.update(bound="hbm", kernel=kname, achieved=byts / sec / 1e9, peak=8000.0,
                       unit="GB/s", algorithmic_bytes_per_launch=byts,
                       # SURVEY 8(d)'s definition: 12 B per non-zero per pass over X
                       survey_8d_bytes_per_pass=12.0 * si["nnz"],
                       survey_8d_rate_GBps=12.0 * si["nnz"] / sec / 1e9)
        elif gram_mode == bb.GRAM_OZAKI:
            rows, kdim = (p, n) if logit else (n, p_loc)
            ops = 16.0 * rows * (rows + 1) * kdim  # 16 exact int8 Grams (lower triangle, 2/MAC)
            kfull = "bb::k_oz_gemm16u"
            out.update(bound="mfma", kernel=("k_oz_gemm16u X'Omega X" if logit else "k_oz_gemm16u")
                       + " (v_mfma_i32_16x16x64_i8)", achieved=ops / sec / 1e12,
                       peak=INT8_MFMA_PEAK_TOPS, unit="TOP/s", ops_per_launch=ops,
                       algorithmic_bytes_per_launch=16.0 * rows * kdim)
        else:
            flops = float(n) * p * (p + 1) if logit else float(n) * (n + 1) * p_loc
            kfull = "bb::k_gram"
            out.update(bound="mfma", kernel="k_gram (v_mfma_f64_16x16x4_f64)",
                       achieved=flops / sec / 1e12, peak=FP64_MFMA_PEAK_TFLOPS, unit="TFLOP/s",
                       ops_per_launch=flops,
                       algorithmic_bytes_per_launch=8.0 * (p if logit else n) * (n if logit else p_loc))
    elif phase == "chol":
        # the per-sweep Cholesky of the n x n Woodbury system (p x p for the logistic path):
        # m^3/3 algorithmic flops; its time is set by the chain of m_pad/64 dependent block
        # steps, reported as the latency model beside the flop rate
        m = p if logit else n
        # the p x p system is factored at round_up(p, 64) (bb_engine.cpp chol_m); the n x n
        # Woodbury system at n_pad = round_up(n, 128)
        m_pad = -(-m // CHOL_NB) * CHOL_NB if logit else -(-n // 128) * 128
        flops = m ** 3 / 3.0
        steps = m_pad // CHOL_NB
        kfull = "bb::k_chol_persistent"
        out.update(bound="mfma", kernel="k_chol_persistent (fp64 MFMA, one launch per factor)",
                   achieved=flops / sec / 1e12, peak=FP64_MFMA_PEAK_TFLOPS, unit="TFLOP/s",
                   ops_per_launch=flops, algorithmic_bytes_per_launch=8.0 * m_pad * m_pad,
                   latency_model={"system": m, "system_padded": m_pad, "block": CHOL_NB,
                                  "dependent_block_steps": steps,
                                  "us_per_step": ms * 1e3 / steps,
                                  "model": "time = steps x (in-LDS elimination of the 64-block "
                                           "+ W = U_kk^-T + U_k,k+1 + next diagonal update) "
                                           "(DESIGN.md s5.2)"})
    elif phase == "eapply":
        # the near-identity solve's pass over X: X diag(D) X' d in one read
        # of X (dense: 8 n_pad p_loc bytes, plus the d vector and the per-workgroup partial
        # n-vectors it writes; sparse: the CSC and CSR non-zeros, 12 B each, plus D, s, d),
        # times the fraction of the launches that ran a pass (the others, past the sweep's
        # iteration count, return at once)
        n_pad = -(-n // 128) * 128
        if sparse:
            si = eng.sparse_info()
            byts = 24.0 * si["nnz"] + 24.0 * p_loc + 16.0 * n_pad
            kname, kfull = "k_sp_eapply_cols + k_sp_eapply_rows (X D X' d)", "bb::k_sp_eapply"
        else:
            byts = 8.0 * n_pad * p_loc + 8.0 * p_loc + 8.0 * n_pad * (1 + ctx.get("ea_parts", 512))
            kname, kfull = "k_eapply (X D X' d, one pass over X)", "bb::k_eapply"
        pf = ctx.get("pass_frac", 1.0)
        # fp32 passes of the mixed plan: X at 4 B per element
        pf32 = 0.0 if sparse else ctx.get("pass32_frac", 0.0)
        byts32 = byts - 4.0 * n_pad * p_loc
        algo = byts * pf + byts32 * pf32
        out.update(bound="hbm", kernel=kname, achieved=algo / sec / 1e9, peak=8000.0,
                   unit="GB/s", algorithmic_bytes_per_launch=algo,
                   bytes_per_pass=byts, passes_per_launch=pf,
                   bytes_per_fp32_pass=byts32, fp32_passes_per_launch=pf32)
    elif phase == "lambda":
        # the tilted-stable draws: VALU-bound arithmetic with a rejection tail.
        # achieved = SIMD issue cycles per launch -- the per-class VALU instruction counts of the
        # committed profile of this workload and tree (rocprofv3 SQ_INSTS_VALU_*) priced at the
        # measured cycles per wave64 instruction (f64 FMA/MUL/ADD 4, f64 rcp/sqrt 16, f32
        # transcendental 8, 32-bit ops 2; profiles/r05_valu_costs.json) -- over the live average
        # launch time, against every SIMD issuing every cycle (1024 SIMDs x 2.4 GHz).  The fused
        # launch (k_lambda_xu, dense near-identity sweeps) also streams X for X u: its HBM rate.
        kfull = ctx.get("instances", {}).get("lambda")
        fused = bool(kfull) and kfull.startswith("bb::k_lambda_xu")
        v, vnote = pmc_valu(n, p, traffic_world, kfull, ctx.get("window"))
        cyc = v.get("issue_cycles") if v else None
        out.update(bound="valu", kernel=kfull,
                   achieved=(cyc / sec / 1e9) if cyc else None, peak=VALU_PEAK_GCYC,
                   unit="G SIMD issue-cycles/s (VALU)", draws_per_launch=p_loc,
                   draws_per_s=p_loc / sec,
                   issue_cycles_per_launch=cyc,
                   frac_bounds=([v["issue_cycles_low"] / sec / 1e9 / VALU_PEAK_GCYC,
                                 v["issue_cycles_high"] / sec / 1e9 / VALU_PEAK_GCYC]
                                if cyc else None),
                   valu_insts_per_launch=v["SQ_INSTS_VALU"] if v else None,
                   valu_class_counts=v.get("class_counts") if v else None,
                   valu_class_cycles=v.get("class_cycles") if v else None,
                   valu_busy_frac=v.get("valu_busy_frac") if v else None,
                   valu_source=v["source"] if v else None, valu_note=vnote,
                   cost_model="INT32 / CVT / unclassified instructions at the average cost of "
                              "their members in the kernel's ISA; frac_bounds price them at 2 "
                              "and 4 cycles (tools/pmc_valu_summary.py)")
        if fused:
            byts = 8.0 * n * p_loc + 32.0 * p_loc
            out["hbm"] = {"algorithmic_bytes_per_launch": byts, "achieved_GBps": byts / sec / 1e9,
                          "peak_GBps": 8000.0, "frac": byts / sec / 1e9 / 8000.0,
                          "note": "X read once for X u (8 B per element) + beta read and "
                                  "lambda, D, u written (8 B each per coefficient)"}
    elif phase == "beta" and not logit:
        # the Woodbury beta update: one read of X for X' w (dense: fused with the
        # next sweep's X beta partials, k_beta_wb_xb; sparse: the CSC non-zeros), D, u read and
        # beta written (8 B each per coefficient)
        if sparse:
            si = eng.sparse_info()
            byts = 12.0 * si["nnz"] + 32.0 * p_loc
            kfull = "bb::k_sp_beta"
        else:
            byts = 8.0 * n * p_loc + 32.0 * p_loc
            kfull = "bb::k_beta_wb"
        out.update(bound="hbm", kernel=kfull, achieved=byts / sec / 1e9, peak=8000.0,
                   unit="GB/s", algorithmic_bytes_per_launch=byts)
    else:
        kfull = {"reduce": "bb::k_oz_crt", "solve": "bb::k_bsolve", "beta": "bb::k_beta"}[phase]
        out.update(bound="latency", kernel=kfull, achieved=None, peak=None, unit=None)
    out["frac"] = (out["achieved"] / out["peak"]) if (out.get("peak") and
                                                       out.get("achieved") is not None) else None
    # the PMC evidence is matched on the exact kernel instance the timed run launched
    # (bb_kernel_instance), never on a name prefix
    inst = ctx.get("instances", {}).get(phase)
    out["kernel_instance"] = inst
    # the per-sweep kernels' traffic from a profile of the same bench window; the Gram, CRT
    # and factor run only on factor sweeps (the fitted-regime run at C3): any window
    tb, tsrc, tnote = pmc_traffic(n, p, traffic_world, inst,
                                  None if phase in ("gram", "reduce", "chol", "solve")
                                  else ctx.get("window"))
    m = re.match(r"(bb::k_eapply<\d+), \d+>$", inst or "")
    if phase == "eapply" and m and (out.get("fp32_passes_per_launch") or 0) > 0:
        # the mixed plan's E-apply phase launches three instances (fp32 / fp64 products, the
        # fp64 residual pass, the fp32 correction products): their dispatch-weighted traffic
        fam = [f"{m.group(1)}, {k}>" for k in (0, 2, 3)]
        tb, tsrc, tnote, per = pmc_traffic_family(n, p, traffic_world, fam, ctx.get("window"))
        out["kernel_instances"] = per
        out["traffic_definition"] = ("HBM bytes per E-apply launch, averaged over the phase's "
                                     "instances weighted by their dispatches in the profiled "
                                     "window (as the live time averages every launch)")
    if out.get("bound") == "mfma":
        mf = pmc_mfma(n, p, traffic_world, inst, ctx.get("gram_name"))
        out["mfma_busy_frac"] = mf["mfma_busy_frac"] if mf else None
        out["mfma_busy"] = mf
    out["traffic"] = tb
    out["traffic_unit"] = "HBM bytes per launch (rocprofv3 PMC)"
    out["traffic_source"] = tsrc
    if tnote:
        out["traffic_note"] = tnote
    return out


def fail(msg, code=2):
    log(f"bench.py: ERROR: {msg}")
    raise SystemExit(code)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # M = 1000 timed sweeps after B = 100 burn-in sweeps
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c3",
                    help="BASELINE config (default c3, the headline metric)")
    ap.add_argument("--rows", type=int, default=None)
    ap.add_argument("--cols", type=int, default=None)
    ap.add_argument("--alpha", type=float, default=None)
    ap.add_argument("--cpu-sweeps", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-literal", action="store_true",
                    help="skip the reference-literal p x p CPU sweep for p > 8000 (C3: ~60 s, "
                         "40 GB of host memory)")
    ap.add_argument("--no-parity-check", action="store_true",
                    help="skip the N > 1 pre-timing check of the sharded chain against one "
                         "device holding the whole problem")
    ap.add_argument("--single-process", action="store_true",
                    help="drive --gpus N devices from ONE process through an RCCL shard group "
                         "(ncclCommInitAll) -- the path the .C entry points use under R; the "
                         "default for --gpus N > 1 without a torch.distributed launcher")
    ap.add_argument("--timing-stride", type=int, default=4,
                    help="bracket the dominant kernel with HIP events in every k-th timed sweep")
    ap.add_argument("--no-fitted", action="store_true",
                    help="skip the fitted-regime measurement that follows the timed run")
    ap.add_argument("--gram", choices=["fp64", "ozaki"], default=None,
                    help="dense Woodbury Gram: fp64 MFMA or Ozaki-II int8 MFMA (default: the "
                         "library default, Ozaki)")
    ap.add_argument("--tuning", action="append", default=[], metavar="KEY=VALUE",
                    help="bb_set_tuning(KEY, VALUE) before the engines are built (A/B runs; "
                         "include/bayesbridge.h lists the keys)")
    args = ap.parse_args()
    wn, wp, walpha, kind = WORKLOADS[args.workload]
    n = args.rows or wn
    p = args.cols or wp
    alpha = args.alpha or walpha
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus < 1:
        fail("--gpus must be >= 1")
    if world_env > 1 and world_env != args.gpus:
        fail(f"launched with WORLD_SIZE={world_env} but --gpus={args.gpus}")
    if kind in ("small", "logit") and args.gpus > 1:
        fail(f"workload {args.workload} does not shard (p <= n: replicas only, DESIGN.md s7); "
             f"run it with --gpus 1")
    if kind == "small":
        return small_chain(args, n, p, alpha)
    if world_env > 1:
        mode = "ranks"  # one process per GPU (torch.distributed launcher), RCCL per rank
    elif args.gpus > 1 or args.single_process:
        mode = "group"  # one process drives every GPU (the .C entry points' path)
    else:
        mode = "single"
    return run_chain(args, n, p, alpha, kind, mode)


def shard_bounds(p, world, r):
    per = (p + world - 1) // world
    j0 = min(p, r * per)
    return j0, min(p, j0 + per)


def make_design(kind, n, p, j0, j1):
    if kind == "sparse":
        return make_sparse_columns(n, j0, j1)
    if kind == "logit":
        return make_logit_problem(n, p)[0]
    return make_columns(n, j0, j1)


def make_y(kind, n, p):
    if kind == "sparse":
        return make_sparse_problem_y(n, p)[0]
    if kind == "logit":
        return make_logit_problem(n, p)[1]
    return make_problem_y(n, p)[0]


def run_chain(args, n, p, alpha, kind, mode):
    """C2-C5: one chain of the p > n Woodbury sampler (or the logistic p <= n sampler) on
    --gpus devices.  mode "single": one engine on one GPU; "ranks": this process is rank
    RANK of a torch.distributed job, one GPU and one column shard per rank, RCCL
    all-reduces between ranks; "group": this process drives N GPUs through an RCCL shard
    group, one enqueue thread per device (bb_group_run).  Timing: W warm-up sweeps, then K
    sweeps between barrier + synchronize fences on every device, max over ranks."""
    import torch

    import bayesbridge_amd as bb

    sparse, logit = kind == "sparse", kind == "logit"
    cpu_sweeps = args.cpu_sweeps if args.cpu_sweeps is not None else \
        (5 if sparse else 40 if logit else 5)
    world = args.gpus
    rank = int(os.environ.get("RANK", "0")) if mode == "ranks" else 0
    local_rank = int(os.environ.get("LOCAL_RANK", "0")) if mode == "ranks" else 0
    ndev = torch.cuda.device_count()
    need = world if mode == "group" else local_rank + 1
    if ndev < need:
        fail(f"--gpus {world} ({mode} mode) needs {need} visible GPU(s), found {ndev}; "
             f"refusing to measure fewer GPUs than requested")
    dist = None
    if mode == "ranks":
        import torch.distributed as dist  # noqa: F811

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    devices = list(range(world)) if mode == "group" else [local_rank]
    torch.cuda.set_device(devices[0])
    bb.set_verbose(0)
    for kv in args.tuning:
        k, v = kv.split("=")
        bb.set_tuning(int(k), int(v))
    gram_mode = None if args.gram is None else (bb.GRAM_OZAKI if args.gram == "ozaki"
                                                else bb.GRAM_FP64)
    shard_world = 1 if mode == "single" else world
    my_ranks = list(range(world)) if mode == "group" else [rank]

    def make_engine(r, dev, cap, world_=None, stream=0):
        w_ = shard_world if world_ is None else world_
        j0, j1 = shard_bounds(p, w_, r)
        X = make_design(kind, n, p, j0, j1)
        cfg = bb.EngineConfig(n=n, p=p, p_local=(p if logit else j1 - j0), j0=j0, rank=r,
                              world=w_, true_alpha=alpha, method=6 if logit else 2,
                              trace_capacity=cap, seed=0xB4E5B41D6E, stream=stream,
                              device=dev, gram_mode=gram_mode)
        return bb.Engine(cfg, X, y)

    t_setup0 = time.perf_counter()
    y = make_y(kind, n, p)
    cap = max(1, min(args.steps, 1000))
    engines = [make_engine(r, devices[i], cap) for i, r in enumerate(my_ranks)]
    eng = engines[0]
    grp = None
    forced_old = None  # key 9's value before BB_FORCE_RCCL forced it (restored at the end)
    if mode == "group":
        grp = bb.ShardGroup(engines, rccl=True)
    elif mode == "ranks":
        obj = [bb.Engine.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        eng.comm_init(obj[0])
    elif os.environ.get("BB_FORCE_RCCL", "0") == "1":
        # per-rank proxy of an N-GPU job: a 1-rank RCCL communicator and
        # the world > 1 near-identity protocol forced on it (bb_set_tuning key 9): the bound
        # sums, X u and every product go through ncclAllReduce and the host waits for each
        # sweep's decision, as every rank of the job does
        forced_old = bb.set_tuning(9, 1)
        eng.comm_init(bb.Engine.comm_unique_id())
    runner = grp or eng
    runner.init_state()
    setup_s = time.perf_counter() - t_setup0
    p_loc = eng.p_local
    log(f"[rank {rank}] setup {setup_s:.2f} s  (workload={args.workload}, mode={mode}, n={n}, "
        f"p={p}, p_local={p_loc}, devices={devices}, method={eng.method()})")

    def sync_all():
        runner.sync()
        for d in devices:
            torch.cuda.synchronize(d)

    def barrier():
        if dist:
            dist.barrier()

    parity = None
    if world > 1 and not args.no_parity_check:
        parity = shard_parity_check(bb, dist, rank, engines, my_ranks, runner, make_engine,
                                    devices[0], p, world)
        if not parity["ok"]:
            if rank == 0:
                log(f"bench.py: ERROR: sharded chain differs from the one-device engine: "
                    f"{json.dumps(parity)}")
            raise SystemExit(3)
        runner.init_state()  # restart the chain from the reference start after the check

    t = 1
    runner.run(t, args.warmup, first_slot=-1)
    t += args.warmup
    sync_all()
    # per-phase breakdown (untimed, an event at every phase start of rank 0's sweeps): it
    # also picks the dominant single-kernel phase, whose launches the timed loop brackets
    nph = max(1, min(args.steps, 20))
    eng.enable_timing(True, phases=True)
    eng.reset_timing()
    ph0 = eng.nid_stats()
    runner.run(t, nph, first_slot=-1)
    t += nph
    sync_all()
    phases = eng.phase_times()
    ph1 = eng.nid_stats()
    # the phase-split sweeps took the near-identity path (their Gram phases are no-ops)
    nid_phase_cheb = ph1["mode"] >= 0 and (ph1["cheb_sweeps"] - ph0["cheb_sweeps"]) * 2 > nph
    _, sweep_ms_phases, _ = eng.kernel_times()
    dom = max((ph for ph in SINGLE_KERNEL_PHASES if ph in phases), key=lambda k: phases[k])
    barrier()
    # every stride-th timed sweep brackets its dominant-phase launch (an event pair costs ~6 us
    # of stream time per bracketed sweep: 1-2 % of a near-identity C3 sweep at stride 1); the
    # E-apply's bytes per launch need every launch counted (pass_frac below)
    stride = 1 if dom == "eapply" else max(1, args.timing_stride)
    eng.enable_timing(True, phases=False, timed_phase=dom, stride=stride)
    eng.reset_timing()
    nid0 = eng.nid_stats()
    mix0 = eng.nid_mixed()
    t0 = time.perf_counter()
    # the timed loop records every sweep's beta / lambda / sig2 / tau into the device trace
    # ring, as the reference's MCMC loop writes its output slots (BridgeWrapper.cpp:287-298)
    runner.run(t, args.steps, first_slot=0)
    sync_all()
    elapsed = time.perf_counter() - t0
    t += args.steps
    if dist:
        dist.barrier()
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    dom_ms, _, _ = eng.kernel_times()
    brackets = eng.timed_brackets()
    # the exact kernel instances the timed sweeps launched (the PMC evidence is matched on them)
    instances = {ph: bb.kernel_instance(ph) for ph in SINGLE_KERNEL_PHASES}
    nid1 = eng.nid_stats()
    mix1 = eng.nid_mixed()
    eng.enable_timing(False)
    nid = None
    ctx_pass_frac = 1.0
    ctx_pass32 = 0.0
    if nid1["mode"] >= 0:
        dc = nid1["cheb_sweeps"] - nid0["cheb_sweeps"]
        dp = nid1["products"] - nid0["products"]
        nid = {"timed_sweeps": args.steps, "chebyshev_sweeps": dc,
               "cholesky_sweeps": nid1["chol_sweeps"] - nid0["chol_sweeps"],
               "eapply_passes_per_chebyshev_sweep": (dp / dc) if dc else None,
               "mixed_plan_sweeps": mix1["mixed_sweeps"] - mix0["mixed_sweeps"],
               "fp32_passes_per_chebyshev_sweep": ((mix1["products32"] - mix0["products32"]) / dc
                                                   if dc else None),
               "eps_last": nid1["eps"],
               "rule": "per sweep on the device: Chebyshev iteration on the certified spectrum "
                       "interval [1, 1 + eps], eps >= lambda_max(X D X') / sig2 (the least of "
                       "the trace and thresholded sums + T Lambda, Lambda >= lambda_max(X X') "
                       "certified at setup), when K iterates (at most the cost model's cap) "
                       "bound the relative error of w by 2^-56; else Gram + Cholesky "
                       "(DESIGN.md s6.5)" + (
                           "; column shards decide from the all-reduced shard sums (every rank "
                           "alike) and exchange X u and each product E d" if world > 1 else "")}
        # E-apply launches past a sweep's iteration count return at once: the roofline's
        # bytes per launch are a pass's bytes x (passes run / launches), its time the average
        # over all launches (what a rocprofv3 kernel trace averages)
        ctx_pass_frac = (dp / brackets) if (dom == "eapply" and brackets) else 1.0
        # the mixed plan's products stream the fp32 copy of X (4 B per element)
        ctx_pass32 = ((mix1["products32"] - mix0["products32"]) / brackets
                      if (dom == "eapply" and brackets) else 0.0)
    flags = eng.error_flags()
    st = eng.state()
    if not (math.isfinite(st["tau"]) and math.isfinite(st["sig2"])) or flags:
        log(f"[rank {rank}] WARNING: state tau={st['tau']} sig2={st['sig2']} flags={flags}")

    gram_name = ("pair-list sparse Gram (fp64)" if sparse else
                 ("X'Omega X " if logit else "") +
                 ("ozaki-II int8 (fp64-accurate)" if eng.gram_mode() == bb.GRAM_OZAKI
                  else "fp64 mfma"))
    ctx = dict(bb=bb, eng=eng, kind=kind, n=n, p=p, p_loc=p_loc, gram_mode=eng.gram_mode(),
               gram_name=gram_name, pass_frac=ctx_pass_frac, pass32_frac=ctx_pass32,
               window=(args.steps, args.warmup),
               nid_cheb=nid_phase_cheb,
               instances=instances)
    fitted = None
    if mode == "single" and not logit and not args.no_fitted:
        fitted = fitted_regime(bb, eng, kind, n, p, alpha, t)
        t += 10000
    ref_proto = None
    if mode == "single" and not args.no_fitted:
        ref_proto = reference_protocol(runner, sync_all)
    # the Gram's instances as launched (by the fitted-regime run when the timed sweeps formed none)
    ctx_gram = dict(ctx, instances=dict(instances, **{
        ph: instances.get(ph) or bb.kernel_instance(ph) for ph in ("gram", "reduce", "chol")}))
    traffic_world = 1 if mode == "single" else world
    roof = roofline_for(dom, dom_ms, ctx, traffic_world)
    roof["timing"] = ("HIP events on rank 0's engine stream around "
                      + ("every timed launch" if stride == 1 else
                         f"the launch of every {stride}th timed sweep ({brackets} launches)"))
    secondary = None
    # the Gram's roofline beside the dominant kernel's: from this run's phase split when its
    # sweeps formed the Gram, else from the fitted-regime run (near-identity sweeps skip it)
    gram_src = (phases, f"HIP events at phase starts, {nph} untimed sweeps")
    if nid_phase_cheb and fitted:
        gram_src = (fitted["phases_ms"], "HIP events at phase starts, fitted-regime run")
    if dom != "gram" and "gram" in gram_src[0] and not (nid_phase_cheb and not fitted):
        secondary = roofline_for("gram", gram_src[0]["gram"], ctx_gram, traffic_world)
        secondary["timing"] = gram_src[1]
    gram_total_ms = sum(phases.get(k, 0.0) for k in ("ozprep", "gram", "reduce"))

    cpu = cpu_more = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and cpu_sweeps > 0:
        cpu, cpu_more = cpu_baselines(args, n, p, alpha, kind, cpu_sweeps)

    value = args.steps / elapsed
    if rank == 0:
        wl = {"c2": "C2 Gaussian bridge", "c3": "C3 Gaussian bridge",
              "c4": "C4 logistic bridge (Polya-Gamma)",
              "c5": f"C5 sparse CSC Gaussian bridge (density {SPARSE_DENSITY})"}[args.workload]
        par = {"single": "one GPU",
               "ranks": f"column-shard x{world}, one process per GPU, RCCL all-reduce",
               "group": f"column-shard x{world}, one process (RCCL shard group, "
                        f"ncclCommInitAll, one enqueue thread per GPU)"}[mode]
        config = {"workload": f"{wl} n={n} p={p} alpha={alpha}", "n": n, "p": p,
                  "alpha": alpha, "mode": mode, "parallelism": par,
                  "beta_step": ("p x p Cholesky of X'Omega X + diag(lambda/tau^2)" if logit
                                else "woodbury (exact, p > n)")}
        config["gram"] = gram_name
        if mode == "single" and os.environ.get("BB_FORCE_RCCL", "0") == "1":
            config["proxy"] = ("one rank's share: a 1-rank RCCL communicator with the column-"
                               "shard protocol forced (bb_set_tuning key 9)")
        if args.tuning:
            config["tuning"] = list(args.tuning)
            if any(kv.split("=")[0] == "16" and kv.split("=")[1] != "0" for kv in args.tuning):
                config["forced_iterates"] = ("bb_set_tuning key 16: the near-identity solve runs "
                                             "this many Chebyshev iterates every sweep instead "
                                             "of its certified count (a timing proxy, not a "
                                             "certified chain)")
        if sparse:
            si = eng.sparse_info()
            config.update(density=SPARSE_DENSITY, nnz_local=si["nnz"], pairs_local=si["pairs"],
                          max_row_nnz=si["max_row"])
        rec = {
            "metric": f"Gibbs sweeps/sec at n={n},p={p},alpha={alpha}",
            "value": value,
            "unit": "sweeps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1000.0 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("synthetic (SURVEY.md 8(d) design, seed 20240501"
                     + (f", Bernoulli({SPARSE_DENSITY}) sparsity)" if sparse else ")")),
            "config": config,
            "roofline": roof,
            "roofline_secondary": secondary,
            "phases_ms": {k: round(v, 4) for k, v in phases.items()},
            "sweep_ms_phase_events": sweep_ms_phases,
            "gram_total_ms": gram_total_ms,
            "cpu_baseline": cpu,
            "parity_check": parity,
            "setup_s": setup_s,
            "near_identity": nid,
            "fitted_regime": fitted,
            "reference_protocol": ref_proto,
        }
        if cpu_more:
            rec["cpu_baselines"] = cpu_more
        print(json.dumps(rec), flush=True)
    if grp:
        grp.close()
    for e in engines:
        e.close()
    if forced_old is not None:
        bb.set_tuning(9, forced_old)  # the setting is process-global
    if dist:
        dist.destroy_process_group()


def reference_protocol(runner, sync_all, burn=500, nsamp=1000):
    """The reference's default call, timed on the same engine:
    bridge.reg.stb(y, X, nsamp = 1000, burn = 500) (BridgeWrapper.R:194-201) from the
    reference start (beta = 0 for p > n, BridgeWrapper.cpp:242-244): burn + 1 burn-in sweeps
    then nsamp - 1 MCMC sweeps recorded into the trace (BridgeWrapper.cpp:266-298).  `value` is
    the post-burn rate the reference's `runtime` out-parameter measures (BridgeWrapper.cpp:
    284-311), `call_sweeps_per_s` the whole call's."""
    runner.init_state()
    sync_all()
    t0 = time.perf_counter()
    runner.run(1, burn + 1, first_slot=-1)
    sync_all()
    t1 = time.perf_counter()
    runner.run(burn + 2, nsamp - 1, first_slot=0)
    sync_all()
    t2 = time.perf_counter()
    return {"value": (nsamp - 1) / (t2 - t1), "unit": "sweeps/s",
            "call_sweeps_per_s": (burn + nsamp) / (t2 - t0),
            "burn": burn, "nsamp": nsamp, "burn_s": t1 - t0, "mcmc_s": t2 - t1,
            "protocol": "bridge.reg.stb defaults (BridgeWrapper.R:194-201): burn-in 500 + 1 "
                        "sweeps, then 999 MCMC sweeps recorded, from the reference start; value = "
                        "MCMC sweeps / post-burn wall time (the reference's runtime is post-burn "
                        "CPU time)"}


def fitted_regime(bb, eng, kind, n, p, alpha, t, warm=20, steps=50):
    """The same engine timed in the fitted regime: the chain restarted at
    the data-generating coefficients with tau = 1e-2, sig2 = 1, `warm` untimed sweeps, then
    `steps` sweeps between stream synchronisations, with the per-phase split and the path the
    Woodbury solve took.  (From the reference start a C3 chain stays in the near-null regime
    for thousands of sweeps; the C5 posterior collapses back to it within a few sweeps,
    whatever the start.)"""
    _, btrue = (make_sparse_problem_y(n, p) if kind == "sparse" else make_problem_y(n, p))
    eng.set_state(btrue[:eng.p_local], 1e-2, 1.0, alpha)
    eng.run(t, warm, first_slot=-1)
    eng.sync()
    s0 = eng.nid_stats()
    t0 = time.perf_counter()
    eng.run(t + warm, steps, first_slot=-1)  # timed without events
    eng.sync()
    el = time.perf_counter() - t0
    s1 = eng.nid_stats()
    st = eng.state()
    eng.enable_timing(True, phases=True)  # then 10 sweeps with the per-phase split
    eng.reset_timing()
    eng.run(t + warm + steps, 10, first_slot=-1)
    eng.sync()
    phases = eng.phase_times()
    eng.enable_timing(False)
    return {"value": steps / el, "unit": "sweeps/s", "ms_per_step": 1e3 * el / steps,
            "steps": steps, "warmup": warm,
            "start": "beta = data-generating coefficients, tau = 1e-2, sig2 = 1",
            "state_after": {"tau": st["tau"], "sig2": st["sig2"],
                            "coefficients_above_1e-3": int(np.sum(np.abs(st["beta"]) > 1e-3))},
            "chebyshev_sweeps": (s1["cheb_sweeps"] - s0["cheb_sweeps"]) if s1["mode"] >= 0 else 0,
            "eps_last": s1["eps"],
            "phases_ms": {k: round(v, 4) for k, v in phases.items()},
            "timing": "wall clock around the timed sweeps (no events); phases_ms from 10 more "
                      "sweeps with an event at every phase start"}


def shard_parity_check(bb, dist, rank, engines, my_ranks, runner, make_engine, dev0, p, world,
                       k0=6, sweeps=2):
    """Before timing an N > 1 run: two teacher-forced sweeps of the sharded chain against ONE
    engine holding the whole problem on rank 0's device (the same counters, so the only
    difference is the fp64 summation order of the Gram, S_alpha and X beta).  Start: the
    one-device chain after k0 sweeps from beta = 0.  Bars as
    tests/test_gpu_parity.py::test_shard_group_matches_single_engine (beta 1e-9 relative L2,
    lambda 1e-10 with no decision flips, tau 1e-12, sig2 1e-11).  Returns a dict with the
    errors and `ok` (the same on every rank)."""
    ref = None
    state = None
    if rank == 0:
        ref = make_engine(0, dev0, 1, world_=1, stream=0)
        ref.init_state()
        ref.run(1, k0, first_slot=-1)
        ref.sync()
        state = ref.state()
    errs = {"beta_rel_l2": 0.0, "lambda_max_rel": 0.0, "lambda_flips": 0, "tau_rel": 0.0,
            "sig2_rel": 0.0}
    for s in range(sweeps):
        if dist:
            obj = [state]
            dist.broadcast_object_list(obj, src=0)
            state = obj[0]
        t = 1_000_000 + s  # counters of their own: the check is not part of the chain
        for e, r in zip(engines, my_ranks):
            j0, j1 = shard_bounds(p, world, r)
            e.set_state(state["beta"][j0:j1], state["tau"], state["sig2"], state["alpha"])
        runner.run(t, 1, first_slot=-1)
        runner.sync()
        parts = [(r, e.state()) for e, r in zip(engines, my_ranks)]
        if dist:
            gathered = [None] * world
            dist.all_gather_object(gathered, parts)
            parts = [x for g in gathered for x in g]
        if rank == 0:
            parts.sort(key=lambda q: q[0])
            bg = np.concatenate([q[1]["beta"] for q in parts])
            lg = np.concatenate([q[1]["lambda"] for q in parts])
            ref.set_state(state["beta"], state["tau"], state["sig2"], state["alpha"])
            ref.run(t, 1, first_slot=-1)
            ref.sync()
            r1 = ref.state()
            lr = np.abs(lg - r1["lambda"]) / np.maximum(np.abs(r1["lambda"]), 1e-300)
            e0 = parts[0][1]
            errs["beta_rel_l2"] = max(errs["beta_rel_l2"], rel_l2(bg, r1["beta"]))
            errs["lambda_max_rel"] = max(errs["lambda_max_rel"], float(lr.max()))
            errs["lambda_flips"] += int(np.sum(lr > 1e-6))
            errs["tau_rel"] = max(errs["tau_rel"], abs(e0["tau"] - r1["tau"]) / r1["tau"])
            errs["sig2_rel"] = max(errs["sig2_rel"], abs(e0["sig2"] - r1["sig2"]) / r1["sig2"])
            state = r1
    ok = None
    if rank == 0:
        ok = (errs["beta_rel_l2"] <= 1e-9 and errs["lambda_max_rel"] <= 1e-10
              and errs["lambda_flips"] == 0 and errs["tau_rel"] <= 1e-12
              and errs["sig2_rel"] <= 1e-11)
        ref.close()
    if dist:
        obj = [(ok, errs)]
        dist.broadcast_object_list(obj, src=0)
        ok, errs = obj[0]
    return dict(ok=bool(ok), sweeps=sweeps, start=f"one-device chain after {k0} sweeps",
                against="one engine holding all p columns on rank 0's device", **errs)


def literal_fits(p):
    """Host memory for the reference-literal chain's two p x p matrices (X'X and the factor)
    with a 2x margin."""
    try:
        import psutil
        return psutil.virtual_memory().available > 4 * 8.0 * p * p
    except Exception:
        return False


def cpu_baselines(args, n, p, alpha, kind, cpu_sweeps):
    """The cpu_baseline leg (rank 0, N = 1 only), timed on this host."""
    sparse, logit = kind == "sparse", kind == "logit"
    log(f"[cpu_baseline] timing {cpu_sweeps} CPU sweeps at n={n}, p={p} ...")
    if sparse:
        per_sweep, threads = cpu_baseline_sparse(n, p, alpha, cpu_sweeps)
        what = ("compiled C sparse Woodbury chain (oracle/bb_cpu_chain.c: OpenMP sparse Gram "
                "by output column + dpotrf, scipy OpenBLAS, OpenMP lambda draws)")
    elif logit:
        per_sweep, threads = cpu_baseline_logit(n, p, alpha, cpu_sweeps)
        what = ("compiled C logistic chain (oracle/bb_cpu_chain.c: dsyrk X'Omega X + dpotrf, "
                "scipy OpenBLAS, OpenMP Polya-Gamma and lambda draws)")
    else:
        per_sweep, threads = cpu_baseline(n, p, alpha, cpu_sweeps)
        what = ("compiled C Woodbury chain (oracle/bb_cpu_chain.c: dsyrk + dpotrf + dgemv, "
                "scipy OpenBLAS, OpenMP lambda draws)")
    cpu = {"value": 1.0 / per_sweep, "unit": "sweeps/s", "cores": threads, "kind": "port",
           "sample": f"{cpu_sweeps} {what} at n={n}, p={p}, {threads} threads; "
                     f"{per_sweep:.3f} s per sweep"}
    # the CPU baseline at 1 core and all cores, for the algorithm-matched
    # Woodbury chain and (p <= 8000) the reference-literal p x p path
    cpu_more = None
    if sparse or logit:
        # the same compiled chain on one core
        ns = max(1, min(cpu_sweeps, 2 if sparse else 3))
        per1, th1 = (cpu_baseline_sparse if sparse else cpu_baseline_logit)(n, p, alpha, ns,
                                                                            threads=1)
        cpu_more = [dict(cpu, path="all cores"),
                    {"value": 1.0 / per1, "unit": "sweeps/s", "cores": th1, "kind": "port",
                     "path": "1 core", "sample": f"{ns} sweeps of the same compiled C chain, "
                                                 f"{per1:.3f} s per sweep"}]
    if kind == "dense":
        cpu_more = [dict(cpu, path="Woodbury (algorithm-matched to the GPU)")]
        variants = [(False, 1, max(1, min(cpu_sweeps, 3)))]
        if p <= 8000:
            variants += [(True, None, 3), (True, 1, 2)]
        elif literal_fits(p) and not args.no_literal:
            # the reference-literal p x p path in the same run (C3: X'X is
            # 20 GB, one dpotrf of p = 50 000 per sweep, ~60 s with its setup on 16 threads)
            variants += [(True, None, 1)]
        for lit, th, ns in variants:
            per_sweep, threads = cpu_baseline(n, p, alpha, ns, threads=th, literal=lit)
            cpu_more.append({
                "value": 1.0 / per_sweep, "unit": "sweeps/s", "cores": threads, "kind": "port",
                "path": ("reference-literal p x p Cholesky (dpotrf p=%d)" % p if lit
                         else "Woodbury (algorithm-matched to the GPU)"),
                "sample": f"{ns} sweeps of the compiled C chain, {per_sweep:.3f} s per sweep"})
    return cpu, cpu_more


def small_phase_model(n, p):
    """The in-kernel phase split of the fused small-p sweep for this (n, p) from the committed
    tools/small_phase_bench output (profiles/r*_c1_small_phases.txt), or None."""
    import glob
    import re

    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_c1_small_phases.txt"))):
        for line in open(f):
            m = re.match(r"n=(\d+) p=(\d+) ortho=0: ([\d.]+) us/sweep \(rss ([\d.]+), "
                         r"tau/sig2 ([\d.]+), lambda ([\d.]+), beta ([\d.]+) us\)", line)
            if m and int(m.group(1)) == n and int(m.group(2)) == p:
                v = [float(m.group(i)) for i in range(3, 8)]
                best = {"source": os.path.relpath(f, ROOT), "us_per_sweep_in_kernel": v[0],
                        "phases_us": {"S_alpha_rss": v[1], "tau_sig2": v[2], "lambda": v[3],
                                      "beta_chol_solves": v[4]}}
    return best


def small_chain(args, n, p, alpha):
    """C1 (BASELINE configs[0], p <= n): the reference-literal p x p path, run as the .C
    driver runs it -- one bridge_reg_stable call, W burn-in and K recorded sweeps; with p <= 32
    every block of sweeps is one single-workgroup launch.  `value` is K / the
    call's post-burn runtime.  The CPU baseline is the compiled reference-literal chain
    (oracle/bb_cpu_chain.c: p x p dpotrf + dtrsm on scipy's OpenBLAS + the C samplers, one
    thread) over a bounded number of sweeps."""
    import torch  # noqa: F401  (device init on the same footing as the other workloads)

    import bayesbridge_amd as bb

    X = make_columns(n, 0, p)
    y, _ = make_problem_y(n, p)
    bb.set_verbose(0)
    bb.set_seed(0xB4E5B41D6E)
    t_setup0 = time.perf_counter()
    out = bb.bridge_reg_stb(y, X, nsamp=args.steps, burn=args.warmup, alpha=alpha)
    wall = time.perf_counter() - t_setup0
    runtime = float(out["runtime"])
    value = args.steps / runtime
    cpu = None
    if not args.no_cpu_baseline:
        import oracle

        ns = args.cpu_sweeps if args.cpu_sweeps is not None else 20000
        r = oracle.cpu_chain(y, X, ns + 1, burn=0, alpha=alpha, method="chol",
                             seed=0xB4E5B41D6E, threads=1, record=False)
        per = r["runtime"] / ns
        cpu = {"value": 1.0 / per, "unit": "sweeps/s", "cores": 1, "kind": "port",
               "sample": f"{ns} sweeps of the compiled C reference-literal chain "
                         f"(oracle/bb_cpu_chain.c: p x p dpotrf + dtrsm, scipy OpenBLAS, "
                         f"1 thread) at n={n}, p={p}"}
    # The fused chain is one workgroup running dependent draws: no flop or byte roofline
    # bounds it (p^3/3 + 3p^2 + 2np = 8e3 flop per sweep at C1).  Its bound is latency: the
    # per-sweep chain of S_alpha/rss -> tau, sig2 -> lambda (p rejection draws in parallel,
    # the slowest decides) -> the p x p Cholesky and solves, measured in-kernel by
    # tools/small_phase_bench (profiles/r03_c1_small_phases.txt, s_memrealtime per phase).
    lat = small_phase_model(n, p)
    roof = {"bound": "latency", "kernel": "k_small_chain (whole sweeps in one workgroup)",
            "achieved": 1e6 / value, "unit": "us per sweep", "peak": None, "frac": None,
            "traffic": None, "latency_model": lat}
    rec = {
        "metric": f"Gibbs sweeps/sec at n={n},p={p},alpha={alpha}",
        "value": value, "unit": "sweeps/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": 1000.0 * runtime / args.steps,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (SURVEY.md 8(d) design, seed 20240501)",
        "config": {"workload": f"C1 Gaussian bridge n={n} p={p} alpha={alpha}", "n": n, "p": p,
                   "alpha": alpha, "beta_step": "p x p Cholesky (reference-literal)",
                   "parallelism": "replicas only (p <= n)",
                   "kernel": "k_small_chain (whole sweeps in one workgroup)"},
        "roofline": roof,
        "cpu_baseline": cpu, "call_wall_s": wall,
    }
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
