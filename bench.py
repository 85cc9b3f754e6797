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


def cpu_baseline_logit(n, p, alpha, sweeps, log_every=True):
    """Oracle logistic sweeps (numpy X'Omega X, LAPACK Cholesky, C PG and tilted-stable
    samplers).  Returns (median s per sweep, threads)."""
    from oracle import gibbs

    X, y, _ = make_logit_problem(n, p)
    beta, tau = np.zeros(p), 1.0
    times = []
    for t in range(1, sweeps + 1):
        t0 = time.perf_counter()
        beta, _, tau, _ = gibbs.logit_sweep(X, y, beta, tau, alpha, t, 1, 0)
        times.append(time.perf_counter() - t0)
        if log_every:
            log(f"[cpu_baseline] logistic sweep {t}: {times[-1]:.3f} s")
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return float(np.median(times)), threads


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


def cpu_baseline_sparse(n, p, alpha, sweeps, log_every=True):
    """Oracle Woodbury sweeps on the sparse design (scipy SpGEMM X diag(D) X', LAPACK
    Cholesky, the C tilted-stable sampler).  Returns (median s per sweep, threads)."""
    import oracle
    from oracle import gibbs

    X = make_sparse_columns(n, 0, p)
    y, _ = make_sparse_problem_y(n, p)
    beta = np.zeros(p)
    times = []
    for t in range(1, sweeps + 1):
        t0 = time.perf_counter()
        tau = oracle.tau_from_sum(oracle.sum_abs_pow(beta, alpha), p, alpha, 2.0, 2.0, 1, 0, t)
        r = y - X @ beta
        sig2 = oracle.sig2_from_rss(float(r @ r), n, 0.0, 0.0, 1, 0, t)
        lam = oracle.sample_lambda(beta, alpha, tau, 1, 0, t)
        z = oracle.normals(p, 1, 0, t, oracle.KIND_BETA_Z)
        d = oracle.normals(n, 1, 0, t, oracle.KIND_DELTA)
        beta = gibbs.beta_step_woodbury(X, y, lam, sig2, tau, z, d)
        times.append(time.perf_counter() - t0)
        if log_every:
            log(f"[cpu_baseline] sparse sweep {t}: {times[-1]:.3f} s")
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return float(np.median(times)), threads


def blas_threads(threads):
    """Context limiting the BLAS pools to `threads` (None: leave them as they are)."""
    import contextlib

    if threads is None:
        return contextlib.nullcontext()
    from threadpoolctl import threadpool_limits
    return threadpool_limits(limits=threads)


def cpu_baseline(n, p, alpha, sweeps, log_every=True, threads=None, literal=False):
    """Oracle sweeps on the host: the CPU restatement of the reference sweep.  Default: the
    Woodbury draw, algorithm-matched to the GPU path (reference-literal p x p Cholesky at
    p=50000 needs a 20 GB Gram and ~4e13 flop per sweep).  literal=True: the reference's own
    p x p path (BridgeRegression.cpp:24-25 X'X and X'y once, then per sweep
    :552-575 dpotrf of X'X + diag(lambda sig2 / tau^2) and three triangular solves).
    threads: BLAS threads (None = the environment's).  Returns (median s per sweep, threads)."""
    import oracle
    from oracle import gibbs

    X = make_columns(n, 0, p)
    y, _ = make_problem_y(n, p)
    beta = np.zeros(p)
    tau, sig2 = 1.0, 1.0
    times = []
    with blas_threads(threads):
        if literal:
            G, c = X.T @ X, X.T @ y
        for t in range(1, sweeps + 1):
            t0 = time.perf_counter()
            tau = oracle.tau_from_sum(oracle.sum_abs_pow(beta, alpha), p, alpha, 2.0, 2.0, 1, 0,
                                      t)
            r = y - X @ beta
            sig2 = oracle.sig2_from_rss(float(r @ r), n, 0.0, 0.0, 1, 0, t)
            lam = oracle.sample_lambda(beta, alpha, tau, 1, 0, t)
            z = oracle.normals(p, 1, 0, t, oracle.KIND_BETA_Z)
            if literal:
                beta = gibbs.beta_step_chol(G, c, lam, sig2, tau, z)
            else:
                d = oracle.normals(n, 1, 0, t, oracle.KIND_DELTA)
                beta = gibbs.beta_step_woodbury(X, y, lam, sig2, tau, z, d)
            times.append(time.perf_counter() - t0)
            if log_every:
                log(f"[cpu_baseline] {'literal' if literal else 'woodbury'} "
                    f"threads={threads or 'env'} sweep {t}: {times[-1]:.3f} s")
    # first sweep starts from beta = 0 (all lambda draws at h = 0); report the median
    per = float(np.median(times))
    if threads is None:
        threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return per, threads


def pmc_traffic(n, p, world, kernel):
    """HBM bytes per k_gram launch from the newest committed PMC summary of this workload
    (profiles/rNN_pmc.json, written by tools/profile_round.sh + tools/profile_summary.py:
    separate FETCH_SIZE / WRITE_SIZE passes, gfx950 x2 read correction).  None if absent or
    for a different workload / world size."""
    import glob

    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        w = d.get("workload", {})
        gk = d.get("gram_kernels", {})
        if w.get("n") != n or w.get("p") != p or world != 1:
            continue
        for k in gk:  # exact name, or the prefix of a template instantiation
            if k == kernel or k.startswith(kernel + "<"):
                best = (gk[k]["hbm_bytes_per_launch"], os.path.relpath(f, ROOT))
    return best


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
    ap.add_argument("--single-process", action="store_true",
                    help="drive --gpus N devices from ONE process through an RCCL shard group "
                         "(ncclCommInitAll) -- the path the .C entry points use under R")
    ap.add_argument("--gram", choices=["fp64", "ozaki"], default=None,
                    help="dense Woodbury Gram: fp64 MFMA or Ozaki-II int8 MFMA (default: the "
                         "library default, Ozaki)")
    args = ap.parse_args()
    wn, wp, walpha, kind = WORKLOADS[args.workload]
    sparse, logit = kind == "sparse", kind == "logit"
    n = args.rows or wn
    p = args.cols or wp
    alpha = args.alpha or walpha
    cpu_sweeps = args.cpu_sweeps if args.cpu_sweeps is not None else \
        (2 if sparse else 20 if logit else 5)

    if kind == "small":
        return small_chain(args, n, p, alpha)
    if args.single_process:
        return single_process(args, n, p, alpha, kind)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE")
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)

    import torch

    import bayesbridge_amd as bb

    # every rank drives its own GPU; torch's current device must match for the
    # torch.cuda.synchronize() fences of the timing protocol
    ndev = max(1, torch.cuda.device_count())
    device = local_rank % ndev
    torch.cuda.set_device(device)

    bb.set_verbose(0)
    per = (p + world - 1) // world
    j0 = min(p, rank * per)
    j1 = min(p, j0 + per)
    p_loc = j1 - j0
    t_setup0 = time.perf_counter()
    if logit and world > 1:
        raise SystemExit("the logistic workload runs on one GPU (replicas only)")
    if sparse:
        X = make_sparse_columns(n, j0, j1)
        y, _ = make_sparse_problem_y(n, p)
        nnz_loc = int(X.nnz)
    elif logit:
        X, y, _ = make_logit_problem(n, p)
        nnz_loc = n * p
    else:
        X = make_columns(n, j0, j1)
        y, _ = make_problem_y(n, p)
        nnz_loc = n * p_loc
    cfg = bb.EngineConfig(n=n, p=p, p_local=p_loc, j0=j0, rank=rank, world=world,
                          true_alpha=alpha, method=6 if logit else 2,
                          trace_capacity=max(1, min(args.steps, 1000)), seed=0xB4E5B41D6E,
                          stream=0, device=device,
                          gram_mode=None if args.gram is None else
                          (bb.GRAM_OZAKI if args.gram == "ozaki" else bb.GRAM_FP64))
    eng = bb.Engine(cfg, X, y)
    del X
    force_rccl = os.environ.get("BB_FORCE_RCCL", "0") == "1"
    if world > 1:
        if rank == 0:
            uid = bb.Engine.comm_unique_id()
            obj = [uid]
        else:
            obj = [None]
        dist.broadcast_object_list(obj, src=0)
        eng.comm_init(obj[0])
    elif force_rccl:
        # exercise the RCCL exchange path on one GPU (1-rank communicator)
        eng.comm_init(bb.Engine.comm_unique_id())
    eng.init_state()
    setup_s = time.perf_counter() - t_setup0
    log(f"[rank {rank}] setup {setup_s:.2f} s  (workload={args.workload}, n={n}, p={p}, "
        f"p_local={p_loc}, method={eng.method()})")

    t = 1
    eng.run(t, args.warmup, first_slot=-1)
    t += args.warmup
    eng.sync()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    # inside the timed region only the Gram kernel is bracketed by HIP events (two per sweep)
    eng.enable_timing(True, phases=False)
    eng.reset_timing()
    t0 = time.perf_counter()
    # the timed loop records every sweep's beta / lambda / sig2 / tau into the device trace
    # ring, as the reference's MCMC loop writes its output slots (BridgeWrapper.cpp:287-298)
    eng.run(t, args.steps, first_slot=0)
    eng.sync()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    t += args.steps
    if dist:
        dist.barrier()
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    gram_ms, _, nsamp = eng.kernel_times()
    # per-phase breakdown from a short untimed run with an event at every phase start
    eng.enable_timing(True, phases=True)
    eng.reset_timing()
    nph = max(1, min(args.steps, 20))
    eng.run(t, nph, first_slot=-1)
    eng.sync()
    t += nph
    phases = eng.phase_times()
    _, sweep_ms, _ = eng.kernel_times()
    eng.enable_timing(False)
    flags = eng.error_flags()
    st = eng.state()
    if not (math.isfinite(st["tau"]) and math.isfinite(st["sig2"])) or flags:
        log(f"[rank {rank}] WARNING: state tau={st['tau']} sig2={st['sig2']} flags={flags}")

    value = args.steps / elapsed
    ms_per_step = 1000.0 * elapsed / args.steps
    gram_mode = eng.gram_mode()
    gram_flops = float(n) * (n + 1) * p_loc
    n_pad = -(-n // 128) * 128
    ntri = n_pad * (n_pad + 1) // 2
    if sparse:
        # Dominant kernel = the pair-list sparse Gram, HBM-bound.  By-column
        # kernel, per launch: the pair stream (8 B product + 2 B row position per pair), the
        # segment starts (4 B per packed entry) and the packed triangle written (8 B per
        # entry), the CSR rows (4 B index + 8 B value per non-zero) and D, u (8 B each per
        # column).  The general kernel streams 4 B column indices instead and gathers D.
        si = eng.sparse_info()
        pairs = si["pairs"]
        if si["col_mode"]:
            kernel_bytes = 10.0 * pairs + 12.0 * ntri + 12.0 * si["nnz"] + 16.0 * p_loc
            kname = "k_sp_gram_col (pair-list Gram by output column)"
            kfull = "bb::k_sp_gram_col"
        else:
            kernel_bytes = 12.0 * pairs + 12.0 * ntri + 8.0 * p_loc
            kname = "k_sp_gram (pair-list Gram)"
            kfull = "bb::k_sp_gram"
        achieved = kernel_bytes / (gram_ms * 1e-3) / 1e9 if gram_ms > 0 else 0.0
        peak, unit, bound = 8000.0, "GB/s", "hbm"
        kernel_ops = kernel_bytes
        alg_bytes = kernel_bytes
        traffic = pmc_traffic(n, p, world, kfull)
    elif logit and gram_mode == bb.GRAM_OZAKI:
        # Dominant kernel = the per-sweep X'Omega X as the Ozaki-II int8 Gram of X' diag(omega)
        # (rows = coefficients, K = observations): kOzMods x p(p+1) n int8 ops per launch
        kernel_ops = 16.0 * p * (p + 1) * n
        achieved = kernel_ops / (gram_ms * 1e-3) / 1e12 if gram_ms > 0 else 0.0
        peak, unit, kname, bound = (INT8_MFMA_PEAK_TOPS, "TOP/s",
                                    "k_oz_gemm16u X'Omega X (v_mfma_i32_16x16x64_i8)", "mfma")
        alg_bytes = 16.0 * n * p
        traffic = pmc_traffic(n, p, world, "bb::k_oz_gemm16u")
    elif logit:
        # Dominant kernel = the per-sweep X'Omega X (fp64 MFMA k_gram over K = n rows):
        # n p (p + 1) algorithmic flops per launch (path p <= n, C4)
        kernel_ops = float(n) * p * (p + 1)
        achieved = kernel_ops / (gram_ms * 1e-3) / 1e12 if gram_ms > 0 else 0.0
        peak, unit, kname, bound = (FP64_MFMA_PEAK_TFLOPS, "TFLOP/s",
                                    "k_gram X'Omega X (v_mfma_f64_16x16x4_f64)", "mfma")
        alg_bytes = 8.0 * n * p
        traffic = pmc_traffic(n, p, world, "bb::k_gram")
    elif gram_mode == bb.GRAM_OZAKI:
        # Dominant kernel = the Gram GEMM: algorithmic int8 ops of one k_oz_gemm launch,
        # kOzMods x n(n+1) p_local (16 exact symmetric int8 Grams).
        kernel_ops = 16.0 * n * (n + 1) * p_loc
        achieved = kernel_ops / (gram_ms * 1e-3) / 1e12 if gram_ms > 0 else 0.0
        peak, unit, kname, bound = (INT8_MFMA_PEAK_TOPS, "TOP/s",
                                    "k_oz_gemm16u (v_mfma_i32_16x16x64_i8)", "mfma")
        alg_bytes = 16.0 * n * p_loc
        traffic = pmc_traffic(n, p, world, "bb::k_oz_gemm16u")
    else:
        # fp64 path: algorithmic fp64 flops of one k_gram launch, n(n+1) p_local
        kernel_ops = gram_flops
        achieved = kernel_ops / (gram_ms * 1e-3) / 1e12 if gram_ms > 0 else 0.0
        peak, unit, kname, bound = (FP64_MFMA_PEAK_TFLOPS, "TFLOP/s",
                                    "k_gram (v_mfma_f64_16x16x4_f64)", "mfma")
        alg_bytes = 8.0 * n * p_loc
        traffic = pmc_traffic(n, p, world, "bb::k_gram")
    gram_total_ms = gram_ms + phases.get("ozprep", 0.0) + phases.get("reduce", 0.0)
    # the dense Gram's fp64-equivalent rate (meaningless for the sparse design)
    if logit:
        gram_flops = float(n) * p * (p + 1)
    fp64_equiv = (gram_flops / (gram_total_ms * 1e-3) / 1e12
                  if gram_total_ms > 0 and kind in ("dense", "logit") else None)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and cpu_sweeps > 0:
        log(f"[cpu_baseline] timing {cpu_sweeps} oracle sweeps at n={n}, p={p} ...")
        if sparse:
            per_sweep, threads = cpu_baseline_sparse(n, p, alpha, cpu_sweeps)
            what = "scipy SpGEMM + LAPACK"
        elif logit:
            per_sweep, threads = cpu_baseline_logit(n, p, alpha, cpu_sweeps)
            what = "numpy X'Omega X + LAPACK + C Polya-Gamma sampler"
        else:
            per_sweep, threads = cpu_baseline(n, p, alpha, cpu_sweeps)
            what = "numpy/OpenBLAS"
        cpu = {"value": 1.0 / per_sweep, "unit": "sweeps/s", "cores": threads, "kind": "port",
               "sample": f"{cpu_sweeps} {'logistic' if logit else 'Woodbury'} sweeps of the "
                         f"oracle ({what}, "
                         f"{threads} threads, + C tilted-stable sampler) at n={n}, p={p}; "
                         f"median sweep {per_sweep:.3f} s"}

    # C2: the CPU baseline at 1 core and all cores, for the Woodbury port and
    # for the reference-literal p x p path (dpotrf at p = 5000)
    cpu_more = None
    if (cpu is not None and args.workload == "c2" and p <= 8000):
        cpu_more = []
        for lit in (False, True):
            for th in (1, None):
                if not lit and th is None:
                    per_sweep, threads = 1.0 / cpu["value"], cpu["cores"]
                else:
                    per_sweep, threads = cpu_baseline(n, p, alpha, cpu_sweeps, threads=th,
                                                      literal=lit)
                cpu_more.append({
                    "value": 1.0 / per_sweep, "unit": "sweeps/s", "cores": threads,
                    "kind": "port",
                    "path": ("reference-literal p x p Cholesky (dpotrf p=%d)" % p if lit
                             else "Woodbury (algorithm-matched to the GPU)"),
                    "sample": f"{cpu_sweeps} sweeps, median {per_sweep:.3f} s"})

    if rank == 0:
        wl = {"c1": "C1 Gaussian bridge", "c2": "C2 Gaussian bridge", "c3": "C3 Gaussian bridge",
              "c4": "C4 logistic bridge (Polya-Gamma)",
              "c5": f"C5 sparse CSC Gaussian bridge (density {SPARSE_DENSITY})"}[args.workload]
        config = {"workload": f"{wl} n={n} p={p} alpha={alpha}",
                  "rccl": bool(world > 1 or force_rccl),
                  "n": n, "p": p, "alpha": alpha,
                  "beta_step": ("p x p Cholesky of X'Omega X + diag(lambda/tau^2)" if logit
                                else "woodbury (exact, p > n)"),
                  "parallelism": f"column-shard x{world}" + (" + RCCL all-reduce"
                                                             if world > 1 else "")}
        if sparse:
            si = eng.sparse_info()
            config.update(gram="pair-list sparse Gram (fp64)", density=SPARSE_DENSITY,
                          nnz_local=si["nnz"], pairs_local=si["pairs"], max_row_nnz=si["max_row"])
        elif logit:
            config["gram"] = ("X'Omega X ozaki-II int8 (fp64-accurate)"
                              if gram_mode == bb.GRAM_OZAKI else "X'Omega X fp64 mfma")
        else:
            config["gram"] = ("ozaki-II int8 (fp64-accurate)" if gram_mode == bb.GRAM_OZAKI
                              else "fp64 mfma")
        rec = {
            "metric": f"Gibbs sweeps/sec at n={n},p={p},alpha={alpha}",
            "value": value,
            "unit": "sweeps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("synthetic (SURVEY.md 8(d) design, seed 20240501"
                     + (f", Bernoulli({SPARSE_DENSITY}) sparsity)" if sparse else ")")),
            "config": config,
            "roofline": {"bound": bound, "kernel": kname,
                         "achieved": achieved, "peak": peak,
                         "unit": unit, "frac": achieved / peak,
                         "traffic": traffic[0] if traffic else None,
                         "traffic_unit": "HBM bytes per launch (rocprofv3 PMC)",
                         "traffic_source": traffic[1] if traffic else None,
                         "algorithmic_bytes_per_launch": alg_bytes,
                         "gram_ms_avg": gram_ms,
                         "sweep_ms_avg_events": sweep_ms,
                         "ops_per_launch": kernel_ops,
                         "gram_fp64_equivalent_tflops": fp64_equiv,
                         "gram_total_ms": gram_total_ms},
            "phases_ms": {k: round(v, 4) for k, v in phases.items()},
            "cpu_baseline": cpu,
            "setup_s": setup_s,
        }
        if cpu_more:
            rec["cpu_baselines"] = cpu_more
        print(json.dumps(rec), flush=True)
    eng.close()
    if dist:
        dist.destroy_process_group()


def small_chain(args, n, p, alpha):
    """C1 (BASELINE configs[0], p <= n): the reference-literal p x p path, run as the .C
    driver runs it -- one bridge_reg_stable call, W burn-in and K recorded sweeps; with p <= 32
    every block of sweeps is one single-workgroup launch.  `value` is K / the
    call's post-burn runtime.  The CPU baseline is the oracle's reference-literal chain
    (gibbs.bridge_regression_stable, method "chol": numpy/LAPACK p x p Cholesky + the C
    samplers, one BLAS thread) over a bounded number of sweeps."""
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
        from oracle import gibbs

        ns = args.cpu_sweeps if args.cpu_sweeps is not None else 2000
        with blas_threads(1):
            t0 = time.perf_counter()
            gibbs.bridge_regression_stable(y, X, ns, burn=0, alpha=alpha, seed=1, stream=0,
                                           method="chol")
            per = (time.perf_counter() - t0) / ns
        cpu = {"value": 1.0 / per, "unit": "sweeps/s", "cores": 1, "kind": "port",
               "sample": f"{ns} sweeps of the oracle's reference-literal chain (numpy/LAPACK "
                         f"p x p Cholesky + C samplers, 1 thread) at n={n}, p={p}"}
    # the p x p path's algorithmic flops per sweep (path p <= n):
    # p^3/3 + 3 p^2 + 2 n p; the fused chain is latency-bound, far from any roofline
    flops = p ** 3 / 3.0 + 3.0 * p * p + 2.0 * n * p
    achieved = flops * value / 1e12
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
        "roofline": {"bound": "mfma", "kernel": "k_small_chain", "achieved": achieved,
                     "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / FP64_MFMA_PEAK_TFLOPS, "traffic": None,
                     "note": "latency-bound: one workgroup, a chain of dependent draws"},
        "cpu_baseline": cpu, "call_wall_s": wall,
    }
    print(json.dumps(rec), flush=True)


def single_process(args, n, p, alpha, kind):
    """--single-process: the .C entry points' multi-GPU path -- one host thread, one engine
    per device holding a column shard, exchanges through an RCCL group (bb_group_create_rccl,
    ncclCommInitAll).  Same workload, timing protocol and JSON line as the default mode."""
    import torch

    import bayesbridge_amd as bb

    if kind == "logit":
        raise SystemExit("the logistic workload runs on one GPU")
    ndev = args.gpus
    if ndev > max(1, torch.cuda.device_count()):
        raise SystemExit(f"--single-process --gpus {ndev}: only {torch.cuda.device_count()} visible")
    bb.set_verbose(0)
    per = (p + ndev - 1) // ndev
    y = make_sparse_problem_y(n, p)[0] if kind == "sparse" else make_problem_y(n, p)[0]
    t_setup0 = time.perf_counter()
    engines = []
    for r in range(ndev):
        j0, j1 = r * per, min(p, (r + 1) * per)
        X = make_sparse_columns(n, j0, j1) if kind == "sparse" else make_columns(n, j0, j1)
        cfg = bb.EngineConfig(n=n, p=p, p_local=j1 - j0, j0=j0, rank=r, world=ndev,
                              true_alpha=alpha, method=2,
                              trace_capacity=max(1, min(args.steps, 1000)), seed=0xB4E5B41D6E,
                              stream=0, device=r)
        engines.append(bb.Engine(cfg, X, y))
        del X
    grp = bb.ShardGroup(engines, rccl=ndev > 1) if ndev > 1 else None
    (grp or engines[0]).init_state()
    setup_s = time.perf_counter() - t_setup0
    runner = grp or engines[0]
    runner.run(1, args.warmup, first_slot=-1)
    runner.sync()
    engines[0].enable_timing(True, phases=False)
    engines[0].reset_timing()
    t0 = time.perf_counter()
    runner.run(1 + args.warmup, args.steps, first_slot=0)
    runner.sync()
    elapsed = time.perf_counter() - t0
    gram_ms, _, _ = engines[0].kernel_times()
    rec = {
        "metric": f"Gibbs sweeps/sec at n={n},p={p},alpha={alpha}",
        "value": args.steps / elapsed, "unit": "sweeps/s", "n_gpus": ndev,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": 1000.0 * elapsed / args.steps, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (SURVEY.md 8(d) design, seed 20240501)",
        "config": {"workload": f"{args.workload} n={n} p={p} alpha={alpha}", "n": n, "p": p,
                   "alpha": alpha, "parallelism": f"column-shard x{ndev}, one process, "
                                                  "RCCL group (ncclCommInitAll)"},
        "roofline": None, "cpu_baseline": None, "gram_ms_rank0": gram_ms, "setup_s": setup_s,
    }
    print(json.dumps(rec), flush=True)
    if grp:
        grp.close()
    for e in engines:
        e.close()


if __name__ == "__main__":
    main()
