#!/usr/bin/env python3
"""Benchmark: Gibbs sweeps/s of the BayesBridge stable sampler on MI355X.

Workload (BASELINE.json metric): Gaussian bridge regression, n=2000, p=50000, alpha=0.5
(SURVEY.md C3), synthetic design of SURVEY.md s8(d).  One step = one full Gibbs sweep
(tau, sig2, all p lambda_j, beta | rest) with X resident in HBM.  At N GPUs the p columns
are sharded across one process per GPU with one RCCL all-reduce per exchange step
(strong scaling: the total problem is fixed).

Defaults follow SURVEY.md 8(d): M = 1000 timed sweeps after B = 100 burn-in sweeps, every
timed sweep recording beta / lambda / sig2 / tau into the device-resident trace.

Prints ONE JSON line (rank 0) with the driver's contract fields plus
  roofline     -- the fp64 MFMA Gram kernel (dominant kernel): algorithmic flops per
                  launch / average launch duration from HIP events on the engine stream
  cpu_baseline -- the oracle's Woodbury sweep (numpy/OpenBLAS + C latent sampler) timed
                  on this host on a bounded number of sweeps (rank 0, N=1 only).
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


def cpu_baseline(n, p, alpha, sweeps, log_every=True):
    """Oracle Woodbury sweeps on the host: the CPU restatement of the reference sweep,
    algorithm-matched to the GPU path (reference-literal p x p Cholesky at p=50000 needs a
    20 GB Gram and ~4e13 flop per sweep)."""
    import oracle
    from oracle import gibbs

    X = make_columns(n, 0, p)
    y, _ = make_problem_y(n, p)
    beta = np.zeros(p)
    tau, sig2 = 1.0, 1.0
    hyper = dict(nu_shape=2.0, nu_rate=2.0, sig2_shape=0.0, sig2_scale=0.0)
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
            log(f"[cpu_baseline] sweep {t}: {times[-1]:.3f} s")
    del hyper
    # first sweep starts from beta = 0 (all lambda draws at h = 0); report the median
    per = float(np.median(times))
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
    ap.add_argument("--rows", type=int, default=2000)
    ap.add_argument("--cols", type=int, default=50000)
    ap.add_argument("--alpha", type=float, default=0.5)
    ap.add_argument("--cpu-sweeps", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--gram", choices=["fp64", "ozaki"], default=None,
                    help="Woodbury Gram: fp64 MFMA or Ozaki-II int8 MFMA (default: env "
                         "BB_GRAM_MODE, else the library default)")
    args = ap.parse_args()

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
    n, p, alpha = args.rows, args.cols, args.alpha
    per = (p + world - 1) // world
    j0 = min(p, rank * per)
    j1 = min(p, j0 + per)
    p_loc = j1 - j0
    t_setup0 = time.perf_counter()
    X = make_columns(n, j0, j1)
    y, _ = make_problem_y(n, p)
    cfg = bb.EngineConfig(n=n, p=p, p_local=p_loc, j0=j0, rank=rank, world=world,
                          true_alpha=alpha, method=2,
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
    log(f"[rank {rank}] setup {setup_s:.2f} s  (n={n}, p={p}, p_local={p_loc}, "
        f"method={eng.method()})")

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
    # Dominant kernel = the Gram GEMM.  fp64 path: algorithmic fp64 flops of one k_gram
    # launch on this rank, n(n+1) p_local.  Ozaki path: algorithmic int8 ops of
    # one k_oz_gemm launch, kOzMods x n(n+1) p_local (16 exact symmetric int8 Grams).
    gram_mode = eng.gram_mode()
    gram_flops = float(n) * (n + 1) * p_loc
    if gram_mode == bb.GRAM_OZAKI:
        kernel_ops = 16.0 * n * (n + 1) * p_loc
        peak, unit, kname = INT8_MFMA_PEAK_TOPS, "TOP/s", "k_oz_gemm16u (v_mfma_i32_16x16x64_i8)"
    else:
        kernel_ops = gram_flops
        peak, unit, kname = FP64_MFMA_PEAK_TFLOPS, "TFLOP/s", "k_gram (v_mfma_f64_16x16x4_f64)"
    achieved = kernel_ops / (gram_ms * 1e-3) / 1e12 if gram_ms > 0 else 0.0
    gram_total_ms = gram_ms + phases.get("ozprep", 0.0) + phases.get("reduce", 0.0)
    fp64_equiv = gram_flops / (gram_total_ms * 1e-3) / 1e12 if gram_total_ms > 0 else 0.0

    traffic = pmc_traffic(n, p, world, "bb::k_oz_gemm16u" if gram_mode == bb.GRAM_OZAKI
                          else "bb::k_gram")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.cpu_sweeps > 0:
        log(f"[cpu_baseline] timing {args.cpu_sweeps} oracle sweeps at n={n}, p={p} ...")
        per_sweep, threads = cpu_baseline(n, p, alpha, args.cpu_sweeps)
        cpu = {"value": 1.0 / per_sweep, "unit": "sweeps/s", "cores": threads, "kind": "port",
               "sample": f"{args.cpu_sweeps} Woodbury sweeps of the oracle (numpy/OpenBLAS "
                         f"{threads} threads + C tilted-stable sampler) at n={n}, p={p}; "
                         f"median sweep {per_sweep:.3f} s"}

    if rank == 0:
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
            "data": "synthetic (SURVEY.md 8(d) Gaussian design, seed 20240501)",
            "config": {"workload": f"C3 Gaussian bridge n={n} p={p} alpha={alpha}",
                       "rccl": bool(world > 1 or force_rccl),
                       "n": n, "p": p, "alpha": alpha,
                       "beta_step": "woodbury (exact, p > n)",
                       "gram": ("ozaki-II int8 (fp64-accurate)" if gram_mode == bb.GRAM_OZAKI
                                else "fp64 mfma"),
                       "parallelism": f"column-shard x{world}" + (" + RCCL all-reduce"
                                                                  if world > 1 else "")},
            "roofline": {"bound": "mfma", "kernel": kname,
                         "achieved": achieved, "peak": peak,
                         "unit": unit, "frac": achieved / peak,
                         "traffic": traffic[0] if traffic else None,
                         "traffic_unit": "HBM bytes per launch (rocprofv3 PMC)",
                         "traffic_source": traffic[1] if traffic else None,
                         "algorithmic_bytes_per_launch": (16.0 * n * p_loc if gram_mode == bb.GRAM_OZAKI
                                                          else 8.0 * n * p_loc),
                         "gram_ms_avg": gram_ms,
                         "sweep_ms_avg_events": sweep_ms,
                         "ops_per_launch": kernel_ops,
                         "gram_fp64_equivalent_tflops": fp64_equiv,
                         "gram_total_ms": gram_total_ms},
            "phases_ms": {k: round(v, 4) for k, v in phases.items()},
            "cpu_baseline": cpu,
            "setup_s": setup_s,
        }
        print(json.dumps(rec), flush=True)
    eng.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
