"""The reference-literal CPU path at C3, timed on the GPU box's host (VERDICT r4 missing #2).

Code/C/BridgeRegression.cpp:24 forms X'X once (p x p, 20 GB at p = 50 000) and every sweep
(:552-575) factors A = X'X + diag(lambda sig2 / tau^2) with chol(U, VInv, 'U') and applies
three triangular solves.  oracle/bb_cpu_chain.c runs exactly that chain (method "chol":
dgemm for X'X, dpotrf + dtrsm / dtrsv per sweep, the oracle's samplers) on scipy's
OpenBLAS.  Here: bench.py's C3 design and key, one burn-in sweep, then `--sweeps` timed
sweeps (the chain's own post-burn clock), on every host thread the box gives the job
(OMP_NUM_THREADS, 16 on the pool) -- outside the driver's bench path: one sweep takes minutes.
Output: one JSON document (stdout, and --out).

    python tools/literal_c3.py [--sweeps 2] [--out profiles/r05_cpu_literal_c3.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    import oracle

    ap = argparse.ArgumentParser()
    ap.add_argument("--sweeps", type=int, default=2)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    n, p, alpha, _ = bench.WORKLOADS["c3"]
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    t0 = time.perf_counter()
    X = bench.make_columns(n, 0, p)
    y, _ = bench.make_problem_y(n, p)
    t_data = time.perf_counter() - t0
    print(f"[literal_c3] data {t_data:.1f} s; X'X ({p} x {p}, {8 * p * p / 1e9:.0f} GB) and "
          f"{a.sweeps + 1} sweeps on {threads} threads ...", file=sys.stderr, flush=True)
    t1 = time.perf_counter()
    r = oracle.cpu_chain(y, X, a.sweeps + 1, burn=0, alpha=alpha, method="chol",
                         seed=0xB4E5B41D6E, threads=threads, record=False)
    wall = time.perf_counter() - t1
    per = r["runtime"] / a.sweeps
    rec = {"workload": f"C3 Gaussian bridge n={n} p={p} alpha={alpha}",
           "path": "reference-literal p x p: X'X once (BridgeRegression.cpp:24), per sweep "
                   "dpotrf of X'X + diag(lambda sig2 / tau^2) and three triangular solves "
                   "(:552-575); oracle/bb_cpu_chain.c method chol on scipy OpenBLAS",
           "threads": threads, "timed_sweeps": a.sweeps, "s_per_sweep": per,
           "sweeps_per_s": 1.0 / per,
           "setup_and_burn_s": wall - r["runtime"],
           "tau_last": float(r["tau"][-1]), "sig2_last": float(r["sig2"][-1]),
           "host": os.uname().nodename}
    js = json.dumps(rec, indent=1)
    print(js, flush=True)
    if a.out:
        with open(os.path.join(ROOT, a.out) if not os.path.isabs(a.out) else a.out, "w") as fh:
            fh.write(js + "\n")


if __name__ == "__main__":
    main()
