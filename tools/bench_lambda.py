"""Microbenchmark of the tilted-stable lambda kernel on a C3-like state (n=2000, p=50000).

The state (beta, tau) comes from three oracle sweeps from beta = 0, so the h = beta^2/tau^2
distribution is the one the sampler meets early in burn-in.  Prints one line per
(group size, inlining) variant with the average launch time and parity vs the oracle.
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bayesbridge_amd as bb  # noqa: E402
import bench  # noqa: E402
import oracle  # noqa: E402
from oracle import gibbs  # noqa: E402


def c3_state(n=2000, p=50000, sweeps=3):
    X = bench.make_columns(n, 0, p)
    y, _ = bench.make_problem_y(n, p)
    beta, tau = np.zeros(p), 1.0
    for t in range(1, sweeps + 1):
        tau = oracle.tau_from_sum(oracle.sum_abs_pow(beta, 0.5), p, 0.5, 2, 2, 1, 0, t)
        r = y - X @ beta
        sig2 = oracle.sig2_from_rss(float(r @ r), n, 0, 0, 1, 0, t)
        lam = oracle.sample_lambda(beta, 0.5, tau, 1, 0, t)
        z = oracle.normals(p, 1, 0, t, oracle.KIND_BETA_Z)
        d = oracle.normals(n, 1, 0, t, oracle.KIND_DELTA)
        beta = gibbs.beta_step_woodbury(X, y, lam, sig2, tau, z, d)
    return beta, tau


def main():
    t0 = time.time()
    beta, tau = c3_state()
    print(f"state ready in {time.time() - t0:.1f}s; tau={tau:.3e}", flush=True)
    reps = 20
    ref = oracle.sample_lambda(beta, 0.5, tau, 1, 0, reps + 1)
    for p in (50000, 6250):
        b = beta[:p]
        r = ref[:p]
        for noinl in (0, 1):
            for g in (1, 2, 4, 8, 16, 32, 64):
                ms, lam = bb.bench_lambda(b, 0.5, tau, g, noinl, reps)
                err = np.max(np.abs(lam - r) / r)
                print(f"p={p:6d} noinline={noinl} G={g:2d}: {ms * 1e3:9.1f} us/launch  "
                      f"max rel err vs oracle {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
