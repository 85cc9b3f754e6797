"""trace.beta timing: the default 401-ratio grid (bridge-trace.R) on a 442 x 10 design (or
n x p: `python tools/bench_trace.py [p [n]]`), one device launch (bb_bridge_em_batch)
against the per-ratio bridge_EM loop, plus the numpy oracle loop (oracle/em.py) for scale."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bayesbridge_amd as bb  # noqa: E402
from oracle import em  # noqa: E402

rng = np.random.default_rng(4)
p = int(sys.argv[1]) if len(sys.argv) > 1 else 10
n = int(sys.argv[2]) if len(sys.argv) > 2 else max(442, 2 * p)
X = rng.standard_normal((n, p))
if p == 10:
    b = np.array([3, -2, 1.5, 0, 0, 0.5, 0, 0, -1, 0.0])
else:
    b = np.zeros(p)
    b[:max(3, p // 10)] = rng.uniform(0.5, 3, max(3, p // 10))
y = X @ b + rng.standard_normal(n)
grid = np.exp(np.arange(-20.0, 20.0 + 1e-9, 0.1))
tol = 1e-9
bb.set_verbose(0)
bb.trace_beta(y, X, ratio_grid=grid[:3])  # warm
t0 = time.perf_counter()
tb = bb.trace_beta(y, X, ratio_grid=grid)
t1 = time.perf_counter()
# large p: the loops run every `stride`-th ratio and their times are scaled to the grid
stride = 1 if p <= 300 else 20
sub = grid[::stride]
loop = np.array([bb.bridge_em(y, X, 0.5, ratio=r, lambda_max=r / tol, tol=tol) for r in sub])
t2 = time.perf_counter()
orc = np.array([em.bridge_em(y, X, r, 0.5, r / tol, tol, 30)[0] for r in sub])
t3 = time.perf_counter()
print(f"trace.beta {grid.size} ratios, p={p}, n={n}: batched {1e3 * (t1 - t0):.1f} ms, "
      f"per-ratio bridge_EM loop {1e3 * (t2 - t1) * stride:.1f} ms, numpy oracle loop "
      f"{1e3 * (t3 - t2) * stride:.1f} ms"
      + (f" (loops timed on every {stride}th ratio, scaled)" if stride > 1 else "")
      + f"; max |batched - loop| {np.max(np.abs(tb['beta'][::stride] - loop)):.2e}, "
      f"max |batched - oracle| {np.max(np.abs(tb['beta'][::stride] - orc)):.2e}", flush=True)
