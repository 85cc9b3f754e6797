"""A/B of the device Cholesky chain variants (bb_set_chol_version): factor + solve times at
the system sizes of the BASELINE configs (C2/C4 m = 1024, C3 2048, C5 5120) and the v2
chain's per-step stamps at m = 2048 (slot 0 step start, 1 last pivot, 5 U complete, 7 end).
Usage: python tools/bench_chol_ab.py"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bayesbridge_amd as bb  # noqa: E402

out = {}
for m in (512, 1024, 2048, 4096, 5120):
    row = {}
    for v in (1, 2, 3):
        bb.set_chol_version(v)
        f, s = bb.bench_chol(m, reps=10)
        row[f"v{v}_factor_us"] = f * 1e3
        row[f"v{v}_solve_us"] = s * 1e3
    out[m] = row
    print(m, json.dumps({k: round(x, 1) for k, x in row.items()}), flush=True)
for v in (2, 3):
    bb.set_chol_version(v)
    f, s, ts = bb.bench_chol(2048, reps=3, trace=True)
    t = ts[:-1, :8].astype(np.int64) * 0.01
    steps = np.diff(t[:, 0])
    lp = t[:-1, 1] - t[:-1, 0]
    u5 = t[:-1, 5] - t[:-1, 1]
    en = t[:-1, 7] - t[:-1, 5]
    print(f"v{v} m=2048 step median {np.median(steps):.2f} us: start->last pivot "
          f"{np.median(lp[1:-1]):.2f}, last pivot->U done {np.median(u5[1:-1]):.2f}, "
          f"U->end {np.median(en[1:-1]):.2f}")
bb.set_chol_version(2)
if False:
    f, s, ts = bb.bench_chol(2048, reps=3, trace=True)
t = ts[:-1, :8].astype(np.int64) * 0.01
steps = np.diff(t[:, 0])
print("v2 m=2048 step us (start-to-start):", np.round(steps[:8], 2).tolist(), "... median",
      round(float(np.median(steps)), 2))
lp = t[:-1, 1] - t[:-1, 0]
u5 = t[:-1, 5] - t[:-1, 1]
en = t[:-1, 7] - t[:-1, 5]
print("  start->last pivot %.2f  last pivot->U done %.2f  U->end %.2f (medians, us)" %
      (np.median(lp[1:-1]), np.median(u5[1:-1]), np.median(en[1:-1])))
