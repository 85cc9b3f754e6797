"""Microbenchmark of the blocked Cholesky + backward solve, plus the per-step critical-path
breakdown from the kernel's s_memrealtime stamps (100 MHz -> 10 ns ticks)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bayesbridge_amd as bb  # noqa: E402

for m in (512, 1024, 2048, 4096):
    f, s, ts = bb.bench_chol(m, reps=10, trace=True)
    print(f"m={m}: factor {f * 1e3:8.1f} us  solve {s * 1e3:7.1f} us", flush=True)
    if m == 2048:
        t = ts.astype(np.int64) * 0.01  # us
        base = t[0, 0]
        print(" kp  wg0start  load  upd  elim  rel | p1start acq done | gap(next wg0 - rel)")
        for k in range(t.shape[0]):
            r = t[k] - base
            nxt = (t[k + 1, 0] - t[k, 4]) if k + 1 < t.shape[0] else float("nan")
            p1 = (f"{r[5]:8.2f} {t[k,6]-t[k,5]:5.2f} {t[k,7]-t[k,6]:5.2f}" if t[k, 5] else
                  "       -     -     -")
            print(f"{k:3d} {r[0]:8.2f} {t[k,1]-t[k,0]:5.2f} {t[k,2]-t[k,1]:5.2f} "
                  f"{t[k,3]-t[k,2]:5.2f} {t[k,4]-t[k,3]:5.2f} | {p1} | {nxt:6.2f}")
