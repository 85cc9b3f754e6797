"""Microbenchmark of the device Cholesky + backward solve, plus the chain workgroup's
per-step critical path from s_memrealtime stamps (100 MHz -> 10 ns ticks):
  0 elim start, 1 elim done, 2 W stores issued, 3 hand-off acquired, 4 tiles loaded,
  5 U_{k,k+1} formed + stored, 6 next diagonal block formed, 7 W and U released."""
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
        print("  k   elim  stW   acqR  load  U+st  D'    rel   | step")
        for k in range(t.shape[0] - 1):
            d = np.diff(t[k])
            print(f"{k:3d} " + " ".join(f"{v:5.2f}" for v in d) +
                  f" | {t[k + 1, 0] - t[k, 0]:6.2f}")
