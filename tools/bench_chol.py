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
        t = ts[:, :8].astype(np.int64) * 0.01  # us
        clk = ts[:, 8:].astype(np.int64)
        print("  k   elim  stW   acqR  load  U+st  D'    rel   | step   | elim MHz")
        for k in range(t.shape[0] - 2):
            d = np.diff(t[k])
            mhz = (clk[k, 1] - clk[k, 0]) / max(d[0], 1e-9)
            print(f"{k:3d} " + " ".join(f"{v:5.2f}" for v in d) +
                  f" | {t[k + 1, 0] - t[k, 0]:6.2f} | {mhz:6.0f}")
        g = ts[:, 16:].astype(np.int64)
        print("elimination groups (us): start offset / length per producer wave, step 5")
        k = 5
        ngr = sum(1 for w in range(8) if g[k, w] > 0 and g[k, 8 + w] >= g[k, w])
        print("  " + "  ".join(f"{(g[k, w] - g[k, 0]) * 0.01:5.2f}/{(g[k, 8 + w] - g[k, w]) * 0.01:4.2f}"
                               for w in range(ngr)) +
              f"   (elim start -> group 0: {(g[k, 0] - ts[k, 0].astype(np.int64)) * 0.01:.2f})")
        o = ts[-1].astype(np.int64)
        kt = 6
        w_pub = ts[kt - 1, 7].astype(np.int64)   # chain released W_{kt-1}, U_{kt-1,kt}
        acq = ts[kt, 3].astype(np.int64)         # chain acquired step kt's hand-off
        rel = lambda v: (v - w_pub) * 0.01
        print(f"owner hops feeding step {kt} (us after the chain released W_{kt-1}):")
        print("  tile (kt-1,kt+1) [updated, stored]: last update acquired %.2f -> stored %.2f" %
              (rel(o[1]), rel(o[4])))
        print("  tile (kt,kt+1) [hand-off; last update from the chain's panels]: waits %.2f -> "
              "acquired %.2f -> loaded %.2f -> updated %.2f -> handed off %.2f;  chain acquired %.2f" %
              (rel(o[8]), rel(o[9]), rel(o[10]), rel(o[11]), rel(o[12]), rel(acq)))
