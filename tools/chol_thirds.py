"""Per-step lengths of the device Cholesky chain at large m, in thirds of the factorisation
(bb.bench_chol trace: slot 0 = step start, 1 = last pivot, 7 = step end; 10 ns ticks), with
the elimination interval (start -> last pivot) split out.  Usage: python tools/chol_thirds.py [m] [chain version]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bayesbridge_amd as bb  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 5120
if len(sys.argv) > 2:
    bb.set_chol_version(int(sys.argv[2]))
f, s, ts = bb.bench_chol(m, reps=3, trace=True)
nblk = (m + 127) // 128 * 128 // 64
t = ts[:nblk, :8].astype(np.int64) * 0.01
clk = ts[:nblk, 8:16].astype(np.int64)  # s_memtime (shader clock) at the same slots
steps = np.diff(t[:, 0])
elim = t[:-1, 1] - t[:-1, 0]
print(f"m={m} v{bb.chol_version()}: factor {f * 1e3:.1f} us, {nblk} steps")
for a, b in ((0, nblk // 3), (nblk // 3, 2 * nblk // 3), (2 * nblk // 3, nblk - 1)):
    mhz = np.mean((clk[a:b, 1] - clk[a:b, 0]) / np.maximum(elim[a:b], 1e-9))
    print(f"  steps {a:3d}-{b:3d}: step {np.mean(steps[a:b]):6.2f} us, start->last pivot "
          f"{np.mean(elim[a:b]):6.2f} us at {mhz:6.0f} MHz")

# owner stamps of the three tiles feeding step kt (the middle step for m >= 48 blocks; see
# k_chol_persistent's OWN_TS): A = (kt-1, kt+1) stored for the merges, B = (kt, kt+1) and
# D = (kt+1, kt+1) the hand-offs.  Slots 0-4 as in bench_chol.py, 6 = tile started (after its
# load).
kt = nblk // 2 if nblk >= 48 else 6
t0 = int(ts[kt, 0])
own = ts[-1].astype(np.int64)
rel = lambda v: round((int(v) - t0) * 0.01, 2) if v else None  # noqa: E731
print(f"step {kt}: previous step end {rel(ts[kt - 1, 7])}, last pivot {rel(ts[kt, 1])}, "
      f"end {rel(ts[kt, 7])} (us after the step start)")
for name, off in (("A", 0), ("B", 8), ("D", 16)):
    print(f"  {name}: started {rel(own[off + 6])}; stamps {[rel(own[off + q]) for q in range(5)]}")
