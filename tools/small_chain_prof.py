"""Profile the small-p path at the diabetes shape: .C bridge_reg_stb / bridge_reg_tri calls
(5000 samples; argument stable | ortho | tri), for rocprofv3 --kernel-trace --stats."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bayesbridge_amd as bb  # noqa: E402
from sklearn.datasets import load_diabetes  # noqa: E402

d = load_diabetes(scaled=False)
X = d.data - d.data.mean(axis=0)
y = d.target - d.target.mean()
bb.set_verbose(0)
mode = sys.argv[1] if len(sys.argv) > 1 else "stable"
for _ in range(2):
    t0 = time.perf_counter()
    if mode == "tri":
        out = bb.bridge_reg_tri(y, X, nsamp=5000, burn=500)
    else:
        out = bb.bridge_reg_stb(y, X, nsamp=5000, burn=500, ortho=(mode == "ortho"))
    print(f"runtime {out['runtime']:.3f} s wall {time.perf_counter() - t0:.3f} s "
          f"-> {5000 / out['runtime']:.0f} sweeps/s", flush=True)
