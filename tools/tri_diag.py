"""Per-slot divergence of the triangle chain: GPU (.C bridge_regression) vs the oracle."""
import sys

import numpy as np

sys.path.insert(0, ".")
import bayesbridge_amd as bb  # noqa: E402
from oracle import gibbs  # noqa: E402
from tests.conftest import synthetic_problem  # noqa: E402

bb.set_verbose(0)
n, p = 100, 20
X, y, _ = synthetic_problem(n, p, seed=5)
e = bb.Engine(bb.EngineConfig(n=n, p=p, method=4), X, y)
basis = e.tri_basis()
for burn in (0, 10):
    bb.set_seed(4321)
    g = bb.bridge_reg_tri(y, X, nsamp=30, burn=burn, extras=True)
    o = gibbs.bridge_regression_tri(y, X, 30, basis, burn=burn, seed=4321, stream=0)
    print("burn", burn)
    for s in range(30):
        r = {k: float(np.max(np.abs(g[k][s] - o[k][s]) / np.maximum(np.abs(o[k][s]), 1e-300)))
             for k in ("beta", "u", "w")}
        r.update({k: abs(g[k][s] - o[k][s]) / abs(o[k][s]) for k in ("tau", "sig2")})
        print(s, " ".join(f"{k}={v:.2e}" for k, v in r.items()),
              int(np.sum(g["shape"][s] != o["shape"][s])))
