"""Triangle-mixture sampler timing: device sweeps/s (Engine, data resident) vs the oracle
(one C call per sweep for the omega/u/beta update + numpy for tau/sig2)."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import bayesbridge_amd as bb  # noqa: E402
from oracle import gibbs  # noqa: E402
from tests.conftest import synthetic_problem  # noqa: E402

bb.set_verbose(0)
for n, p, ortho in [(100, 20, 0), (442, 10, 0), (1000, 100, 0), (2000, 500, 0), (2000, 500, 1)]:
    X, y, _ = synthetic_problem(n, p, seed=1)
    t0 = time.perf_counter()
    e = bb.Engine(bb.EngineConfig(n=n, p=p, method=4, ortho=bool(ortho)), X, y)
    setup = time.perf_counter() - t0
    e.init_state()
    e.run(1, 20)
    e.sync()
    K = 200 if p <= 100 else 50
    t0 = time.perf_counter()
    e.run(21, K)
    e.sync()
    dt = (time.perf_counter() - t0) / K
    basis = e.tri_basis()
    Ko = 20 if p <= 100 else 3
    t0 = time.perf_counter()
    gibbs.bridge_regression_tri(y, X, Ko, basis, burn=0, seed=1, ortho=bool(ortho))
    do = (time.perf_counter() - t0) / (Ko - 1)
    print(f"n={n} p={p} ortho={ortho}: device {1e3 * dt:.3f} ms/sweep ({1 / dt:.0f} sweeps/s), "
          f"oracle {1e3 * do:.2f} ms/sweep, setup {setup:.2f} s, flags {e.error_flags()}",
          flush=True)
