"""Diagnose triangle-sampler parity at wide p: one teacher-forced sweep, GPU vs oracle,
for several (n, p, betaburn); prints relative errors, error flags and the coordinates of z
that differ most."""
import sys
import numpy as np

sys.path.insert(0, ".")
import bayesbridge_amd as bb  # noqa: E402
from oracle import gibbs  # noqa: E402
from tests.conftest import synthetic_problem  # noqa: E402

bb.set_verbose(0)
for (n, p, bburn) in [(900, 517, 2), (900, 517, 0), (700, 300, 2), (900, 513, 0), (900, 512, 0),
                      (900, 511, 0), (1200, 1000, 0)]:
    X, y, _ = synthetic_problem(n, p, seed=5)
    cfg = bb.EngineConfig(n=n, p=p, method=4, seed=777, stream=0, betaburn=bburn,
                          trace_capacity=1)
    e = bb.Engine(cfg, X, y)
    tV, a, d = e.tri_basis()
    e.init_state()
    o = gibbs.bridge_regression_tri(y, X, 3, (tV, a, d), burn=0, betaburn=bburn, seed=777,
                                    stream=0)
    i = 1
    e.set_state(o["beta"][i - 1], o["tau"][i - 1], o["sig2"][i - 1], 0.5)
    e.set_tri_state(o["u"][i - 1])
    e.run(i, 1, first_slot=0, slot_step=0, mcmc_phase=1)
    g = e.trace(0, 1)
    bg, bo = g["beta"][:, 0], o["beta"][i]
    zg, zo = tV @ bg, tV @ bo
    dz = np.abs(zg - zo)
    top = np.argsort(-dz)[:5]
    print(f"n={n} p={p} betaburn={bburn}: beta relL2 {np.linalg.norm(bg - bo) / np.linalg.norm(bo):.3e}"
          f" flags={e.error_flags()} top dz idx {top.tolist()} vals {dz[top].tolist()}",
          flush=True)
    e.close()
