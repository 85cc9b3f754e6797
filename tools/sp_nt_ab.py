"""A/B of the sparse Gram kernels (bb_set_tuning key 3: 0 lanes per entry, 1 the same with
non-temporal loads, 2 the flat chunked stream) on one C5 engine (n = 5000, p = 200000,
density 0.01); prints the gram phase (HIP events at phase starts, 10 sweeps each),
alternating, and the largest difference between the variants' Grams on one D.
Usage: python tools/sp_nt_ab.py [variants, default 0,2,0,2]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import bayesbridge_amd as bb  # noqa: E402

n, p = 5000, 200000
bb.set_verbose(0)
X = bench.make_sparse_columns(n, 0, p)
y, _ = bench.make_sparse_problem_y(n, p)
e = bb.Engine(bb.EngineConfig(n=n, p=p, true_alpha=0.3, method=2, seed=0xB4E5B41D6E), X, y)
e.init_state()
t = 1
e.run(t, 10, first_slot=-1)
t += 10
e.sync()
variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,2,0,2").split(",")]
for nt in variants:
    bb.set_tuning(3, nt)
    e.enable_timing(True, phases=True)
    e.reset_timing()
    e.run(t, 10, first_slot=-1)
    t += 10
    e.sync()
    ph = e.phase_times()
    print(f"nt={nt}: gram {ph['gram']:.4f} ms  beta {ph.get('beta', float('nan')):.4f} ms",
          flush=True)
bb.set_tuning(3, 0)
e.close()
import numpy as np  # noqa: E402
import scipy.sparse as sps  # noqa: E402

Xs = sps.csc_matrix(sps.hstack(X) if isinstance(X, list) else X)
rng = np.random.default_rng(5)
D = 10.0 ** rng.uniform(-8, 0, p)
outs = {}
for v in sorted(set(variants)):
    bb.set_tuning(3, v)
    outs[v] = bb.sparse_gram(Xs, D)[0]
bb.set_tuning(3, 0)
base = outs[min(outs)]
for v, C in outs.items():
    print(f"variant {v}: max |C - C0| / max|C0| = "
          f"{np.max(np.abs(C - base)) / np.max(np.abs(base)):.3e}", flush=True)
