"""A/B of non-temporal pair-list loads in the sparse Gram (bb_set_tuning key 3) on one C5
engine (n = 5000, p = 200000, density 0.01); prints the gram phase (HIP events at phase
starts, 10 sweeps each), alternating.  Usage: python tools/sp_nt_ab.py"""
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
for nt in (0, 1, 0, 1):
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
