"""A/B of the Ozaki residue-plane stores (bb_set_tuning key 1: ordinary, non-temporal, and
non-temporal with non-temporal X loads) on
one C3 engine (n = 2000, p = 50000), alternating variants; prints the ozprep and gram phase
times (HIP events at phase starts, 20 sweeps each).  Usage: python tools/res_nt_ab.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import bayesbridge_amd as bb  # noqa: E402

n, p = 2000, 50000
bb.set_verbose(0)
y, _ = bench.make_problem_y(n, p)
e = bb.Engine(bb.EngineConfig(n=n, p=p, true_alpha=0.5, method=2, seed=0xB4E5B41D6E),
              bench.make_columns(n, 0, p), y)
e.init_state()
t = 1
e.run(t, 30, first_slot=-1)
t += 30
e.sync()
for nt in (0, 1, 2, 0, 1, 2):
    bb.set_tuning(1, nt)
    bb.set_tuning(2, 1 if nt == 2 else 0)
    e.enable_timing(True, phases=True)
    e.reset_timing()
    e.run(t, 20, first_slot=-1)
    t += 20
    e.sync()
    ph = e.phase_times()
    print(f"nt={nt}: ozprep {ph['ozprep']:.4f} ms  gram {ph['gram']:.4f} ms  beta "
          f"{ph['beta']:.4f} ms (nt X loads {nt == 2})", flush=True)
bb.set_tuning(1, 2)
bb.set_tuning(2, 1)
e.close()
