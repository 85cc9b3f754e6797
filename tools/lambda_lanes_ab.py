"""A/B of the speculative lambda launch's lanes per coefficient (bb_set_tuning key 5: 0 = the
default policy, L = 64 up to p = 1024, 16 up to 40 000, 8 above; 4 / 8 / 16 / 32 / 64
forced, 4 = one outer attempt of 4 inner attempts per round) on the C2, C3
and C4 engines from a steady state reached after 30 sweeps.  Alternates the lane counts and
prints the lambda phase time (HIP events at phase starts, 20 sweeps each), after checking
that one sweep from the same state draws bit-identical beta under every lane count.
Usage: python tools/lambda_lanes_ab.py [c2|c3|c4 ...]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import bayesbridge_amd as bb  # noqa: E402

bb.set_verbose(0)
ok = True
for wl in sys.argv[1:] or ["c3", "c2", "c4"]:
    n, p, alpha, kind = bench.WORKLOADS[wl]
    logit = kind == "logit"
    e = bb.Engine(bb.EngineConfig(n=n, p=p, true_alpha=alpha, method=6 if logit else 2,
                                  seed=0xB4E5B41D6E),
                  bench.make_design(kind, n, p, 0, p), bench.make_y(kind, n, p))
    e.init_state()
    t = 1
    e.run(t, 30, first_slot=-1)
    t += 30
    e.sync()
    st = e.state()
    lanes = (64, 32, 16) if logit else (8, 4, 16)
    outs = []
    for L in lanes:
        bb.set_tuning(5, L)
        e.set_state(st["beta"], st["tau"], st["sig2"], st["alpha"])
        e.run(t, 1, first_slot=-1)
        e.sync()
        outs.append(e.state()["beta"].copy())
    same = all(np.array_equal(outs[0], o) for o in outs[1:])
    ok &= same
    print(f"{wl}: one sweep from the same state, beta bit-identical across L {lanes}: {same}",
          flush=True)
    t += 1
    for _ in range(2):
        for L in lanes:
            bb.set_tuning(5, L)
            e.enable_timing(True, phases=True)
            e.reset_timing()
            e.run(t, 20, first_slot=-1)
            t += 20
            e.sync()
            ph = e.phase_times()
            print(f"{wl} L={L:2d}: lambda {ph['lambda']:.4f} ms  sweep {sum(ph.values()):.4f} ms",
                  flush=True)
    bb.set_tuning(5, 0)
    e.close()
sys.exit(0 if ok else 1)
