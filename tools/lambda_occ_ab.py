"""A/B of the lambda launches' occupancy (bb_set_tuning key 4: 0 = the register-minimal
instances at 3 waves per SIMD, 3 = both capped at 128 VGPRs for 4 waves per SIMD) on the C3
(k_lambda_spec<16>) and C5 (k_lambda_cb<8>) engines, from a steady state reached after 30
sweeps; alternates the variants and prints the lambda phase time (HIP events at phase starts,
20 sweeps each).  It also checks that both variants draw the same chain: one sweep from the
same state under each must give bit-identical beta.
Usage: python tools/lambda_occ_ab.py [c3|c5 ...]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import bayesbridge_amd as bb  # noqa: E402

bb.set_verbose(0)
for wl in sys.argv[1:] or ["c3", "c5"]:
    n, p, alpha, kind = bench.WORKLOADS[wl]
    e = bb.Engine(bb.EngineConfig(n=n, p=p, true_alpha=alpha, method=2, seed=0xB4E5B41D6E),
                  bench.make_design(kind, n, p, 0, p), bench.make_y(kind, n, p))
    e.init_state()
    t = 1
    e.run(t, 30, first_slot=-1)
    t += 30
    e.sync()
    st = e.state()
    outs = []
    for occ in (0, 3):
        bb.set_tuning(4, occ)
        e.set_state(st["beta"], st["tau"], st["sig2"], st["alpha"])
        e.run(t, 1, first_slot=-1)
        e.sync()
        outs.append(e.state()["beta"].copy())
    same = bool(np.array_equal(outs[0], outs[1]))
    print(f"{wl}: one sweep from the same state, beta bit-identical across variants: {same}",
          flush=True)
    t += 1
    for occ in (0, 3, 0, 3, 0, 3):
        bb.set_tuning(4, occ)
        e.enable_timing(True, phases=True)
        e.reset_timing()
        e.run(t, 20, first_slot=-1)
        t += 20
        e.sync()
        ph = e.phase_times()
        print(f"{wl} occ={occ}: lambda {ph['lambda']:.4f} ms  sweep {sum(ph.values()):.4f} ms",
              flush=True)
    bb.set_tuning(4, 2)
    e.close()
    if not same:
        sys.exit(1)
