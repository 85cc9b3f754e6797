"""A/B of the Cholesky chain's tagged-word hand-offs (bb_set_tuning key 21) and the backward
solve's (key 20): bb.bench_chol factor and solve times at m = 1024, 2048, 4096, alternating."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bayesbridge_amd as bb  # noqa: E402

for rnd in range(2):
    for v in (1, 0):
        o21, o20 = bb.set_tuning(21, v), bb.set_tuning(20, v)
        try:
            for m in (1024, 2048, 4096):
                f, s = bb.bench_chol(m, reps=10)[:2]
                print(f"ll={v} m={m}: factor {f * 1e3:7.1f} us  solve {s * 1e3:6.1f} us", flush=True)
        finally:
            bb.set_tuning(21, o21)
            bb.set_tuning(20, o20)
