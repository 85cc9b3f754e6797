"""Ozaki int8 GEMM timing and ablations at the C3 shape (n=2000, p_local=50000)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bayesbridge_amd as bb  # noqa: E402

n, k = 2000, 50000
ops = 16.0 * n * (n + 1) * k
for dbg, name in [(0, "full"), (1, "no LDS-DMA refill"), (2, "no fragment reads"),
                  (4, "no waits/barrier"), (8, "refill from one chunk"), (3, "no DMA, no reads"), (7, "MFMA only")]:
    for S in (0, 1, 2, 4, 8):
        ms = bb.bench_ozaki(n, k, nsplit=S, dbg=dbg, reps=10)
        print(f"{name:20s} S={S}: {ms * 1e3:8.1f} us  {ops / ms / 1e9:7.0f} TOP/s", flush=True)
        if dbg:
            break
