"""Microbenchmark of the blocked Cholesky + backward solve (factor / solve ms)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bayesbridge_amd as bb  # noqa: E402

for m in (1024, 2048):
    for nt in (128, 256, 512, 1024):
        f, s = bb.bench_chol(m, nt, reps=5)
        print(f"m={m} diag_threads={nt:4d}: factor {f * 1e3:8.1f} us  solve {s * 1e3:7.1f} us",
              flush=True)
