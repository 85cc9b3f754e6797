"""Why k_oz_gemm16u reads ~2x its residue planes: the GEMM at the C3
shape (n = 2000, K = 50 000) with and without its diagonal-pair workgroups (bb_bench_ozaki
dbg 16: the pairs idle).  Run under `rocprofv3 --pmc TCC_MISS_sum TCC_HIT_sum` (own pass);
each variant is launched `reps` times, so the per-dispatch counters of k_oz_gemm16u<0> and
k_oz_gemm16u<16> compare the two.  Also prints the kernel times."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bayesbridge_amd as bb  # noqa: E402

n, k = 2000, 50000
for dbg, name in ((0, "production"), (16, "pairs idle")):
    ms = bb.bench_ozaki(n, k, nsplit=0, dbg=dbg, reps=5)
    print(f"{name:12s} dbg={dbg}: {ms * 1e3:8.1f} us", flush=True)
