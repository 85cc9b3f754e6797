"""A/B of k_oz_gemm16u's K rotation (bb_ozaki.hip): the C3-shaped GEMM (n = 2000,
K = 50 000, random residues) without rotation (dbg 999) and with the diagonal pairs' lead L
and the per-earlier-pair-round start shift T, both in 1/1000 of a pass (dbg 1000000 +
1000 T + L).  Run under `rocprofv3 --pmc TCC_MISS_sum TCC_HIT_sum` (own pass) for the L2
misses per dispatch; each variant is 1 warm-up + `reps` dispatches, in the printed order.
Also prints the kernel times (HIP events).
Usage: python tools/oz_lead_probe.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bayesbridge_amd as bb  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
n, k = 2000, 50000
VARIANTS = [(999, "no rotation")] + [
    (1000000 + 1000 * t + l, f"late {t} lead {l}")
    for t, l in ((62, 30), (50, 30), (75, 30), (90, 30), (62, 40), (75, 40), (90, 40), (62, 20))
] + [(999, "no rotation")]
for dbg, name in VARIANTS:
    ms = bb.bench_ozaki(n, k, nsplit=0, dbg=dbg, reps=reps)
    print(f"{name:18s} dbg={dbg}: {ms * 1e3:8.1f} us  ({1 + reps} dispatches)", flush=True)
