"""A/B of the device Cholesky chain variants (bb_set_chol_version): factor + solve times at
the system sizes of the BASELINE configs (C2/C4 m = 1024, C3 2048, C5 5120) and the v2 /
v3 chains' per-step stamps at m = 2048 (slot 0 step start, 1 last pivot; the rest relative
to the last pivot).
Usage: python tools/bench_chol_ab.py"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bayesbridge_amd as bb  # noqa: E402

out = {}
VERSIONS = tuple(int(v) for v in os.environ.get("CHOL_VERSIONS", "1,2,3").split(","))
for m in (512, 1024, 2048, 4096, 5120):
    row = {}
    for v in VERSIONS:
        bb.set_chol_version(v)
        f, s = bb.bench_chol(m, reps=10)
        row[f"v{v}_factor_us"] = f * 1e3
        row[f"v{v}_solve_us"] = s * 1e3
    out[m] = row
    print(m, json.dumps({k: round(x, 1) for k, x in row.items()}), flush=True)
NAMES = {2: "wave7 W stored", 3: "wave7 U rb3 put", 4: "wave4 Q loaded", 5: "U complete (B1)",
         6: "wave0 Q loaded", 7: "step end"}
for v in [v for v in VERSIONS if v in (2, 3)]:
    bb.set_chol_version(v)
    f, s, ts = bb.bench_chol(2048, reps=3, trace=True)
    t = ts[:-1, :8].astype(np.int64) * 0.01
    steps = np.diff(t[:, 0])
    lp = t[:-1, 1] - t[:-1, 0]
    rel = {NAMES[j]: round(float(np.median((t[:-1, j] - t[:-1, 1])[1:-1])), 2) for j in NAMES}
    print(f"v{v} m=2048 step median {np.median(steps):.2f} us, start->last pivot "
          f"{np.median(lp[1:-1]):.2f}; after the last pivot (us): {json.dumps(rel)}", flush=True)
bb.set_chol_version(1)

# the step-6 hand-offs against the chain: owner stamps of tiles A = (5, 7) (stored tile,
# slots 0-3 its last standard update, 4 flag), B = (6, 7) (merge: 0 start, 1 W_5 / H_5 seen,
# 2 U_{5,7} formed, 3 merged, 4 released) and D = (7, 7) (dmerge, same slots), relative to
# the start of chain step 6 (us)
kt = 6
for v in VERSIONS:
    bb.set_chol_version(v)
    f, s, ts = bb.bench_chol(2048, reps=3, trace=True)
    t0 = int(ts[kt, 0])
    rel = lambda x: round((int(x) - t0) * 0.01, 2) if x else None  # noqa: E731
    own = ts[-1]
    print(f"v{v} step {kt}: prev step end {rel(ts[kt - 1, 7])}, last pivot {rel(ts[kt, 1])}, "
          f"end {rel(ts[kt, 7])}; A {[rel(x) for x in own[0:5]]} B {[rel(x) for x in own[8:13]]} "
          f"D {[rel(x) for x in own[16:21]]}", flush=True)
bb.set_chol_version(1)

# v1 elimination: producer-group start / end stamps (trace slots 16-23 / 24-31)
# relative to the step start, medians over the steps (us)
for v in [v for v in VERSIONS if v == 1]:
    bb.set_chol_version(v)
    f, s, ts = bb.bench_chol(2048, reps=3, trace=True)
    t = ts[1:-2].astype(np.int64)
    st = np.median((t[:, 16:24] - t[:, [0]]) * 0.01, axis=0)
    en = np.median((t[:, 24:32] - t[:, [0]]) * 0.01, axis=0)
    steps = np.diff(ts[:-1, 0].astype(np.int64)) * 0.01
    print(f"v{v} groups start", np.round(st, 2).tolist(), "end", np.round(en, 2).tolist(),
          "last pivot", round(float(np.median((t[:, 1] - t[:, 0]) * 0.01)), 2),
          "step median", round(float(np.median(steps)), 2), flush=True)
bb.set_chol_version(1)

# v4 (16-column leaf pipeline, bb_chol4.h) per-step stamps, medians over the inner steps (us
# after the step's leaf-0 start); slot names in bb_chol4.h
V4_SLOTS = {1: "leaf3 done", 2: "W rel", 3: "S acq", 4: "U rel", 5: "D00 ready", 6: "leaf1 start",
            7: "leaf2 start", 24: "s3 UU", 25: "s2 UU", 26: "S free",
            27: "s1 UU", 28: "s0 US0", 29: "s0 US3", 30: "s0 UU", 31: "w4 UU"}
for t in range(4):
    V4_SLOTS[8 + 4 * t] = f"L{t} piv"
    V4_SLOTS[9 + 4 * t] = f"L{t} W"
    if t < 3:
        V4_SLOTS[10 + 4 * t] = f"X{t}"
        V4_SLOTS[11 + 4 * t] = f"upd{t + 1}"
for v in [v for v in VERSIONS if v == 4]:
    bb.set_chol_version(v)
    for m in (1024, 2048):
        f, s, ts = bb.bench_chol(m, reps=3, trace=True)
        nb = m // 64
        t = ts[:nb].astype(np.int64)
        steps = np.diff(t[:, 0]) * 0.01
        print(f"v4 m={m} factor {f * 1e3:.1f} us; step median {np.median(steps[1:]):.2f} "
              f"(min {steps[1:].min():.2f} max {steps[1:].max():.2f})", flush=True)
        inner = t[1:-1]
        rel = {}
        for j, name in sorted(V4_SLOTS.items(), key=lambda kv: np.median(inner[:, kv[0]] - inner[:, 0])):
            d = (inner[:, j] - inner[:, 0]) * 0.01
            d = d[inner[:, j] > 0]
            if len(d):
                rel[name] = round(float(np.median(d)), 2)
        print("  " + json.dumps(rel), flush=True)
        if m == 2048:  # the traced owner hop's step (owner stamps B / D above are for step 6)
            row = t[6]
            print("  step 6: " + json.dumps({name: round(float((row[j] - row[0]) * 0.01), 2)
                                            for j, name in V4_SLOTS.items() if row[j] > 0}), flush=True)
bb.set_chol_version(1)
