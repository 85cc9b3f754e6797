"""Per-dispatch durations of one kernel, in launch order, from a rocprofv3 --kernel-trace
CSV (the *kernel_trace.csv under a -d directory): shows whether a kernel's avg/min spread is
a within-launch tail or a change of regime between sweeps (e.g. the first sweeps from
beta = 0).  Usage: python tools/dispatch_series.py <dir> <kernel-substring> [skip]"""
import csv
import glob
import sys

import numpy as np


def main():
    d, name = sys.argv[1], sys.argv[2]
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if name in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    us = np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows])
    print(f"{name}: {len(us)} dispatches; first 12 (us): {np.round(us[:12], 1).tolist()}")
    s = us[skip:]
    print(f"after skipping {skip}: mean {s.mean():.1f} min {s.min():.1f} max {s.max():.1f} "
          f"median {np.median(s):.1f} us")
    step = max(1, len(us) // 25)
    print("means per block of", step, "dispatches:",
          [round(float(us[i:i + step].mean()), 1) for i in range(0, len(us), step)])


if __name__ == "__main__":
    main()
