"""Summarise a rocprofv3 kernel_stats.csv: per-kernel calls, average and total time."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    name = r["Name"].split("(")[0][:56]
    print(f"{name:56s} calls={r['Calls']:>6} avg_us={float(r['AverageNs']) / 1e3:9.2f} "
          f"min_us={float(r['MinNs']) / 1e3:9.2f} tot_ms={float(r['TotalDurationNs']) / 1e6:9.2f} "
          f"{100 * float(r['TotalDurationNs']) / tot:5.1f}%")
