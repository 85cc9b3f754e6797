"""Per-sweep kernel timeline from a rocprofv3 --kernel-trace database (rocpd sqlite):
durations and the gap before each kernel, for the sweeps around the n-th launch of a kernel.
usage: python tools/rocpd_timeline.py DB [anchor-substring] [index] [count]"""
import sqlite3
import sys

db = sys.argv[1]
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_lambda_xu"
idx = int(sys.argv[3]) if len(sys.argv) > 3 else 20
cnt = int(sys.argv[4]) if len(sys.argv) > 4 else 30
con = sqlite3.connect(db)
rows = con.execute(
    "select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
    "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start").fetchall()
pos = [i for i, r in enumerate(rows) if anchor in r[0]]
print(f"{len(rows)} dispatches, {len(pos)} of {anchor}")
i0 = pos[min(idx, len(pos) - 1)]
prev = None
for name, s, e in rows[i0 - 2:i0 + cnt]:
    gap = (s - prev) / 1000 if prev else 0.0
    print(f"{name.split('(')[0][:44]:44s} dur {(e - s) / 1000:8.2f} gap {gap:7.2f}")
    prev = e
