"""Average each PMC counter per kernel over dispatches: python tools/pmc_show.py <dir>..."""
import csv
import glob
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    tot, cnt = defaultdict(float), defaultdict(int)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = (r["Kernel_Name"].split("(")[0][-24:], r["Counter_Name"])
            tot[k] += float(r["Counter_Value"])
            cnt[k] += 1
    for k in sorted(tot):
        print(f"{d.split('/')[-1]:6s} {k[0]:24s} {k[1]:22s} {tot[k] / cnt[k]:16.1f}")
