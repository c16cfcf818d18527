"""Average each counter of a rocprofv3 --pmc CSV over the launches of one kernel.

python tools/sq_summary.py <dir> <kernel-substring>
"""
import csv
import glob
import sys
from collections import defaultdict

d, pat = sys.argv[1], sys.argv[2]
vals = defaultdict(list)
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(vals):
    v = vals[k]
    print(f"{k:24s} n={len(v):3d} avg={sum(v) / len(v):.4g}")
