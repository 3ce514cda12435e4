"""Average rocprofv3 PMC counters per dispatch for kernels whose name
contains a pattern.  Usage: python tools/pmc_summary.py OUTDIR PATTERN"""
import collections
import csv
import glob
import os
import sys

root, pat = sys.argv[1], sys.argv[2]
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        if pat in k:
            agg[k[:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in agg.items():
        print(k, {c: round(sum(v) / len(v), 1) for c, v in sorted(d.items())})
