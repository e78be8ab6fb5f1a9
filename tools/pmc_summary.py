"""Summarise rocprofv3 --pmc CSVs per kernel: python tools/pmc_summary.py DIR [name-substring]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if sub and sub not in r["Kernel_Name"]:
            continue
        k = r["Kernel_Name"][:60]
        agg[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
per = collections.defaultdict(lambda: collections.defaultdict(list))
for (k, _), cs in agg.items():
    for c, v in cs.items():
        per[k][c].append(v)
for k, cs in per.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} mean {sum(v) / len(v):.4g}  (n={len(v)})")
