"""Median per-dispatch value of one rocprofv3 PMC counter for every kernel in a run
(summed over the counter's instances), in KB and as a ratio to a given byte count.

usage: python tools/pmc_by_kernel.py DIR COUNTER [alg_bytes] [x2]   (x2: FETCH_SIZE's gfx950 correction)
"""
import collections
import csv
import glob
import statistics
import sys


def main():
    d, counter = sys.argv[1], sys.argv[2]
    alg = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
    mul = 2.0 if len(sys.argv) > 4 and sys.argv[4] == "x2" else 1.0
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                per[r["Kernel_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for k, v in sorted(per.items()):
        m = statistics.median(v.values()) * 1024 * mul
        print(f"{k[:90]:90s} n={len(v):3d}  {m / 1e9:8.3f} GB" + (f"  {m / alg:.4f}x" if alg else ""))


if __name__ == "__main__":
    main()
