"""Per-kernel dispatch statistics from a rocprofv3 --kernel-trace CSV, warm-up excluded:
for every kernel, the median / min / mean duration of its last N dispatches (N = the bench's
timed steps), so the profile can be set beside the bench line it was recorded with.

    python tools/trace_summary.py run_kernel_trace.csv [N] > kernel_medians.json
"""
import csv
import json
import statistics
import sys


def main():
    path = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    by = {}
    for r in rows:
        by.setdefault(r["Kernel_Name"], []).append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    out = {}
    for name, d in by.items():
        if not (name.startswith("_ZN2hg") or name.startswith("void hg::")):
            continue
        t = d[-last:]
        out[name] = {"dispatches": len(d), "last_n": len(t), "median_ms": round(statistics.median(t), 4),
                     "min_ms": round(min(t), 4), "mean_ms": round(sum(t) / len(t), 4)}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
