#!/usr/bin/env python3
"""Per-step instruction mix of a streaming kernel's row loop, from device assembly.

    hipcc --offload-arch=gfx950 ... --cuda-device-only -S fused.hip -o f.s
    python tools/loop_mix.py f.s <kernel-name-substring> [steps_per_trip] [min_pk] [nloops]

Finds every loop (a label with a later branch back to it) in the first kernel whose
name contains the substring, keeps the innermost ones (no loop nested inside) and
reports the one with the most instructions, per step (trip / steps_per_trip, default
12): mnemonic counts plus an issue-cycle estimate from the measured 4-waves-per-SIMD
costs of profiles/r02/probe/issue_wps.txt and profiles/r03/probe/pk_issue_wps_1.txt.
"""
import re
import sys
from collections import Counter

COST = {"pk": 4.49, "dpp": 5.1, "valu": 2.85, "cvt_pk": 5.13, "nop": 4.0}


def kernel_lines(lines, pat):
    start = None
    for i, ln in enumerate(lines):
        m = re.match(r"^(_Z\w+):", ln)
        if m and start is None and pat in m.group(1):
            start, name = i, m.group(1)
        elif start is not None and ln.strip().startswith(".Lfunc_end"):
            return name, lines[start:i]
    raise SystemExit(f"no kernel matches {pat!r}")


def main():
    path, pat = sys.argv[1], sys.argv[2]
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    name, body = kernel_lines(open(path).read().splitlines(), pat)
    labels = {}
    loops = []
    for i, ln in enumerate(body):
        m = re.match(r"^(\.LBB\w+):", ln)
        if m:
            labels[m.group(1)] = i
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", ln)
        if m:
            tgt = m.group(1) or m.group(2)
            if tgt in labels and labels[tgt] < i:
                loops.append((labels[tgt], i))
    inner = [(a, b) for a, b in loops if not any(a < c and d < b for c, d in loops if (c, d) != (a, b))]
    if not inner:
        raise SystemExit("no loop")
    inner.sort(key=lambda ab: ab[1] - ab[0], reverse=True)
    nloops = int(sys.argv[5]) if len(sys.argv) > 5 else 1      # report the N largest loops
    for a, b in inner[:nloops]:
        report(name, body, a, b, steps)


def report(name, body, a, b, steps):
    cnt = Counter()
    for ln in body[a:b + 1]:
        t = ln.strip()
        if not t or t.startswith((";", ".")):
            continue
        cnt[t.split()[0]] += 1
    print(f"{name}: loop lines {a}-{b}, per step (/{steps}):")
    cyc = 0.0
    cls = Counter()
    for op, n in cnt.most_common():
        ps = n / steps
        if op.startswith("v_pk_"):
            k = "pk"
        elif "dpp" in op:
            k = "dpp"
        elif op.startswith("v_cvt_pk"):
            k = "cvt_pk"
        elif op.startswith("v_"):
            k = "valu"
        elif op.startswith("s_nop"):
            k = "nop"
        else:
            k = None
        if k:
            cyc += ps * COST[k]
            cls[k] += ps
        print(f"  {op:28s} {ps:7.2f}")
    print("  classes: " + ", ".join(f"{k} {v:.2f}" for k, v in cls.items()))
    print(f"  VALU issue estimate: {cyc:.0f} cycles per wave-step (4 waves/SIMD costs)")


if __name__ == "__main__":
    main()
