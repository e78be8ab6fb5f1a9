#!/usr/bin/env python3
"""Instruction mix of a kernel's loops from a device assembly file.

    hipcc --offload-arch=gfx950 ... --cuda-device-only -S x.hip -o x.s
    python tools/isa_stats.py x.s <kernel-name-substring> [--all]

For every backward branch (a loop) prints the body's instruction count per class
(VALU plain / VALU DPP / packed / VMEM / SMEM / SALU / LDS / waitcnt / nop), which is
what the issue-floor estimates in DESIGN.md are computed from.
"""
import re
import sys
from collections import Counter


def kernel_body(lines, name):
    start = None
    for i, ln in enumerate(lines):
        if start is None and ln.split(";")[0].strip() == name + ":":
            start = i
        elif start is not None and ln.strip().startswith(".Lfunc_end"):
            return lines[start:i]
    raise SystemExit(f"kernel {name!r} not found")


def classify(ins):
    op = ins.split()[0]
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        if "_dpp" in op or " wave_sh" in ins or " row_sh" in ins or "quad_perm" in ins:
            return "valu_dpp"
        if op.startswith("v_pk_"):
            return "valu_pk"
        if op.startswith(("v_readlane", "v_readfirstlane", "v_writelane")):
            return "valu_lane"
        return "valu"
    return "other"


def main():
    path, pat = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    names = [m.group(1) for m in (re.match(r"^(_Z\w+):", ln) for ln in lines) if m and pat in m.group(1)]
    if not names:
        raise SystemExit("no kernel matches")
    for name in names if "--all" in sys.argv else names[:1]:
        body = kernel_body(lines, name)
        labels = {}
        insts = []      # (index, text)
        for ln in body:
            s = ln.split(";")[0].strip()
            if not s or s.startswith((";", ".")) and not s.startswith(".LBB"):
                continue
            if s.startswith(".LBB") and s.endswith(":"):
                labels[s[:-1]] = len(insts)
                continue
            insts.append(s.split(";")[0].strip())
        print(f"== {name}: {len(insts)} instructions")
        for j, ins in enumerate(insts):
            m = re.match(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", ins)
            if not m:
                continue
            tgt = m.group(1) or m.group(2)
            if tgt in labels and labels[tgt] <= j:
                seg = insts[labels[tgt]:j + 1]
                c = Counter(classify(x) for x in seg)
                print(f"  loop {tgt}: {len(seg)} instrs  " +
                      "  ".join(f"{k}={v}" for k, v in sorted(c.items())))
                ops = Counter(x.split()[0] for x in seg if classify(x).startswith("valu"))
                print("     top VALU: " + ", ".join(f"{k}:{v}" for k, v in ops.most_common(14)))


if __name__ == "__main__":
    main()
