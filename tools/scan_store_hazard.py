"""Scan gfx950 device assembly for the store-data hazard seen in k_tri_up (r05): a MUBUF store
of more than 8 bytes (buffer_store_dwordx3 / x4) whose soffset is an SGPR, followed directly
(no wait state) by a VALU instruction that writes one of the store's data VGPRs.  LLVM's hazard
recognizer inserts the wait state only when soffset is not a register; on the MI355X the
store was observed to send the overwritten value (tests/test_gpu_triup.py, bf16 -> f32).
usage: python tools/scan_store_hazard.py FILE.s ...   (hipcc -S --cuda-device-only output)"""
import re
import sys

STORE = re.compile(r"^\s*buffer_store_dwordx([34])\s+v\[(\d+):(\d+)\],\s*\S+,\s*s\[\d+:\d+\],\s*(\S+)")
VALU = re.compile(r"^\s*(v_\S+)\s+v\[?(\d+)(?::(\d+))?\]?")


def scan(path):
    hits = []
    fn = "?"
    lines = open(path).read().splitlines()
    for i, ln in enumerate(lines):
        if re.match(r"^_Z\S+:", ln):
            fn = ln.split(":")[0]
        m = STORE.match(ln)
        if not m or not m.group(4).startswith("s"):
            continue
        lo, hi = int(m.group(2)), int(m.group(3))
        j = i + 1
        while j < len(lines) and (not lines[j].strip() or lines[j].lstrip().startswith((";", "."))):
            j += 1
        if j >= len(lines):
            continue
        v = VALU.match(lines[j])
        if v and not v.group(1).startswith(("v_cmp", "v_cmpx", "v_readfirstlane", "v_readlane")):
            d0 = int(v.group(2))
            d1 = int(v.group(3)) if v.group(3) else d0
            if d0 <= hi and d1 >= lo:
                hits.append((fn, i + 1, ln.strip(), lines[j].strip()))
    return hits


if __name__ == "__main__":
    total = 0
    for p in sys.argv[1:]:
        for fn, ln, st, nx in scan(p):
            total += 1
            print(f"{p}:{ln}: {fn}\n    {st}\n    {nx}")
    print(f"{total} hazards")
    sys.exit(1 if total else 0)
