"""Scan gfx950 device assembly for the store-data hazard seen in k_tri_up (r05): a MUBUF store
of more than 8 bytes (buffer_store_dwordx3 / x4) whose soffset is an SGPR, followed directly
(no wait state) by a VALU instruction that writes one of the store's data VGPRs.  LLVM's hazard
recognizer inserts the wait state only when soffset is not a register; on the MI355X the
store was observed to send the overwritten value (tests/test_gpu_triup.py, bf16 -> f32).
usage: python tools/scan_store_hazard.py FILE.s ...   (hipcc -S --cuda-device-only output)
       python tools/scan_store_hazard.py --lib LIB.so   (every gfx950 code object in the library's
                                                          .hip_fatbin, via clang-offload-bundler and
                                                          llvm-objdump)"""
import concurrent.futures
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"

STORE = re.compile(r"^\s*buffer_store_dwordx([34])\s+v\[(\d+):(\d+)\],\s*\S+,\s*s\[\d+:\d+\],\s*(\S+)")
VALU = re.compile(r"^\s*(v_\S+)\s+v\[?(\d+)(?::(\d+))?\]?")


def scan(path):
    hits = []
    fn = "?"
    lines = open(path).read().splitlines()
    for i, ln in enumerate(lines):
        if re.match(r"^_Z\S+:", ln):
            fn = ln.split(":")[0]
        elif re.match(r"^[0-9a-f]+ <_Z\S+>:", ln):          # llvm-objdump label
            fn = ln.split("<")[1].split(">")[0]
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


def split_bundles(lib, out_dir):
    """The library's gfx950 code objects (one per offload bundle of .hip_fatbin) in out_dir."""
    fat = os.path.join(out_dir, "fatbin.bin")
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fat], check=True)
    data = open(fat, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    offs, i = [], data.find(magic)
    while i >= 0:
        offs.append(i)
        i = data.find(magic, i + 1)
    cos = []
    for k, o in enumerate(offs):
        b = os.path.join(out_dir, f"b{k}.bin")
        co = os.path.join(out_dir, f"co{k}.o")
        open(b, "wb").write(data[o:offs[k + 1] if k + 1 < len(offs) else len(data)])
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={b}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        cos.append(co)
    return cos


def disassemble_lib(lib, out_dir):
    """The library's device code objects as llvm-objdump listings in out_dir (one per bundle)."""
    cos = split_bundles(lib, out_dir)

    def one(co):
        s_path = co[:-2] + ".s"
        with open(s_path, "w") as f:
            subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], stdout=f, check=True)
        return s_path

    with concurrent.futures.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        return list(ex.map(one, cos))


if __name__ == "__main__":
    total = 0
    paths = sys.argv[1:]
    tmp = None
    if paths[:1] == ["--lib"]:
        tmp = tempfile.TemporaryDirectory()
        paths = disassemble_lib(paths[1], tmp.name)
    for p in paths:
        for fn, ln, st, nx in scan(p):
            total += 1
            print(f"{p}:{ln}: {fn}\n    {st}\n    {nx}")
    print(f"{total} hazards")
    sys.exit(1 if total else 0)
