"""Scan gfx950 device assembly for the store-data hazard class seen in k_tri_up (r05): a vector
memory store of more than 8 bytes (MUBUF buffer_store_dwordx3/x4 and _format_xyz(w), MTBUF
tbuffer_store_format_xyz(w), global_ / flat_ / scratch_store_dwordx3/x4), followed with no wait
state by a VALU instruction that writes one of the store's data registers (VGPRs or AGPRs).
The ISA requires one wait state there; LLVM's hazard recognizer inserts it only for MUBUF / MTBUF
stores whose soffset is not a register and for FLAT-family stores, and on the MI355X a MUBUF
store with an SGPR soffset sent the overwritten value (tests/test_gpu_triup.py, bf16 -> f32).
The check here is the class, whatever the soffset form: the next instruction after the store
(labels, comments and directives skipped, so a write after a fall-through label counts; a
branch or any other instruction between them is one wait state, `s_nop N` N + 1).
usage: python tools/scan_store_hazard.py FILE.s|FILE.o ...   (hipcc -S --cuda-device-only output,
                                                              or a code object: disassembled)
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

WIDE_STORE = re.compile(r"^\s*((?:t?buffer_store_(?:dwordx[34]|format_xyzw?))|"
                        r"(?:(?:global|flat|scratch)_store_dwordx[34]))\s+(.*)$")
REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+))")
INSN = re.compile(r"^\s*([a-z_][a-z0-9_]*)\b(.*)$")
WAIT_STATES = 1          # the ISA's requirement between the store and a VALU write of its data


def _regs(tok):
    """('v' | 'a', lo, hi) of one register operand token, or None."""
    m = REG.match(tok.strip())
    if not m:
        return None
    lo = int(m.group(2) if m.group(2) is not None else m.group(4))
    hi = int(m.group(3)) if m.group(3) is not None else lo
    return m.group(1), lo, hi


def _operands(rest):
    return [t for t in rest.split("//")[0].split(",")]


def store_data(mnemonic, rest):
    """The data register range of a > 8-byte store: the first 3- or 4-register v / a range."""
    for tok in _operands(rest):
        r = _regs(tok.strip().split()[0] if tok.strip() else "")
        if r and r[2] - r[1] + 1 in (3, 4):
            return r
    return None


def valu_dest(mnemonic, rest):
    """The v / a register range a VALU instruction writes (its first operand), or None."""
    if not mnemonic.startswith("v_") or mnemonic.startswith(("v_cmp", "v_readlane", "v_readfirstlane",
                                                             "v_nop")):
        return None
    ops = _operands(rest)
    if not ops or not ops[0].strip():
        return None
    return _regs(ops[0].strip().split()[0])


def _is_code(ln):
    t = ln.strip()
    if not t or t.startswith((";", "//", ".", "#")) or t.endswith(":"):
        return False
    if re.match(r"^[0-9a-f]+ <.*>:$", t):          # llvm-objdump symbol line
        return False
    return True


def scan(path):
    hits = []
    fn = "?"
    lines = open(path).read().splitlines()
    for i, ln in enumerate(lines):
        if re.match(r"^_Z\S+:", ln):
            fn = ln.split(":")[0]
        elif re.match(r"^[0-9a-f]+ <\S+>:", ln):          # llvm-objdump label
            fn = ln.split("<")[1].split(">")[0]
        m = WIDE_STORE.match(ln)
        if not m:
            continue
        data = store_data(m.group(1), m.group(2))
        if data is None:
            continue
        waits, j = 0, i + 1
        while j < len(lines) and waits < WAIT_STATES:
            if not _is_code(lines[j]):
                j += 1
                continue
            im = INSN.match(lines[j])
            if not im:
                j += 1
                continue
            mn, rest = im.group(1), im.group(2)
            if mn == "s_endpgm":
                break
            d = valu_dest(mn, rest)
            if d and d[0] == data[0] and d[1] <= data[2] and d[2] >= data[1]:
                hits.append((fn, i + 1, ln.strip(), lines[j].strip()))
                break
            if mn == "s_nop":
                n = re.match(r"\s*(\d+|0x[0-9a-fA-F]+)", rest)
                waits += (int(n.group(1), 0) if n else 0) + 1
            else:
                waits += 1
            j += 1
    return hits


def disassemble(co, s_path):
    with open(s_path, "w") as f:
        subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], stdout=f, check=True)
    return s_path


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
        return disassemble(co, co[:-2] + ".s")

    with concurrent.futures.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        return list(ex.map(one, cos))


if __name__ == "__main__":
    total = 0
    paths = sys.argv[1:]
    tmp = None
    tmp = tempfile.TemporaryDirectory()
    if paths[:1] == ["--lib"]:
        paths = disassemble_lib(paths[1], tmp.name)
    else:
        paths = [disassemble(p, os.path.join(tmp.name, f"o{k}.s")) if p.endswith(".o") else p
                 for k, p in enumerate(paths)]
    for p in paths:
        for fn, ln, st, nx in scan(p):
            total += 1
            print(f"{p}:{ln}: {fn}\n    {st}\n    {nx}")
    print(f"{total} hazards")
    sys.exit(1 if total else 0)
