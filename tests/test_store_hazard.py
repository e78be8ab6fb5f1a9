"""The shipped gfx950 code has no unguarded store-data hazard (CPU check of the built library).

A vector memory store of more than 8 bytes followed, with no wait state, by a VALU write of its
data registers stored the overwritten value on the MI355X (k_tri_up bf16 -> f32, round 5;
DESIGN.md §8c).  tools/scan_store_hazard.py disassembles every code object of
libhygrid_hip.so and looks for the whole class: MUBUF / MTBUF / global / flat / scratch stores,
any soffset form, across fall-through labels.  The scanner itself is checked on a test-only
code object assembled here with seeded violations (and guarded sequences it must accept).
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd", "HyGrid",
                   "_lib", "libhygrid_hip.so")
LLVM = "/opt/rocm/lib/llvm/bin"
sys.path.insert(0, os.path.join(ROOT, "tools"))

# each seeded case: (assembly between the kernel label and s_endpgm, hazards expected)
SEEDED = [
    # the round-5 instance: SGPR soffset, data VGPR written by the very next VALU
    ("buffer_store_dwordx4 v[0:3], v4, s[0:3], s8 offen\n  v_mov_b32 v2, v5", 1),
    # the same store with soffset 0 and the wait state the compiler inserts for it
    ("buffer_store_dwordx4 v[0:3], v4, s[0:3], 0 offen\n  s_nop 0\n  v_mov_b32 v1, 0", 0),
    # 12-byte MUBUF store, write of its last register
    ("buffer_store_dwordx3 v[0:2], v4, s[0:3], 0 offen\n  v_add_f32 v2, v1, v1", 1),
    # global and flat stores (data is the second operand)
    ("global_store_dwordx4 v[6:7], v[8:11], off\n  v_add_f32 v9, v1, v1", 1),
    ("flat_store_dwordx4 v[6:7], v[8:11]\n  v_mul_f32 v11, v1, v1", 1),
    # MTBUF, packed VALU overlapping the data range
    ("tbuffer_store_format_xyzw v[12:15], v4, s[0:3], 0 "
     "format:[BUF_DATA_FORMAT_32_32_32_32,BUF_NUM_FORMAT_FLOAT] offen\n"
     "  v_pk_mov_b32 v[14:15], v[0:1], v[0:1] op_sel:[0,1]", 1),
    # a write of an unrelated register, and an 8-byte store: no hazard
    ("buffer_store_dwordx4 v[0:3], v4, s[0:3], s8 offen\n  v_mov_b32 v5, v6", 0),
    ("buffer_store_dwordx2 v[0:1], v4, s[0:3], s8 offen\n  v_mov_b32 v0, v6", 0),
    # one instruction between them is one wait state; v_cmp writes no VGPR
    ("buffer_store_dwordx4 v[0:3], v4, s[0:3], s8 offen\n  s_add_u32 s9, s9, 4\n  v_mov_b32 v0, v6", 0),
    ("buffer_store_dwordx4 v[0:3], v4, s[0:3], s8 offen\n  v_cmp_eq_u32 vcc, v0, v1\n  v_mov_b32 v0, v6", 0),
]


def _tools_ok():
    return all(os.path.exists(f"{LLVM}/{t}") for t in ("llvm-mc", "llvm-objdump"))


@pytest.mark.skipif(not _tools_ok(), reason="needs the ROCm LLVM tools")
def test_scanner_catches_seeded_violations(tmp_path):
    from scan_store_hazard import disassemble, scan
    for k, (body, want) in enumerate(SEEDED):
        src = tmp_path / f"seed{k}.s"
        src.write_text('.amdgcn_target "amdgcn-amd-amdhsa--gfx950"\n.text\n.globl seeded\n'
                       ".p2align 8\n.type seeded,@function\nseeded:\n  " + body + "\n  s_endpgm\n")
        obj = tmp_path / f"seed{k}.o"
        subprocess.run([f"{LLVM}/llvm-mc", "-triple=amdgcn-amd-amdhsa", "-mcpu=gfx950",
                        "-filetype=obj", str(src), "-o", str(obj)], check=True)
        got = scan(disassemble(str(obj), str(tmp_path / f"seed{k}.dis")))
        assert len(got) == want, (body, got)


def test_scanner_follows_fallthrough_labels(tmp_path):
    """Compiler (-S) listings: a label between the store and the write is no wait state."""
    from scan_store_hazard import scan
    p = tmp_path / "k.s"
    p.write_text("_Z1kv:\n  buffer_store_dwordx4 v[4:7], v0, s[0:3], 0 offen\n.LBB0_2:\n"
                 "  ; %bb.3\n  v_mov_b32_e32 v6, 0\n  s_endpgm\n")
    assert len(scan(str(p))) == 1
    p.write_text("_Z1kv:\n  buffer_store_dwordx4 v[4:7], v0, s[0:3], 0 offen\n"
                 "  s_cbranch_scc1 .LBB0_2\n.LBB0_2:\n  v_mov_b32_e32 v6, 0\n  s_endpgm\n")
    assert scan(str(p)) == []


@pytest.mark.skipif(not os.path.exists(LIB) or shutil.which("objcopy") is None or not _tools_ok(),
                    reason="needs the built library and the ROCm LLVM tools")
def test_no_store_data_hazard_in_library():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "scan_store_hazard.py"), "--lib", LIB],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and r.stdout.strip().endswith("0 hazards"), r.stdout[-3000:] + r.stderr[-2000:]
