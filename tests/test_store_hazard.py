"""The shipped gfx950 code has no unguarded store-data hazard (CPU check of the built library).

A MUBUF store of more than 8 bytes with an SGPR soffset, followed directly by a VALU write of
its data registers, stored the overwritten value on the MI355X (k_tri_up bf16 -> f32, round 5;
DESIGN.md §8c).  tools/scan_store_hazard.py disassembles every code object of
libhygrid_hip.so and looks for that pattern.
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd", "HyGrid",
                   "_lib", "libhygrid_hip.so")


@pytest.mark.skipif(not os.path.exists(LIB) or shutil.which("objcopy") is None
                    or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"),
                    reason="needs the built library and the ROCm LLVM tools")
def test_no_store_data_hazard_in_library():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "scan_store_hazard.py"), "--lib", LIB],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and r.stdout.strip().endswith("0 hazards"), r.stdout[-3000:] + r.stderr[-2000:]
