"""Per-kernel scratch and spill counts of the built library, from the code-object metadata
(`llvm-readobj --notes`: .private_segment_fixed_size, .sgpr_spill_count, .vgpr_spill_count) of
every gfx950 code object in libhygrid_hip.so's .hip_fatbin.  Round 5 found a run-time array
index (128 B of scratch per lane) and register-cap spills in hot kernels this way.
usage: python tools/kernel_resources.py LIB.so [--all]   (default: only kernels with scratch or spills)"""
import os
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from scan_store_hazard import LLVM, split_bundles  # noqa: E402


def resources(lib):
    """{kernel symbol: (scratch bytes per lane, sgpr spills, vgpr spills)}"""
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        for co in split_bundles(lib, tmp):
            txt = subprocess.run([f"{LLVM}/llvm-readobj", "--notes", co], capture_output=True,
                                 text=True, check=True).stdout
            name, vals = None, {}
            for ln in txt.splitlines():
                ln = ln.strip()
                if ln.startswith(".name:"):
                    name, vals = ln.split(":", 1)[1].strip(), {}
                elif name and ln.split(":")[0] in (".private_segment_fixed_size", ".sgpr_spill_count",
                                                   ".vgpr_spill_count"):
                    vals[ln.split(":")[0]] = int(ln.split(":")[1])
                    if len(vals) == 3:
                        out[name] = (vals[".private_segment_fixed_size"], vals[".sgpr_spill_count"],
                                     vals[".vgpr_spill_count"])
                        name = None
    return out


if __name__ == "__main__":
    res = resources(sys.argv[1])
    show_all = "--all" in sys.argv
    for k, (scr, ss, vs) in sorted(res.items()):
        if show_all or scr or ss or vs:
            print(f"{scr:6d} B scratch  {ss:4d} sgpr spills  {vs:4d} vgpr spills  {k}")
    print(f"{len(res)} kernels")
