"""Kernel-source digest (no torch import): shared by _abi.py (runtime check against the
library's stamp) and csrc/Makefile (the stamp compiled into libhygrid_hip.so).

usage: python3 HyGrid/_digest.py  -> prints the digest of the csrc/ tree next to it."""
import hashlib
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(_HERE), "csrc")
HEADER = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "hygrid.h")


def kernel_source_digest(csrc=CSRC, header=HEADER):
    """sha256 (16 hex digits) over the kernel sources (csrc/*.hip, *.h, Makefile, the C-ABI
    header): ties a library (hg_build_digest) and a profile (profiles/*/pmc_traffic.json) to
    the code they came from, also where no git metadata travels (the GPU box gets a bare
    snapshot)."""
    h = hashlib.sha256()
    files = sorted(os.path.join(csrc, f) for f in os.listdir(csrc)
                   if f.endswith((".hip", ".h", "Makefile")))
    for f in files + ([header] if os.path.exists(header) else []):
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(kernel_source_digest())
