"""HBM read / write bytes of the fused kernel per library variant (FETCH_SIZE and WRITE_SIZE in
separate rocprofv3 passes over tools/prof_pipeline.py fused B 2; the reads corrected x2 as
tools/pmc_traffic.py does), against the algorithmic bytes of a 4K RGB bf16 batch of B.

usage: python tools/traffic_ab.py OUTDIR B name[%VAR=value] ...   ('base' = the in-tree lib)
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from pmc_traffic import read  # noqa: E402

LIBDIR = os.path.join(ROOT, "hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd",
                      "HyGrid", "_lib")


def main():
    out, batch, names = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
    alg_r = alg_w = batch * 3 * 2160 * 3840 * 2
    for n in names:
        lib, _, env = n.partition("%")
        path = os.path.join(LIBDIR, "libhygrid_hip.so") if lib == "base" else \
            os.path.join(LIBDIR, "variants", f"libhygrid_{lib}.so")
        e = dict(os.environ, HYGRID_LIB=path)
        if env:
            k, v = env.split("=")
            e[k] = v
        got = {}
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(out, f"{n.replace('%', '_').replace('=', '_')}_{c}")
            cmd = ["rocprofv3", "--pmc", c, "--output-format", "csv", "-d", d, "-o", "run", "--",
                   sys.executable, os.path.join(ROOT, "tools", "prof_pipeline.py"), "fused",
                   str(batch), "2"]
            subprocess.run(cmd, check=True, timeout=90, env=e, stdout=subprocess.DEVNULL,
                           stderr=subprocess.DEVNULL)
            got[c] = read(d, "k_fused", c)[0] * 1024
        rd, wr = got["FETCH_SIZE"] * 2, got["WRITE_SIZE"]
        print(f"{n:28s} reads {rd / alg_r:.4f}x  writes {wr / alg_w:.4f}x  total "
              f"{(rd + wr) / (alg_r + alg_w):.4f}x", flush=True)


if __name__ == "__main__":
    main()
