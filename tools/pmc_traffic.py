"""HBM traffic per launch from rocprofv3 PMC counters -> profiles/pmc_traffic.json.

Runs on the GPU box (this driver itself never touches the GPU; every profiled run is a
child process with the program directly after `--`):

    python tools/pmc_traffic.py OUTDIR [batch] [--summarise-only]

Per stage of tools/prof_pipeline.py it makes two separate passes, `--pmc FETCH_SIZE` and
`--pmc WRITE_SIZE` (they cannot share a pass on gfx950), and converts them as
MI355X_MICROARCH.md §HBM prescribes: bytes = counter x 1024, with FETCH_SIZE doubled
(gfx950 tallies 128-B streaming read requests at 64 B).  Two known-byte runs (a torch bf16
clone and the nearest rect->hex copy, each one read + one write of the batch) are profiled
beside the hot-path kernels and their measured/known ratios are written out with the
numbers, so the correction can be checked for this access pattern.
"""
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STAGES = {   # json key -> (prof_pipeline stage, kernel-name substring[, algorithmic bytes])
    "pipeline_r2h_conv_h2r": ("fused", "k_fused"),
    "rect_to_hex": ("r2h", "k_r2h_stream"),
    "hexconv2d": ("conv", "k_fused"),           # HexConv2d 3->3 runs on k_fused MD 1
    "hex_to_rect": ("h2r", "k_h2r_stream"),
    "calib_torch_copy": ("copy", "__amd_rocclr_copyBuffer"),
    "calib_r2h_nearest": ("r2h_nearest", "k_resample_nearest"),
    # round 6: the config-2 round trip and config-5 level 0, each on its own bytes
    # (algorithmic read bytes, write bytes)
    "pipeline_r2h_h2r": ("rt", "k_fused", (32 * 3 * 1080 * 1920 * 4, 32 * 3 * 1080 * 1920 * 4)),
    "pyramid_level0_from_rect": ("pyr0", "k_fused", (8 * 3 * 4320 * 7680 * 2, 8 * 3 * 2160 * 3840 * 2)),
}
# The FETCH_SIZE x2 correction was calibrated at the headline kernel's own access width (8 B per
# lane, dwordx2) in round 6: tools/microbench/walk8.hip's one-shot copy8 reads 1.0000x its bytes
# (profiles/r06/walk8_pmc.txt), as the 16-B copy does.
CAL_8B = {"copy8_fetch_x2_over_bytes": 1.0000, "copy16_fetch_x2_over_bytes": 1.0000,
          "source": "profiles/r06/walk8_pmc.txt (tools/microbench/walk8.hip)"}


def run_pass(out, stage, counter, batch):
    d = os.path.join(out, f"{stage}_{counter}")
    cmd = ["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "run",
           "--", sys.executable, os.path.join(ROOT, "tools", "prof_pipeline.py"), stage,
           str(batch), "2"]
    subprocess.run(cmd, check=True, timeout=300, stdout=subprocess.DEVNULL)
    return d


def read(d, sub, counter):
    vals = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"] and r["Counter_Name"] == counter:
                key = r["Dispatch_Id"]
                vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    if not vals:
        raise RuntimeError(f"no {counter} rows for {sub} in {d}")
    v = sorted(vals.values())
    if "copyBuffer" in sub:              # clone = small setup blits + the one big copy
        return v[-1], len(v)
    return v[len(v) // 2], len(v)        # median over dispatches


def main():
    out = sys.argv[1]
    batch = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 128
    only = "--summarise-only" in sys.argv       # re-read the CSVs of an earlier run
    os.makedirs(out, exist_ok=True)
    H, W, C = 2160, 3840, 3
    known = 2 * batch * C * H * W * 2        # one bf16 read + one bf16 write of the batch
    res = {}
    for key, spec in STAGES.items():
        stage, sub = spec[0], spec[1]
        alg_r, alg_w = spec[2] if len(spec) > 2 else (known / 2, known / 2)
        alg = alg_r + alg_w
        dirs = [os.path.join(out, f"{stage}_{c}") if only else run_pass(out, stage, c, batch)
                for c in ("FETCH_SIZE", "WRITE_SIZE")]
        f, nf = read(dirs[0], sub, "FETCH_SIZE")
        w, nw = read(dirs[1], sub, "WRITE_SIZE")
        fetch_b, write_b = 2.0 * f * 1024, w * 1024
        res[key] = {"FETCH_SIZE_KB": f, "WRITE_SIZE_KB": w, "dispatches": [nf, nw],
                    "read_bytes_corrected": fetch_b, "write_bytes": write_b,
                    "hbm_bytes_per_launch": fetch_b + write_b,
                    "alg_bytes_per_launch": alg,
                    "traffic_over_alg": (fetch_b + write_b) / alg,
                    "reads_over_alg_reads": fetch_b / alg_r,
                    "writes_over_alg_writes": write_b / alg_w}
        print(key, json.dumps(res[key]), flush=True)
    sys.path[:0] = [os.path.join(ROOT, "hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd")]
    from HyGrid._abi import kernel_source_digest
    doc = {"kernel_source_digest": kernel_source_digest(),
           "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, "
                     f"tools/prof_pipeline.py <stage> {batch} 2 (4K RGB bf16)",
           "correction": "bytes = KB x 1024; FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md §HBM)",
           "calibration_8B_lanes": CAL_8B,
           "batch": batch, "kernels": res}
    with open(os.path.join(out, "pmc_traffic.json"), "w") as fh:
        json.dump(doc, fh, indent=1)


if __name__ == "__main__":
    main()
