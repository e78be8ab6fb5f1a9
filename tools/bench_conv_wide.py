"""Wide-channel HexConv2d (HexConvModule in segmentation models, HexModules.py:97-288):
the MFMA implicit-GEMM kernel (conv_mfma.hip) against the generic LDS kernel
(HYGRID_CONV_MFMA=0), HIP events, median over rounds; TFLOP/s counted as 2*O*7*C per
output sample (the dense hex contraction), against the f32 matrix peak (157.3 TF).

usage: python tools/bench_conv_wide.py [rounds]     -> one JSON line per shape
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd")]

import torch  # noqa: E402

from HyGrid import ops  # noqa: E402

F32_MFMA_PEAK_TF = 157.3


def run(B, C, O, H, W, dt, rounds):
    dev = torch.device("cuda:0")
    x = (torch.rand((B, C, H, W), device=dev) - 0.5).to(dt)
    k = (torch.rand((O, C, 1, 7), device=dev) - 0.5) * 0.1
    b = torch.rand((O,), device=dev) - 0.5
    res = {}
    for r in range(rounds + 1):
        for mode in ("1", "0"):
            if mode == "0" and r > 2:
                continue        # the generic kernel is slow: 2 timed rounds are enough
            os.environ["HYGRID_CONV_MFMA"] = mode
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.hexconv2d(x, k, b, 0, 2, padding=1, out_dtype=dt)
            e1.record()
            e1.synchronize()
            if r:
                res.setdefault(mode, []).append(e0.elapsed_time(e1))
    os.environ.pop("HYGRID_CONV_MFMA", None)
    flops = 2.0 * O * 7 * C * B * H * W
    out = {"shape": f"B{B} C{C} O{O} {H}x{W}", "dtype": str(dt)}
    for mode, name in (("1", "mfma"), ("0", "generic")):
        ms = statistics.median(res[mode])
        out[name] = {"ms": round(ms, 4), "TFLOP_s": round(flops / ms / 1e9, 2)}
    out["mfma"]["frac_f32_mfma_peak"] = round(out["mfma"]["TFLOP_s"] / F32_MFMA_PEAK_TF, 4)
    out["speedup"] = round(out["generic"]["ms"] / out["mfma"]["ms"], 2)
    print(json.dumps(out), flush=True)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    for (B, C, O, H, W) in [(4, 64, 64, 1080, 1920), (8, 32, 32, 540, 960),
                            (2, 128, 128, 540, 960), (4, 16, 32, 1080, 1920)]:
        for dt in (torch.bfloat16, torch.float32):
            run(B, C, O, H, W, dt, rounds)


if __name__ == "__main__":
    main()
