"""A/B timing of the HexConv2d kernels that hg_hexconv2d can pick for a radius-2,
stride-1, padding-1 layer: the two-column streaming kernel (k_fused MD 1, fused_conv.hip)
and the register-streaming kernel (k_hexconv_stream, conv_stream.hip, HYGRID_FCONV=0).
Interleaved in one process, HIP events on the launch stream, median over rounds.

usage: python tools/ab_conv.py [rounds] [batch]     (4K RGB, C=O=3, groups 1 and 3)
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd")]

import torch  # noqa: E402

from HyGrid import ops  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    H, W, C = 2160, 3840, 3
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(2)
    x32 = torch.rand((B, C, H, W), generator=g, device=dev)
    combos = [(torch.float32, torch.float32), (torch.bfloat16, torch.bfloat16),
              (torch.bfloat16, torch.float32), (torch.float16, torch.float16)]
    for groups in (1, 3):
        k = (torch.rand((3, 3 // groups, 1, 7), device=dev) - 0.5)
        b = torch.rand((3,), device=dev) - 0.5
        for dti, dto in combos:
            x = x32.to(dti)
            res = {}
            for r in range(rounds + 1):
                for mode in ("1", "0"):
                    os.environ["HYGRID_FCONV"] = mode
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record()
                    ops.hexconv2d(x, k, b, 0, 2, padding=1, groups=groups, out_dtype=dto)
                    e1.record()
                    e1.synchronize()
                    if r:
                        res.setdefault(mode, []).append(e0.elapsed_time(e1))
            nbytes = B * C * H * W * (x.element_size() + torch.empty((), dtype=dto).element_size())
            out = {"groups": groups, "in": str(dti), "out": str(dto), "batch": B}
            for mode, t in res.items():
                ms = statistics.median(t)
                out["fconv" if mode == "1" else "conv_stream"] = {
                    "ms": round(ms, 4), "GB_per_s": round(nbytes / ms / 1e6, 1)}
            print(json.dumps(out), flush=True)
            del x
    os.environ.pop("HYGRID_FCONV", None)


if __name__ == "__main__":
    main()
