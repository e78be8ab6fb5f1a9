"""Profiling driver: runs one operator of the hot path a few times on a synthetic
4K bf16 batch so that rocprofv3 (kernel trace / PMC passes) can attribute it.

usage: python tools/prof_pipeline.py [fused|r2h|conv|h2r|r2h_nearest|copy|rt|pyr0] [batch] [iters]
(rt and pyr0 use their own configs: 1080p fp32 b32, 8K fp16 b8)

`copy` (torch bf16 clone) and `r2h_nearest` (one read + one write of every element) are
the known-byte calibration runs for the FETCH_SIZE/WRITE_SIZE counters.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd")]

import torch  # noqa: E402

from HyGrid import ops  # noqa: E402
from HyGrid.HexFrames import HexConv2d  # noqa: E402
from HyGrid.pipeline import rect_hex_conv_rect  # noqa: E402


def main():
    what = sys.argv[1] if len(sys.argv) > 1 else "fused"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    dev = torch.device("cuda:0")
    H, W = 2160, 3840
    x = torch.rand((B, 3, H, W), device=dev, dtype=torch.bfloat16)
    torch.manual_seed(3)
    conv = HexConv2d(3, 3, 0, 2, padding=1, bias=True).to(dev)
    conv.out_dtype = torch.bfloat16
    with torch.no_grad():
        for _i in range(iters):
            if what == "fused":
                rect_hex_conv_rect(x, conv, out_dtype=torch.bfloat16)
            elif what == "r2h":
                ops.rect_to_hex(x, (H, W), out_dtype=torch.bfloat16)
            elif what == "conv":
                conv(x)
            elif what == "h2r":
                ops.hex_to_rect(x, (H, W), out_dtype=torch.bfloat16)
            elif what == "r2h_nearest":
                ops.rect_to_hex(x, (H, W), interp=0)
            elif what == "copy":
                x.clone()
            elif what == "rt":          # config 2: 1080p RGB fp32 b32 round trip (k_fused MD 2)
                if _i == 0:
                    xr = torch.rand((32, 3, 1080, 1920), device=dev)
                ops.pipeline_r2h_h2r(xr)
            elif what == "pyr0":        # config 5 level 0: 8K RGB fp16 b8 from the rect image (MD 3)
                if _i == 0:
                    xp = torch.rand((8, 3, 4320, 7680), device=dev, dtype=torch.float16)
                    kp = torch.tensor([1, 1, 1, 6, 1, 1, 1], dtype=torch.float32,
                                      device=dev).div_(12).expand(3, 7).contiguous()
                ops.hex_pyramid_level(xp, kp, None, (2160, 3840), 0, from_rect=True,
                                      out_dtype=torch.float16)
            else:
                raise SystemExit(f"unknown stage {what!r}")
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
