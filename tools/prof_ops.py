"""Profiling driver for the secondary lines: runs one call a few times so rocprofv3 (kernel
trace / PMC passes) can attribute its kernel.

usage: python tools/prof_ops.py OP [iters]
  rt   config 2: fused rect -> hex -> rect round trip, 1080p fp32 b32 (k_fused MD 2)
  pyr0 config 5 level 0 from the rect image, 8K fp16 b8 (k_fused MD 3)
  pyr1 config 5 level 1 (4K -> 2K from a hex image)
  hr0  hexresize 8K -> 4K fp16 b8 (the pyramid chain's level-0 hexresize); hr1 4K -> 2K,
       hr2 2K -> 1K (levels 1, 2)
  up   hex (1080, 1920) -> rect (2160, 3840) bf16 b32
  wide HexConv2d(64, 64, 0, 2, padding=1) bf16, 4 x 64 x 1080 x 1920 (the bench's wide line)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd")]

import torch  # noqa: E402

from HyGrid import ops  # noqa: E402
from HyGrid.pipeline import rect_hex_rect  # noqa: E402


def main():
    op = sys.argv[1]
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda:0")
    if op == "rt":
        x = torch.rand((32, 3, 1080, 1920), device=dev)
        fn = lambda: rect_hex_rect(x)  # noqa: E731
    elif op in ("pyr0", "pyr1"):
        shape = (8, 3, 4320, 7680) if op == "pyr0" else (8, 3, 2160, 3840)
        x = torch.rand(shape, device=dev, dtype=torch.float16)
        taps = (torch.tensor([1, 1, 1, 6, 1, 1, 1], dtype=torch.float32, device=dev) / 12).repeat(3, 1)
        H, W = shape[-2:]
        fn = lambda: ops.hex_pyramid_level(x, taps, None, (H // 2, W // 2), 0,  # noqa: E731
                                           from_rect=(op == "pyr0"), out_dtype=torch.float16)
    elif op in ("hr0", "hr1", "hr2"):
        H, W = {"hr0": (4320, 7680), "hr1": (2160, 3840), "hr2": (1080, 1920)}[op]
        x = torch.rand((8, 3, H, W), device=dev, dtype=torch.float16)
        fn = lambda: ops.hexresize(x, (H // 2, W // 2), out_dtype=torch.float16)  # noqa: E731
    elif op == "up":
        x = torch.rand((32, 3, 1080, 1920), device=dev, dtype=torch.bfloat16)
        fn = lambda: ops.hex_to_rect(x, (2160, 3840))  # noqa: E731
    elif op == "wide":
        from HyGrid.HexFrames import HexConv2d
        x = (torch.rand((4, 64, 1080, 1920), device=dev) - 0.5).to(torch.bfloat16)
        torch.manual_seed(5)
        conv = HexConv2d(64, 64, 0, 2, padding=1, bias=True).to(dev)
        conv.out_dtype = torch.bfloat16
        fn = lambda: conv(x)  # noqa: E731
    else:
        raise SystemExit(f"unknown op {op}")
    with torch.no_grad():
        for _ in range(iters):
            fn()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
