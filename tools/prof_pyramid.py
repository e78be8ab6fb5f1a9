"""Profiling driver for the config-5 hex pyramid (rocprofv3 kernel trace / PMC passes):
python tools/prof_pyramid.py [fused|unfused] [batch] [iters]   (8K RGB fp16, Gaussian taps)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd")]

import torch  # noqa: E402

from HyGrid.HexFrames import HexConv2d  # noqa: E402
from HyGrid.pipeline import hex_pyramid  # noqa: E402


def main():
    what = sys.argv[1] if len(sys.argv) > 1 else "fused"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    dev = torch.device("cuda:0")
    x = torch.rand((B, 3, 4320, 7680), device=dev, dtype=torch.float16)
    conv = HexConv2d(3, 3, 0, 2, padding=1, groups=3, bias=False).to(dev)
    with torch.no_grad():
        conv.kernel.copy_(torch.tensor([1, 1, 1, 6, 1, 1, 1], dtype=torch.float32,
                                       device=dev).div_(12).expand_as(conv.kernel))
        for _ in range(iters):
            hex_pyramid(x, conv, 3, fused=(what == "fused"))
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
