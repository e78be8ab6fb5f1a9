"""A/B of the config-5 pyramid paths in one process (HIP events, median of rounds):
fused levels with rect->hex inside level 0, fused levels after a separate rect->hex, and
the operator chain.   python tools/ab_pyramid.py [rounds] [batch]"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd")]

import torch  # noqa: E402

from HyGrid.HexFrames import HexConv2d  # noqa: E402
from HyGrid.pipeline import hex_pyramid  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    dev = torch.device("cuda:0")
    x = torch.rand((B, 3, 4320, 7680), device=dev, dtype=torch.float16)
    conv = HexConv2d(3, 3, 0, 2, padding=1, groups=3, bias=False).to(dev)
    with torch.no_grad():
        conv.kernel.copy_(torch.tensor([1, 1, 1, 6, 1, 1, 1], dtype=torch.float32,
                                       device=dev).div_(12).expand_as(conv.kernel))
    variants = {"fused_l0_from_rect": dict(fused=True, l0_from_rect=True),
                "fused_after_r2h": dict(fused=True, l0_from_rect=False),
                "operator_chain": dict(fused=False)}
    t = {k: [] for k in variants}
    with torch.no_grad():
        for r in range(rounds + 1):
            for k, kw in variants.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                hex_pyramid(x, conv, 3, **kw)
                e1.record()
                e1.synchronize()
                if r:
                    t[k].append(e0.elapsed_time(e1))
    for k, v in t.items():
        print(f"{k:22s} median {statistics.median(v):.4f} ms  min {min(v):.4f} ms", flush=True)


if __name__ == "__main__":
    main()
