"""Config 5 (8K fp16 b8, 3 fused pyramid levels): the levels as ONE chained launch
(hg_hex_pyramid_chain, HYGRID_PYR_CHAIN=1) against one launch per level, interleaved in one
process on the same buffers, HIP events on the caller's stream around each step; median / min
of the rounds, outputs compared bit for bit.
    python tools/pyramid_chain_probe.py [rounds] [batch]"""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd"))


def main():
    from HyGrid.HexFrames import HexConv2d
    from HyGrid.pipeline import hex_pyramid
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    dev = torch.device("cuda:0")
    H, W = 4320, 7680
    x = torch.rand((B, 3, H, W), device=dev, dtype=torch.float16)
    conv = HexConv2d(3, 3, 0, 2, padding=1, groups=3, bias=False).to(dev)
    with torch.no_grad():
        conv.kernel.copy_(torch.tensor([1, 1, 1, 6, 1, 1, 1], dtype=torch.float32, device=dev)
                          .div_(12).expand_as(conv.kernel))
    alg = sum(B * 3 * (h * w + (h // 2) * (w // 2)) * 2
              for h, w in ((H, W), (H // 2, W // 2), (H // 4, W // 4)))

    def step(chain):
        if chain:
            os.environ["HYGRID_PYR_CHAIN"] = "1"
        else:
            os.environ.pop("HYGRID_PYR_CHAIN", None)
        return hex_pyramid(x, conv, levels=3, out_dtype=torch.float16)

    t = {True: [], False: []}
    with torch.no_grad():
        a, b = step(True), step(False)
        same = all(torch.equal(u, v) for u, v in zip(a, b))
        print(f"chain == per-level launches: {same}", flush=True)
        for _ in range(3):
            step(True)
            step(False)
        torch.cuda.synchronize()
        for r in range(rounds):
            for chain in ((True, False) if r % 2 == 0 else (False, True)):
                step(chain)   # warm the path
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                step(chain)
                e1.record()
                e1.synchronize()
                t[chain].append(e0.elapsed_time(e1))
    os.environ.pop("HYGRID_PYR_CHAIN", None)
    for chain in (True, False):
        med = statistics.median(t[chain])
        print(f"{'chain (one launch)  ' if chain else 'one launch per level'}: {med:.4f} ms "
              f"(min {min(t[chain]):.4f})  {alg / (med * 1e-3) / 8e12:.3f} of 8 TB/s", flush=True)
    ratio = statistics.median([u / v for u, v in zip(t[True], t[False])])
    print(f"chain / per-level (median of round ratios): {ratio:.4f}")
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
