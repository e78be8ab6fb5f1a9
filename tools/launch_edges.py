"""Launch ramp and tail of the short launches (config 2's 0.3 ms round trip, the pyramid levels):
each kernel timed at several batch sizes, t(B) = a + b * B fitted; `a` is what a launch costs
beyond its per-image work (dispatch ramp, the partly filled last round of waves, the drain).
A one-shot 16-B-per-lane device copy of the same bytes (torch's copy_ and a clone) beside it.
HIP events, median of 20 per point.
    python tools/launch_edges.py"""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd"))


def timed(fn, n=20):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        t.append(e0.elapsed_time(e1))
    return statistics.median(t)


def fit(pts):
    n = len(pts)
    mx = sum(b for b, _ in pts) / n
    my = sum(t for _, t in pts) / n
    sxx = sum((b - mx) ** 2 for b, _ in pts)
    sxy = sum((b - mx) * (t - my) for b, t in pts)
    slope = sxy / sxx
    return my - slope * mx, slope


def main():
    from HyGrid import ops
    dev = torch.device("cuda:0")
    C, H, W = 3, 1080, 1920
    xs = torch.rand((128, C, H, W), device=dev)
    ys = torch.empty_like(xs)
    lines = {}
    for name, fn in (
            ("roundtrip fp32 1080p (MD 2)", lambda x: ops.pipeline_r2h_h2r(x)),
            ("copy_ fp32 (same bytes)", lambda x: ys[:x.shape[0]].copy_(x))):
        pts = []
        for B in (8, 16, 32, 64, 128):
            x = xs[:B]
            t = timed(lambda: fn(x))
            pts.append((B, t))
            print(f"{name:34s} B {B:4d}  {t:.4f} ms  {B * C * H * W * 8 / t / 1e9:.0f} GB/s", flush=True)
        a, b = fit(pts)
        lines[name] = (a, b)
        print(f"{name:34s} fit: {a * 1e3:.1f} us + {b * 1e3:.2f} us per image "
              f"(B=32: edges {a / (a + 32 * b) * 100:.1f} % of the launch)", flush=True)
    f16 = torch.float16
    xp = torch.rand((16, C, 4320, 7680), device=dev, dtype=f16)
    k = torch.tensor([1, 1, 1, 6, 1, 1, 1], dtype=torch.float32, device=dev).div_(12).expand(3, 1, 1, 7).contiguous()
    for lv, (hi, wi, fr) in enumerate(((4320, 7680, True), (2160, 3840, False), (1080, 1920, False))):
        src = xp if fr else torch.rand((16, C, hi, wi), device=dev, dtype=f16)
        pts = []
        for B in (2, 4, 8, 16):
            x = src[:B]
            t = timed(lambda: ops.hex_pyramid_level(x, k, None, (hi // 2, wi // 2), 0, from_rect=fr,
                                                     out_dtype=f16))
            pts.append((B, t))
            print(f"pyramid level {lv} ({hi}x{wi} fp16)      B {B:4d}  {t:.4f} ms", flush=True)
        a, b = fit(pts)
        print(f"pyramid level {lv} fit: {a * 1e3:.1f} us + {b * 1e3:.2f} us per image "
              f"(B=8: edges {a / (a + 8 * b) * 100:.1f} %)", flush=True)


if __name__ == "__main__":
    main()
