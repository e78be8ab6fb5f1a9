"""Practical HBM ceiling at the bench lines' own sizes: a device-to-device copy (torch clone)
moving the same bytes as each line's kernel (read once + write once), HIP events, median of
20 after 10 warmup copies.  usage: python tools/copy_ceiling.py"""
import json
import statistics

import torch


def copy_rate(shape, dt):
    x = torch.rand(shape, device="cuda").to(dt)
    y = torch.empty_like(x)
    for _ in range(10):
        y.copy_(x)
    ts = []
    for _ in range(20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        y.copy_(x)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = statistics.median(ts)
    gb = 2 * x.numel() * x.element_size() / 1e9
    return {"shape": list(shape), "dtype": str(dt), "GB": round(gb, 4), "ms": round(ms, 4),
            "GB_per_s": round(gb / ms * 1e3, 1), "frac_of_8TBs": round(gb / ms * 1e3 / 8000, 4)}


if __name__ == "__main__":
    out = {"config3_4K_bf16_b128": copy_rate((128, 3, 2160, 3840), torch.bfloat16),
           "config2_1080p_f32_b32": copy_rate((32, 3, 1080, 1920), torch.float32),
           "config5_8K_f16_b8": copy_rate((8, 3, 4320, 7680), torch.float16)}
    print(json.dumps(out, indent=1))
