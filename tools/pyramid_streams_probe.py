"""Config 5 (8K fp16 b8, 3 fused pyramid levels): does splitting the batch into image groups on
separate HIP streams hide the launches' ramp and tail (profiles/r06/launch_edges.txt: ~86 us of
fixed cost per step)?  One step = 3 dependent level launches per group; the groups are
independent images.  HIP events on the caller's stream around the fork / join, median of 20.
    python tools/pyramid_streams_probe.py"""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd"))


def main():
    from HyGrid import ops
    dev = torch.device("cuda:0")
    f16 = torch.float16
    B, C, H, W = 8, 3, 4320, 7680
    xp = torch.rand((B, C, H, W), device=dev, dtype=f16)
    k = torch.tensor([1, 1, 1, 6, 1, 1, 1], dtype=torch.float32, device=dev).div_(12).expand(3, 7).contiguous()
    main_st = torch.cuda.current_stream(dev)
    pool = [torch.cuda.Stream(dev) for _ in range(8)]

    def chain(x):
        cur, h_, w_ = x, H, W
        for lv in range(3):
            h_, w_ = h_ // 2, w_ // 2
            cur = ops.hex_pyramid_level(cur, k, None, (h_, w_), 0, from_rect=(lv == 0), out_dtype=f16)
        return cur

    def step(groups, order):
        if groups == 1:
            chain(xp)
            return
        per = B // groups
        fork = torch.cuda.Event()
        fork.record(main_st)
        for g in range(groups):
            s = pool[g]
            s.wait_event(fork)
            with torch.cuda.stream(s):
                if order == "interleave":
                    pass
                chain(xp[g * per:(g + 1) * per])
        for g in range(groups):
            main_st.wait_stream(pool[g])

    def timed(fn, n=20):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        t = []
        for _ in range(n):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main_st)
            fn()
            e1.record(main_st)
            e1.synchronize()
            t.append(e0.elapsed_time(e1))
        return statistics.median(t), min(t)

    alg = sum(B * C * (h * w + (h // 2) * (w // 2)) * 2 for h, w in ((H, W), (H // 2, W // 2), (H // 4, W // 4)))
    for rep in range(2):
        for groups in (1, 2, 4, 8):
            med, mn = timed(lambda: step(groups, "chain"))
            print(f"image groups on streams {groups}: {med:.4f} ms (min {mn:.4f})  "
                  f"{alg / (med * 1e-3) / 8e12:.3f} of 8 TB/s", flush=True)


if __name__ == "__main__":
    main()
