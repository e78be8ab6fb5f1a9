"""What the bench's per-step collective costs on the GPU: the row-sample reduction (every 64th
output row of the 128 x 3 x 2160 x 3840 bf16 batch) in a few torch forms, and the world-1 RCCL
all-gather of its 128 x 3 fp32 result.  HIP events, median of 30.
    python tools/step_sums_probe.py"""
import statistics

import torch
import torch.distributed as dist


def timed(fn, n=30):
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


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=dev)
    y = torch.rand((128, 3, 2160, 3840), device=dev, dtype=torch.bfloat16)
    forms = {
        "sum((2,3)) of y[:, :, ::64]": lambda: torch.sum(y[:, :, ::64], (2, 3), dtype=torch.float32),
        "sum(-1).sum(-1) of y[:, :, ::64]": lambda: torch.sum(y[:, :, ::64], -1, dtype=torch.float32).sum(-1),
        "sum(-1) of y[:, :, ::64, :].view rows": lambda: torch.sum(
            y.view(128, 3, 2160 // 8, 8, 3840)[:, :, ::8, 0], (2, 3), dtype=torch.float32),
        "sum((2,3)) of y[:, :, 0] (one row)": lambda: torch.sum(y[:, :, 0], -1, dtype=torch.float32),
    }
    for k, f in forms.items():
        print(f"{k:44s} {timed(f):.4f} ms", flush=True)
    s = torch.sum(y[:, :, ::64], -1, dtype=torch.float32).sum(-1)
    out = torch.empty_like(s)
    print(f"{'all_gather_into_tensor, world 1 (RCCL)':44s} "
          f"{timed(lambda: dist.all_gather_into_tensor(out, s)):.4f} ms", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
