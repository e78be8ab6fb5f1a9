"""HBM write ceilings at the inverse-lattice line's shape (32 x 3 x 2160 x 3840 bf16 output,
1.59 GB): torch fill_ (pure writes), a 4:1 write:read copy (x read once, written 4x as
the 2x-upsampled image would be), and a plain copy; median of 9 launches after warm-up."""
import statistics
import torch

dev = torch.device("cuda:0")
y = torch.empty((32, 3, 2160, 3840), dtype=torch.bfloat16, device=dev)
x = torch.rand((32, 3, 1080, 1920), device=dev).to(torch.bfloat16)
z = torch.empty_like(y)


def t(fn, n=9):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record(); b.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts)


GB = y.numel() * 2 / 1e9
ms = t(lambda: y.fill_(1.0))
print(f"fill_ (writes only)      {ms:.4f} ms  {GB / ms:.2f} TB/s  {GB / ms / 8:.3f} of 8 TB/s")
ms = t(lambda: y.view(32, 3, 1080, 2, 1920, 2).copy_(x[:, :, :, None, :, None].expand(32, 3, 1080, 2, 1920, 2)))
gb = GB + x.numel() * 2 / 1e9
print(f"2x nearest upsample copy {ms:.4f} ms  {gb / ms:.2f} TB/s  {gb / ms / 8:.3f} of 8 TB/s")
ms = t(lambda: z.copy_(y))
print(f"copy_ (1 read : 1 write) {ms:.4f} ms  {2 * GB / ms:.2f} TB/s  {2 * GB / ms / 8:.3f} of 8 TB/s")
