"""Locate the samples where k_hexresize_down differs from the general kernel at a shape."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from HyGrid import ops  # noqa: E402
from oracle import oracle as O  # noqa: E402

B, C, h, w = (int(v) for v in sys.argv[1:5])
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(h + w)
x = torch.rand((B, C, h, w), generator=g, device=dev).to(torch.float16)
size = (h // 2, w // 2)
y = ops.hexresize(x, size, out_dtype=torch.float16)
os.environ["HYGRID_DOWN"] = "0"
r = ops.hexresize(x, size, out_dtype=torch.float16)
del os.environ["HYGRID_DOWN"]
torch.cuda.synchronize()
bad = (y.view(torch.int16) != r.view(torch.int16))
print("mismatches", int(bad.sum()))
idx = bad.nonzero()
if idx.numel():
    print("planes", torch.unique(idx[:, 0] * C + idx[:, 1]).tolist()[:40])
    print("rows min/max", int(idx[:, 2].min()), int(idx[:, 2].max()), "rows mod 4 hist",
          torch.bincount(idx[:, 2] % 4).tolist())
    print("cols min/max", int(idx[:, 3].min()), int(idx[:, 3].max()), "col mod 62 hist",
          torch.bincount(idx[:, 3] % 62, minlength=62).tolist())
    rows = torch.unique(idx[:, 2]).tolist()
    print("distinct rows", len(rows), rows[:20])
    for k in range(min(8, idx.shape[0])):
        b_, c_, a_, q_ = (int(v) for v in idx[k])
        print("at", (b_, c_, a_, q_), "stream", float(y[b_, c_, a_, q_]), "general", float(r[b_, c_, a_, q_]))
    b_, c_ = int(idx[0, 0]), int(idx[0, 1])
    ref = O.hexresize(x[b_, c_].double().cpu().numpy(), size, 1)
    a_, q_ = int(idx[0, 2]), int(idx[0, 3])
    print("oracle", ref[a_, q_], "plane err stream", np.abs(y[b_, c_].double().cpu().numpy() - ref).max(),
          "general", np.abs(r[b_, c_].double().cpu().numpy() - ref).max())
