"""Which of the two GPU paths (k_tri_up / the general kernel) matches the exact fp32 blend of the
oracle's fp64 lattice (weights cast to fp32, alpha*p1 + beta*p2 + gamma*p3 rounded per
operation, geometry_np.py:347-354), for one hexresize / hex->rect linear call.
usage: python tools/dbg_triup.py OP h w h1 w1 [in_dtype out_dtype]   (OP: resize | h2r)"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd"))
from oracle import oracle as O  # noqa: E402
from HyGrid import ops  # noqa: E402

DT = {"bf16": torch.bfloat16, "f16": torch.float16, "f32": torch.float32}


def main():
    op, h, w, h1, w1 = sys.argv[1], *map(int, sys.argv[2:6])
    dt = DT[sys.argv[6]] if len(sys.argv) > 6 else torch.bfloat16
    od = DT[sys.argv[7]] if len(sys.argv) > 7 else torch.float32
    fn = ops.hexresize if op == "resize" else ops.hex_to_rect
    maps = O.hexresize_maps(h, w, h1, w1) if op == "resize" else O.h2r_maps(h, w, h1, w1)
    g = torch.Generator(device="cuda").manual_seed(h * 17 + w)
    x = torch.rand((2, 3, h, w), generator=g, device="cuda").to(dt)
    y_up = fn(x, (h1, w1), out_dtype=od).float().cpu().numpy()
    os.environ["HYGRID_DOWN"] = "0"
    y_gen = fn(x, (h1, w1), out_dtype=od).float().cpu().numpy()
    del os.environ["HYGRID_DOWN"]
    xs = x.float().cpu().numpy()
    i_n, j_n, flag, valid = (maps[k].astype(np.int64) for k in ("i_n", "j_n", "flag", "valid"))
    s1 = ((i_n + 1) / 2.0).astype(np.int64)
    s2 = ((i_n + 2) / 2.0).astype(np.int64)
    r = [i_n, np.where(flag == 1, i_n + 1, i_n), i_n + 1]
    c = [j_n - s1, np.where(flag == 1, j_n - s2, j_n + 1 - s1), j_n + 1 - s2]
    vb = [valid & 1, np.where(flag == 1, (valid >> 1) & 1, (valid >> 2) & 1), (valid >> 3) & 1]
    wts = [maps[k].astype(np.float32) for k in ("alpha", "beta", "gamma")]
    acc = None
    for v in range(3):
        ok = vb[v] == 1
        rr, cc = np.clip(r[v], 0, h - 1), np.clip(c[v], 0, w - 1)
        val = np.where(ok, xs[:, :, rr, cc], np.float32(0)).astype(np.float32)
        term = (wts[v] * val).astype(np.float32)
        acc = term if acc is None else (acc + term).astype(np.float32)
    ref = torch.from_numpy(acc).to(od).float().numpy()
    for name, y in (("tri_up", y_up), ("general", y_gen)):
        bad = np.argwhere(y.view(np.uint32) != ref.view(np.uint32))
        print(f"{name:8s} differs from the exact fp32 blend at {len(bad)} elements")
        for p in bad[:4]:
            b_, c_, a, bb = p
            print(f"   (a={a}, b={bb}) got {y[tuple(p)]!r} exact {ref[tuple(p)]!r} "
                  f"flag {flag[a, bb]} valid {valid[a, bb]} w {[float(t[a, bb]) for t in wts]}")
    print("tri_up vs general:", int((y_up.view(np.uint32) != y_gen.view(np.uint32)).sum()), "elements differ")
    reps = int(os.environ.get("DBG_REPS", "0"))   # repeat both paths: run-to-run differences
    for name, env in (("tri_up", None), ("general", "0")):
        nbad = 0
        for _ in range(reps):
            if env:
                os.environ["HYGRID_DOWN"] = env
            junk = torch.full((2, 3, h1, w1), float("nan"), device="cuda", dtype=od)   # dirty the allocator
            del junk
            y = fn(x, (h1, w1), out_dtype=od).float().cpu().numpy()
            os.environ.pop("HYGRID_DOWN", None)
            nbad += int((y.view(np.uint32) != ref.view(np.uint32)).any())
        if reps:
            print(f"{name}: {nbad} of {reps} repeated runs differ from the exact blend")


if __name__ == "__main__":
    main()
