"""Interleaved A/B timing of fused-kernel variants in ONE process (same GPU, same clocks):
each round launches every variant library three times back to back (the last launch is
timed) in a shuffled order on the same device buffers; reports the median / min per-launch
time over the rounds (HIP events on the launch stream) and the median of the per-round
ratios to the first variant named.

usage: python tools/ab_fused.py [rounds] name1 name2 ...   (name 'base' = the in-tree lib;
       others = HyGrid/_lib/variants/libhygrid_<name>.so); env AB_BATCH (default 128).
"""
import ctypes
import os
import random
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd",
                      "HyGrid", "_lib")
_i64, _int, _vp, _dbl = ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_double


def load(name):
    name = name.split("%")[0]        # name%VAR=value: the library with an A/B switch set
    path = os.path.join(LIBDIR, "libhygrid_hip.so") if name == "base" else \
        os.path.join(LIBDIR, "variants", f"libhygrid_{name}.so")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    f = lib.hg_pipeline_r2h_conv_h2r
    f.argtypes = [_vp, _vp, _vp, _vp, _int, _int] + [_i64] * 9 + [_int, _int, _int, _dbl, _vp]
    f.restype = _int
    return f


def main():
    rounds = int(sys.argv[1])
    names = sys.argv[2:]
    B, C, H, W = int(os.environ.get("AB_BATCH", "128")), 3, 2160, 3840
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(2)
    x = torch.rand((B, C, H, W), generator=g, device=dev, dtype=torch.bfloat16)
    y = torch.empty_like(x)
    torch.manual_seed(3)
    k = (torch.rand((3, 21), device=dev) - 0.5) * 0.5
    b = torch.rand((3,), device=dev) - 0.5
    st = torch.cuda.current_stream()
    fns = {n: load(n) for n in names}
    args = lambda: (x.data_ptr(), k.data_ptr(), b.data_ptr(), y.data_ptr(), 7, 7, B, C, C, H, W,
                    H, W, H, W, 1, 1, 0, 0.0, st.cuda_stream)
    times = {n: [] for n in names}
    ratios = {n: [] for n in names}
    sums = {}
    rng = random.Random(7)
    for r in range(rounds + 1):
        order = list(fns.items())
        rng.shuffle(order)               # no fixed position in the round (clock / heat drift)
        rt = {}
        for n, f in order:
            env = [kv.split("=") for kv in n.split("%")[1:]]   # name%VAR=VAL[%VAR2=VAL2...]
            for k_, v_ in env:
                os.environ[k_] = v_
            for rep in range(3):         # back-to-back launches; the last one is timed
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                rc = f(*args())
                e1.record()
                if rc != 0:
                    raise SystemExit(f"{n}: status {rc}")
            for k_, _ in env:
                del os.environ[k_]
            e1.synchronize()
            rt[n] = e0.elapsed_time(e1)
            if r == rounds:
                sums[n] = float(y.float().sum().item())
        if r > 0:
            for n in names:
                times[n].append(rt[n])
                ratios[n].append(rt[n] / rt[names[0]])
    alg = 2.0 * B * C * H * W * 2
    for n in names:
        t = times[n]
        print(f"{n:14s} median {statistics.median(t):.4f} ms  min {min(t):.4f} ms  "
              f"{alg / statistics.median(t) / 1e6:.0f} GB/s  vs {names[0]} {statistics.median(ratios[n]):.4f}  "
              f"checksum {sums[n]:.6e}", flush=True)


if __name__ == "__main__":
    main()
