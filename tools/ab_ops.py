"""Interleaved in-process A/B timing of library variants for the unfused hot-path operators
(one process, same device buffers, HIP events on the launch stream; each round runs every
variant three times back to back in a shuffled order and times the last launch; median /
min per launch and the median per-round ratio to the first variant named).

usage: python tools/ab_ops.py OP ROUNDS name1 name2 ...
  OP: r2h | h2r | conv | wide (HexConv2d 64->64, 1080p bf16 b4) | stem / stem32 (HexConv2d 3->64, 1080p b4, bf16 / f32) | r2h32 | h2r32 | rt | pyr | pyrfr | pyr1 | pyr2   (bf16 4K b128 for
      r2h/h2r/conv; fp32 1080p b32 for r2h32/h2r32 and rt, the fused round trip; pyr = config-5 pyramid level 0, 8K fp16 b8 -> 4K from a
      hex image, pyrfr = the same from the rect image, pyr1 = level 1, 4K -> 2K, pyr2 = level 2, 2K -> 1K;
      hr0 / hr1 / hr2 = hexresize alone at those three levels (fp16); hrb = 4K -> 2K bf16 b32; up = hex (h/2, w/2) -> rect (h, w)
      linear at 4K bf16 b32, the inverse of ConvertToHexagon's lattice)
  name 'base' = the in-tree library; others = HyGrid/_lib/variants/libhygrid_<name>.so;
  'name%VAR=VAL' runs that library with the environment variable VAR=VAL set around its calls
  (the library's A/B switches, e.g. base%HYGRID_PYR_KERNEL=lds)
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
    name = name.split("%")[0]
    path = os.path.join(LIBDIR, "libhygrid_hip.so") if name == "base" else \
        os.path.join(LIBDIR, "variants", f"libhygrid_{name}.so")
    return ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)


def main():
    op, rounds, names = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    libs = {n: load(n) for n in names}
    sys.path[:0] = [os.path.join(ROOT, "hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd")]
    from HyGrid import _abi
    dt = {torch.bfloat16: _abi.HG_BF16, torch.float16: _abi.HG_F16, torch.float32: _abi.HG_F32}
    g = torch.Generator(device=dev).manual_seed(2)
    if op in ("r2h", "h2r", "conv"):
        B, C, H, W, t = 128, 3, 2160, 3840, torch.bfloat16
    elif op in ("r2h32", "h2r32", "rt"):
        B, C, H, W, t = 32, 3, 1080, 1920, torch.float32
    elif op == "wide":
        B, C, H, W, t = 4, 64, 1080, 1920, torch.bfloat16
    elif op in ("stem", "stem32"):     # an mmseg stem: HexConv2d(3 -> 64), 1080p b4
        B, C, H, W, t = 4, 3, 1080, 1920, torch.bfloat16 if op == "stem" else torch.float32
    elif op in ("pyr1", "hr1"):
        B, C, H, W, t = 8, 3, 2160, 3840, torch.float16
    elif op in ("pyr2", "hr2"):
        B, C, H, W, t = 8, 3, 1080, 1920, torch.float16
    elif op == "up":
        B, C, H, W, t = 32, 3, 1080, 1920, torch.bfloat16
    elif op == "upn":
        B, C, H, W, t = 32, 3, 1080, 1920, torch.uint8
    elif op == "hrb":                  # the bench's hexresize_2x line: 4K -> 2K bf16 b32
        B, C, H, W, t = 32, 3, 2160, 3840, torch.bfloat16
    else:
        B, C, H, W, t = 8, 3, 4320, 7680, torch.float16
    if t == torch.uint8:
        x = torch.randint(0, 256, (B, C, H, W), generator=g, device=dev, dtype=t)
        dt[t] = _abi.HG_U8
    else:
        x = torch.rand((B, C, H, W), generator=g, device=dev, dtype=t)
    taps = (torch.tensor([1, 1, 1, 6, 1, 1, 1], dtype=torch.float32, device=dev) / 12).repeat(C)
    if op.startswith("pyr") or op.startswith("hr"):
        y = torch.empty((B, C, H // 2, W // 2), device=dev, dtype=t)
    elif op in ("up", "upn"):
        y = torch.empty((B, C, 2 * H, 2 * W), device=dev, dtype=t)
    elif op in ("stem", "stem32"):
        y = torch.empty((B, 64, H, W), device=dev, dtype=t)
    else:
        y = torch.empty_like(x)
    kc = C if op == "wide" else 3
    ko = 64 if op in ("stem", "stem32") else kc
    k = (torch.rand((ko, 7 * kc), generator=g, device=dev) - 0.5) * (0.5 if kc == 3 else 0.05)
    b = torch.rand((ko,), generator=g, device=dev) - 0.5
    s = st.cuda_stream

    def call(lib):
        if op in ("r2h", "r2h32"):
            f = lib.hg_rect_to_hex
            f.argtypes = [_vp, _vp, _int, _int] + [_i64] * 5 + [_int, _vp]
            return f(x.data_ptr(), y.data_ptr(), dt[t], dt[t], B * C, H, W, H, W, 1, s)
        if op in ("h2r", "h2r32"):
            f = lib.hg_hex_to_rect
            f.argtypes = [_vp, _vp, _int, _int] + [_i64] * 5 + [_int, _vp]
            return f(x.data_ptr(), y.data_ptr(), dt[t], dt[t], B * C, H, W, H, W, 1, s)
        if op == "rt":
            f = lib.hg_pipeline_r2h_h2r
            f.argtypes = [_vp, _vp, _int, _int] + [_i64] * 5 + [_vp]
            return f(x.data_ptr(), y.data_ptr(), dt[t], dt[t], B * C, H, W, H, W, s)
        if op.startswith("hr"):
            f = lib.hg_hexresize
            f.argtypes = [_vp, _vp, _int, _int] + [_i64] * 5 + [_int, _vp]
            return f(x.data_ptr(), y.data_ptr(), dt[t], dt[t], B * C, H, W, H // 2, W // 2, 1, s)
        if op in ("up", "upn"):
            f = lib.hg_hex_to_rect
            f.argtypes = [_vp, _vp, _int, _int] + [_i64] * 5 + [_int, _vp]
            return f(x.data_ptr(), y.data_ptr(), dt[t], dt[t], B * C, H, W, 2 * H, 2 * W,
                     0 if op == "upn" else 1, s)
        if op in ("conv", "wide", "stem", "stem32"):
            f = lib.hg_hexconv2d
            f.argtypes = [_vp] * 4 + [_int] * 3 + [_i64] * 5 + [_int] * 7 + [_dbl, _vp]
            return f(x.data_ptr(), k.data_ptr(), b.data_ptr(), y.data_ptr(), dt[t], _abi.HG_F32,
                     dt[t], B, C, ko, H, W, 2, 1, 1, 1, 1, 0, 0, 0.0, s)
        f = lib.hg_hex_pyramid_level
        f.argtypes = [_vp, _vp, _int, _int] + [_i64] * 6 + [_vp, _vp, _int, _int, _vp]
        return f(x.data_ptr(), y.data_ptr(), dt[t], dt[t], B, C, H, W, H // 2, W // 2,
                 taps.data_ptr(), None, 0, 1 if op == "pyrfr" else 0, s)

    times = {n: [] for n in names}
    ratios = {n: [] for n in names}
    sums = {}
    outs = {}
    rng = random.Random(7)
    for r in range(rounds + 1):
        order = list(libs.items())
        rng.shuffle(order)               # no fixed position in the round (clock / heat drift)
        rt = {}
        for n, lib in order:
            env = [kv.split("=") for kv in n.split("%")[1:]]   # name%VAR=VAL[%VAR2=VAL2...]
            for k_, v_ in env:
                os.environ[k_] = v_
            for rep in range(3):         # back-to-back launches; the last one is timed
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                rc = call(lib)
                e1.record()
                if rc != 0:
                    raise SystemExit(f"{n}: status {rc}")
            for k_, _ in env:
                del os.environ[k_]
            e1.synchronize()
            rt[n] = e0.elapsed_time(e1)
            if r == rounds:
                sums[n] = float(y.double().sum().item())
                if op in ("stem", "stem32"):       # element-wise against the first variant named
                    outs[n] = y.float().clone()
        if r > 0:
            for n in names:
                times[n].append(rt[n])
                ratios[n].append(rt[n] / rt[names[0]])
    alg = x.numel() * x.element_size() + y.numel() * y.element_size()
    for n in names:
        tm = times[n]
        print(f"{op:6s} {n:14s} median {statistics.median(tm):.4f} ms  min {min(tm):.4f} ms  "
              f"{alg / statistics.median(tm) / 1e6:.0f} GB/s  vs {names[0]} "
              f"{statistics.median(ratios[n]):.4f}  checksum {sums[n]:.9e}", flush=True)
    if outs:
        ref = outs[names[0]]
        for n in names[1:]:
            d = (outs[n] - ref).abs().max().item() / max(ref.abs().max().item(), 1e-30)
            print(f"{op:6s} {n:14s} max |diff| / max |{names[0]}| = {d:.3e}", flush=True)


if __name__ == "__main__":
    main()
