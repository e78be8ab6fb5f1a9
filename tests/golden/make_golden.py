#!/usr/bin/env python3
"""Generate the golden vectors for the hot path from the reference itself.

CONTAINER-ONLY fixture generator (needs /root/reference; never runs on the GPU box).
It imports the reference's own `HyGrid.geometry_np` and `HyGrid.HexFrames` (a stub
`cv2` module is inserted first: cv2 is only used by the off-path `heximpad`), runs
them on small seeded inputs and freezes inputs + outputs + the reference's own
integer lattice index maps into `tests/golden/*.npz`.

The integer maps are not recomputed here: they are read out of the reference
function's own local variables (`i_n`, `j_n`, `up_down_flag`, `valid_indices*`,
`min_indices`, ...) with a `sys.setprofile` return hook, so the fixtures hold
exactly what the reference computed.

Reference call sites exercised (paths relative to /root/reference):
  rect_to_hex_resample   HyGrid/geometry_np.py:358-519
  hex_to_rect_resample   HyGrid/geometry_np.py:191-356 (linear)
  hex_to_square_resample HyGrid/geometry_torch.py:191-358 (nearest; the numpy twin
                         raises at geometry_np.py:339).  Executed from its source
                         text with device 'cuda'->'cpu' and torch.linspace bound to
                         numpy's linspace so the lattice is the geometry_np one.
  hexresize              HyGrid/geometry_np.py:520-681
  HexConv2d              HyGrid/HexFrames.py:22-185 (+ heximage_to_type1 :417-445)
  image_geometric_transformation  HyGrid/geometry_np.py:6-189
  HexPool2d / HexAdaptivePool2d / HexGlobalPool2d  HyGrid/HexFrames.py:255-410, :461-479

Usage:  python tests/golden/make_golden.py   (writes next to this file)
"""
import json
import os
import sys
import types

sys.dont_write_bytecode = True
REF = os.environ.get("HYGRID_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))

import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.modules.setdefault("cv2", types.ModuleType("cv2"))
sys.path.insert(0, REF)
import HyGrid.geometry_np as G  # noqa: E402
import HyGrid.HexFrames as HF  # noqa: E402


class Capture:
    """Grab ndarray/tensor locals of a named reference function at its return."""

    def __init__(self, name):
        self.name = name
        self.locals = {}

    def __call__(self, frame, event, arg):
        if event == "return" and frame.f_code.co_name == self.name:
            self.locals = {k: v for k, v in frame.f_locals.items()
                           if isinstance(v, (np.ndarray, torch.Tensor))}

    def run(self, fn, *a, **kw):
        sys.setprofile(self)
        try:
            return fn(*a, **kw)
        finally:
            sys.setprofile(None)


def np_(v):
    return v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else np.asarray(v)


def valid_mask(loc, n):
    m = np.zeros(np_(loc["valid_indices1"]).shape, np.int32)
    for k in range(1, n + 1):
        m |= np_(loc[f"valid_indices{k}"]).astype(np.int32) << (k - 1)
    return m


def make_input(rng, shape, dtype):
    if dtype == "u8":
        return rng.integers(0, 256, size=shape, dtype=np.uint8)
    if dtype == "f16":
        return rng.random(shape).astype(np.float16)
    if dtype == "f32":
        return rng.random(shape).astype(np.float32)
    return rng.random(shape)


def load_geometry_torch_cpu():
    """geometry_torch executed from its source text on the CPU (no GPU here).

    Two substitutions only: device 'cuda' -> 'cpu', and `torch.linspace` is
    served by numpy's linspace (float64) so that the sampling lattice equals
    geometry_np's; everything else (neighbour choice, argmin rule) is the
    reference's own code.
    """
    src = open(os.path.join(REF, "HyGrid", "geometry_torch.py")).read()
    src = src.replace("'cuda'", "'cpu'").replace('"cuda"', '"cpu"')

    class TorchProxy(types.ModuleType):
        def __getattr__(self, k):
            return getattr(torch, k)

    tp = TorchProxy("torch")
    tp.linspace = lambda a, b, n: torch.from_numpy(np.linspace(a, b, n))
    ns = {"__name__": "geometry_torch_cpu"}
    exec(compile(src, "geometry_torch.py", "exec"), ns)
    ns["torch"] = tp
    return ns


R2H_CASES = [  # (C, H, W, H1, W1, dtype)
    (1, 16, 20, 8, 10, "f64"),
    (3, 15, 17, 15, 17, "f32"),
    (3, 9, 12, 20, 25, "f64"),
    (1, 64, 64, 32, 32, "u8"),
    (2, 7, 5, 7, 5, "f64"),
    (1, 1, 1, 1, 1, "f64"),
    (1, 3, 4, 1, 6, "f64"),
    (1, 5, 4, 6, 1, "f64"),
    (3, 12, 16, 12, 16, "f16"),
    (3, 30, 40, 61, 79, "f32"),
    (1, 256, 256, 256, 256, "u8"),   # BASELINE config 1
]
H2R_CASES = [  # (C, H, W, H1, W1, dtype): hex (H,W) -> rect (H1,W1)
    (1, 16, 20, 8, 10, "f64"),
    (3, 15, 17, 15, 17, "f32"),
    (3, 9, 12, 20, 25, "f64"),
    (1, 64, 64, 32, 32, "u8"),
    (2, 7, 5, 7, 5, "f64"),
    (1, 1, 1, 1, 1, "f64"),
    (1, 3, 4, 1, 6, "f64"),
    (1, 5, 4, 6, 1, "f64"),
    (3, 12, 16, 12, 16, "f16"),
    (3, 30, 40, 61, 79, "f32"),
]
RESIZE_CASES = [
    (3, 16, 20, 8, 10, "f64"),
    (3, 17, 23, 9, 12, "f32"),
    (3, 8, 10, 16, 20, "f64"),
    (1, 33, 47, 17, 24, "f64"),
    (2, 9, 9, 9, 9, "f32"),
    (1, 40, 64, 20, 32, "u8"),
]


def gen_r2h(rng):
    arrs, index = {}, []
    for ci, (c, h, w, h1, w1, dt) in enumerate(R2H_CASES):
        x = make_input(rng, (c, h, w), dt)
        arrs[f"c{ci}_x"] = x
        for mode in ("bilinear", "nearest"):
            cap = Capture("rect_to_hex_resample")
            y = cap.run(G.rect_to_hex_resample, x, (h1, w1), mode)
            L = cap.locals
            tag = f"c{ci}_{mode}"
            arrs[tag + "_y"] = np.asarray(y).reshape(c, h1, w1)
            arrs[tag + "_i_n"] = np_(L["i_n"]).astype(np.int32)
            arrs[tag + "_j_n"] = np_(L["j_n"]).astype(np.int32)
            arrs[tag + "_i_f"] = np_(L["i_f"])
            arrs[tag + "_j_f"] = np_(L["j_f"])
            arrs[tag + "_valid"] = valid_mask(L, 4)
            if mode == "nearest":
                arrs[tag + "_argmin"] = np_(L["min_indices"]).astype(np.int32)
            index.append(dict(case=ci, mode=mode, c=c, h=h, w=w, h1=h1, w1=w1, dtype=dt,
                              out_dtype=str(np.asarray(y).dtype), out_shape=list(np.shape(y))))
    return arrs, index


def gen_h2r(rng, gt):
    arrs, index = {}, []
    for ci, (c, h, w, h1, w1, dt) in enumerate(H2R_CASES):
        x = make_input(rng, (c, h, w), dt)
        arrs[f"c{ci}_x"] = x
        # linear: the numpy reference
        cap = Capture("hex_to_rect_resample")
        y = cap.run(G.hex_to_rect_resample, x, (h1, w1), "linear")
        L = cap.locals
        tag = f"c{ci}_linear"
        arrs[tag + "_y"] = np.asarray(y).reshape(c, h1, w1)
        for k in ("i_n", "j_n"):
            arrs[tag + "_" + k] = np_(L[k]).astype(np.int32)
        arrs[tag + "_flag"] = np_(L["up_down_flag"]).astype(np.int32)
        arrs[tag + "_i_f"] = np_(L["i_f"])
        arrs[tag + "_j_f"] = np_(L["j_f"])
        arrs[tag + "_valid"] = valid_mask(L, 4)
        for k in ("alpha", "beta", "gamma"):
            arrs[tag + "_" + k] = np_(L[k])[..., 0]
        arrs[tag + "_S"] = np.stack([np_(L["S1"]), np_(L["S2"]), np_(L["S3"])])
        index.append(dict(case=ci, mode="linear", c=c, h=h, w=w, h1=h1, w1=w1, dtype=dt,
                          out_dtype=str(np.asarray(y).dtype), out_shape=list(np.shape(y))))
        # nearest: the torch twin (geometry_np's nearest raises, :339)
        cap = Capture("hex_to_square_resample")
        y = cap.run(gt["hex_to_square_resample"], x, (h1, w1), "nearest")
        L = cap.locals
        tag = f"c{ci}_nearest"
        arrs[tag + "_y"] = np.asarray(y).reshape(c, h1, w1)
        for k in ("i_n", "j_n"):
            arrs[tag + "_" + k] = np_(L[k]).astype(np.int32)
        arrs[tag + "_flag"] = np_(L["up_down_flag"]).astype(np.int32)
        arrs[tag + "_valid"] = valid_mask(L, 4)
        arrs[tag + "_argmin"] = np_(L["min_indices"]).astype(np.int32)
        index.append(dict(case=ci, mode="nearest", c=c, h=h, w=w, h1=h1, w1=w1, dtype=dt,
                          out_dtype=str(np.asarray(y).dtype), out_shape=list(np.shape(y)),
                          source="geometry_torch.hex_to_square_resample (cpu exec, numpy linspace)"))
    return arrs, index


def gen_resize(rng):
    arrs, index = {}, []
    for ci, (c, h, w, h1, w1, dt) in enumerate(RESIZE_CASES):
        x = make_input(rng, (c, h, w), dt)
        arrs[f"c{ci}_x"] = x
        cap = Capture("hexresize")
        y = cap.run(G.hexresize, x, (h1, w1), "linear")
        L = cap.locals
        tag = f"c{ci}_linear"
        arrs[tag + "_y"] = np.asarray(y).reshape(c, h1, w1)
        for k in ("i_n", "j_n"):
            arrs[tag + "_" + k] = np_(L[k]).astype(np.int32)
        arrs[tag + "_flag"] = np_(L["up_down_flag"]).astype(np.int32)
        arrs[tag + "_i_f"] = np_(L["i_f"])
        arrs[tag + "_j_f"] = np_(L["j_f"])
        arrs[tag + "_valid"] = valid_mask(L, 4)
        for k in ("alpha", "beta", "gamma"):
            arrs[tag + "_" + k] = np_(L[k])[..., 0]
        index.append(dict(case=ci, mode="linear", c=c, h=h, w=w, h1=h1, w1=w1, dtype=dt,
                          out_dtype=str(np.asarray(y).dtype), out_shape=list(np.shape(y))))
    return arrs, index


def conv_cases():
    """Deterministic subset of the HexConv2d parameter space."""
    cases = []
    i = 0
    for r in (2, 3):
        for off in (0, 1):
            for pad in (0, 1, 2):
                for (h, w) in ((8, 10), (7, 9)):
                    for stride in (1, 2):
                        groups = (1, 3)[i % 2]
                        dil = (1, 1, 2)[i % 3]
                        out_c = (3, 6)[(i // 2) % 2]
                        bias = (i % 5) != 0
                        pval = (0.0, 0.5)[(i // 3) % 2]
                        cases.append(dict(r=r, off=off, pad=pad, h=h, w=w, stride=stride,
                                          groups=groups, dilation=dil, out_c=out_c, bias=bias,
                                          padding_mode="constant", padding_value=pval))
                        i += 1
    # the bench configuration's layer, larger image
    cases.append(dict(r=2, off=0, pad=1, h=24, w=40, stride=1, groups=1, dilation=1, out_c=3,
                      bias=True, padding_mode="constant", padding_value=0.0))
    # depthwise Gaussian (pyramid config) shape
    cases.append(dict(r=2, off=0, pad=1, h=16, w=18, stride=1, groups=3, dilation=1, out_c=3,
                      bias=False, padding_mode="constant", padding_value=0.0))
    # other torch padding modes
    for mode in ("reflect", "replicate", "circular"):
        for off in (0, 1):
            cases.append(dict(r=2, off=off, pad=1, h=9, w=11, stride=1, groups=1, dilation=1,
                              out_c=4, bias=True, padding_mode=mode, padding_value=0.0))
    # wider channels
    cases.append(dict(r=2, off=1, pad=1, h=12, w=14, stride=1, groups=2, dilation=1, out_c=8,
                      bias=True, padding_mode="constant", padding_value=0.0, in_c=6))
    cases.append(dict(r=4, off=0, pad=3, h=13, w=15, stride=1, groups=1, dilation=1, out_c=2,
                      bias=True, padding_mode="constant", padding_value=0.0))
    return cases


def gen_conv():
    arrs, index = {}, []
    for ci, p in enumerate(conv_cases()):
        torch.manual_seed(1000 + ci)
        p = dict(p)
        in_c = p.setdefault("in_c", 3)
        try:
            m = HF.HexConv2d(in_c, p["out_c"], p["off"], p["r"], stride=p["stride"],
                             padding=p["pad"], dilation=p["dilation"], groups=p["groups"],
                             bias=p["bias"], padding_mode=p["padding_mode"],
                             padding_value=p["padding_value"])
            x = torch.rand(2, in_c, p["h"], p["w"])
            with torch.no_grad():
                y = m(x)
        except Exception as e:  # configurations the reference itself rejects
            index.append(dict(case=ci, **p, error=type(e).__name__))
            continue
        arrs[f"c{ci}_x"] = x.numpy()
        arrs[f"c{ci}_kernel"] = m.kernel.detach().numpy()
        if m.bias is not None:
            arrs[f"c{ci}_bias"] = m.bias.detach().numpy()
        arrs[f"c{ci}_y"] = y.numpy()
        index.append(dict(case=ci, **p, out_shape=list(y.shape),
                          out_dtype=str(y.dtype)))
    return arrs, index


def gen_conv_bwd():
    """HexConv2d gradients from the reference's own autograd graph (pad -> type1 ->
    two strided F.conv2d -> interleave, HexFrames.py:96-169) for a seeded upstream
    gradient: d input, d kernel, d bias of every forward case above."""
    arrs, index = {}, []
    for ci, p in enumerate(conv_cases()):
        torch.manual_seed(1000 + ci)
        p = dict(p)
        in_c = p.setdefault("in_c", 3)
        try:
            m = HF.HexConv2d(in_c, p["out_c"], p["off"], p["r"], stride=p["stride"],
                             padding=p["pad"], dilation=p["dilation"], groups=p["groups"],
                             bias=p["bias"], padding_mode=p["padding_mode"],
                             padding_value=p["padding_value"])
            x = torch.rand(2, in_c, p["h"], p["w"]).requires_grad_(True)
            y = m(x)
            g = torch.Generator().manual_seed(5000 + ci)
            gy = torch.randn(y.shape, generator=g)
            y.backward(gy)
        except Exception as e:  # configurations the reference itself rejects
            index.append(dict(case=ci, **p, error=type(e).__name__))
            continue
        arrs[f"c{ci}_x"] = x.detach().numpy()
        arrs[f"c{ci}_kernel"] = m.kernel.detach().numpy()
        if m.bias is not None:
            arrs[f"c{ci}_bias"] = m.bias.detach().numpy()
            arrs[f"c{ci}_dbias"] = m.bias.grad.numpy()
        arrs[f"c{ci}_gy"] = gy.numpy()
        arrs[f"c{ci}_dx"] = x.grad.numpy()
        arrs[f"c{ci}_dkernel"] = m.kernel.grad.numpy()
        index.append(dict(case=ci, **p, out_shape=list(y.shape)))
    return arrs, index


def igt_cases():
    """(c, h, w, H, dtype) for image_geometric_transformation (hex -> hex homography)."""
    th = np.deg2rad(30.0)
    rot = np.array([[np.cos(th), -np.sin(th), 0.0], [np.sin(th), np.cos(th), 0.0], [0, 0, 1.0]])
    return [
        (1, 8, 10, np.eye(3), "f64"),
        (3, 9, 12, np.diag([0.5, 0.5, 1.0]), "f64"),
        (3, 12, 16, np.diag([2.0, 1.5, 1.0]), "f32"),
        (2, 11, 13, rot, "f64"),
        (1, 16, 16, np.array([[1.0, 0.3, 0.0], [0.2, 1.0, 0.0], [0, 0, 1.0]]), "f64"),
        (3, 10, 14, np.array([[0.9, 0.0, 1.25], [0.0, 1.1, -2.5], [0, 0, 1.0]]), "u8"),
        (1, 7, 9, np.array([[1.3, -0.4, 0.7], [0.5, 0.8, 0.3], [0, 0, 1.0]]), "f32"),
    ]


def gen_igt(rng):
    """geometry_np.image_geometric_transformation (:6-189), 'linear', with the reference's
    own lattice locals (its 'nearest' raises at :172, 'bilinear' returns np.empty)."""
    arrs, index = {}, []
    for ci, (c, h, w, Hm, dt) in enumerate(igt_cases()):
        x = make_input(rng, (c, h, w), dt)
        arrs[f"c{ci}_x"] = x
        arrs[f"c{ci}_H"] = Hm
        cap = Capture("image_geometric_transformation")
        y = cap.run(G.image_geometric_transformation, x, Hm, "linear")
        L = cap.locals
        tag = f"c{ci}"
        h1, w1 = np_(L["i_n"]).shape
        arrs[tag + "_y"] = np.asarray(y).reshape(c, h1, w1)
        for k in ("i_n", "j_n"):
            arrs[tag + "_" + k] = np_(L[k]).astype(np.int32)
        arrs[tag + "_flag"] = np_(L["up_down_flag"]).astype(np.int32)
        arrs[tag + "_valid"] = valid_mask(L, 4)
        arrs[tag + "_x_"] = np_(L["x_"])
        arrs[tag + "_y_"] = np_(L["y_"])
        for k in ("alpha", "beta", "gamma"):
            arrs[tag + "_" + k] = np_(L[k])[..., 0]
        for k in ("p1_x", "p1_y", "p2_x", "p2_y", "p3_x", "p3_y"):
            arrs[tag + "_" + k] = np_(L[k])
        entry = dict(case=ci, c=c, h=h, w=w, h1=int(h1), w1=int(w1), dtype=dt,
                     out_dtype=str(np.asarray(y).dtype), out_shape=list(np.shape(y)))
        try:
            G.image_geometric_transformation(x, Hm, "nearest")
            entry["nearest"] = "ok"
        except Exception as e:  # the reference's tuple-unpacking of np.min (:172)
            entry["nearest"] = type(e).__name__
        entry["bilinear_shape"] = list(np.shape(G.image_geometric_transformation(x, Hm, "bilinear")))
        index.append(entry)
    return arrs, index


def pool_cases():
    """HexPool2d configurations (HexFrames.py:255-343).  stride is always given: the
    reference's stride=None path crashes (:270-276)."""
    return [
        dict(method="max", k=2, s=2, pad=0, h=8, w=11),
        dict(method="min", k=2, s=2, pad=0, h=9, w=12),
        dict(method="average", k=2, s=2, pad=0, h=8, w=12),
        dict(method="max", k=3, s=2, pad=1, h=10, w=13),
        dict(method="average", k=3, s=3, pad=1, h=12, w=16, mode="reflect"),
        dict(method="max", k=[2, 3], s=[2, 3], pad=0, h=9, w=14),
        dict(method="average", k=2, s=2, pad=0, h=9, w=13, ceil=True),
        dict(method="average", k=2, s=2, pad=0, h=9, w=13, ceil=True, cip=False),
        dict(method="max", k=3, s=3, pad=0, h=11, w=16, ceil=True, cip=False),
        dict(method="average", k=2, s=1, pad=1, h=7, w=9, mode="replicate"),
        dict(method="min", k=2, s=2, pad=2, h=6, w=8, mode="constant", value=0.5),
        dict(method="max", k=2, s=2, pad=0, h=8, w=10, allnan=True),
        dict(method="average", k=2, s=2, pad=0, h=8, w=10, allnan=True),
        dict(method="max", k=4, s=2, pad=0, h=9, w=12),
        dict(method="average", k=2, s=2, pad=1, h=7, w=9, mode="circular"),
        dict(method="max", k=3, s=2, pad=1, h=10, w=12),
        dict(method="average", k=3, s=2, pad=0, h=9, w=10, ceil=True, cip=False),
        dict(method="min", k=[3, 2], s=[2, 3], pad=1, h=11, w=15, ceil=True),
        dict(method="max", k=2, s=3, pad=0, h=10, w=14),
    ]


def _nan_input(shape, seed, allnan=False):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(shape, generator=g, dtype=torch.float64)
    m = torch.rand(shape, generator=g) < 0.15
    x[m] = float("nan")
    if allnan:
        x[..., 0:2, 0:4] = float("nan")      # whole windows of NaN
    return x


def gen_pool():
    """HexPool2d / HexAdaptivePool2d / HexGlobalPool2d outputs and input gradients from the
    reference's own forward and autograd (NaN-aware max/min/average, :461-479).  The
    adaptive / global modules cannot be constructed in the reference (their method dict
    names the undefined centroid_pooling, :354-358, :401-405); their forward (:359-396,
    :406-410) is run on instances built with nn.Module.__init__ and the method set."""
    arrs, index = {}, []
    ci = 0
    for p in pool_cases():
        x = _nan_input((2, 3, p["h"], p["w"]), 500 + ci, p.get("allnan", False))
        entry = dict(kind="pool", case=ci, **p)
        try:
            m = HF.HexPool2d(p["method"], kernel_size=p["k"], stride=p["s"], padding=p["pad"],
                             padding_mode=p.get("mode", "constant"),
                             padding_value=p.get("value", 0), ceil_mode=p.get("ceil", False),
                             count_include_pad=p.get("cip", True))
            xr = x.clone().requires_grad_(True)
            y = m(xr)
            gy = torch.randn(y.shape, generator=torch.Generator().manual_seed(900 + ci),
                             dtype=torch.float64)
            y.backward(gy)
            arrs[f"p{ci}_x"] = x.numpy()
            arrs[f"p{ci}_y"] = y.detach().numpy()
            arrs[f"p{ci}_gy"] = gy.numpy()
            arrs[f"p{ci}_dx"] = xr.grad.numpy()
            entry["out_shape"] = list(y.shape)
        except Exception as e:
            entry["error"] = type(e).__name__
        index.append(entry)
        ci += 1
    for kind, cls, args in (("adaptive", "HexAdaptivePool2d", [(2, 9, 12), (3, 12, 20),
                                                                  (4, 8, 9), (1, 6, 7)]),
                            ("global", "HexGlobalPool2d", [(1, 5, 7), (1, 16, 20)])):
        for a in args:
            for method in ("max", "min", "average"):
                entry = dict(kind=kind, case=ci, method=method, outsize=a[0], h=a[1], w=a[2])
                try:
                    getattr(HF, cls)(a[0], method) if kind == "adaptive" else getattr(HF, cls)(method)
                    entry["construct"] = "ok"
                except Exception as e:
                    entry["construct"] = type(e).__name__
                m = getattr(HF, cls).__new__(getattr(HF, cls))
                torch.nn.Module.__init__(m)
                m.hn, m.wn = a[0], a[0]
                m.method = {"max": HF.max_pooling, "min": HF.min_pooling,
                            "average": HF.average_pooling}[method]
                x = _nan_input((2, 3, a[1], a[2]), 700 + ci)
                xr = x.clone().requires_grad_(True)
                try:
                    y = m(xr)
                    gy = torch.randn(y.shape, generator=torch.Generator().manual_seed(ci),
                                     dtype=torch.float64)
                    y.backward(gy)
                    arrs[f"p{ci}_x"] = x.numpy()
                    arrs[f"p{ci}_y"] = y.detach().numpy()
                    arrs[f"p{ci}_gy"] = gy.numpy()
                    arrs[f"p{ci}_dx"] = xr.grad.numpy()
                    entry["out_shape"] = list(y.shape)
                except Exception as e:
                    entry["error"] = type(e).__name__
                index.append(entry)
                ci += 1
    return arrs, index


def gen_taps():
    """Impulse tap tables: output (r,q) of tap t reads input flat index table[t,r,q] (-1: zero)."""
    arrs, index = {}, []
    i = 0
    for off in (0, 1):
        for pad in (0, 1, 2):
            for (h, w) in ((8, 10), (7, 9)):
                x = (torch.arange(h * w, dtype=torch.float32) + 1).reshape(1, 1, h, w)
                tabs = []
                for t in range(7):
                    m = HF.HexConv2d(1, 1, off, 2, padding=pad, bias=False)
                    with torch.no_grad():
                        m.kernel.zero_()
                        m.kernel[0, 0, 0, t] = 1.0
                        y = m(x)[0, 0].numpy()
                    tabs.append(np.rint(y).astype(np.int32) - 1)
                arrs[f"t{i}_table"] = np.stack(tabs)
                index.append(dict(case=i, off=off, pad=pad, h=h, w=w))
                i += 1
    return arrs, index


def gen_kats(gt):
    kat = {}
    ones = np.ones((1, 12, 16))
    y = G.rect_to_hex_resample(ones, None, "bilinear")
    kat["r2h_ones"] = dict(col0_max=float(np.abs(y[:, 0]).max()),
                           colN_max=float(np.abs(y[:, -1]).max()),
                           interior_min=float(y[1:-1, 1:-1].min()),
                           interior_max=float(y[1:-1, 1:-1].max()),
                           row0_col1=float(y[0, 1]))
    y = G.hex_to_rect_resample(ones, None, "linear")
    kat["h2r_ones"] = dict(min=float(y.min()), max=float(y.max()))
    x = np.random.default_rng(7).random((2, 11, 13))
    kat["offset_dead"] = dict(
        r2h=bool(np.array_equal(G.rect_to_hex_resample(x, (9, 14), "bilinear", 0),
                                G.rect_to_hex_resample(x, (9, 14), "bilinear", 1))),
        h2r=bool(np.array_equal(G.hex_to_rect_resample(x, (9, 14), "linear", 0),
                                G.hex_to_rect_resample(x, (9, 14), "linear", 1))),
        hexresize=bool(np.array_equal(G.hexresize(x, (9, 14), "linear", 0),
                                      G.hexresize(x, (9, 14), "linear", 1))))
    errs = {}
    probes = {
        "r2h_linear": lambda: G.rect_to_hex_resample(x, None, "linear"),
        "r2h_2d": lambda: G.rect_to_hex_resample(x[0], None, "bilinear"),
        "r2h_4d": lambda: G.rect_to_hex_resample(x[None], None, "bilinear"),
        "h2r_nearest": lambda: G.hex_to_rect_resample(x, (9, 14), "nearest"),
        "h2r_unknown": lambda: G.hex_to_rect_resample(x, (9, 14), "cubic"),
        "hexresize_nearest": lambda: G.hexresize(x, (9, 14), "nearest"),
        "conv_bad_groups": lambda: HF.HexConv2d(3, 4, 0, 2, groups=3),
    }
    for k, f in probes.items():
        try:
            f()
            errs[k] = None
        except Exception as e:
            errs[k] = type(e).__name__
    kat["errors"] = errs
    # h2r 'bilinear' (method 2) runs no blend and returns np.empty transposed (W1,C,H1)
    y = G.hex_to_rect_resample(x, (8, 10), "bilinear")
    kat["h2r_bilinear_shape"] = list(y.shape)
    # HexConv2d surface
    m = HF.HexConv2d(3, 6, 0, 2, padding=1, groups=3)
    kat["conv_repr"] = repr(m)
    kat["conv_state_keys"] = sorted(m.state_dict().keys())
    kat["conv_kernel_shape"] = list(m.kernel.shape)
    for r in (1, 2, 3, 4):
        mm = HF.HexConv2d(1, 1, 0, r)
        kat[f"conv_kernelnum_r{r}"] = [mm.kernelnum, mm.k_h, mm.k_w]
    # type1 / type2 format conversions
    t = torch.arange(2 * 5 * 4, dtype=torch.float32).reshape(1, 2, 5, 4)
    for off in (0, 1):
        kat[f"type1_off{off}"] = HF.heximage_to_type1(t, off).numpy().tolist()
        kat[f"type2_off{off}_shape"] = list(HF.heximage_to_type2(t, off).shape)
    return kat


def main():
    rng = np.random.default_rng(20260109)
    gt = load_geometry_torch_cpu()
    meta = {"reference": REF, "numpy": np.__version__, "torch": torch.__version__}
    for name, fn in (("r2h", lambda: gen_r2h(rng)), ("h2r", lambda: gen_h2r(rng, gt)),
                     ("hexresize", lambda: gen_resize(rng)), ("hexconv", gen_conv),
                     ("hexconv_bwd", gen_conv_bwd), ("igt", lambda: gen_igt(rng)),
                     ("pool", gen_pool), ("taps", gen_taps)):
        arrs, index = fn()
        np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **arrs)
        meta[name] = index
        print(name, len(index), "cases")
    meta["kat"] = gen_kats(gt)
    with open(os.path.join(OUT, "index.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
