"""Tensor-level entry points: torch device tensors in, torch device tensors out.

Thin layer over the C ABI (`_abi`): shape/dtype policy, output allocation (the
caller — here torch's caching allocator — owns every buffer), and the current
HIP stream.  The reference-compatible surfaces (geometry_np, geometry_torch,
HexFrames, ...) are built on these.

Layout: a raster batch is any tensor (..., H, W); all leading dims are flattened
into `planes`, which the kernels walk with the lattice maps computed once.
"""
import ctypes

import torch

from . import _abi

_FLOATS = (torch.float16, torch.bfloat16, torch.float32, torch.float64)


def _planes(x):
    if x.dim() < 2:
        raise ValueError(f"expected a raster (..., H, W), got shape {tuple(x.shape)}")
    x = x.contiguous()
    lead = tuple(x.shape[:-2])
    planes = 1
    for d in lead:
        planes *= d
    return x, lead, planes


_RESAMPLE_OP = {"hg_rect_to_hex": _abi.HG_OP_RECT_TO_HEX, "hg_hex_to_rect": _abi.HG_OP_HEX_TO_RECT,
                "hg_hexresize": _abi.HG_OP_HEXRESIZE}


class _ResampleFn(torch.autograd.Function):
    """Autograd of a resample: backward = hg_resample_backward (the transpose of the
    forward's lattice weights)."""

    @staticmethod
    def forward(ctx, x, fn_name, size, interp, out_dtype):
        ctx.meta = (_RESAMPLE_OP[fn_name], tuple(x.shape), x.dtype, int(interp))
        return _resample_raw(fn_name, x, size, interp, out_dtype)

    @staticmethod
    def backward(ctx, gy):
        op, shape, xdt, interp = ctx.meta
        acc = torch.float64 if torch.float64 in (gy.dtype, xdt) else torch.float32
        g = gy.contiguous().to(acc)
        h, w = shape[-2], shape[-1]
        h1, w1 = int(g.shape[-2]), int(g.shape[-1])
        planes = 1
        for d in shape[:-2]:
            planes *= d
        dx = torch.empty(shape, dtype=acc, device=gy.device)
        st = _abi.lib().hg_resample_backward(op, _abi.ptr(g), _abi.ptr(dx), _abi.dtype_code(acc),
                                             planes, h, w, h1, w1, interp, _abi.stream_of(g))
        _abi.check(st, "hg_resample_backward")
        return dx.to(xdt), None, None, None, None


def _resample(fn_name, x, size, interp, out_dtype):
    if torch.is_grad_enabled() and x.requires_grad and x.is_floating_point():
        return _ResampleFn.apply(x, fn_name, size, interp, out_dtype)
    return _resample_raw(fn_name, x, size, interp, out_dtype)


def _resample_raw(fn_name, x, size, interp, out_dtype):
    _abi.require_device(x)
    x = x.detach()
    x, lead, planes = _planes(x)
    h, w = int(x.shape[-2]), int(x.shape[-1])
    h1, w1 = (h, w) if size is None else (int(size[0]), int(size[1]))
    if interp == _abi.HG_NEAREST:
        out_dtype = x.dtype
    elif out_dtype is None:
        out_dtype = x.dtype if x.dtype in _FLOATS else torch.float32
    y = torch.empty(lead + (h1, w1), dtype=out_dtype, device=x.device)
    st = getattr(_abi.lib(), fn_name)(
        _abi.ptr(x), _abi.ptr(y), _abi.dtype_code(x.dtype), _abi.dtype_code(out_dtype),
        planes, h, w, h1, w1, int(interp), _abi.stream_of(x))
    _abi.check(st, fn_name)
    return y


def rect_to_hex(x, size=None, interp=_abi.HG_LINEAR, out_dtype=None):
    """rect (..., H, W) -> hex (..., H1, W1); geometry_np.py:358-519."""
    return _resample("hg_rect_to_hex", x, size, interp, out_dtype)


def hex_to_rect(x, size=None, interp=_abi.HG_LINEAR, out_dtype=None):
    """hex (..., H, W) -> rect (..., H1, W1); geometry_np.py:191-356."""
    return _resample("hg_hex_to_rect", x, size, interp, out_dtype)


def hexresize(x, size, interp=_abi.HG_LINEAR, out_dtype=None):
    """hex (..., H, W) -> hex (..., H1, W1); geometry_np.py:520-681."""
    return _resample("hg_hexresize", x, size, interp, out_dtype)


_OPS = {"rect_to_hex": _abi.HG_OP_RECT_TO_HEX, "hex_to_rect": _abi.HG_OP_HEX_TO_RECT,
        "hexresize": _abi.HG_OP_HEXRESIZE}


def lattice_maps(op, h, w, h1, w1, device=None):
    """The integer lattice maps + fp64 coefficients a resample uses (parity tests)."""
    device = torch.device("cuda") if device is None else torch.device(device)
    if not torch.cuda.is_available():
        raise RuntimeError("HyGrid needs a HIP device (MI355X); none is available.")
    im = torch.empty((5, h1, w1), dtype=torch.int32, device=device)
    fm = torch.empty((5, h1, w1), dtype=torch.float64, device=device)
    st = _abi.lib().hg_lattice_maps(_OPS[op], h, w, h1, w1, _abi.ptr(im), _abi.ptr(fm),
                                    _abi.stream_of(im))
    _abi.check(st, "hg_lattice_maps")
    keys = ("i_n", "j_n", "flag", "valid", "argmin")
    out = {k: im[i] for i, k in enumerate(keys)}
    out.update({k: fm[i] for i, k in enumerate(("i_f", "j_f", "alpha", "beta", "gamma"))})
    return out


def homography_plan(h, w, H):
    """Host planning of image_geometric_transformation (geometry_np.py:56-102): the
    output axes of the transformed corners and inv(H), in NumPy exactly as the
    reference computes them (O(h1 + w1) work).  Returns (xs, ys, hinv) as float64
    ndarrays; h1 = len(xs), w1 = len(ys)."""
    import numpy as np
    H = np.asarray(H.detach().cpu() if isinstance(H, torch.Tensor) else H, dtype=np.float64)
    if H.shape != (3, 3):
        raise ValueError(f"H must be 3x3, got shape {H.shape}")
    corner = np.array([[-(h / 2 - 0.5), -((w + 0.5) / 2 - 0.5), 1.],
                       [-(h / 2 - 0.5), (w + 0.5) / 2 - 0.5, 1.],
                       [h / 2 - 0.5, -((w + 0.5) / 2 - 0.5), 1.],
                       [h / 2 - 0.5, (w + 0.5) / 2 - 0.5, 1.]]).transpose()
    c = np.matmul(H, corner)
    h1_inf, w1_inf = np.min(c[0], axis=-1), np.min(c[1], axis=-1)
    h1_sup, w1_sup = np.max(c[0], axis=-1), np.max(c[1], axis=-1)
    xs = np.arange(h1_inf, h1_sup + 1, 1).astype(np.float64)
    ys = np.arange(w1_inf, w1_sup + 0.5, 1).astype(np.float64)
    hinv = np.ascontiguousarray(np.linalg.inv(H), dtype=np.float64)
    return xs, ys, hinv


def _homography_args(x, H):
    import numpy as np
    h, w = int(x.shape[-2]), int(x.shape[-1])
    xs, ys, hinv = homography_plan(h, w, H)
    dxs = torch.from_numpy(xs).to(x.device)
    dys = torch.from_numpy(ys).to(x.device)
    return h, w, dxs, dys, hinv.ctypes.data_as(ctypes.c_void_p), hinv


def hex_homography(x, H, interp=_abi.HG_LINEAR, out_dtype=None):
    """hex (..., H, W) -> hex (..., h1, w1) under the affine map H
    (image_geometric_transformation, geometry_np.py:6-189), by hg_hex_homography.
    'linear' blends in fp64 and returns out_dtype (default: x's float dtype, float32 for
    integer input); 'nearest' copies the first-minimum vertex (geometry_torch.py:165-173)."""
    _abi.require_device(x)
    x = x.detach()
    x, lead, planes = _planes(x)
    h, w, dxs, dys, hptr, _keep = _homography_args(x, H)
    h1, w1 = int(dxs.numel()), int(dys.numel())
    if interp == _abi.HG_NEAREST:
        out_dtype = x.dtype
    elif out_dtype is None:
        out_dtype = x.dtype if x.dtype in _FLOATS else torch.float32
    y = torch.empty(lead + (h1, w1), dtype=out_dtype, device=x.device)
    st = _abi.lib().hg_hex_homography(
        _abi.ptr(x), _abi.ptr(y), _abi.dtype_code(x.dtype), _abi.dtype_code(out_dtype),
        planes, h, w, h1, w1, _abi.ptr(dxs), _abi.ptr(dys), hptr, int(interp),
        _abi.stream_of(x))
    _abi.check(st, "hg_hex_homography")
    return y


def homography_maps(h, w, H, device=None):
    """Lattice maps of one image_geometric_transformation (parity tests): the keys of
    lattice_maps plus the inverse-mapped point x_, y_ (geometry_np.py:104-105)."""
    device = torch.device("cuda") if device is None else torch.device(device)
    if not torch.cuda.is_available():
        raise RuntimeError("HyGrid needs a HIP device (MI355X); none is available.")
    probe = torch.empty((h, w), device=device)
    h, w, dxs, dys, hptr, _keep = _homography_args(probe, H)
    h1, w1 = int(dxs.numel()), int(dys.numel())
    im = torch.empty((5, h1, w1), dtype=torch.int32, device=device)
    fm = torch.empty((7, h1, w1), dtype=torch.float64, device=device)
    st = _abi.lib().hg_hex_homography_maps(h, w, h1, w1, _abi.ptr(dxs), _abi.ptr(dys), hptr,
                                           _abi.ptr(im), _abi.ptr(fm), _abi.stream_of(im))
    _abi.check(st, "hg_hex_homography_maps")
    keys = ("i_n", "j_n", "flag", "valid", "argmin")
    out = {k: im[i] for i, k in enumerate(keys)}
    out.update({k: fm[i] for i, k in enumerate(("i_f", "j_f", "alpha", "beta", "gamma",
                                                 "x_", "y_"))})
    return out


POOL_METHODS = {"max": 0, "min": 1, "average": 2}
_POOL_PAD_MODES = _abi.PAD_MODES


def pool_plan(h, w, kh, kw, sh, sw, padding=0, ceil_mode=False, count_include_pad=True):
    """HexPool2d's window geometry (HexFrames.py:286-319): the padded frame, the ceil-mode
    extension (F.pad(input, (0, ph, 0, pw)) — ph columns on the right, pw rows at the
    bottom, as the reference passes them, :295-300) and the output size.  Returns
    dict(hn, wn, ext_h, ext_w, ext_value).  Raises IndexError where the reference's
    gather would index outside the frame."""
    H0, W0 = h + 2 * padding, w + 2 * padding
    ext_h = ext_w = 0
    ext_value = 0.0
    if ceil_mode:
        hn0 = H0 // sh
        wn0 = (W0 - sw // 2 - sw) // sw + 1
        ph = (kh - H0 + hn0 * sh) % kh
        pw = (kw - W0 + (wn0 * sw + sw // 2)) % kw
        ext_w, ext_h = ph, pw
        ext_value = 0.0 if count_include_pad else float("nan")
    H, W = H0 + ext_h, W0 + ext_w
    hn = (H - kh) // sh + 1
    wn = (W - sw // 2) // sw
    if hn < 0 or wn < 0:
        raise RuntimeError(f"hex pooling: window {kh}x{kw} / stride {sh}x{sw} does not fit "
                           f"a {H}x{W} frame")
    if hn > 0 and wn > 0:
        shift = sw // 2 if hn >= 2 else 0
        if (hn - 1) * sh + kh > H or (wn - 1) * sw + shift + kw > W:
            raise IndexError(f"hex pooling: windows ({kh}x{kw}, stride {sh}x{sw}) reach "
                             f"outside the {H}x{W} frame (the reference's gather raises)")
    return dict(hn=hn, wn=wn, ext_h=ext_h, ext_w=ext_w, ext_value=ext_value)


def _pool_args(x, method, kh, kw, sh, sw, hn, wn, pad, pad_mode, pad_value, ext_h, ext_w,
               ext_value):
    h, w = int(x.shape[-2]), int(x.shape[-1])
    return (POOL_METHODS[method], h, w, int(pad), _POOL_PAD_MODES[pad_mode], float(pad_value),
            int(ext_h), int(ext_w), float(ext_value), int(kh), int(kw), int(sh), int(sw),
            int(hn), int(wn))


def _pool_raw(x, args):
    _abi.require_device(x)
    if x.dtype not in _FLOATS:
        raise TypeError(f"hex pooling needs a floating-point raster, got {x.dtype} (the "
                        f"reference's NaN masking, HexFrames.py:461-479)")
    x, lead, planes = _planes(x.detach())
    m, h, w, pad, mode, pv, eh, ew, ev, kh, kw, sh, sw, hn, wn = args
    y = torch.empty(lead + (hn, wn), dtype=x.dtype, device=x.device)
    st = _abi.lib().hg_hex_pool2d(_abi.ptr(x), _abi.ptr(y), _abi.dtype_code(x.dtype), m, planes,
                                  h, w, pad, mode, pv, eh, ew, ev, kh, kw, sh, sw, hn, wn,
                                  _abi.stream_of(x))
    _abi.check(st, "hg_hex_pool2d")
    return y


class _HexPoolFn(torch.autograd.Function):
    """Autograd of hex pooling: hg_hex_pool2d_backward (gy to the selected element of a
    max / min window, gy / count to the non-NaN elements of an average window, folded
    back through the padding) — the reference's autograd of HexFrames.py:286-343."""

    @staticmethod
    def forward(ctx, x, args):
        ctx.save_for_backward(x)
        ctx.args = args
        return _pool_raw(x, args)

    @staticmethod
    def backward(ctx, gy):
        (x,) = ctx.saved_tensors
        m, h, w, pad, mode, pv, eh, ew, ev, kh, kw, sh, sw, hn, wn = ctx.args
        acc = torch.float64 if x.dtype == torch.float64 else torch.float32
        xc, lead, planes = _planes(x.detach())
        g = gy.contiguous().to(acc)
        dx = torch.empty(tuple(x.shape), dtype=acc, device=x.device)
        st = _abi.lib().hg_hex_pool2d_backward(
            _abi.ptr(xc), _abi.ptr(g), _abi.ptr(dx), _abi.dtype_code(x.dtype),
            _abi.dtype_code(acc), m, planes, h, w, pad, mode, pv, eh, ew, ev, kh, kw, sh, sw,
            hn, wn, _abi.stream_of(xc))
        _abi.check(st, "hg_hex_pool2d_backward")
        return dx.to(x.dtype), None


def hex_pool2d(x, method, kh, kw, sh, sw, hn, wn, pad=0, pad_mode="constant", pad_value=0.0,
               ext_h=0, ext_w=0, ext_value=0.0):
    """Hex pooling of (..., h, w) -> (..., hn, wn) by hg_hex_pool2d (geometry: pool_plan).
    Differentiable in x."""
    if pad_mode not in _POOL_PAD_MODES:
        raise NotImplementedError(f"padding mode {pad_mode!r}")
    if _POOL_PAD_MODES[pad_mode] != 0 and pad_value not in (0, None):
        raise RuntimeError(f'Padding mode "{pad_mode}" doesn\'t take in value argument')
    args = _pool_args(x, method, kh, kw, sh, sw, hn, wn, pad, pad_mode,
                      0.0 if pad_value is None else pad_value, ext_h, ext_w, ext_value)
    if torch.is_grad_enabled() and x.requires_grad:
        return _HexPoolFn.apply(x, args)
    return _pool_raw(x, args)


def reduce_last(x, method):
    """The reference's max_pooling / min_pooling / average_pooling (HexFrames.py:461-479):
    NaN-aware reduction over the last dim, as a 1 x n window of hg_hex_pool2d."""
    n = int(x.shape[-1])
    y = hex_pool2d(x.unsqueeze(-2), method, 1, n, 1, max(n, 1), 1, 1)
    return y[..., 0, 0]


def hexconv2d_out_shape(h, w, radius, stride=1, padding=0, dilation=1):
    ho, wo = ctypes.c_int64(), ctypes.c_int64()
    st = _abi.lib().hg_hexconv2d_out_shape(h, w, radius, stride, padding, dilation,
                                          ctypes.byref(ho), ctypes.byref(wo))
    _abi.check(st, "hexconv2d_out_shape")
    return ho.value, wo.value


def hexconv2d(x, kernel, bias, even_odd_offset, radius, stride=1, padding=0, dilation=1,
              groups=1, padding_mode="constant", padding_value=0.0, out_dtype=None,
              epilogue=None):
    """HexConv2d forward (HexFrames.py:96-169) on (B, C, H, W) -> (B, O, Ho, Wo).

    kernel: (O, C/groups, 1, K) or (O, C/groups, K) float32/float64 — the
    accumulation dtype, as the reference's `input.to(self.kernel.dtype)` (:107).
    epilogue: None or (scale, shift, act, slope) — per-channel affine (tensors (O,) or
    None) and hg_act activation fused into the store (hg_hexconv2d_epilogue).
    """
    _abi.require_device(x)
    while x.dim() < 4:
        x = x.unsqueeze(0)
    x = x.contiguous()
    B, C, h, w = (int(s) for s in x.shape)
    k = kernel.detach()
    if k.dtype not in (torch.float32, torch.float64):
        k = k.float()
    k = k.reshape(k.shape[0], k.shape[1], -1).contiguous()
    O = int(k.shape[0])
    if int(k.shape[1]) * groups != C:
        raise ValueError(f"kernel expects {int(k.shape[1]) * groups} input channels, got {C}")
    b = None
    if bias is not None:
        b = bias.detach().to(k.dtype).contiguous()
    if out_dtype is None:
        out_dtype = torch.get_default_dtype()
    ho, wo = hexconv2d_out_shape(h, w, radius, stride, padding, dilation)
    y = torch.empty((B, O, ho, wo), dtype=out_dtype, device=x.device)
    pm = _abi.PAD_MODES.get(padding_mode)
    if pm is None:
        raise ValueError(f"unsupported padding_mode {padding_mode!r}")
    if epilogue is None:
        st = _abi.lib().hg_hexconv2d(
            _abi.ptr(x), _abi.ptr(k), _abi.ptr(b), _abi.ptr(y), _abi.dtype_code(x.dtype),
            _abi.dtype_code(k.dtype), _abi.dtype_code(out_dtype), B, C, O, h, w, radius, stride,
            padding, dilation, groups, int(even_odd_offset), pm, float(padding_value),
            _abi.stream_of(x))
        _abi.check(st, "hg_hexconv2d")
        return y
    scale, shift, act, slope = epilogue
    sc = None if scale is None else scale.detach().to(k.dtype).contiguous()
    sf = None if shift is None else shift.detach().to(k.dtype).contiguous()
    for t in (sc, sf):
        if t is not None and t.numel() != O:
            raise ValueError(f"epilogue scale/shift must have {O} elements")
    st = _abi.lib().hg_hexconv2d_epilogue(
        _abi.ptr(x), _abi.ptr(k), _abi.ptr(b), _abi.ptr(y), _abi.dtype_code(x.dtype),
        _abi.dtype_code(k.dtype), _abi.dtype_code(out_dtype), B, C, O, h, w, radius, stride,
        padding, dilation, groups, int(even_odd_offset), pm, float(padding_value),
        _abi.ptr(sc), _abi.ptr(sf), int(act), float(slope), _abi.stream_of(x))
    _abi.check(st, "hg_hexconv2d_epilogue")
    return y


def hexconv2d_backward(gy, x, kernel, bias, cfg, need_x=True, need_k=True, need_b=True):
    """Gradients of hexconv2d (hg_hexconv2d_backward): (d x, d kernel, d bias).

    gy: (B, O, ho, wo); x: the forward input (B, C, H, W); kernel: the parameter
    (O, C/groups, 1, K) (its dtype, float32 or float64, is the accumulation dtype, as
    the forward's `input.to(self.kernel.dtype)`, HexFrames.py:107).  Returns None for
    the gradients not requested; d x has x's dtype, d kernel / d bias the parameters'.
    """
    _abi.require_device(gy)
    while x.dim() < 4:
        x = x.unsqueeze(0)
    x = x.contiguous()
    B, C, h, w = (int(s) for s in x.shape)
    k = kernel.detach()
    if k.dtype not in (torch.float32, torch.float64):
        k = k.float()
    kshape = tuple(kernel.shape)
    k = k.reshape(k.shape[0], k.shape[1], -1).contiguous()
    O, K = int(k.shape[0]), int(k.shape[2])
    g = gy.detach().to(k.dtype).contiguous()
    dx = torch.empty_like(x) if need_x else None
    dk = torch.empty((O, int(k.shape[1]), K), dtype=k.dtype, device=x.device) if need_k else None
    db = (torch.empty((O,), dtype=k.dtype, device=x.device)
          if (need_b and bias is not None) else None)
    pm = _abi.PAD_MODES.get(cfg["padding_mode"])
    if pm is None:
        raise ValueError(f"unsupported padding_mode {cfg['padding_mode']!r}")
    st = _abi.lib().hg_hexconv2d_backward(
        _abi.ptr(x), _abi.ptr(k), _abi.ptr(g), _abi.ptr(dx), _abi.ptr(dk), _abi.ptr(db),
        _abi.dtype_code(x.dtype), _abi.dtype_code(k.dtype), B, C, O, h, w, cfg["r"],
        cfg["stride"], cfg["pad"], cfg["dilation"], cfg["groups"], int(cfg["off"]), pm,
        float(cfg["padding_value"]), _abi.stream_of(x))
    _abi.check(st, "hg_hexconv2d_backward")
    gk = dk.reshape(kshape).to(kernel.dtype) if dk is not None else None
    gb = db.to(bias.dtype) if db is not None else None
    return dx, gk, gb


def hex_to_type1(x, even_odd_offset, row_repeat=1, out_dtype=None):
    """Offset-row hex raster (..., H, W) -> type1 (..., H*row_repeat, 2W+1) on the GPU
    (hg_hex_to_type1): row_repeat 1 = HexFrames.heximage_to_type1 (HexFrames.py:417-445),
    2 = heximage_to_type2 (:446-449).  out_dtype converts first (the reference's torch
    version returns the default float dtype)."""
    _abi.require_device(x)
    if out_dtype is not None and x.dtype != out_dtype:
        x = x.to(out_dtype)
    x, lead, planes = _planes(x)
    h, w = int(x.shape[-2]), int(x.shape[-1])
    y = torch.empty(lead + (h * row_repeat, 2 * w + 1), dtype=x.dtype, device=x.device)
    st = _abi.lib().hg_hex_to_type1(_abi.ptr(x), _abi.ptr(y), x.element_size(), planes, h, w,
                                    int(even_odd_offset) & 1, int(row_repeat), _abi.stream_of(x))
    _abi.check(st, "hg_hex_to_type1")
    return y


def strided_copy2d(x, row_start, row_step, col_start, col_step, h_out=None, w_out=None):
    """Contiguous x[..., row_start::row_step, col_start::col_step] (bounded by h_out /
    w_out) by one gfx950 gather (hg_strided_copy2d): type1 / type2 decoding
    (HexImage.py:108-111, HexFrames.py:450-458) into a kernel-ready raster."""
    _abi.require_device(x)
    x, lead, planes = _planes(x)
    H, W = int(x.shape[-2]), int(x.shape[-1])
    if h_out is None:
        h_out = len(range(row_start, H, row_step))
    if w_out is None:
        w_out = len(range(col_start, W, col_step))
    y = torch.empty(lead + (h_out, w_out), dtype=x.dtype, device=x.device)
    st = _abi.lib().hg_strided_copy2d(_abi.ptr(x), _abi.ptr(y), x.element_size(), planes, H, W,
                                      row_start, row_step, col_start, col_step, h_out, w_out,
                                      _abi.stream_of(x))
    _abi.check(st, "hg_strided_copy2d")
    return y


HG_EUNSUP = _abi.HG_EUNSUP


def pipeline_r2h_h2r(x, hex_size=None, out_dtype=None):
    """Fused rect -> hex (bilinear) -> rect (linear) round trip, no conv: the same result as
    hex_to_rect(rect_to_hex(x, hex_size), hex_size) (geometry_np.py:358-519, :191-356) with
    the hex image kept in fp32 on chip.  x: (..., h, w) device tensor -> (..., h1, w1).

    Returns None when the fused kernel does not cover the geometry / dtypes (the caller then
    runs the two resamplers); raises on argument errors.
    """
    _abi.require_device(x)
    x = x.contiguous()
    h, w = int(x.shape[-2]), int(x.shape[-1])
    planes = x.numel() // max(h * w, 1)
    h1, w1 = (h, w) if hex_size is None else (int(hex_size[0]), int(hex_size[1]))
    if out_dtype is None:
        out_dtype = x.dtype if x.dtype in (torch.bfloat16, torch.float16) else torch.float32
    y = torch.empty(tuple(x.shape[:-2]) + (h1, w1), dtype=out_dtype, device=x.device)
    st = _abi.lib().hg_pipeline_r2h_h2r(_abi.ptr(x), _abi.ptr(y), _abi.dtype_code(x.dtype),
                                        _abi.dtype_code(out_dtype), planes, h, w, h1, w1,
                                        _abi.stream_of(x))
    if st in (HG_EUNSUP, _abi.HG_EDTYPE):
        return None
    _abi.check(st, "hg_pipeline_r2h_h2r")
    return y


def pipeline_r2h_conv_h2r(x, kernel, bias, hex_size=None, rect_size=None, padding=1, groups=1,
                          even_odd_offset=0, padding_value=0.0, out_dtype=None):
    """Fused rect -> hex (bilinear) -> HexConv2d (radius 2) -> hex -> rect (linear).

    Returns None when the fused kernel does not cover the geometry / dtypes (the
    caller then runs the three operators); raises on argument errors.
    """
    _abi.require_device(x)
    while x.dim() < 4:
        x = x.unsqueeze(0)
    x = x.contiguous()
    B, C, h, w = (int(s) for s in x.shape)
    h1, w1 = (h, w) if hex_size is None else (int(hex_size[0]), int(hex_size[1]))
    ho, wo = hexconv2d_out_shape(h1, w1, 2, 1, padding, 1)
    h2, w2 = (ho, wo) if rect_size is None else (int(rect_size[0]), int(rect_size[1]))
    k = kernel.detach().float().reshape(kernel.shape[0], -1).contiguous()
    O = int(k.shape[0])
    b = bias.detach().float().contiguous() if bias is not None else None
    if out_dtype is None:
        out_dtype = x.dtype if x.dtype in (torch.bfloat16, torch.float16) else torch.float32
    y = torch.empty((B, O, h2, w2), dtype=out_dtype, device=x.device)
    st = _abi.lib().hg_pipeline_r2h_conv_h2r(
        _abi.ptr(x), _abi.ptr(k), _abi.ptr(b), _abi.ptr(y), _abi.dtype_code(x.dtype),
        _abi.dtype_code(out_dtype), B, C, O, h, w, h1, w1, h2, w2, int(padding), int(groups),
        int(even_odd_offset), float(padding_value), _abi.stream_of(x))
    if st in (HG_EUNSUP, _abi.HG_EDTYPE):
        return None
    _abi.check(st, "hg_pipeline_r2h_conv_h2r")
    return y


# one int32 workspace per (device, stream) for hg_hex_pyramid_chain (each call zeroes it on the
# stream first; calls on one stream are ordered, so they can share it)
_CHAIN_WS = {}


def chain_workspace(device, stream, nbytes):
    """The (device, stream)'s pyramid-chain workspace, at least nbytes (int [1] after a call:
    the chain's fault word, 0 unless a workgroup waited > ~1 s for its input)."""
    key = (device.index, int(stream.value or 0))
    ws = _CHAIN_WS.get(key)
    if ws is None or ws.numel() * 4 < nbytes:
        ws = torch.zeros(max(nbytes // 4 + 4, 1024), dtype=torch.int32, device=device)
        _CHAIN_WS[key] = ws
    return ws


def hex_pyramid_chain(x, taps, bias=None, levels=3, even_odd_offset=0):
    """`levels` pyramid levels from the rect image x in ONE launch (hg_hex_pyramid_chain):
    level 0 = hex_pyramid_level(x, from_rect=True), level l = hex_pyramid_level(level l - 1),
    each (h // 2, w // 2) of the one before, all in x's dtype (16-bit), bit-identical to those
    calls.  Returns the list of levels, or None outside the chain's domain (levels 2-3, C = 3,
    every level on the fused kernel: the caller then runs the levels one launch each)."""
    _abi.require_device(x)
    while x.dim() < 4:
        x = x.unsqueeze(0)
    x = x.contiguous()
    B, C, h, w = (int(s) for s in x.shape)
    if x.dtype not in (torch.float16, torch.bfloat16) or not 2 <= levels <= 3:
        return None
    k = taps.detach().float().reshape(C, 7).contiguous()
    b = bias.detach().float().contiguous() if bias is not None else None
    outs, hl, wl = [], h, w
    for _ in range(levels):
        hl, wl = hl // 2, wl // 2
        outs.append(torch.empty((B, C, hl, wl), dtype=x.dtype, device=x.device))
    L = _abi.lib()
    need = int(L.hg_hex_pyramid_chain_workspace(int(levels), B, h))
    if need < 0:
        _abi.check(need, "hg_hex_pyramid_chain_workspace")
    st_ = _abi.stream_of(x)
    ws = chain_workspace(x.device, st_, need)
    ys = (ctypes.c_void_p * levels)(*[o.data_ptr() for o in outs])
    st = L.hg_hex_pyramid_chain(_abi.ptr(x), ys, int(levels), _abi.dtype_code(x.dtype), B, C, h,
                                w, _abi.ptr(k), _abi.ptr(b), int(even_odd_offset), _abi.ptr(ws),
                                ws.numel() * 4, st_)
    if st in (HG_EUNSUP, _abi.HG_EDTYPE):
        return None
    _abi.check(st, "hg_hex_pyramid_chain")
    return outs


def hex_pyramid_level(x, taps, bias=None, size=None, even_odd_offset=0, from_rect=False,
                      out_dtype=None, out=None):
    """One hex Gaussian pyramid level in one pass: hexresize(HexConv2d_depthwise(x))
    (geometry_np.py:520-681 after HexFrames.py:96-169, radius 2, padding 1, pad value 0),
    with rect_to_hex(x) (geometry_np.py:358-519) first when from_rect.

    x: (B, C, h, w) device tensor; taps: the depthwise kernel (C, 1, 1, 7) or (C, 7);
    size: (h1, w1), default (h // 2, w // 2).  out: an optional contiguous (B, C, h1, w1)
    tensor of out_dtype to write into (e.g. a slice of a larger batch).  Returns None when the
    fused kernel does not cover the geometry / dtypes (the caller then runs the operators).
    """
    _abi.require_device(x)
    while x.dim() < 4:
        x = x.unsqueeze(0)
    x = x.contiguous()
    B, C, h, w = (int(s) for s in x.shape)
    h1, w1 = (h // 2, w // 2) if size is None else (int(size[0]), int(size[1]))
    k = taps.detach().float().reshape(C, 7).contiguous()
    b = bias.detach().float().contiguous() if bias is not None else None
    if out_dtype is None:
        out_dtype = x.dtype if x.dtype in (torch.bfloat16, torch.float16) else torch.float32
    if out is None:
        y = torch.empty((B, C, h1, w1), dtype=out_dtype, device=x.device)
    else:
        if (tuple(out.shape) != (B, C, h1, w1) or out.dtype != out_dtype
                or out.device != x.device or not out.is_contiguous()):
            raise ValueError(f"hex_pyramid_level: out must be a contiguous {(B, C, h1, w1)} "
                             f"{out_dtype} tensor on {x.device}")
        y = out
    st = _abi.lib().hg_hex_pyramid_level(
        _abi.ptr(x), _abi.ptr(y), _abi.dtype_code(x.dtype), _abi.dtype_code(out_dtype), B, C,
        h, w, h1, w1, _abi.ptr(k), _abi.ptr(b), int(even_odd_offset), int(bool(from_rect)),
        _abi.stream_of(x))
    if st in (HG_EUNSUP, _abi.HG_EDTYPE):
        return None
    _abi.check(st, "hg_hex_pyramid_level")
    return y
