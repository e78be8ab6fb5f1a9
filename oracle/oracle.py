"""ctypes front-end of the CPU restatement in hg_oracle.c.

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product package.  Parity of every
function here is pinned by tests/test_oracle_golden.py against golden vectors
captured from the reference (tests/golden/make_golden.py).

Each function mirrors one reference entry point (paths under /root/reference):
  rect_to_hex   HyGrid/geometry_np.py:358-519
  hex_to_rect   HyGrid/geometry_np.py:191-356 (linear); nearest per
                HyGrid/geometry_torch.py:335-347
  hexresize     HyGrid/geometry_np.py:520-681
  hexconv2d     HyGrid/HexFrames.py:96-169
  hexconv2d_backward  the adjoint of hexconv2d (reference: torch autograd of :96-169)
  rect_to_hex_backward / hex_to_rect_backward / hexresize_backward  the adjoints of the
                three resamplers (reference: torch autograd through the indexing of
                HyGrid/geometry_torch.py:322-325; weights geometry_np.py:514-517, :347-354)
  image_geometric_transformation  HyGrid/geometry_np.py:6-189 (NumPy restatement;
                nearest per HyGrid/geometry_torch.py:165-173)
  hex_pool2d    HyGrid/HexFrames.py:286-343 windows, :461-479 reductions, and their
                autograd (hex_pool2d_backward)
Inputs are (planes, h, w) arrays of any real dtype; outputs are float64.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libhg_oracle.so")
_lib = None

_i64 = ctypes.c_int64
_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int32)

PAD_MODES = {"constant": 0, "zeros": 0, "reflect": 1, "replicate": 2, "circular": 3}


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.or_linspace.restype = ctypes.c_double
        L.or_linspace.argtypes = [ctypes.c_double, ctypes.c_double, _i64, _i64]
        for name in ("or_r2h_maps", "or_h2r_maps", "or_hexresize_maps"):
            getattr(L, name).argtypes = [_i64] * 4 + [_ip, _dp]
            getattr(L, name).restype = None
        for name in ("or_rect_to_hex", "or_hex_to_rect", "or_hexresize",
                     "or_rect_to_hex_backward", "or_hex_to_rect_backward",
                     "or_hexresize_backward"):
            getattr(L, name).argtypes = [_dp, _dp] + [_i64] * 5 + [ctypes.c_int]
            getattr(L, name).restype = None
        L.or_hexconv2d_out_shape.argtypes = [_i64, _i64] + [ctypes.c_int] * 4 + [
            ctypes.POINTER(_i64), ctypes.POINTER(_i64)]
        L.or_hexconv2d.argtypes = [_dp, _dp, _dp, _dp] + [_i64] * 5 + [ctypes.c_int] * 7 + [
            ctypes.c_double]
        L.or_hexconv2d_backward.argtypes = [_dp] * 6 + [_i64] * 5 + [ctypes.c_int] * 7 + [
            ctypes.c_double]
        L.or_heximage_to_type1.argtypes = [_dp, _dp, _i64, _i64, _i64, ctypes.c_int]
        L.or_heximage_to_type1.restype = None
        L.or_num_threads.restype = ctypes.c_int
        L.or_set_num_threads.argtypes = [ctypes.c_int]
        L.or_set_num_threads.restype = None
        _lib = L
    return _lib


def set_num_threads(n):
    lib().or_set_num_threads(int(n))


def num_threads():
    return lib().or_num_threads()


def _dptr(a):
    return a.ctypes.data_as(_dp)


def _as_planes(x):
    x = np.ascontiguousarray(np.asarray(x), dtype=np.float64)
    if x.ndim == 2:
        x = x[None]
    return x.reshape(-1, x.shape[-2], x.shape[-1]), x.shape[:-2]


def linspace(start, stop, n):
    return np.array([lib().or_linspace(start, stop, n, k) for k in range(n)])


def _maps(fn, nf, h, w, h1, w1):
    im = np.zeros((5, h1, w1), np.int32)
    fm = np.zeros((nf, h1, w1), np.float64)
    fn(h, w, h1, w1, im.ctypes.data_as(_ip), _dptr(fm))
    keys = ("i_n", "j_n", "flag", "valid", "argmin")
    out = {k: im[i] for i, k in enumerate(keys)}
    fkeys = ("i_f", "j_f", "alpha", "beta", "gamma")[:nf]
    out.update({k: fm[i] for i, k in enumerate(fkeys)})
    return out


def r2h_maps(h, w, h1, w1):
    return _maps(lib().or_r2h_maps, 2, h, w, h1, w1)


def h2r_maps(h, w, h1, w1):
    return _maps(lib().or_h2r_maps, 5, h, w, h1, w1)


def hexresize_maps(h, w, h1, w1):
    return _maps(lib().or_hexresize_maps, 5, h, w, h1, w1)


def _resample(fn, x, size, interp):
    planes, lead = _as_planes(x)
    n, h, w = planes.shape
    h1, w1 = (h, w) if size is None else size
    out = np.empty((n, h1, w1), np.float64)
    fn(_dptr(planes), _dptr(out), n, h, w, h1, w1, int(interp))
    return out.reshape(tuple(lead) + (h1, w1))


def rect_to_hex(x, size=None, interp=1):
    return _resample(lib().or_rect_to_hex, x, size, interp)


def hex_to_rect(x, size=None, interp=1):
    return _resample(lib().or_hex_to_rect, x, size, interp)


def hexresize(x, size, interp=1):
    return _resample(lib().or_hexresize, x, size, interp)


def _resample_backward(fn, gy, size, interp):
    """gx (planes, h, w) = R^T gy for a resample from (h, w) to gy's (h1, w1)."""
    planes, lead = _as_planes(gy)
    n, h1, w1 = planes.shape
    h, w = size
    out = np.empty((n, h, w), np.float64)
    fn(_dptr(planes), _dptr(out), n, h, w, h1, w1, int(interp))
    return out.reshape(tuple(lead) + (h, w))


def rect_to_hex_backward(gy, src_size, interp=1):
    return _resample_backward(lib().or_rect_to_hex_backward, gy, src_size, interp)


def hex_to_rect_backward(gy, src_size, interp=1):
    return _resample_backward(lib().or_hex_to_rect_backward, gy, src_size, interp)


def hexresize_backward(gy, src_size, interp=1):
    return _resample_backward(lib().or_hexresize_backward, gy, src_size, interp)


def hexconv2d_out_shape(h, w, r, stride=1, padding=0, dilation=1):
    ho, wo = _i64(), _i64()
    st = lib().or_hexconv2d_out_shape(h, w, r, stride, padding, dilation, ctypes.byref(ho),
                                      ctypes.byref(wo))
    if st:
        raise ValueError(f"hexconv2d: input too small or bad params (status {st})")
    return ho.value, wo.value


def hexconv2d(x, kernel, bias, even_odd_offset, radius, stride=1, padding=0, dilation=1,
              groups=1, padding_mode="constant", padding_value=0.0):
    x = np.ascontiguousarray(x, np.float64)
    while x.ndim < 4:
        x = x[None]
    B, C, h, w = x.shape
    k = np.ascontiguousarray(kernel, np.float64)
    O = k.shape[0]
    ho, wo = hexconv2d_out_shape(h, w, radius, stride, padding, dilation)
    y = np.empty((B, O, ho, wo), np.float64)
    bp = None
    if bias is not None:
        bias = np.ascontiguousarray(bias, np.float64)
        bp = _dptr(bias)
    st = lib().or_hexconv2d(_dptr(x), _dptr(k), bp, _dptr(y), B, C, O, h, w, radius, stride,
                            padding, dilation, groups, int(even_odd_offset),
                            PAD_MODES[padding_mode], float(padding_value))
    if st:
        raise ValueError(f"hexconv2d oracle status {st}")
    return y


def hexconv2d_backward(x, kernel, gy, even_odd_offset, radius, stride=1, padding=0,
                       dilation=1, groups=1, padding_mode="constant", padding_value=0.0):
    """(dx, dkernel, dbias) of hexconv2d for upstream gradient gy (all float64)."""
    x = np.ascontiguousarray(x, np.float64)
    while x.ndim < 4:
        x = x[None]
    B, C, h, w = x.shape
    k = np.ascontiguousarray(kernel, np.float64)
    O = k.shape[0]
    gy = np.ascontiguousarray(gy, np.float64)
    dx = np.empty_like(x)
    dk = np.empty_like(k)
    db = np.empty((O,), np.float64)
    st = lib().or_hexconv2d_backward(_dptr(x), _dptr(k), _dptr(gy), _dptr(dx), _dptr(dk),
                                     _dptr(db), B, C, O, h, w, radius, stride, padding,
                                     dilation, groups, int(even_odd_offset),
                                     PAD_MODES[padding_mode], float(padding_value))
    if st:
        raise ValueError(f"hexconv2d_backward oracle status {st}")
    return dx, dk, db


def heximage_to_type1(x, even_odd_offset):
    planes, lead = _as_planes(x)
    n, h, w = planes.shape
    t = np.empty((n, h, 2 * w + 1), np.float64)
    lib().or_heximage_to_type1(_dptr(planes), _dptr(t), n, h, w, int(even_odd_offset))
    return t.reshape(tuple(lead) + (h, 2 * w + 1))


def image_geometric_transformation(x, H, interp=1):
    """NumPy restatement of geometry_np.image_geometric_transformation (:6-189) on
    (planes, h, w) input; returns (y (planes, h1, w1), maps dict).  Output lattice: the
    arange axes of the transformed corners (:56-87, odd rows +0.5); each sample is mapped
    by inv(H) (:97-102) and blended from its triangle of input hexagons (:107-187).
    interp 1 = 'linear' (fp64), 0 = nearest (first minimum, geometry_torch.py:165-173)."""
    planes, lead = _as_planes(x)
    n, h, w = planes.shape
    H = np.asarray(H, np.float64)
    hx, wy = h / 2 - 0.5, (w + 0.5) / 2 - 0.5
    corners = np.array([[-hx, -wy, 1.], [-hx, wy, 1.], [hx, -wy, 1.], [hx, wy, 1.]]).T
    c = np.matmul(H, corners)
    xs = np.arange(c[0].min(), c[0].max() + 1, 1)
    ys = np.arange(c[1].min(), c[1].max() + 0.5, 1)
    X = np.repeat(xs[:, None], ys.size, axis=1)
    Y = np.repeat(ys[None, :], xs.size, axis=0)
    Y[1::2] += 0.5
    Hi = np.linalg.inv(H)
    xm = (Hi[0, 0] * X + Hi[0, 1] * Y) + Hi[0, 2]
    ym = (Hi[1, 0] * X + Hi[1, 1] * Y) + Hi[1, 2]
    fi = xm + (h - 1) * 0.5
    fj = 0.5 * fi + ym + (w - 0.5) * 0.5
    i_n, j_n = fi.astype(np.int64), fj.astype(np.int64)
    flag = (fi - i_n) > (fj - j_n)
    half1 = ((i_n + 1) / 2).astype(np.int64)
    half2 = ((i_n + 2) / 2).astype(np.int64)
    # vertices: p1 = (i, j - half1); p2 = flag ? (i+1, j - half2) : (i, j+1 - half1);
    # p3 = (i+1, j+1 - half2)
    rows = [i_n, np.where(flag, i_n + 1, i_n), i_n + 1]
    cols = [j_n - half1, np.where(flag, j_n - half2, j_n + 1 - half1), j_n + 1 - half2]
    ok = [(r >= 0) & (r < h) & (q >= 0) & (q < w) for r, q in zip(rows, cols)]
    f = flag.astype(np.float64)
    cx = (h - 1) / 2
    cy = (w - 0.5) / 2
    px = [i_n - cx, (i_n + f) - cx, (i_n + 1) - cx]
    py = [j_n - i_n / 2 - cy, (j_n + 1 - f) - (i_n + f) / 2 - cy, (j_n + 1) - (i_n + 1) / 2 - cy]
    dx = [xm - p for p in px]
    dy = [ym - p for p in py]

    def area(a, b):
        return 0.5 * np.abs(dx[a] * dy[b] - dy[a] * dx[b])
    S1, S2, S3 = area(1, 2), area(0, 2), area(0, 1)
    S = S1 + S2 + S3
    wts = [S1 / S, S2 / S, S3 / S]
    d = np.stack([dx[k] * dx[k] + dy[k] * dy[k] for k in range(3)])
    amin = np.argmin(d, axis=0)
    vals = []
    for k in range(3):
        v = np.zeros((n,) + xm.shape, planes.dtype)
        r, q = np.where(ok[k], rows[k], 0), np.where(ok[k], cols[k], 0)
        v[:] = np.where(ok[k], planes[:, r, q], 0)
        vals.append(v)
    if interp == 1:
        y = (wts[0] * vals[0] + wts[1] * vals[1]) + wts[2] * vals[2]
    else:
        y = np.choose(amin, vals) if n else np.zeros((0,) + xm.shape, planes.dtype)
    cand = [(i_n, j_n - half1), (i_n + 1, j_n - half2), (i_n, j_n + 1 - half1),
            (i_n + 1, j_n + 1 - half2)]
    valid4 = sum((((r >= 0) & (r < h) & (q >= 0) & (q < w)).astype(np.int32) << k)
                 for k, (r, q) in enumerate(cand))
    maps = dict(i_n=i_n, j_n=j_n, flag=flag.astype(np.int32), argmin=amin, valid=valid4,
                alpha=wts[0], beta=wts[1], gamma=wts[2], x_=xm, y_=ym)
    return y.reshape(tuple(lead) + xm.shape), maps


_PAD_NP = {"constant": "constant", "zeros": "constant", "reflect": "reflect",
           "replicate": "edge", "circular": "wrap"}


def _pool_frame(x, pad, mode, value, ext_h, ext_w, ext_value):
    """The reference's padded (+ ceil-mode extended) input (:289, :300), with the index
    of each frame element in x (-1 outside x) for the backward fold."""
    n, h, w = x.shape
    idx = np.arange(h * w, dtype=np.int64).reshape(h, w)
    if pad:
        m = _PAD_NP[mode]
        if m == "constant":
            f = np.pad(x, ((0, 0), (pad, pad), (pad, pad)), constant_values=value)
            idx = np.pad(idx, pad, constant_values=-1)
        else:
            f = np.pad(x, ((0, 0), (pad, pad), (pad, pad)), mode=m)
            idx = np.pad(idx, pad, mode=m)
    else:
        f = x
    if ext_h or ext_w:
        f = np.pad(f, ((0, 0), (0, ext_h), (0, ext_w)), constant_values=ext_value)
        idx = np.pad(idx, ((0, ext_h), (0, ext_w)), constant_values=-1)
    return f, idx


def _pool_windows(hn, wn, kh, kw, sh, sw):
    """Frame (row, col) of every window element, (hn, wn, kh*kw) each (:307-325)."""
    i = np.arange(hn)[:, None, None]
    j = np.arange(wn)[None, :, None]
    k = np.arange(kh * kw)[None, None, :]
    rows = i * sh + k // kw
    cols = (i % 2) * sw // 2 + j * sw + k % kw
    return np.broadcast_to(rows, (hn, wn, kh * kw)), np.broadcast_to(cols, (hn, wn, kh * kw))


def hex_pool2d(x, method, kh, kw, sh, sw, hn, wn, pad=0, mode="constant", value=0.0,
               ext_h=0, ext_w=0, ext_value=0.0):
    """NumPy restatement of hex pooling on (..., h, w) float64 input -> (..., hn, wn):
    window gather (:307-325) then max_pooling / min_pooling / average_pooling
    (:461-479: NaN -> -inf / +inf, first extreme; mean of the non-NaN values)."""
    planes, lead = _as_planes(x)
    f, _ = _pool_frame(planes, pad, mode, value, ext_h, ext_w, ext_value)
    r, c = _pool_windows(hn, wn, kh, kw, sh, sw)
    g = f[:, r, c]                                         # (n, hn, wn, K)
    nan = np.isnan(g)
    if method == "max":
        y = np.where(nan, -np.inf, g).max(axis=-1) if g.shape[-1] else None
    elif method == "min":
        y = np.where(nan, np.inf, g).min(axis=-1) if g.shape[-1] else None
    else:
        cnt = (~nan).sum(axis=-1)
        ssum = np.where(nan, 0.0, g).sum(axis=-1)
        with np.errstate(invalid="ignore", divide="ignore"):
            y = ssum / cnt
        y[cnt == 0] = np.nan
    return y.reshape(tuple(lead) + (hn, wn))


def hex_pool2d_backward(x, gy, method, kh, kw, sh, sw, hn, wn, pad=0, mode="constant",
                        value=0.0, ext_h=0, ext_w=0, ext_value=0.0):
    """d x of hex_pool2d (the reference's autograd): max / min give gy to the first
    extreme unless it is NaN or padding; average gives gy / count to each non-NaN
    element; padded positions fold back onto x (reflect / replicate / circular)."""
    planes, lead = _as_planes(x)
    gyp = np.asarray(gy, np.float64).reshape(-1, hn, wn)
    n = planes.shape[0]
    f, idx = _pool_frame(planes, pad, mode, value, ext_h, ext_w, ext_value)
    r, c = _pool_windows(hn, wn, kh, kw, sh, sw)
    g = f[:, r, c]
    src = idx[r, c]                                        # (hn, wn, K)
    nan = np.isnan(g)
    dx = np.zeros(planes.shape[0:1] + (planes.shape[1] * planes.shape[2],))
    if method in ("max", "min"):
        u = np.where(nan, -np.inf if method == "max" else np.inf, g)
        sel = u.argmax(axis=-1) if method == "max" else u.argmin(axis=-1)
        s = np.take_along_axis(src[None].repeat(n, 0), sel[..., None], -1)[..., 0]
        ok = (s >= 0) & ~np.take_along_axis(nan, sel[..., None], -1)[..., 0]
        for p in range(n):
            np.add.at(dx[p], s[p][ok[p]], gyp[p][ok[p]])
    else:
        cnt = (~nan).sum(axis=-1)
        with np.errstate(invalid="ignore", divide="ignore"):
            gs = gyp / cnt
        contrib = np.where(nan | (src[None] < 0), 0.0, gs[..., None])
        for p in range(n):
            m = (src >= 0) & ~nan[p]
            np.add.at(dx[p], src[m], contrib[p][m])
    return dx.reshape(np.shape(x))
