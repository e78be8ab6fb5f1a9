"""ctypes binding of libhygrid_hip.so (C ABI: include/hygrid.h).

This is the only module that touches the native library.  Everything above it
(geometry_np, geometry_torch, HexFrames, ...) goes through `ops`, which calls
these entry points on torch device buffers and torch's current HIP stream.

There is no CPU fallback: if the library or a HIP device is missing, the call
raises.  (The CPU restatement under oracle/ is test infrastructure only.)
"""
import ctypes
import os

import torch  # noqa: F401  — load torch's HIP runtime before ours (shared SONAME)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HYGRID_LIB", os.path.join(_HERE, "_lib", "libhygrid_hip.so"))

CSRC = os.path.join(os.path.dirname(_HERE), "csrc")


from ._digest import kernel_source_digest  # noqa: E402  (re-exported)


# dtype codes (enum hg_dtype)
HG_U8, HG_I8, HG_U16, HG_I16, HG_I32, HG_I64, HG_F16, HG_BF16, HG_F32, HG_F64 = range(10)
HG_NEAREST, HG_LINEAR = 0, 1
HG_OP_RECT_TO_HEX, HG_OP_HEX_TO_RECT, HG_OP_HEXRESIZE = 0, 1, 2
HG_KERNEL_GENERAL, HG_KERNEL_NEAREST, HG_KERNEL_STREAM, HG_KERNEL_DOWN, HG_KERNEL_UP = range(5)
HG_PYR_FUSED, HG_PYR_FUSED_SHORT, HG_PYR_STREAM, HG_PYR_LDS = range(4)
HG_OK, HG_EINVAL, HG_EDTYPE, HG_ESHAPE, HG_EUNSUP, HG_EOVERFLOW = 0, -1, -2, -3, -4, -5
PAD_MODES = {"constant": 0, "zeros": 0, "reflect": 1, "replicate": 2, "circular": 3}
HG_ACT_NONE, HG_ACT_RELU, HG_ACT_LEAKY_RELU, HG_ACT_RELU6, HG_ACT_SIGMOID, HG_ACT_TANH = range(6)

TORCH_DTYPE = {
    torch.uint8: HG_U8, torch.int8: HG_I8, torch.int16: HG_I16, torch.int32: HG_I32,
    torch.int64: HG_I64, torch.float16: HG_F16, torch.bfloat16: HG_BF16,
    torch.float32: HG_F32, torch.float64: HG_F64,
}
if hasattr(torch, "uint16"):
    TORCH_DTYPE[torch.uint16] = HG_U16

# Every symbol include/hygrid.h declares, with its ctypes signature.
_i64, _int, _vp, _dbl = ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_double
_RESAMPLE = ([_vp, _vp, _int, _int, _i64, _i64, _i64, _i64, _i64, _int, _vp], _int)
SIGNATURES = {
    "hg_abi_version": ([], _int),
    "hg_build_digest": ([], ctypes.c_char_p),
    "hg_fused_layout": ([_int, ctypes.POINTER(_int), ctypes.POINTER(_int), ctypes.POINTER(_int)],
                        _int),
    "hg_strerror": ([_int], ctypes.c_char_p),
    "hg_rect_to_hex": _RESAMPLE,
    "hg_hex_to_rect": _RESAMPLE,
    "hg_hexresize": _RESAMPLE,
    "hg_resample_backward": ([_int, _vp, _vp, _int] + [_i64] * 5 + [_int, _vp], _int),
    "hg_lattice_maps": ([_int, _i64, _i64, _i64, _i64, _vp, _vp, _vp], _int),
    "hg_resample_kernel": ([_int, _int, _int] + [_i64] * 5 + [_int], _int),
    "hg_hexconv2d_out_shape": ([_i64, _i64, _int, _int, _int, _int,
                                ctypes.POINTER(_i64), ctypes.POINTER(_i64)], _int),
    "hg_hexconv2d": ([_vp, _vp, _vp, _vp, _int, _int, _int, _i64, _i64, _i64, _i64, _i64,
                      _int, _int, _int, _int, _int, _int, _int, _dbl, _vp], _int),
    "hg_hexconv2d_epilogue": ([_vp, _vp, _vp, _vp, _int, _int, _int, _i64, _i64, _i64, _i64,
                               _i64, _int, _int, _int, _int, _int, _int, _int, _dbl, _vp, _vp,
                               _int, _dbl, _vp], _int),
    "hg_hexconv2d_backward": ([_vp] * 6 + [_int, _int] + [_i64] * 5 + [_int] * 7 + [_dbl, _vp],
                              _int),
    "hg_hex_to_type1": ([_vp, _vp, _int] + [_i64] * 3 + [_int, _int, _vp], _int),
    "hg_strided_copy2d": ([_vp, _vp, _int] + [_i64] * 9 + [_vp], _int),
    "hg_hex_homography": ([_vp, _vp, _int, _int] + [_i64] * 5 + [_vp] * 3 + [_int, _vp], _int),
    "hg_hex_homography_maps": ([_i64] * 4 + [_vp] * 5 + [_vp], _int),
    "hg_hex_pool2d": ([_vp, _vp, _int, _int] + [_i64] * 3 + [_int, _int, _dbl, _i64, _i64, _dbl]
                      + [_int] * 4 + [_i64, _i64, _vp], _int),
    "hg_hex_pool2d_backward": ([_vp, _vp, _vp, _int, _int, _int] + [_i64] * 3
                               + [_int, _int, _dbl, _i64, _i64, _dbl] + [_int] * 4
                               + [_i64, _i64, _vp], _int),
    "hg_hex_pyramid_level": ([_vp, _vp, _int, _int] + [_i64] * 6 + [_vp, _vp, _int, _int, _vp],
                             _int),
    "hg_hex_pyramid_level_kernel": ([_int, _int] + [_i64] * 6 + [_int, _int], _int),
    "hg_hex_pyramid_chain_workspace": ([_int, _i64, _i64], _i64),
    "hg_hex_pyramid_chain": ([_vp, ctypes.POINTER(_vp), _int, _int] + [_i64] * 4 +
                             [_vp, _vp, _int, _vp, _i64, _vp], _int),
    "hg_pipeline_r2h_h2r": ([_vp, _vp, _int, _int] + [_i64] * 5 + [_vp], _int),
    "hg_pipeline_r2h_conv_h2r": ([_vp, _vp, _vp, _vp, _int, _int] + [_i64] * 9 +
                                 [_int, _int, _int, _dbl, _vp], _int),
}
ABI_VERSION = 1

_lib = None


class HyGridError(RuntimeError):
    """A HIP runtime error reported by the native library."""


def lib():
    """Load the native library once (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"HyGrid native library not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        v = L.hg_abi_version()
        if v != ABI_VERSION:
            raise ImportError(f"libhygrid_hip.so ABI {v}, expected {ABI_VERSION}")
        # refuse a library built from other sources than the tree it is loaded from (a
        # stale pushed .so must not produce a parity result or a bench line)
        built, here = L.hg_build_digest().decode(), kernel_source_digest()
        if built != here:
            raise ImportError(f"{LIB_PATH} was built from kernel sources {built}, but this "
                              f"tree's are {here}: rebuild (make -C csrc)")
        _lib = L
    return _lib


def fused_layout(md):
    """(band_rows, window_owned_columns, window_left_halo) of the streaming fused kernel's
    mode md (0 pipeline, 1 HexConv2d, 2 round trip): where its bands and windows end."""
    rows, own, halo = _int(), _int(), _int()
    check(lib().hg_fused_layout(int(md), ctypes.byref(rows), ctypes.byref(own),
                                ctypes.byref(halo)), "hg_fused_layout")
    return rows.value, own.value, halo.value


def resample_kernel(op, src_dtype, dst_dtype, planes, h, w, h1, w1, interp=HG_LINEAR):
    """Which kernel a resample call would run (HG_KERNEL_*; nothing is launched)."""
    st = lib().hg_resample_kernel(int(op), int(src_dtype), int(dst_dtype), int(planes), int(h),
                                  int(w), int(h1), int(w1), int(interp))
    if st < 0:
        check(st, "hg_resample_kernel")
    return st


def pyramid_level_kernel(x_dtype, y_dtype, batch, channels, h, w, h1, w1, even_odd_offset=0,
                         from_rect=False):
    """Which kernel hg_hex_pyramid_level would run (HG_PYR_*; nothing is launched)."""
    st = lib().hg_hex_pyramid_level_kernel(int(x_dtype), int(y_dtype), int(batch), int(channels),
                                           int(h), int(w), int(h1), int(w1), int(even_odd_offset),
                                           int(bool(from_rect)))
    if st < 0:
        check(st, "hg_hex_pyramid_level_kernel")
    return st


def strerror(status):
    return lib().hg_strerror(int(status)).decode()


def check(status, what):
    """Map a C-ABI status onto the reference's exception types."""
    if status == 0:
        return
    msg = f"{what}: {strerror(status)} (status {status})"
    if status < 0:
        raise ValueError(msg)
    raise HyGridError(msg)


def dtype_code(dt):
    try:
        return TORCH_DTYPE[dt]
    except KeyError:
        raise TypeError(f"HyGrid: unsupported dtype {dt}") from None


def require_device(t):
    """The product path runs on the GPU only; fail loudly otherwise."""
    if not torch.cuda.is_available():
        raise RuntimeError("HyGrid needs a HIP device (MI355X); none is available. "
                           "There is no CPU fallback.")
    if not t.is_cuda:
        raise RuntimeError("HyGrid op received a CPU tensor; move it to the GPU first")


def stream_of(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None
