"""Kernel dispatch of the resamplers, checked on the host (no GPU needed): which kernel
hg_rect_to_hex / hg_hex_to_rect / hg_hexresize pick for the lattices of the reference's
entry points (hg_resample_kernel: the dispatch without a launch).  The GPU parity tests
compare those kernels with the general ones (tests/test_gpu_down.py, test_gpu_stream.py);
this pins that the specialised kernel is the one they exercise."""
import os

import pytest

from HyGrid import _abi

OPS = (_abi.HG_OP_RECT_TO_HEX, _abi.HG_OP_HEX_TO_RECT, _abi.HG_OP_HEXRESIZE)


def _kernel(*a, **env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return _abi.resample_kernel(*a)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.mark.parametrize("h,w,interp,dt", [
    (2160, 3840, _abi.HG_NEAREST, _abi.HG_U8),    # ConvertToHexagon on a 4K u8 image
    (512, 683, _abi.HG_NEAREST, _abi.HG_U8),      # ... on the demo's ADE image
    (2160, 3840, _abi.HG_NEAREST, _abi.HG_BF16),
    (2160, 3840, _abi.HG_LINEAR, _abi.HG_BF16),   # the demo's bilinear ratio at 4K
    (512, 683, _abi.HG_LINEAR, _abi.HG_F16)])     # the demo's own (256, 341)
def test_downsample_lattices_take_the_streaming_kernel(h, w, interp, dt):
    args = (_abi.HG_OP_RECT_TO_HEX, dt, dt, 3, h, w, h // 2, w // 2, interp)
    assert _kernel(*args) == _abi.HG_KERNEL_DOWN
    assert _kernel(*args, HYGRID_DOWN="0") in (_abi.HG_KERNEL_NEAREST, _abi.HG_KERNEL_GENERAL)


def test_same_size_keeps_its_kernels():
    for op in (_abi.HG_OP_RECT_TO_HEX, _abi.HG_OP_HEX_TO_RECT):
        assert _kernel(op, _abi.HG_BF16, _abi.HG_BF16, 3, 2160, 3840, 2160, 3840,
                       _abi.HG_LINEAR) == _abi.HG_KERNEL_STREAM
    assert _kernel(_abi.HG_OP_HEXRESIZE, _abi.HG_F16, _abi.HG_F16, 3, 4320, 7680, 2160, 3840,
                   _abi.HG_LINEAR) == _abi.HG_KERNEL_GENERAL


def test_outside_the_domain():
    # f64 (bit-exact NumPy path) and 3x ratios stay on the general kernels
    assert _kernel(_abi.HG_OP_RECT_TO_HEX, _abi.HG_F64, _abi.HG_F64, 1, 2160, 3840, 1080, 1920,
                   _abi.HG_LINEAR) == _abi.HG_KERNEL_GENERAL
    assert _kernel(_abi.HG_OP_RECT_TO_HEX, _abi.HG_BF16, _abi.HG_BF16, 1, 2160, 3840, 720, 1280,
                   _abi.HG_LINEAR) == _abi.HG_KERNEL_GENERAL
    assert _kernel(_abi.HG_OP_RECT_TO_HEX, _abi.HG_U8, _abi.HG_U8, 1, 4, 8, 2, 4,
                   _abi.HG_NEAREST) == _abi.HG_KERNEL_NEAREST   # rows narrower than a chunk
    for op in OPS:
        with pytest.raises(ValueError):
            _abi.resample_kernel(op, _abi.HG_U8, _abi.HG_F32, 1, 8, 8, 4, 4, _abi.HG_NEAREST)
