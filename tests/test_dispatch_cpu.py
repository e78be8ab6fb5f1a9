"""Kernel dispatch of the resamplers, checked on the host (no GPU needed): which kernel
hg_rect_to_hex / hg_hex_to_rect / hg_hexresize pick for the lattices of the reference's
entry points (hg_resample_kernel: the dispatch without a launch).  The GPU parity tests
compare those kernels with the general ones (tests/test_gpu_down.py, test_gpu_stream.py);
this pins that the specialised kernel is the one they exercise."""
import ctypes
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
    # hexresize at the pyramid's 2x ratio: the streaming hexresize kernel (hexresize_down.hip);
    # fp32 in, fp64 out (the NumPy API's bit-exact path) and 4x keep the general kernel
    for h, w in ((4320, 7680), (2160, 3840), (1080, 1920), (35, 126), (9, 22)):
        for dt, ot in ((_abi.HG_F16, _abi.HG_F16), (_abi.HG_BF16, _abi.HG_F32)):
            assert _kernel(_abi.HG_OP_HEXRESIZE, dt, ot, 24, h, w, h // 2, w // 2,
                           _abi.HG_LINEAR) == _abi.HG_KERNEL_DOWN
        assert _kernel(_abi.HG_OP_HEXRESIZE, _abi.HG_F16, _abi.HG_F16, 24, h, w, h // 2, w // 2,
                       _abi.HG_LINEAR, HYGRID_DOWN="0") == _abi.HG_KERNEL_GENERAL
    for dt, ot in ((_abi.HG_F32, _abi.HG_F32), (_abi.HG_F16, _abi.HG_F64)):
        assert _kernel(_abi.HG_OP_HEXRESIZE, dt, ot, 3, 2160, 3840, 1080, 1920,
                       _abi.HG_LINEAR) == _abi.HG_KERNEL_GENERAL
    # odd input widths (rows not dword-aligned for LDS-DMA) keep the general kernel
    assert _kernel(_abi.HG_OP_HEXRESIZE, _abi.HG_F16, _abi.HG_F16, 3, 33, 125, 16, 62,
                   _abi.HG_LINEAR) == _abi.HG_KERNEL_GENERAL
    # any ratio whose window of >= 32 output columns keeps its vertices in the wave's 528
    # input columns (4x: 128 columns per wave, 16x: 32); 32x does not fit
    for h1, w1 in ((540, 960), (135, 240)):
        assert _kernel(_abi.HG_OP_HEXRESIZE, _abi.HG_F16, _abi.HG_F16, 3, 2160, 3840, h1, w1,
                       _abi.HG_LINEAR) == _abi.HG_KERNEL_DOWN
    assert _kernel(_abi.HG_OP_HEXRESIZE, _abi.HG_F16, _abi.HG_F16, 3, 2160, 3840, 68, 120,
                   _abi.HG_LINEAR) == _abi.HG_KERNEL_GENERAL
    # hex (h/2, w/2) -> rect (h, w), the inverse of ConvertToHexagon's lattice: the upsampling
    # triangle kernel (tri_up.hip), linear and nearest; HYGRID_UP=0 falls back to the
    # downsampling triangle kernel (linear) / the general nearest kernel; fp64 out keeps the
    # general one
    for h, w in ((2160, 3840), (540, 964), (1080, 1920), (10, 20)):
        for dt, ot in ((_abi.HG_BF16, _abi.HG_BF16), (_abi.HG_F16, _abi.HG_F32),
                       (_abi.HG_F32, _abi.HG_BF16)):
            assert _kernel(_abi.HG_OP_HEX_TO_RECT, dt, ot, 96, h // 2, w // 2, h, w,
                           _abi.HG_LINEAR) == _abi.HG_KERNEL_UP
        assert _kernel(_abi.HG_OP_HEX_TO_RECT, _abi.HG_BF16, _abi.HG_BF16, 96, h // 2, w // 2, h,
                       w, _abi.HG_LINEAR, HYGRID_UP="0") in (_abi.HG_KERNEL_DOWN, _abi.HG_KERNEL_GENERAL)
        assert _kernel(_abi.HG_OP_HEX_TO_RECT, _abi.HG_BF16, _abi.HG_F64, 96, h // 2, w // 2, h,
                       w, _abi.HG_LINEAR) == _abi.HG_KERNEL_GENERAL
        for dt in (_abi.HG_U8, _abi.HG_BF16, _abi.HG_I32):
            if (w // 2) * {_abi.HG_U8: 1, _abi.HG_BF16: 2, _abi.HG_I32: 4}[dt] % 4:
                continue     # input rows not dword-aligned for LDS-DMA
            assert _kernel(_abi.HG_OP_HEX_TO_RECT, dt, dt, 96, h // 2, w // 2, h, w,
                           _abi.HG_NEAREST) == _abi.HG_KERNEL_UP
            assert _kernel(_abi.HG_OP_HEX_TO_RECT, dt, dt, 96, h // 2, w // 2, h, w,
                           _abi.HG_NEAREST, HYGRID_UP="0") == _abi.HG_KERNEL_NEAREST
    # an output width no K divides: one column per lane
    assert _kernel(_abi.HG_OP_HEX_TO_RECT, _abi.HG_BF16, _abi.HG_BF16, 3, 5, 10, 10, 19,
                   _abi.HG_LINEAR) == _abi.HG_KERNEL_UP
    # hexresize upsampling takes it too; downsampling never does
    assert _kernel(_abi.HG_OP_HEXRESIZE, _abi.HG_F16, _abi.HG_F16, 3, 540, 960, 1080, 1920,
                   _abi.HG_LINEAR) == _abi.HG_KERNEL_UP
    assert _kernel(_abi.HG_OP_HEX_TO_RECT, _abi.HG_U8, _abi.HG_U8, 3, 1080, 1920, 540, 960,
                   _abi.HG_NEAREST) == _abi.HG_KERNEL_NEAREST
    # odd input widths: rows not dword-aligned for 16-bit LDS-DMA
    assert _kernel(_abi.HG_OP_HEX_TO_RECT, _abi.HG_BF16, _abi.HG_BF16, 3, 33, 125, 66, 250,
                   _abi.HG_LINEAR) != _abi.HG_KERNEL_UP


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
    # linear needs a floating output, as the launching call (resample() returns HG_EDTYPE)
    for op in OPS:
        for dt in (_abi.HG_U8, _abi.HG_I32):
            with pytest.raises(ValueError, match="dtype"):
                _abi.resample_kernel(op, _abi.HG_BF16, dt, 1, 64, 64, 64, 64, _abi.HG_LINEAR)


def _pyr(*a, **env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return _abi.lib().hg_hex_pyramid_level_kernel(*a)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def test_pyramid_levels_take_the_fused_row_walk():
    """Config 5's three levels (8 x 3 x 4320 x 7680 fp16: level 0 from the rect image) run
    on k_fused (MD 3, then MD 4 / MD 5 for levels too small to fill the chip at 60-row bands);
    HYGRID_PYR_KERNEL restricts the choice (exact values only)."""
    F16, F32 = _abi.HG_F16, _abi.HG_F32
    fused = (_abi.HG_PYR_FUSED, _abi.HG_PYR_FUSED_SHORT)
    assert _pyr(F16, F16, 8, 3, 4320, 7680, 2160, 3840, 0, 1) == _abi.HG_PYR_FUSED
    assert _pyr(F16, F16, 8, 3, 2160, 3840, 1080, 1920, 0, 0) in fused
    assert _pyr(F16, F16, 8, 3, 1080, 1920, 540, 960, 0, 0) == _abi.HG_PYR_FUSED_SHORT
    assert _pyr(F16, F16, 8, 3, 1080, 1920, 540, 960, 0, 0, HYGRID_PYR_SHORT="0") == _abi.HG_PYR_FUSED
    assert _pyr(F16, F16, 8, 3, 2160, 3840, 1080, 1920, 0, 0,
                HYGRID_PYR_KERNEL="stream") == _abi.HG_PYR_STREAM
    assert _pyr(F16, F16, 8, 3, 2160, 3840, 1080, 1920, 0, 0,
                HYGRID_PYR_KERNEL="lds") == _abi.HG_PYR_LDS
    # a value that is not exactly a kernel name restricts nothing
    assert _pyr(F16, F16, 8, 3, 2160, 3840, 1080, 1920, 0, 0, HYGRID_PYR_KERNEL="l") in fused
    # fp32 levels: only the LDS kernel; restricted to the fused kernel the call declines
    assert _pyr(F32, F32, 2, 3, 540, 960, 270, 480, 1, 1) == _abi.HG_PYR_LDS
    assert _pyr(F32, F32, 2, 3, 540, 960, 270, 480, 1, 1,
                HYGRID_PYR_KERNEL="fused") == _abi.HG_EUNSUP
    # > 2x downsampling overflows every tile: declined up front by the exact host bound
    assert _pyr(F32, F32, 1, 3, 540, 960, 100, 180, 0, 0) == _abi.HG_EUNSUP
    assert _pyr(_abi.HG_U8, F32, 1, 3, 64, 64, 32, 32, 0, 0) == -2   # HG_EDTYPE


def test_pyramid_chain_workspace_and_validation():
    """hg_hex_pyramid_chain's host side (no launch): the workspace is 2 ints (ticket, fault)
    plus one counter per (image, band) of every level but the last (level 0 on 60-row bands of
    the conv image, later levels on 24-row bands), padded to whole 16-byte blocks, and argument
    errors return before any HIP call."""
    L = _abi.lib()
    # config 5: 8 x 4320-row images, 3 levels: 8 * 72 + 8 * 90 counters
    assert L.hg_hex_pyramid_chain_workspace(3, 8, 4320) == 4 * 1300      # 2 + 576 + 720 -> 1300
    assert L.hg_hex_pyramid_chain_workspace(2, 1, 70) == 4 * 4
    assert L.hg_hex_pyramid_chain_workspace(1, 4, 100) == 4 * 4
    assert L.hg_hex_pyramid_chain_workspace(0, 4, 100) == _abi.HG_EINVAL
    fake = ctypes.c_void_p(16)
    ys = (ctypes.c_void_p * 3)(16, 16, 16)
    args = [fake, ys, 3, _abi.HG_F16, 2, 3, 136, 250, fake, None]
    assert L.hg_hex_pyramid_chain(fake, ys, 0, _abi.HG_F16, 2, 3, 136, 250, fake, None, 0, fake,
                                  64, None) == _abi.HG_EINVAL
    assert L.hg_hex_pyramid_chain(*args, 2, fake, 64, None) == _abi.HG_EINVAL   # offset class
    assert L.hg_hex_pyramid_chain(fake, ys, 3, _abi.HG_U8, 2, 3, 136, 250, fake, None, 0, fake,
                                  64, None) == _abi.HG_EDTYPE
    assert L.hg_hex_pyramid_chain(None, None, 3, _abi.HG_F16, 0, 3, 136, 250, None, None, 0,
                                  None, 0, None) == _abi.HG_OK                  # nothing to do
