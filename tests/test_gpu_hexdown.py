"""GPU parity of the ~2x downsampling hexresize kernel (csrc/hexresize_down.hip).

hexresize (geometry_np.py:520-681, 'linear') at (h // 2, w // 2) is every level of the
config-5 pyramid's operator chain; hg_hexresize routes those lattices (16-bit inputs,
fp32 accumulation) to k_hexresize_down.  It evaluates the general kernel's per-sample fp64
triangle records cast to fp32 and its blend alpha*p1 + beta*p2 + gamma*p3 in the same order,
with 0 for vertices outside the raster, so it is asserted BIT-IDENTICAL to the general
kernel (k_resample_lds, selected with HYGRID_DOWN=0, read on every call), NaN / Inf included,
and within one output rounding of the fp64 oracle (oracle/hg_oracle.c or_hexresize, pinned to
geometry_np.py:520-681 by tests/golden).  The dispatch itself is pinned on the host
(tests/test_dispatch_cpu.py); here it is asserted to be the streaming kernel that ran.
"""
import os

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - collected only with -m gpu
    pytest.skip("needs a HIP device", allow_module_level=True)

from HyGrid import _abi, ops  # noqa: E402

DEV = torch.device("cuda:0")


def _general(fn, *args, **kw):
    old = os.environ.get("HYGRID_DOWN")
    os.environ["HYGRID_DOWN"] = "0"
    try:
        out = fn(*args, **kw)
        torch.cuda.synchronize()
        return out
    finally:
        if old is None:
            del os.environ["HYGRID_DOWN"]
        else:
            os.environ["HYGRID_DOWN"] = old


def _bits(t):
    t = t.contiguous()
    return t.view(torch.int16 if t.element_size() == 2 else torch.int32)


def _same_bits(a, b):
    assert a.shape == b.shape and a.dtype == b.dtype
    nbad = int((_bits(a) != _bits(b)).sum().item())
    assert nbad == 0, f"{nbad} elements differ from the general kernel"


def _kernel(x, size, out_dtype):
    B, C, h, w = x.shape
    return _abi.resample_kernel(_abi.HG_OP_HEXRESIZE, _abi.dtype_code(x.dtype),
                                _abi.dtype_code(out_dtype), B * C, h, w, size[0], size[1])


# (h, w): exact halvings, odd sizes (h // 2, w // 2 floor), windows (62 output columns) and
# 4-row units ending inside the raster, one-window images, the pyramid's level shapes
SHAPES = [(4, 4), (6, 10), (9, 22), (17, 40), (33, 124), (35, 126), (64, 66), (65, 130), (100, 1000),
          (128, 250), (256, 256), (270, 480), (540, 960)]
PAIRS = [(torch.float16, torch.float16), (torch.bfloat16, torch.bfloat16),
         (torch.float16, torch.float32), (torch.bfloat16, torch.float32),
         (torch.float16, torch.bfloat16), (torch.bfloat16, torch.float16)]


@pytest.mark.parametrize("h,w", SHAPES)
@pytest.mark.parametrize("pair", PAIRS)
def test_hexresize_2x_bit_identical_and_vs_oracle(h, w, pair):
    dt, od = pair
    g = torch.Generator(device=DEV).manual_seed(h * 31 + w)
    x = torch.rand((2, 3, h, w), generator=g, device=DEV).to(dt)
    size = (h // 2, w // 2)
    assert _kernel(x, size, od) == _abi.HG_KERNEL_DOWN
    y = ops.hexresize(x, size, out_dtype=od)
    torch.cuda.synchronize()
    _same_bits(y, _general(ops.hexresize, x, size, out_dtype=od))
    ref = O.hexresize(x[1].double().cpu().numpy(), size, 1)
    got = y[1].double().cpu().numpy()
    scale = max(np.abs(ref).max(), 1e-30)
    if od == torch.float32:
        np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5 * scale)
    else:   # one 16-bit rounding of an fp32 result
        ulp = 2.0 ** (-8 if od == torch.bfloat16 else -11)
        assert np.abs(got - ref).max() <= ulp * scale


@pytest.mark.parametrize("B,C,h,w", [(8, 3, 4320, 7680), (8, 3, 2160, 3840), (8, 3, 1080, 1920)])
def test_hexresize_pyramid_levels_full_size(B, C, h, w):
    """The bench's unfused pyramid levels (8 x 3 fp16 planes per launch, plane chunks of the
    whole batch): bit-identical to the general kernel; first and last image vs the oracle."""
    g = torch.Generator(device=DEV).manual_seed(h + w)
    x = torch.rand((B, C, h, w), generator=g, device=DEV).to(torch.float16)
    size = (h // 2, w // 2)
    assert _kernel(x, size, torch.float16) == _abi.HG_KERNEL_DOWN
    y = ops.hexresize(x, size, out_dtype=torch.float16)
    torch.cuda.synchronize()
    _same_bits(y, _general(ops.hexresize, x, size, out_dtype=torch.float16))
    del x
    if h <= 2160:
        xs = torch.rand((B, C, h, w), generator=torch.Generator(device=DEV).manual_seed(h + w),
                        device=DEV).to(torch.float16)
        for i in (0, B - 1):
            ref = O.hexresize(xs[i, 0].double().cpu().numpy(), size, 1)
            got = y[i, 0].double().cpu().numpy()
            assert np.abs(got - ref).max() <= 2.0 ** -11 * np.abs(ref).max()


@pytest.mark.parametrize("h,w,h1,w1", [(256, 1024, 64, 256), (256, 1024, 32, 128),
                                       (512, 2048, 32, 128), (130, 520, 26, 104)])
def test_hexresize_strong_downsampling(h, w, h1, w1):
    """4x / 8x / 16x / 5x: narrower windows (K = 4 down to 1 column per lane) on the same
    kernel, bit-identical to the general kernel and within one rounding of the oracle."""
    g = torch.Generator(device=DEV).manual_seed(h1 * 7 + w1)
    x = torch.rand((2, 3, h, w), generator=g, device=DEV).to(torch.float16)
    assert _kernel(x, (h1, w1), torch.float16) == _abi.HG_KERNEL_DOWN
    y = ops.hexresize(x, (h1, w1), out_dtype=torch.float16)
    torch.cuda.synchronize()
    _same_bits(y, _general(ops.hexresize, x, (h1, w1), out_dtype=torch.float16))
    ref = O.hexresize(x[1].double().cpu().numpy(), (h1, w1), 1)
    assert np.abs(y[1].double().cpu().numpy() - ref).max() <= 2.0 ** -11 * np.abs(ref).max()


def test_hexresize_base_not_16b_aligned():
    """A source 4-B but not 16-B aligned takes the 4-B-piece configuration (128 + 16 input
    columns per wave); results bit-identical to the general kernel."""
    h, w = 96, 512
    flat = torch.rand(2 * 3 * h * w + 2, device=DEV).to(torch.bfloat16)
    x = flat[2:].view(2, 3, h, w)
    assert x.data_ptr() % 16 == 4
    for od in (torch.bfloat16, torch.float32):
        y = ops.hexresize(x, (h // 2, w // 2), out_dtype=od)
        torch.cuda.synchronize()
        _same_bits(y, _general(ops.hexresize, x, (h // 2, w // 2), out_dtype=od))


def test_hexresize_nonfinite_bit_identical():
    """NaN / Inf inputs (raster corners and edges, window and unit boundaries) reach exactly
    the outputs the general kernel's taps reach."""
    h, w = 130, 260
    x = torch.rand((2, h, w), device=DEV).to(torch.bfloat16)
    for (p, r, c, v) in [(0, 0, 0, "inf"), (0, 7, 9, "nan"), (0, 64, 259, "-inf"),
                         (0, 129, 100, "nan"), (1, 8, 123, "nan"), (1, 9, 124, "inf"),
                         (1, 129, 259, "nan"), (1, 0, 124, "-inf")]:
        x[p, r, c] = float(v)
    for od in (torch.bfloat16, torch.float32):
        y = ops.hexresize(x, (h // 2, w // 2), out_dtype=od)
        torch.cuda.synchronize()
        _same_bits(y, _general(ops.hexresize, x, (h // 2, w // 2), out_dtype=od))


def test_hexresize_outside_domain_keeps_general_kernel():
    """fp32 inputs, fp64 outputs (the NumPy API's bit-exact path), odd input widths and ratios
    whose window of 32 output columns no longer fits the wave's input columns stay on the
    general kernel."""
    x = torch.rand((1, 1, 64, 66), device=DEV)
    assert _kernel(x, (32, 33), torch.float32) == _abi.HG_KERNEL_GENERAL
    xh = x.half()
    assert _kernel(xh, (32, 33), torch.float64) == _abi.HG_KERNEL_GENERAL
    assert _kernel(xh, (4, 4), torch.float16) == _abi.HG_KERNEL_GENERAL     # 16x, 4-B pieces
    # odd input widths: rows not dword-aligned for LDS-DMA
    xo = torch.rand((1, 1, 33, 125), device=DEV).half()
    assert _kernel(xo, (16, 62), torch.float16) == _abi.HG_KERNEL_GENERAL


# hex (h, w) -> rect (2h, 2w) and near: the inverse of ConvertToHexagon's lattice
# (Image.py:111-116 read backwards; hex_to_rect_resample, geometry_np.py:191-356), two output
# columns per lane; odd output widths end on a single column
UP_SHAPES = [(2, 2, 4, 4), (5, 10, 10, 19), (8, 12, 16, 23), (17, 40, 34, 80), (32, 34, 65, 67),
             (60, 100, 120, 200), (100, 1000, 200, 2000), (135, 240, 270, 480)]


@pytest.mark.parametrize("shape", UP_SHAPES)
@pytest.mark.parametrize("pair", PAIRS)
def test_h2r_2x_up_bit_identical_and_vs_oracle(shape, pair):
    h, w, h1, w1 = shape
    dt, od = pair
    g = torch.Generator(device=DEV).manual_seed(h * 17 + w)
    x = torch.rand((2, 3, h, w), generator=g, device=DEV).to(dt)
    B, C = x.shape[:2]
    k = _abi.resample_kernel(_abi.HG_OP_HEX_TO_RECT, _abi.dtype_code(dt), _abi.dtype_code(od),
                             B * C, h, w, h1, w1)
    assert k == _abi.HG_KERNEL_UP        # the upsampling kernel (tests/test_gpu_triup.py)
    y = ops.hex_to_rect(x, (h1, w1), out_dtype=od)
    torch.cuda.synchronize()
    _same_bits(y, _general(ops.hex_to_rect, x, (h1, w1), out_dtype=od))
    ref = O.hex_to_rect(x[1].double().cpu().numpy(), (h1, w1), 1)
    got = y[1].double().cpu().numpy()
    scale = max(np.abs(ref).max(), 1e-30)
    if od == torch.float32:
        np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5 * scale)
    else:
        ulp = 2.0 ** (-8 if od == torch.bfloat16 else -11)
        assert np.abs(got - ref).max() <= ulp * scale


def test_h2r_2x_up_4k_batch_and_nonfinite():
    """The bench's inverse-lattice line (hex 1080 x 1920 -> rect 2160 x 3840, bf16, 32 x 3
    planes): bit-identical to the general kernel; NaN / Inf planted at corners, edges and
    window boundaries reach exactly the outputs the general kernel's taps reach."""
    g = torch.Generator(device=DEV).manual_seed(4)
    x = torch.rand((32, 3, 1080, 1920), generator=g, device=DEV).to(torch.bfloat16)
    for (b_, c, r, q, v) in [(0, 0, 0, 0, "inf"), (0, 1, 7, 63, "nan"), (5, 2, 540, 64, "-inf"),
                             (31, 2, 1079, 1919, "nan"), (17, 0, 300, 1000, "inf")]:
        x[b_, c, r, q] = float(v)
    y = ops.hex_to_rect(x, (2160, 3840))
    torch.cuda.synchronize()
    _same_bits(y, _general(ops.hex_to_rect, x, (2160, 3840)))
