"""GPU parity of the ~2x downsampling rect->hex kernel (csrc/resample_down.hip).

The reference's own entry points resample at a ratio of ~2: IMAGE.ConvertToHexagon
(Image.py:111-116: rect_to_hex_resample(image, (h//2, w//2), 'nearest') on the image's own
dtype) and the geometry_np demo (geometry_np.py:772-776: bilinear to (256, 341) from an ADE
image).  hg_rect_to_hex routes those lattices to k_r2h_down.  Its bilinear path evaluates the
general kernel's fp32 blend in the same order and its nearest path copies the same tap, so
it is asserted BIT-IDENTICAL to the general kernels (selected with HYGRID_DOWN=0, read on
every call), NaN/Inf included; nearest is also bit-exact against the fp64 oracle
(oracle/hg_oracle.c, pinned to geometry_np.py:358-519 by tests/golden), bilinear within the
north_star tolerance (rtol 1e-5 of max|ref| for fp32 outputs, one output rounding for 16-bit).
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
    if t.element_size() == 1:
        return t.view(torch.uint8)
    return t.view(torch.int16 if t.element_size() == 2 else torch.int32)


def _same_bits(a, b):
    assert a.shape == b.shape and a.dtype == b.dtype
    nbad = int((_bits(a) != _bits(b)).sum().item())
    assert nbad == 0, f"{nbad} elements differ from the general kernel"


# (h, w) -> (h // 2, w // 2) and the demo's exact shape; ragged widths (w1 not a multiple of
# the lane's 2 / 4 columns), band edges (32-row bands), windows past the raster, 4K
SHAPES = [(4, 8), (9, 22), (17, 40), (64, 66), (65, 130), (100, 1000), (256, 256),
          (512, 683), (130, 2050), (2160, 3840)]


def _u8(shape, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return torch.randint(0, 256, shape, generator=g, device=DEV, dtype=torch.uint8)


@pytest.mark.parametrize("h,w", SHAPES)
def test_convert_to_hexagon_nearest_u8(h, w):
    """ConvertToHexagon's call: u8 planes, nearest to (h//2, w//2): the streaming kernel,
    the general kernel and the oracle agree bit for bit."""
    x = _u8((2, 3, h, w), h * 7 + w)
    size = (h // 2, w // 2)
    y = ops.rect_to_hex(x, size, interp=_abi.HG_NEAREST)
    torch.cuda.synchronize()
    _same_bits(y, _general(ops.rect_to_hex, x, size, interp=_abi.HG_NEAREST))
    if h * w <= 1 << 20:
        ref = O.rect_to_hex(x[0].cpu().numpy().astype(np.float64), size, 0)
        np.testing.assert_array_equal(y[0].cpu().numpy().astype(np.float64), ref)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.int16])
@pytest.mark.parametrize("h,w", [(9, 22), (64, 66), (512, 683), (2160, 3840)])
def test_nearest_16bit(h, w, dt):
    g = torch.Generator(device=DEV).manual_seed(h + w)
    x = (torch.randn((2, h, w), generator=g, device=DEV) * 100).to(dt)
    size = (h // 2, w // 2)
    y = ops.rect_to_hex(x, size, interp=_abi.HG_NEAREST)
    torch.cuda.synchronize()
    _same_bits(y, _general(ops.rect_to_hex, x, size, interp=_abi.HG_NEAREST))


@pytest.mark.parametrize("out", [None, torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("h,w,size", [(9, 22, (4, 11)), (64, 66, (32, 33)), (512, 683, (256, 341)),
                                      (130, 2050, (65, 1025)), (100, 1000, (50, 500)),
                                      (2160, 3840, (1080, 1920))])
def test_bilinear_2x(h, w, size, dt, out):
    """The demo's bilinear downsample (geometry_np.py:772-776 at its own (512, 683) ->
    (256, 341) and at 4K): bit-identical to the general kernel, within the north_star
    tolerance of the fp64 oracle."""
    g = torch.Generator(device=DEV).manual_seed(h * 3 + w)
    x = torch.rand((2, 3, h, w), generator=g, device=DEV).to(dt)
    y = ops.rect_to_hex(x, size, out_dtype=out)
    torch.cuda.synchronize()
    _same_bits(y, _general(ops.rect_to_hex, x, size, out_dtype=out))
    if h * w <= 1 << 20:
        ref = O.rect_to_hex(x[1].double().cpu().numpy(), size, 1)
        got = y[1].double().cpu().numpy()
        scale = np.abs(ref).max()
        if out == torch.float32:
            np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5 * scale)
        else:   # one 16-bit rounding of an fp32 result (in the output's dtype)
            od = dt if out is None else out
            ulp = 2.0 ** (-8 if od == torch.bfloat16 else -11)
            assert np.abs(got - ref).max() <= ulp * scale


def test_nonfinite_bit_identical():
    """NaN / Inf inputs reach exactly the outputs the general kernel's taps reach."""
    h, w = 130, 260
    x = torch.rand((1, h, w), device=DEV).to(torch.bfloat16)
    x[0, 7, 9] = float("nan")
    x[0, 0, 0] = float("inf")
    x[0, 64, 259] = float("-inf")
    x[0, 129, 100] = float("nan")
    for interp in (_abi.HG_LINEAR, _abi.HG_NEAREST):
        y = ops.rect_to_hex(x, (h // 2, w // 2), interp=interp)
        torch.cuda.synchronize()
        _same_bits(y, _general(ops.rect_to_hex, x, (h // 2, w // 2), interp=interp))
