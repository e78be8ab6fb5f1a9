"""GPU parity of the upsampling triangle kernel (csrc/tri_up.hip).

hex_to_rect_resample (geometry_np.py:191-356) from hex (h/2, w/2) to rect (h, w) — the inverse
of IMAGE.ConvertToHexagon's lattice (Image.py:111-116) — and hexresize upsampling
(:520-681), 'linear' (the triangle blend, :347-354) and 'nearest' (geometry_torch.py:335-347).
The kernel evaluates the general kernels' per-sample fp64 triangle records (weights cast to
fp32, the blend in the same order, 0 for vertices outside the raster; nearest copies the
chosen element's bits), so it is asserted BIT-IDENTICAL to the general kernels (selected with
HYGRID_DOWN=0, read on every call), NaN / Inf included, and against the fp64 oracle
(oracle/hg_oracle.c, pinned to the reference by tests/golden): linear within one output
rounding, nearest exactly.  The dispatch is pinned on the host (tests/test_dispatch_cpu.py);
here it is asserted to be the upsampling kernel that ran.
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
OPS = {"h2r": (ops.hex_to_rect, _abi.HG_OP_HEX_TO_RECT, O.hex_to_rect),
       "resize": (ops.hexresize, _abi.HG_OP_HEXRESIZE, O.hexresize)}


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
    return t.view({1: torch.uint8, 2: torch.int16, 4: torch.int32}[t.element_size()])


def _same_bits(a, b):
    assert a.shape == b.shape and a.dtype == b.dtype
    nbad = int((_bits(a) != _bits(b)).sum().item())
    assert nbad == 0, f"{nbad} elements differ from the general kernel"


def _kernel(op, x, size, out_dtype, interp):
    B, C, h, w = x.shape
    return _abi.resample_kernel(op, _abi.dtype_code(x.dtype), _abi.dtype_code(out_dtype),
                                B * C, h, w, size[0], size[1], interp)


def _rand(shape, dt, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    if dt == torch.uint8:
        return torch.randint(0, 256, shape, generator=g, device=DEV, dtype=torch.uint8)
    if dt == torch.int32:
        return torch.randint(-2 ** 31, 2 ** 31 - 1, shape, generator=g, device=DEV, dtype=torch.int32)
    return torch.rand(shape, generator=g, device=DEV).to(dt)


# (h, w, h1, w1): exact doublings, odd output sizes (one column per lane when no K divides
# w1), windows of 256 / 512 output columns ending inside the raster, 2-row units ending on
# the last row, one-window and several-window images, ratios between 1 and 2
SHAPES = [(2, 2, 4, 4), (5, 10, 10, 19), (8, 12, 16, 23), (17, 40, 34, 80), (32, 34, 65, 67),
          (60, 100, 120, 200), (100, 1000, 200, 2000), (135, 240, 270, 480), (64, 128, 96, 192),
          (33, 260, 65, 520), (40, 96, 41, 97)]
PAIRS = [(torch.bfloat16, torch.bfloat16), (torch.float16, torch.float16),
         (torch.bfloat16, torch.float32), (torch.float16, torch.bfloat16),
         (torch.float32, torch.float32), (torch.float32, torch.bfloat16)]


@pytest.mark.parametrize("op", ["h2r", "resize"])
@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("pair", PAIRS)
def test_linear_up_bit_identical_and_vs_oracle(op, shape, pair):
    fn, code, ofn = OPS[op]
    h, w, h1, w1 = shape
    dt, od = pair
    x = _rand((2, 3, h, w), dt, h * 17 + w)
    assert _kernel(code, x, (h1, w1), od, _abi.HG_LINEAR) == _abi.HG_KERNEL_UP
    y = fn(x, (h1, w1), out_dtype=od)
    torch.cuda.synchronize()
    _same_bits(y, _general(fn, x, (h1, w1), out_dtype=od))
    ref = ofn(x[1].double().cpu().numpy(), (h1, w1), 1)
    got = y[1].double().cpu().numpy()
    scale = max(np.abs(ref).max(), 1e-30)
    if od == torch.float32:
        np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5 * scale)
    else:   # one 16-bit rounding of an fp32 result
        ulp = 2.0 ** (-8 if od == torch.bfloat16 else -11)
        assert np.abs(got - ref).max() <= ulp * scale


@pytest.mark.parametrize("op", ["h2r", "resize"])
@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("dt", [torch.uint8, torch.bfloat16, torch.int32])
def test_nearest_up_bit_identical_and_vs_oracle(op, shape, dt):
    fn, code, ofn = OPS[op]
    h, w, h1, w1 = shape
    x = _rand((2, 3, h, w), dt, h * 29 + w)
    esz = x.element_size()
    k = _kernel(code, x, (h1, w1), dt, _abi.HG_NEAREST)
    if (w * esz) % 4:
        assert k == _abi.HG_KERNEL_NEAREST      # rows not dword-aligned: the general kernel
    elif 2 * (h - 1) <= h1:
        assert k == _abi.HG_KERNEL_UP           # ~2x: 4-row bands read <= 4 input rows
    else:   # ratios near 1: a 4-row band may read 5 input rows (host check: general kernel)
        assert k in (_abi.HG_KERNEL_UP, _abi.HG_KERNEL_NEAREST)
    y = fn(x, (h1, w1), interp=_abi.HG_NEAREST)
    torch.cuda.synchronize()
    _same_bits(y, _general(fn, x, (h1, w1), interp=_abi.HG_NEAREST))
    if dt != torch.int32:      # the oracle blends in fp64: exact for u8 / bf16 values
        ref = ofn(x[1].double().cpu().numpy(), (h1, w1), 0)
        np.testing.assert_array_equal(y[1].double().cpu().numpy(), ref)


def test_4k_batch_linear_and_nearest_and_nonfinite():
    """The bench's inverse-lattice lines (hex 1080 x 1920 -> rect 2160 x 3840, 32 x 3 planes,
    bf16 linear and u8 nearest): bit-identical to the general kernels; NaN / Inf planted at
    corners, edges and window boundaries reach exactly the outputs the general kernel's taps
    reach; first and last plane of the launch against the oracle."""
    x = _rand((32, 3, 1080, 1920), torch.bfloat16, 4)
    for (b_, c, r, q, v) in [(0, 0, 0, 0, "inf"), (0, 1, 7, 63, "nan"), (5, 2, 540, 64, "-inf"),
                             (31, 2, 1079, 1919, "nan"), (17, 0, 300, 1000, "inf"),
                             (9, 1, 301, 127, "nan"), (9, 1, 302, 128, "-inf")]:
        x[b_, c, r, q] = float(v)
    assert _kernel(_abi.HG_OP_HEX_TO_RECT, x, (2160, 3840), x.dtype, _abi.HG_LINEAR) == _abi.HG_KERNEL_UP
    y = ops.hex_to_rect(x, (2160, 3840))
    torch.cuda.synchronize()
    _same_bits(y, _general(ops.hex_to_rect, x, (2160, 3840)))
    for (b_, c) in ((0, 0), (31, 2)):
        ref = O.hex_to_rect(x[b_, c].double().cpu().numpy(), (2160, 3840), 1).reshape(2160, 3840)
        got = y[b_, c].double().cpu().numpy()
        fin = np.isfinite(ref)
        assert np.array_equal(np.isnan(got), np.isnan(ref))
        assert np.abs(got[fin] - ref[fin]).max() <= 2.0 ** -8 * np.abs(ref[fin]).max()
    del y
    xu = _rand((32, 3, 1080, 1920), torch.uint8, 5)
    assert _kernel(_abi.HG_OP_HEX_TO_RECT, xu, (2160, 3840), xu.dtype, _abi.HG_NEAREST) == _abi.HG_KERNEL_UP
    yu = ops.hex_to_rect(xu, (2160, 3840), interp=_abi.HG_NEAREST)
    torch.cuda.synchronize()
    _same_bits(yu, _general(ops.hex_to_rect, xu, (2160, 3840), interp=_abi.HG_NEAREST))
    ref = O.hex_to_rect(xu[31, 2].double().cpu().numpy(), (2160, 3840), 0).reshape(2160, 3840)
    np.testing.assert_array_equal(yu[31, 2].double().cpu().numpy(), ref)


def test_unaligned_source_declines():
    """A source that is not 4-B aligned cannot be moved by LDS-DMA: the call still returns the
    general kernels' result (the kernel declines at launch)."""
    flat = _rand((2 * 3 * 40 * 96 + 1,), torch.bfloat16, 7)
    x = flat[1:].view(2, 3, 40, 96)
    assert x.data_ptr() % 4 == 2
    y = ops.hex_to_rect(x, (80, 192))
    torch.cuda.synchronize()
    _same_bits(y, _general(ops.hex_to_rect, x, (80, 192)))
