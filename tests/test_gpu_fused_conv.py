"""GPU parity of HexConv2d on the two-column streaming kernel (csrc/fused_conv.hip).

hg_hexconv2d routes radius 2 / stride 1 / padding 1 / pad value 0 / no-epilogue calls
with even widths and C/O/groups in {3/3/1, 3/3/3, 1/1/1} to k_fused<..., MD=1>.  Its
sums run in a different order from the other conv kernels, so it is checked against
the fp64 oracle (oracle/hg_oracle.c, pinned to HexFrames.py:96-169 by
tests/golden/hexconv.npz) at the north_star tolerance for fp32 (rtol 1e-5,
atol 1e-5*max|ref|), and for 16-bit outputs against the register-streaming kernel
(HYGRID_FCONV=0) within one output rounding.
"""
import os

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - collected only with -m gpu
    pytest.skip("needs a HIP device", allow_module_level=True)

from HyGrid import ops  # noqa: E402

DEV = torch.device("cuda:0")


def _other_kernel(fn, *args, **kw):
    old = os.environ.get("HYGRID_FCONV")
    os.environ["HYGRID_FCONV"] = "0"
    try:
        out = fn(*args, **kw)
        torch.cuda.synchronize()
        return out
    finally:
        if old is None:
            del os.environ["HYGRID_FCONV"]
        else:
            os.environ["HYGRID_FCONV"] = old


def _weights(O_, cg, seed):
    g = torch.Generator().manual_seed(seed)
    k = (torch.rand((O_, cg, 1, 7), generator=g) - 0.5).to(DEV)
    b = (torch.rand((O_,), generator=g) - 0.5).to(DEV)
    return k, b


# (B, C, O, groups, h, w): ragged widths vs the 120-column window, odd heights, band
# edges (126-row bands), tiny rasters
CASES = [(2, 3, 3, 1, 7, 8), (1, 3, 3, 1, 9, 10), (2, 3, 3, 1, 127, 242), (1, 3, 3, 3, 130, 250),
         (3, 1, 1, 1, 33, 122), (1, 3, 3, 1, 253, 360), (1, 1, 1, 1, 1, 2), (1, 3, 3, 3, 2, 4)]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("off", [0, 1])
@pytest.mark.parametrize("bias", [True, False])
def test_fused_conv_fp32_vs_oracle(case, off, bias):
    B, C, O_, G, h, w = case
    k, b = _weights(O_, C // G, h * 31 + w + off)
    if not bias:
        b = None
    rng = np.random.default_rng(h + 7 * w)
    x = rng.random((B, C, h, w), dtype=np.float64).astype(np.float32)
    y = ops.hexconv2d(torch.from_numpy(x).to(DEV), k, b, off, 2, padding=1, groups=G,
                      out_dtype=torch.float32).cpu().numpy()
    ref = O.hexconv2d(x.astype(np.float64), k.cpu().double().numpy(),
                      None if b is None else b.cpu().double().numpy(), off, 2, padding=1,
                      groups=G)
    scale = max(np.abs(ref).max(), 1e-30)
    np.testing.assert_allclose(y, ref, rtol=1e-5, atol=1e-5 * scale)


@pytest.mark.parametrize("dt_in,dt_out", [(torch.bfloat16, torch.bfloat16),
                                          (torch.bfloat16, torch.float32),
                                          (torch.float16, torch.float16),
                                          (torch.float16, torch.float32)])
@pytest.mark.parametrize("off", [0, 1])
def test_fused_conv_16bit_vs_stream_kernel(dt_in, dt_out, off):
    B, C, O_, h, w = 2, 3, 3, 130, 250
    k, b = _weights(O_, C, 5 + off)
    g = torch.Generator(device=DEV).manual_seed(11)
    x = torch.rand((B, C, h, w), generator=g, device=DEV).to(dt_in)
    y = ops.hexconv2d(x, k, b, off, 2, padding=1, out_dtype=dt_out)
    ref = _other_kernel(ops.hexconv2d, x, k, b, off, 2, padding=1, out_dtype=dt_out)
    ulp = {torch.bfloat16: 2.0 ** -8, torch.float16: 2.0 ** -11, torch.float32: 1e-5}[dt_out]
    scale = float(ref.float().abs().max())
    torch.testing.assert_close(y.float(), ref.float(), rtol=ulp, atol=ulp * scale)


def test_fused_conv_4k_batch_matches_stream_kernel():
    """BASELINE size (4K RGB, bf16 in, fp32 out) against the register-streaming kernel."""
    k, b = _weights(3, 3, 3)
    g = torch.Generator(device=DEV).manual_seed(2)
    x = torch.rand((2, 3, 2160, 3840), generator=g, device=DEV, dtype=torch.bfloat16)
    y = ops.hexconv2d(x, k, b, 0, 2, padding=1, out_dtype=torch.float32)
    ref = _other_kernel(ops.hexconv2d, x, k, b, 0, 2, padding=1, out_dtype=torch.float32)
    scale = float(ref.abs().max())
    torch.testing.assert_close(y, ref, rtol=1e-5, atol=1e-5 * scale)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("off", [0, 1])
def test_fused_conv_nan_inf_positions_match_stream_kernel(dt, off):
    """Non-finite inputs on the raster border, at the 120-column window edges and at the
    126-row band edges: MD 1 builds its padding by selecting zeros (fused_kernel.h), so a
    boundary row's or column's NaN must reach exactly the outputs whose taps read it,
    as in the register-streaming kernel (HYGRID_FCONV=0)."""
    B, C, h, w = 2, 3, 260, 372
    k, b = _weights(3, 3, 17 + off)
    g = torch.Generator(device=DEV).manual_seed(13)
    x = torch.rand((B, C, h, w), generator=g, device=DEV)
    nan, inf = float("nan"), float("inf")
    x[0, 0, 0, :] = nan                   # first row
    x[0, 1, h - 1, 5] = inf               # last row
    x[0, 2, 40, 0] = -inf                 # first column
    x[1, 0, 77, w - 1] = nan              # last column
    for c0 in (119, 120, 239, 240, 359, 360):   # window edges (owned columns 0..119, ...)
        x[1, 1, 30 + c0 % 7, c0] = nan
    for r0 in (125, 126, 251, 252):       # band edges (126-row bands)
        x[1, 2, r0, 61 + r0 % 5] = inf
    x = x.to(dt)
    y = ops.hexconv2d(x, k, b, off, 2, padding=1, out_dtype=torch.float32)
    ref = _other_kernel(ops.hexconv2d, x, k, b, off, 2, padding=1, out_dtype=torch.float32)
    assert torch.equal(torch.isnan(y), torch.isnan(ref))
    assert torch.equal(torch.isinf(y), torch.isinf(ref))
    assert torch.equal(torch.sign(y[torch.isinf(y)]), torch.sign(ref[torch.isinf(ref)]))
    fin = torch.isfinite(ref)
    scale = float(ref[fin].abs().max())
    torch.testing.assert_close(y[fin], ref[fin], rtol=1e-5, atol=1e-5 * scale)


# (Round 5's four-column HexConv2d kernel, k_fused4 MD 1, opt-in and measured 1.7 % slower
# than k_fused MD 1, was removed in round 6: layout modes 7 and 8 are gone.)


def test_removed_layout_modes_are_invalid():
    from HyGrid import _abi
    for md in (7, 8):
        with pytest.raises(ValueError):
            _abi.fused_layout(md)
