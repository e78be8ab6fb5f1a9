"""GPU parity of the row-streaming resample kernels (csrc/resample_stream.hip).

hg_rect_to_hex / hg_hex_to_rect route near-identity lattices (same-size resamples) to
k_r2h_stream / k_h2r_stream.  Those evaluate the general kernels' fp32 expressions in
the same order, so they are asserted BIT-IDENTICAL to the general LDS kernels
(selected with HYGRID_STREAM=0, read on every call), NaN/Inf positions included, and
within the north_star tolerance (rtol 1e-5, atol 1e-5*max|ref|) of the fp64 oracle
(oracle/hg_oracle.c, pinned to geometry_np.py:191-519 by tests/golden).
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
DT = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}


def _general(fn, *args, **kw):
    old = os.environ.get("HYGRID_STREAM")
    os.environ["HYGRID_STREAM"] = "0"
    try:
        out = fn(*args, **kw)
        torch.cuda.synchronize()
        return out
    finally:
        if old is None:
            del os.environ["HYGRID_STREAM"]
        else:
            os.environ["HYGRID_STREAM"] = old


def _same_bits(a, b):
    assert a.shape == b.shape and a.dtype == b.dtype
    ia = a.contiguous().view(torch.int16 if a.element_size() == 2 else torch.int32)
    ib = b.contiguous().view(torch.int16 if b.element_size() == 2 else torch.int32)
    nbad = int((ia != ib).sum().item())
    assert nbad == 0, f"{nbad} elements differ from the general kernel"


def _close(y, ref, rtol=1e-5):
    y = np.asarray(y, np.float64)
    scale = max(np.abs(ref).max(), 1e-30)
    np.testing.assert_allclose(y, ref, rtol=rtol, atol=rtol * scale)


# (h, w, h1, w1): same-size, ragged widths (not a multiple of the 256-column window),
# odd heights, band edges (128-row bands), and a near-identity r2h with h1 != h
SHAPES_R2H = [(7, 8, 7, 8), (16, 20, 16, 20), (33, 260, 33, 260), (129, 516, 129, 516),
              (130, 1000, 130, 1000), (255, 256, 255, 256), (64, 300, 65, 300),
              (90, 512, 91, 516)]
SHAPES_H2R = [(7, 8), (16, 20), (33, 260), (129, 516), (130, 1000), (255, 256), (2, 4)]
PAIRS = [("f32", "f32"), ("bf16", "bf16"), ("f16", "f16"), ("bf16", "f32"), ("f16", "f32"),
         ("f32", "bf16"), ("f32", "f16")]


@pytest.mark.parametrize("shape", SHAPES_R2H)
@pytest.mark.parametrize("pair", PAIRS)
def test_r2h_stream_bit_identical_to_general(shape, pair):
    h, w, h1, w1 = shape
    g = torch.Generator(device=DEV).manual_seed(h * 1000 + w)
    x = torch.rand((3, 2, h, w), generator=g, device=DEV).to(DT[pair[0]])
    y = ops.rect_to_hex(x, (h1, w1), out_dtype=DT[pair[1]])
    ref = _general(ops.rect_to_hex, x, (h1, w1), out_dtype=DT[pair[1]])
    _same_bits(y, ref)


@pytest.mark.parametrize("shape", SHAPES_H2R)
@pytest.mark.parametrize("pair", PAIRS)
def test_h2r_stream_bit_identical_to_general(shape, pair):
    h, w = shape
    g = torch.Generator(device=DEV).manual_seed(h * 1000 + w + 1)
    x = torch.rand((2, 3, h, w), generator=g, device=DEV).to(DT[pair[0]])
    y = ops.hex_to_rect(x, (h, w), out_dtype=DT[pair[1]])
    ref = _general(ops.hex_to_rect, x, (h, w), out_dtype=DT[pair[1]])
    _same_bits(y, ref)


@pytest.mark.parametrize("op", ["rect_to_hex", "hex_to_rect"])
def test_stream_nan_inf_positions_match_general(op):
    h, w = 40, 264
    g = torch.Generator(device=DEV).manual_seed(7)
    x = torch.rand((2, h, w), generator=g, device=DEV)
    x[0, 5, 17] = float("nan")
    x[0, 0, 0] = float("inf")
    x[1, h - 1, w - 1] = float("-inf")
    x[1, 20, 255] = float("nan")      # window edge column
    x[1, 21, 256] = float("nan")
    fn = getattr(ops, op)
    y = fn(x, (h, w))
    ref = _general(fn, x, (h, w))
    _same_bits(y, ref)


@pytest.mark.parametrize("shape", [(33, 260, 33, 260), (64, 300, 65, 300), (129, 516, 129, 516)])
def test_r2h_stream_vs_oracle(shape):
    h, w, h1, w1 = shape
    rng = np.random.default_rng(h + w)
    x = rng.random((2, h, w), dtype=np.float64).astype(np.float32)
    y = ops.rect_to_hex(torch.from_numpy(x).to(DEV), (h1, w1)).cpu().numpy()
    ref = O.rect_to_hex(x.astype(np.float64), (h1, w1), 1)
    _close(y, ref)


@pytest.mark.parametrize("shape", [(33, 260), (129, 516), (255, 256)])
def test_h2r_stream_vs_oracle(shape):
    h, w = shape
    rng = np.random.default_rng(h * w)
    x = rng.random((2, h, w), dtype=np.float64).astype(np.float32)
    y = ops.hex_to_rect(torch.from_numpy(x).to(DEV), (h, w)).cpu().numpy()
    ref = O.hex_to_rect(x.astype(np.float64), (h, w), 1)
    _close(y, ref)


def test_stream_at_4k_matches_general():
    """BASELINE size (4K, 2 images x 3 channels, bf16) through both kernels."""
    g = torch.Generator(device=DEV).manual_seed(2)
    x = torch.rand((2, 3, 2160, 3840), generator=g, device=DEV, dtype=torch.bfloat16)
    u = ops.rect_to_hex(x, (2160, 3840))
    _same_bits(u, _general(ops.rect_to_hex, x, (2160, 3840)))
    r = ops.hex_to_rect(u, (2160, 3840))
    _same_bits(r, _general(ops.hex_to_rect, u, (2160, 3840)))
