"""GPU parity of the wide-channel HexConv2d path (csrc/conv_mfma.hip: implicit GEMM on
v_mfma_f32_16x16x4_f32, dense radius 2 / stride 1 / dilation 1, O >= 16; C < 8 zero-padded) against
the fp64 oracle (oracle/hg_oracle.c, pinned to HexFrames.py:96-169 by
tests/golden/hexconv.npz) at the north_star fp32 tolerance (rtol 1e-5, atol 1e-5*max|ref|),
and against the generic LDS kernel (HYGRID_CONV_MFMA=0) for 16-bit outputs and the fused
HexConvModule epilogue."""
import os

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a HIP device", allow_module_level=True)

from HyGrid import ops  # noqa: E402

DEV = torch.device("cuda:0")


def _generic(fn, *args, **kw):
    old = os.environ.get("HYGRID_CONV_MFMA")
    os.environ["HYGRID_CONV_MFMA"] = "0"
    try:
        out = fn(*args, **kw)
        torch.cuda.synchronize()
        return out
    finally:
        if old is None:
            del os.environ["HYGRID_CONV_MFMA"]
        else:
            os.environ["HYGRID_CONV_MFMA"] = old


def _weights(O_, C, seed):
    g = torch.Generator().manual_seed(seed)
    bound = 1.0 / np.sqrt(7 * C)
    k = ((torch.rand((O_, C, 1, 7), generator=g) * 2 - 1) * bound).to(DEV)
    b = ((torch.rand((O_,), generator=g) * 2 - 1) * bound).to(DEV)
    return k, b


CASES = [  # (B, C, O, h, w)
    (2, 8, 16, 9, 10), (1, 16, 16, 33, 70), (1, 32, 64, 20, 130), (2, 64, 64, 17, 64),
    (1, 13, 20, 12, 21), (1, 24, 100, 11, 75), (1, 70, 33, 6, 9),
    # narrow inputs (round 6): a 3-channel stem, 1 and 5 channels (zero-padded chunk)
    (2, 3, 64, 20, 130), (1, 1, 16, 9, 10), (1, 5, 40, 14, 33),
]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("pad", [0, 1, 2])
@pytest.mark.parametrize("off", [0, 1])
def test_mfma_conv_fp32_vs_oracle(case, pad, off):
    B, C, O_, h, w = case
    k, b = _weights(O_, C, h * 13 + w + pad)
    rng = np.random.default_rng(h + w * 3 + off)
    x = rng.random((B, C, h, w)).astype(np.float32) - 0.5
    y = ops.hexconv2d(torch.from_numpy(x).to(DEV), k, b, off, 2, padding=pad,
                      out_dtype=torch.float32).cpu().numpy()
    ref = O.hexconv2d(x.astype(np.float64), k.cpu().double().numpy(),
                      b.cpu().double().numpy(), off, 2, padding=pad)
    scale = max(np.abs(ref).max(), 1e-30)
    np.testing.assert_allclose(y, ref, rtol=1e-5, atol=1e-5 * scale)


@pytest.mark.parametrize("mode", ["constant", "reflect", "replicate", "circular"])
def test_mfma_conv_pad_modes_vs_oracle(mode):
    B, C, O_, h, w = 1, 16, 32, 14, 40
    k, b = _weights(O_, C, 7)
    rng = np.random.default_rng(5)
    x = rng.random((B, C, h, w)).astype(np.float32)
    pv = 0.3 if mode == "constant" else 0.0
    y = ops.hexconv2d(torch.from_numpy(x).to(DEV), k, b, 0, 2, padding=1, padding_mode=mode,
                      padding_value=pv, out_dtype=torch.float32).cpu().numpy()
    ref = O.hexconv2d(x.astype(np.float64), k.cpu().double().numpy(), b.cpu().double().numpy(),
                      0, 2, padding=1, padding_mode=mode, padding_value=pv)
    scale = max(np.abs(ref).max(), 1e-30)
    np.testing.assert_allclose(y, ref, rtol=1e-5, atol=1e-5 * scale)


@pytest.mark.parametrize("dt_in,dt_out", [(torch.bfloat16, torch.bfloat16),
                                          (torch.bfloat16, torch.float32),
                                          (torch.float16, torch.float16),
                                          (torch.float32, torch.bfloat16)])
def test_mfma_conv_16bit_vs_generic(dt_in, dt_out):
    B, C, O_, h, w = 2, 32, 48, 30, 100
    k, b = _weights(O_, C, 3)
    g = torch.Generator(device=DEV).manual_seed(9)
    x = (torch.rand((B, C, h, w), generator=g, device=DEV) - 0.5).to(dt_in)
    y = ops.hexconv2d(x, k, b, 0, 2, padding=1, out_dtype=dt_out)
    ref = _generic(ops.hexconv2d, x, k, b, 0, 2, padding=1, out_dtype=dt_out)
    ulp = {torch.bfloat16: 2.0 ** -8, torch.float16: 2.0 ** -11, torch.float32: 1e-5}[dt_out]
    scale = float(ref.float().abs().max())
    torch.testing.assert_close(y.float(), ref.float(), rtol=ulp, atol=ulp * scale)


@pytest.mark.parametrize("act", ["ReLU", "LeakyReLU", "Sigmoid"])
def test_mfma_hexconvmodule_epilogue_vs_generic(act):
    """HexConvModule's fused conv + eval BatchNorm + activation on the MFMA kernel."""
    from HyGrid.HexModules import HexConvModule
    torch.manual_seed(2)
    m = HexConvModule(16, 32, 0, 2, padding=1, norm_cfg=dict(type="BN"),
                      act_cfg=dict(type=act)).to(DEV).eval()
    with torch.no_grad():
        m.norm.running_mean.uniform_(-0.2, 0.2)
        m.norm.running_var.uniform_(0.5, 1.5)
        x = torch.rand((2, 16, 24, 50), device=DEV)
        y = m(x)
        ref = _generic(m, x)
    torch.testing.assert_close(y, ref, rtol=1e-5, atol=1e-5 * float(ref.abs().max()))


@pytest.mark.parametrize("shape", [(2, 3, 64, 24, 100), (1, 3, 32, 17, 37), (1, 16, 48, 9, 38)])
@pytest.mark.parametrize("dt_in", [torch.bfloat16, torch.float16])
def test_mfma_column_store_epilogue_vs_generic(shape, dt_in):
    """16-bit outputs take the [column][channel] accumulator and its 8-B column stores (round 6,
    CM_TD), widths that are not a multiple of 4 its scalar stores; with the fused BN-affine +
    LeakyReLU epilogue on both kernels (bf16 in: the DMA kernel, f16 in: the f32-MFMA kernel)."""
    B, C, O_, h, w = shape
    k, b = _weights(O_, C, 21 + w)
    g = torch.Generator(device=DEV).manual_seed(w)
    x = (torch.rand((B, C, h, w), generator=g, device=DEV) - 0.5).to(dt_in)
    scale = torch.rand((O_,), generator=g, device=DEV) + 0.5
    shift = torch.rand((O_,), generator=g, device=DEV) - 0.5
    epi = (scale, shift, 2, 0.1)          # hg_act 2: LeakyReLU
    for od in (dt_in, torch.float32):
        y = ops.hexconv2d(x, k, b, 0, 2, padding=1, out_dtype=od, epilogue=epi)
        ref = _generic(ops.hexconv2d, x, k, b, 0, 2, padding=1, out_dtype=od, epilogue=epi)
        ulp = {torch.bfloat16: 2.0 ** -8, torch.float16: 2.0 ** -11, torch.float32: 1e-5}[od]
        sc = float(ref.float().abs().max())
        torch.testing.assert_close(y.float(), ref.float(), rtol=ulp, atol=ulp * sc)


def test_mfma_conv_nan_positions_match_generic():
    B, C, O_, h, w = 1, 16, 16, 20, 70
    k, b = _weights(O_, C, 4)
    x = torch.rand((B, C, h, w), device=DEV)
    x[0, 3, 0, 5] = float("nan")
    x[0, 7, 19, 69] = float("inf")
    y = ops.hexconv2d(x, k, b, 1, 2, padding=1, out_dtype=torch.float32)
    ref = _generic(ops.hexconv2d, x, k, b, 1, 2, padding=1, out_dtype=torch.float32)
    assert torch.equal(torch.isnan(y), torch.isnan(ref))
    assert torch.equal(torch.isinf(y), torch.isinf(ref))


# ---- bf16 inputs: the split-weight bf16 MFMA kernel (k_hexconv_mfma_bf16) ----------------

def _bf16_input(shape, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return (torch.rand(shape, generator=g, device=DEV) - 0.5).to(torch.bfloat16)


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("pad", [0, 1, 2])
@pytest.mark.parametrize("off", [0, 1])
def test_mfma_bf16_conv_vs_oracle(case, pad, off):
    """bf16 input (exact in fp64), fp32 output: W = Wh + Wm + Wl in bf16 parts on
    v_mfma_f32_16x16x32_bf16 must keep the fp32 kernel's 1e-5 against the fp64 oracle."""
    B, C, O_, h, w = case
    k, b = _weights(O_, C, h * 13 + w + pad)
    x = _bf16_input((B, C, h, w), h + w * 3 + off)
    y = ops.hexconv2d(x, k, b, off, 2, padding=pad, out_dtype=torch.float32).cpu().numpy()
    ref = O.hexconv2d(x.double().cpu().numpy(), k.cpu().double().numpy(),
                      b.cpu().double().numpy(), off, 2, padding=pad)
    scale = max(np.abs(ref).max(), 1e-30)
    np.testing.assert_allclose(y, ref, rtol=1e-5, atol=1e-5 * scale)


@pytest.mark.parametrize("mode,pv", [("constant", 0.5), ("constant", 0.3), ("reflect", 0.0),
                                     ("replicate", 0.0), ("circular", 0.0)])
def test_mfma_bf16_pad_modes_vs_oracle(mode, pv):
    """A pad value that is not a bf16 (0.3) keeps the f32 kernel; either way 1e-5."""
    B, C, O_, h, w = 1, 16, 32, 14, 40
    k, b = _weights(O_, C, 7)
    x = _bf16_input((B, C, h, w), 5)
    y = ops.hexconv2d(x, k, b, 0, 2, padding=1, padding_mode=mode, padding_value=pv,
                      out_dtype=torch.float32).cpu().numpy()
    ref = O.hexconv2d(x.double().cpu().numpy(), k.cpu().double().numpy(),
                      b.cpu().double().numpy(), 0, 2, padding=1, padding_mode=mode,
                      padding_value=pv)
    scale = max(np.abs(ref).max(), 1e-30)
    np.testing.assert_allclose(y, ref, rtol=1e-5, atol=1e-5 * scale)


def test_mfma_bf16_vs_f32_kernel_and_weight_split():
    """The bf16 kernel against the f32 MFMA kernel (HYGRID_CONV_MFMA_BF16=0) at the wide
    bench shape's channel counts, with weights whose bf16 split needs all three parts."""
    B, C, O_, h, w = 1, 64, 64, 24, 150
    g = torch.Generator().manual_seed(11)
    k = ((torch.rand((O_, C, 1, 7), generator=g) - 0.5) * 0.3 + 1e-3).to(DEV)
    b = (torch.rand((O_,), generator=g) - 0.5).to(DEV)
    x = _bf16_input((B, C, h, w), 3)
    y = ops.hexconv2d(x, k, b, 0, 2, padding=1, out_dtype=torch.float32)
    old = os.environ.get("HYGRID_CONV_MFMA_BF16")
    os.environ["HYGRID_CONV_MFMA_BF16"] = "0"
    try:
        ref = ops.hexconv2d(x, k, b, 0, 2, padding=1, out_dtype=torch.float32)
        torch.cuda.synchronize()
    finally:
        if old is None:
            del os.environ["HYGRID_CONV_MFMA_BF16"]
        else:
            os.environ["HYGRID_CONV_MFMA_BF16"] = old
    assert not torch.equal(y, ref)   # a different kernel (summation order) ran
    torch.testing.assert_close(y, ref, rtol=1e-5, atol=1e-5 * float(ref.abs().max()))


def test_mfma_bf16_nan_positions_match_generic():
    B, C, O_, h, w = 1, 16, 16, 20, 70
    k, b = _weights(O_, C, 4)
    x = _bf16_input((B, C, h, w), 8)
    x[0, 3, 0, 5] = float("nan")
    x[0, 7, 19, 69] = float("inf")
    x[0, 9, 10, 30] = float("-inf")
    y = ops.hexconv2d(x, k, b, 1, 2, padding=1, out_dtype=torch.float32)
    ref = _generic(ops.hexconv2d, x, k, b, 1, 2, padding=1, out_dtype=torch.float32)
    # the same non-finite positions; an infinite input times a weight part that is exactly 0
    # (a weight with fewer than 17 significant bits) is NaN where one fp32 product is +-Inf
    assert torch.equal(~torch.isfinite(y), ~torch.isfinite(ref))
    assert torch.equal(torch.isnan(ref) & ~torch.isnan(y), torch.zeros_like(y, dtype=torch.bool))
    fin = torch.isfinite(ref)
    torch.testing.assert_close(y[fin], ref[fin], rtol=1e-5, atol=1e-5 * float(ref[fin].abs().max()))


def test_mfma_bf16_exact_weights_keep_inf():
    """Weights exactly representable in bf16 (Gaussian-style taps 1/4, 1/8, ..., and zeros):
    every chunk's second and third weight parts are 0, so the kernel runs only the first
    part's MFMAs (conv_mfma.hip: nparts) and an infinite input times a weight stays +-Inf,
    exactly as the generic kernel's fp32 products: the same NaN and Inf positions and signs,
    finite outputs within 1e-5."""
    B, C, O_, h, w = 1, 16, 16, 20, 70
    g = torch.Generator().manual_seed(21)
    k = (torch.randint(-4, 5, (O_, C, 1, 7), generator=g).float() / 8.0).to(DEV)
    b = (torch.randint(-4, 5, (O_,), generator=g).float() / 4.0).to(DEV)
    x = _bf16_input((B, C, h, w), 9)
    x[0, 3, 0, 5] = float("nan")
    x[0, 7, 19, 69] = float("inf")
    x[0, 9, 10, 30] = float("-inf")
    y = ops.hexconv2d(x, k, b, 1, 2, padding=1, out_dtype=torch.float32)
    ref = _generic(ops.hexconv2d, x, k, b, 1, 2, padding=1, out_dtype=torch.float32)
    assert torch.equal(torch.isnan(y), torch.isnan(ref))
    assert torch.equal(torch.isinf(y), torch.isinf(ref))
    assert torch.equal(y[torch.isinf(ref)], ref[torch.isinf(ref)])
    fin = torch.isfinite(ref)
    torch.testing.assert_close(y[fin], ref[fin], rtol=1e-5, atol=1e-5 * float(ref[fin].abs().max()))


# ---- bf16 inputs staged by LDS-DMA (k_hexconv_mfma_bf16d, round 4) ------------------------

def _with_env(name, value, fn, *args, **kw):
    old = os.environ.get(name)
    os.environ[name] = value
    try:
        out = fn(*args, **kw)
        torch.cuda.synchronize()
        return out
    finally:
        if old is None:
            del os.environ[name]
        else:
            os.environ[name] = old


DMA_CASES = [  # (B, C, O, h, w): interior tiles (DMA-staged P) and border tiles in each
    (1, 64, 64, 40, 300), (2, 13, 20, 30, 260), (1, 70, 33, 17, 202), (1, 24, 100, 21, 196),
    (1, 8, 16, 12, 140), (1, 3, 64, 30, 260), (2, 1, 16, 12, 140)]


@pytest.mark.parametrize("case", DMA_CASES)
@pytest.mark.parametrize("pad", [0, 1, 2])
@pytest.mark.parametrize("off", [0, 1])
def test_mfma_bf16_dma_bit_identical_to_register_staging(case, pad, off):
    """The LDS-DMA-staged kernel issues the register-staged kernel's MFMAs on the same
    fragments in the same order: outputs bit-identical (HYGRID_CONV_DMA=0 selects the latter),
    bf16 and fp32 outputs, partial channel chunks and output-channel tiles included."""
    B, C, O_, h, w = case
    k, b = _weights(O_, C, h * 7 + w + pad)
    x = _bf16_input((B, C, h, w), h + w + off)
    for od in (torch.float32, torch.bfloat16):
        y = ops.hexconv2d(x, k, b, off, 2, padding=pad, out_dtype=od)
        torch.cuda.synchronize()
        ref = _with_env("HYGRID_CONV_DMA", "0", ops.hexconv2d, x, k, b, off, 2, padding=pad, out_dtype=od)
        assert torch.equal(y.view(torch.int16 if od == torch.bfloat16 else torch.int32),
                           ref.view(torch.int16 if od == torch.bfloat16 else torch.int32))


@pytest.mark.parametrize("case", DMA_CASES)
@pytest.mark.parametrize("env", [("HYGRID_CONV_NT", "2")])
def test_mfma_bf16_dma_weight_buffering_and_tiles_bit_identical(case, env):
    """Two output-channel tiles per workgroup (HYGRID_CONV_NT=2) compute each output's sum in
    the same order as four: bit-identical outputs.  (Round 5's double-buffered weight chunks and
    3-column-tile build, both slower, were removed in round 6.)"""
    B, C, O_, h, w = case
    k, b = _weights(O_, C, h * 3 + w)
    x = _bf16_input((B, C, h, w), h + 2 * w)
    for od in (torch.float32, torch.bfloat16):
        y = ops.hexconv2d(x, k, b, 0, 2, padding=1, out_dtype=od)
        torch.cuda.synchronize()
        ref = _with_env(env[0], env[1], ops.hexconv2d, x, k, b, 0, 2, padding=1, out_dtype=od)
        assert torch.equal(y.view(torch.int16 if od == torch.bfloat16 else torch.int32),
                           ref.view(torch.int16 if od == torch.bfloat16 else torch.int32))


def test_mfma_bf16_dma_vs_oracle_and_unaligned():
    """1e-5 against the fp64 oracle on a shape with many interior tiles; a source that is
    2-B aligned only (odd element offset) keeps the register staging, same results."""
    B, C, O_, h, w = 1, 32, 48, 36, 330
    k, b = _weights(O_, C, 77)
    x = _bf16_input((B, C, h, w), 31)
    y = ops.hexconv2d(x, k, b, 0, 2, padding=1, out_dtype=torch.float32)
    ref = O.hexconv2d(x.double().cpu().numpy(), k.cpu().double().numpy(),
                      b.cpu().double().numpy(), 0, 2, padding=1)
    scale = max(np.abs(ref).max(), 1e-30)
    np.testing.assert_allclose(y.cpu().numpy(), ref, rtol=1e-5, atol=1e-5 * scale)
    flat = torch.empty(B * C * h * w + 1, device=DEV, dtype=torch.bfloat16)
    xu = flat[1:].view(B, C, h, w)
    xu.copy_(x)
    yu = ops.hexconv2d(xu, k, b, 0, 2, padding=1, out_dtype=torch.float32)
    torch.cuda.synchronize()
    assert torch.equal(yu, y)
