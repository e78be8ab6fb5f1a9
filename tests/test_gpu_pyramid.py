"""BASELINE config 5 as a chain: the 8K fp16 hex Gaussian pyramid the bench times
(rect->hex bilinear at full size, then 3 x [depthwise HexConv2d(3,3,0,2,padding=1,
groups=3) with taps [1,1,1,6,1,1,1]/12 -> hexresize to (h//2, w//2) linear]) against the
fp64 oracle chain (geometry_np.py:358-519, HexFrames.py:96-169, geometry_np.py:520-681).

Every stage stores fp16, so the oracle chain rounds to fp16 after each stage too (the
same storage points); the remaining differences are one fp16 rounding per stored stage
that the fp32 arithmetic of the kernels moves across a rounding boundary.  Tolerance:
7 stored stages x half an fp16 ulp at the top of the range (2^-11), i.e.
atol = 7 * 2^-11 * max|ref|; the unrounded fp64 chain is checked at 2^-8."""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a HIP device", allow_module_level=True)

from HyGrid import _abi, ops  # noqa: E402
from HyGrid.HexFrames import HexConv2d  # noqa: E402
from HyGrid.pipeline import hex_pyramid  # noqa: E402

DEV = torch.device("cuda:0")
TAPS = [1, 1, 1, 6, 1, 1, 1]


def gaussian_conv():
    conv = HexConv2d(3, 3, 0, 2, padding=1, groups=3, bias=False).to(DEV)
    with torch.no_grad():
        conv.kernel.copy_(torch.tensor(TAPS, dtype=torch.float32, device=DEV).div_(12)
                          .expand_as(conv.kernel))
    conv.out_dtype = torch.float16
    return conv


def gpu_chain(x, conv, levels=3):
    """The bench's unfused pyramid (bench.py run_pyramid), level outputs returned."""
    H, W = x.shape[-2:]
    with torch.no_grad():
        hx = ops.rect_to_hex(x, (H, W), out_dtype=torch.float16)
        outs = []
        h_, w_ = H, W
        for _ in range(levels):
            hx = conv(hx)
            h_, w_ = h_ // 2, w_ // 2
            hx = ops.hexresize(hx, (h_, w_), out_dtype=torch.float16)
            outs.append(hx)
    return outs


def oracle_chain(x, kern, levels=3, f16=True):
    rnd = (lambda a: a.astype(np.float16).astype(np.float64)) if f16 else (lambda a: a)
    H, W = x.shape[-2:]
    hx = rnd(O.rect_to_hex(x, (H, W), 1))
    outs = []
    h_, w_ = H, W
    for _ in range(levels):
        hx = rnd(O.hexconv2d(hx, kern, None, 0, 2, padding=1, groups=3))
        h_, w_ = h_ // 2, w_ // 2
        hx = rnd(O.hexresize(hx, (h_, w_), 1))
        outs.append(hx)
    return outs


def check(outs, refs, atol_ulps):
    for lv, (y, ref) in enumerate(zip(outs, refs)):
        y = y.double().cpu().numpy().reshape(ref.shape)
        scale = np.abs(ref).max()
        err = np.abs(y - ref).max()
        assert err <= atol_ulps * scale, f"level {lv}: max err {err:.3e} > {atol_ulps * scale:.3e}"


@pytest.mark.parametrize("H,W", [(540, 960), (136, 250), (70, 90)])
def test_pyramid_chain_vs_oracle(H, W):
    conv = gaussian_conv()
    gen = torch.Generator(device=DEV).manual_seed(5)
    x = torch.rand((2, 3, H, W), generator=gen, device=DEV, dtype=torch.float16)
    outs = gpu_chain(x, conv)
    xd = x.double().cpu().numpy()
    kern = conv.kernel.detach().cpu().numpy()
    check(outs, [r.reshape(o.shape) for r, o in zip(oracle_chain(xd, kern), outs)], 7 * 2 ** -11)
    check(outs, [r.reshape(o.shape) for r, o in zip(oracle_chain(xd, kern, f16=False), outs)],
          2 ** -8)


def test_pyramid_8k_full_image_vs_oracle():
    """One full 4320x7680 RGB image through all three levels (config 5's geometry)."""
    conv = gaussian_conv()
    gen = torch.Generator(device=DEV).manual_seed(5)
    x = torch.rand((1, 3, 4320, 7680), generator=gen, device=DEV, dtype=torch.float16)
    outs = gpu_chain(x, conv)
    assert [tuple(o.shape) for o in outs] == [(1, 3, 2160, 3840), (1, 3, 1080, 1920),
                                              (1, 3, 540, 960)]
    xd = x.double().cpu().numpy()
    refs = oracle_chain(xd, conv.kernel.detach().cpu().numpy())
    check(outs, [r.reshape(o.shape) for r, o in zip(refs, outs)], 7 * 2 ** -11)


def oracle_levels(x, kern, levels=3):
    """The fused pyramid's storage points: rect -> hex -> conv -> hexresize in fp64 with no
    rounding inside a level (the kernels keep fp32 intermediates on chip), one fp16
    rounding per stored level."""
    rnd = lambda a: a.astype(np.float16).astype(np.float64)  # noqa: E731
    H, W = x.shape[-2:]
    cur = O.rect_to_hex(x, (H, W), 1)
    outs = []
    h_, w_ = H, W
    for _ in range(levels):
        h_, w_ = h_ // 2, w_ // 2
        cur = rnd(O.hexresize(O.hexconv2d(cur, kern, None, 0, 2, padding=1, groups=3),
                              (h_, w_), 1))
        outs.append(cur)
    return outs


def level_kernel(x, size, off=0, from_rect=False, out_dtype=None):
    """hg_hex_pyramid_level_kernel for this call: the HG_PYR_* kernel that would run, or a
    negative status (HG_EUNSUP when HYGRID_PYR_KERNEL excludes every kernel that could)."""
    B, C, h, w = x.shape
    y_dt = out_dtype or (x.dtype if x.dtype in (torch.float16, torch.bfloat16) else torch.float32)
    return _abi.lib().hg_hex_pyramid_level_kernel(
        _abi.dtype_code(x.dtype), _abi.dtype_code(y_dt), B, C, h, w, size[0], size[1], off,
        int(bool(from_rect)))


def run_level_on(kernel, monkeypatch, x, taps, bias, size, off=0, from_rect=False,
                 out_dtype=None):
    """One hex_pyramid_level call restricted to `kernel` ("fused" | "stream" | "lds",
    HYGRID_PYR_KERNEL); returns (HG_PYR_* that ran, output), or (status, None) when that
    kernel declines the call."""
    monkeypatch.setenv("HYGRID_PYR_KERNEL", kernel)
    try:
        k = level_kernel(x, size, off, from_rect, out_dtype)
        y = ops.hex_pyramid_level(x, taps, bias, size, off, from_rect=from_rect, out_dtype=out_dtype)
    finally:
        monkeypatch.delenv("HYGRID_PYR_KERNEL")
    assert (k < 0) == (y is None), (kernel, k)
    return k, y


def fused_levels_only(x, conv, monkeypatch):
    """hex_pyramid's levels restricted to the fused row walk (HYGRID_PYR_KERNEL=fused; level
    0 k_fused MD 3 from the rect image, levels 1-2 MD 4 / MD 5 from the hex image), each level
    asserted to be that kernel (hg_hex_pyramid_level_kernel)."""
    H, W = x.shape[-2:]
    cur, outs, h_, w_ = x, [], H, W
    with torch.no_grad():
        for lv in range(3):
            h_, w_ = h_ // 2, w_ // 2
            k, y = run_level_on("fused", monkeypatch, cur, conv.kernel, None, (h_, w_), 0,
                                from_rect=(lv == 0), out_dtype=torch.float16)
            assert k in (_abi.HG_PYR_FUSED, _abi.HG_PYR_FUSED_SHORT), f"level {lv}: kernel {k}"
            outs.append(y)
            cur = y
    return outs


def test_hex_pyramid_8k_fused_full_size(monkeypatch):
    """The bench's config-5 path at full size: hex_pyramid on one 4320x7680 fp16 RGB image
    (level 0 = k_fused MD 3 from the rect image, levels 1-2 MD 4 / MD 5 from the hex image)
    against the oracle with fp64 intermediates and one fp16 rounding per stored level; the
    fused kernel is asserted to be what ran, and hex_pyramid (no restriction) equals it bit
    for bit.
    Tolerance: one fp16 rounding per stored level plus fp32 arithmetic, 3 * 2^-11 of max|ref|."""
    conv = gaussian_conv()
    gen = torch.Generator(device=DEV).manual_seed(5)
    x = torch.rand((1, 3, 4320, 7680), generator=gen, device=DEV, dtype=torch.float16)
    outs = fused_levels_only(x, conv, monkeypatch)
    with torch.no_grad():
        entry = hex_pyramid(x, conv, levels=3)
    for a, b in zip(entry, outs):
        assert torch.equal(a, b)
    refs = oracle_levels(x.double().cpu().numpy(), conv.kernel.detach().cpu().numpy())
    check(outs, [r.reshape(o.shape) for r, o in zip(refs, outs)], 3 * 2 ** -11)


def test_hex_pyramid_8k_batch8_first_last(monkeypatch):
    """The bench's own launch shape (8 x 3 x 4320 x 7680 fp16, one launch per level): the
    first and the last image against the oracle (32-bit offset / descriptor range errors at
    the end of the batch would show here), and every image equals its single-image launch."""
    conv = gaussian_conv()
    gen = torch.Generator(device=DEV).manual_seed(8)
    x = torch.rand((8, 3, 4320, 7680), generator=gen, device=DEV, dtype=torch.float16)
    outs = fused_levels_only(x, conv, monkeypatch)
    assert [tuple(o.shape) for o in outs] == [(8, 3, 2160, 3840), (8, 3, 1080, 1920),
                                              (8, 3, 540, 960)]
    kern = conv.kernel.detach().cpu().numpy()
    for i in (0, 7):
        refs = oracle_levels(x[i:i + 1].double().cpu().numpy(), kern)
        check([o[i:i + 1] for o in outs], [r.reshape(o[i:i + 1].shape) for r, o in zip(refs, outs)],
              3 * 2 ** -11)
        single = fused_levels_only(x[i:i + 1], conv, monkeypatch)
        for a, b in zip(single, outs):
            assert torch.equal(a[0], b[i])


def test_pyramid_level_out_slices():
    """hex_pyramid_level(out=) writes into slices of one batch output (round 6) the same bits
    as separate calls, and rejects a wrong out."""
    conv = gaussian_conv()
    gen = torch.Generator(device=DEV).manual_seed(21)
    x = torch.rand((4, 3, 272, 480), generator=gen, device=DEV, dtype=torch.float16)
    with torch.no_grad():
        ref = ops.hex_pyramid_level(x, conv.kernel, None, (136, 240), 0, from_rect=True,
                                    out_dtype=torch.float16)
        out = torch.full((4, 3, 136, 240), float("nan"), device=DEV, dtype=torch.float16)
        for s0 in (0, 2):
            y = ops.hex_pyramid_level(x[s0:s0 + 2], conv.kernel, None, (136, 240), 0,
                                      from_rect=True, out_dtype=torch.float16, out=out[s0:s0 + 2])
            assert y.data_ptr() == out[s0:s0 + 2].data_ptr()
        with pytest.raises(ValueError):
            ops.hex_pyramid_level(x, conv.kernel, None, (136, 240), 0, from_rect=True,
                                  out_dtype=torch.float16, out=out[:, :, :, :120])
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


@pytest.mark.parametrize("H,W", [(540, 960), (136, 250)])
def test_hex_pyramid_entry_matches_chain(H, W):
    """HyGrid.pipeline.hex_pyramid (the bench's config-5 step) gives the operator chain's
    levels bit for bit, or within one fp16 rounding per stage where it fuses stages."""
    conv = gaussian_conv()
    gen = torch.Generator(device=DEV).manual_seed(7)
    x = torch.rand((2, 3, H, W), generator=gen, device=DEV, dtype=torch.float16)
    outs = gpu_chain(x, conv)
    with torch.no_grad():
        got = hex_pyramid(x, conv, levels=3)
    for a, b in zip(got, outs):
        assert a.shape == b.shape and a.dtype == b.dtype
        scale = b.double().abs().max().item()
        assert (a.double() - b.double()).abs().max().item() <= 7 * 2 ** -11 * scale


LEVEL_CASES = [  # (B, C, h, w, h1, w1)
    (2, 3, 64, 130, 32, 65), (1, 3, 37, 53, 18, 26), (1, 1, 200, 250, 100, 125),
    (2, 3, 33, 500, 16, 250), (1, 3, 17, 9, 8, 4), (1, 2, 70, 90, 35, 45), (1, 3, 40, 70, 40, 70),
]


@pytest.mark.parametrize("case", LEVEL_CASES)
@pytest.mark.parametrize("from_rect", [False, True])
@pytest.mark.parametrize("off", [0, 1])
def test_pyramid_level_fp32_vs_oracle(case, from_rect, off):
    """hg_hex_pyramid_level (fp32 in/out) against the oracle chain at rtol 1e-5: ragged
    tiles (16 x 62 outputs), odd sizes, upsampling-free sizes, 1-3 channels, with bias."""
    B, C, h, w, h1, w1 = case
    g = torch.Generator().manual_seed(h * 7 + w + off)
    taps = (torch.rand((C, 1, 1, 7), generator=g) - 0.3).to(DEV)
    bias = (torch.rand((C,), generator=g) - 0.5).to(DEV)
    x = torch.rand((B, C, h, w), generator=g).to(DEV)
    y = ops.hex_pyramid_level(x, taps, bias, (h1, w1), off, from_rect=from_rect,
                              out_dtype=torch.float32)
    assert y is not None
    xd = x.double().cpu().numpy()
    hx = O.rect_to_hex(xd, (h, w), 1) if from_rect else xd
    c = O.hexconv2d(hx, taps.cpu().double().numpy(), bias.cpu().double().numpy(), off, 2,
                    padding=1, groups=C)
    ref = O.hexresize(c, (h1, w1), 1)
    got = y.double().cpu().numpy()
    scale = max(np.abs(ref).max(), 1e-30)
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5 * scale)


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
def test_pyramid_level_16bit_and_nan(dt):
    """16-bit in/out within one output rounding of the fp64 chain; a NaN in the input
    reaches exactly the outputs whose taps read it (as in the operator chain)."""
    B, C, h, w = 1, 3, 96, 200
    g = torch.Generator().manual_seed(3)
    taps = (torch.rand((C, 1, 1, 7), generator=g) - 0.3).to(DEV)
    x = torch.rand((B, C, h, w), generator=g).to(DEV).to(dt)
    x[0, 1, 50, 100] = float("nan")
    y = ops.hex_pyramid_level(x, taps, None, (h // 2, w // 2), 0, from_rect=False)
    assert y is not None and y.dtype == dt
    with torch.no_grad():
        conv = HexConv2d(3, 3, 0, 2, padding=1, groups=3, bias=False).to(DEV)
        conv.kernel.copy_(taps)
        ref = ops.hexresize(conv(x.float()), (h // 2, w // 2), out_dtype=torch.float32)
    assert torch.equal(torch.isnan(y), torch.isnan(ref))
    fin = torch.isfinite(ref)
    ulp = 2.0 ** -8 if dt == torch.bfloat16 else 2.0 ** -11
    scale = float(ref[fin].abs().max())
    torch.testing.assert_close(y.float()[fin], ref[fin], rtol=ulp, atol=ulp * scale)


STREAM_CASES = [  # (B, C, h, w): 2x downsamples the row-streaming level kernel takes
    (2, 3, 64, 130), (1, 1, 200, 250), (2, 3, 34, 500), (1, 3, 10, 8), (1, 3, 540, 960),
    (1, 1, 122, 244),
]


@pytest.mark.parametrize("case", STREAM_CASES)
@pytest.mark.parametrize("off", [0, 1])
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("from_rect", [False, True])
def test_pyramid_level_kernels_vs_oracle(case, off, dt, from_rect, monkeypatch):
    """Every level kernel on the 2x downsamples the streaming ones take, each restricted with
    HYGRID_PYR_KERNEL and asserted to be what ran: k_fused MD 3 / 4 / 5, k_pyr_stream
    (pyramid_stream.hip) and the LDS-tiled k_pyr_level, each against the fp64 oracle chain
    within one output rounding of the fp32 result and against each other within two: ragged
    bands / windows, 1 and 3 channels, both tap classes, bias; from_rect: the level input made
    on the fly from the rect image (rect_to_hex, geometry_np.py:358-519, same size) against the
    oracle's r2h -> conv -> hexresize."""
    B, C, h, w = case
    h1, w1 = h // 2, w // 2
    g = torch.Generator().manual_seed(h * 3 + w + off)
    taps = (torch.rand((C, 1, 1, 7), generator=g) - 0.3).to(DEV)
    bias = (torch.rand((C,), generator=g) - 0.5).to(DEV)
    x = torch.rand((B, C, h, w), generator=g).to(DEV).to(dt)
    want = {"fused": (_abi.HG_PYR_FUSED, _abi.HG_PYR_FUSED_SHORT), "stream": (_abi.HG_PYR_STREAM,),
            "lds": (_abi.HG_PYR_LDS,)}
    ys = {}
    for name, kinds in want.items():
        k, y = run_level_on(name, monkeypatch, x, taps, bias, (h1, w1), off, from_rect)
        assert k in kinds, (name, k)
        assert y.dtype == dt
        ys[name] = y
    xd = x.double().cpu().numpy()
    hx = O.rect_to_hex(xd, (h, w), 1).reshape(xd.shape) if from_rect else xd
    c = O.hexconv2d(hx, taps.cpu().double().numpy(), bias.cpu().double().numpy(), off, 2,
                    padding=1, groups=C)
    ref = O.hexresize(c, (h1, w1), 1).reshape(B, C, h1, w1)
    ulp = 2.0 ** -8 if dt == torch.bfloat16 else 2.0 ** -11
    scale = float(np.abs(ref).max())
    for name, y in ys.items():
        np.testing.assert_allclose(y.double().cpu().numpy(), ref, rtol=ulp, atol=ulp * scale,
                                   err_msg=name)
    for name in ("stream", "lds"):
        torch.testing.assert_close(ys["fused"].float(), ys[name].float(), rtol=2 * ulp,
                                   atol=2 * ulp * scale)
    # the unrestricted call takes the fused kernel and gives its result bit for bit
    assert level_kernel(x, (h1, w1), off, from_rect) in want["fused"]
    assert torch.equal(ops.hex_pyramid_level(x, taps, bias, (h1, w1), off, from_rect=from_rect),
                       ys["fused"])


@pytest.mark.parametrize("dt", [torch.float32, torch.float16])
def test_pyramid_lds_overflow_is_an_error(dt, monkeypatch):
    """k_pyr_level's footprint overflow is a reported error, not a silent result: with a
    test-only tile cap of 4 Y rows (HYGRID_PYR_LDS_FORCE_CAP; the host bound is skipped) every
    tile overflows, the kernel raises the call's fault flag and hg_hex_pyramid_level returns
    HG_EOVERFLOW (ValueError here).  Without the cap the same call passes the host bound and
    matches the oracle."""
    B, C, h, w = 1, 3, 64, 130
    g = torch.Generator().manual_seed(11)
    taps = (torch.rand((C, 1, 1, 7), generator=g) - 0.3).to(DEV)
    x = torch.rand((B, C, h, w), generator=g).to(DEV).to(dt)
    monkeypatch.setenv("HYGRID_PYR_LDS_FORCE_CAP", "4")
    with pytest.raises(ValueError, match="overflow"):
        run_level_on("lds", monkeypatch, x, taps, None, (h // 2, w // 2))
    monkeypatch.delenv("HYGRID_PYR_LDS_FORCE_CAP")
    k, y = run_level_on("lds", monkeypatch, x, taps, None, (h // 2, w // 2),
                        out_dtype=torch.float32)
    assert k == _abi.HG_PYR_LDS
    c = O.hexconv2d(x.double().cpu().numpy(), taps.cpu().double().numpy(), None, 0, 2,
                    padding=1, groups=C)
    ref = O.hexresize(c, (h // 2, w // 2), 1).reshape(y.shape)
    tol = 2.0 ** -11 if dt == torch.float16 else 1e-5
    scale = float(np.abs(ref).max())
    np.testing.assert_allclose(y.double().cpu().numpy(), ref, rtol=tol, atol=tol * scale)


@pytest.mark.parametrize("case", STREAM_CASES + [(8, 3, 1080, 1920)])
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
def test_pyramid_level_short_bands_vs_oracle(case, dt, monkeypatch):
    """A level from a hex image on the fused row walk with 60-row bands (MD 4) and with the
    short bands small levels take (MD 5, HYGRID_PYR_SHORT=1), each asserted to be what ran:
    bit-identical to each other (a band split changes no output's arithmetic) and within one
    output rounding of the fp64 oracle chain.  (8, 3, 1080, 1920) is the bench's level 2 at
    full size."""
    B, C, h, w = case
    h1, w1 = h // 2, w // 2
    g = torch.Generator().manual_seed(h + 7 * w)
    taps = (torch.rand((C, 1, 1, 7), generator=g) - 0.3).to(DEV)
    bias = (torch.rand((C,), generator=g) - 0.5).to(DEV)
    x = torch.rand((B, C, h, w), generator=g).to(DEV).to(dt)
    outs = []
    for short, kind in (("0", _abi.HG_PYR_FUSED), ("1", _abi.HG_PYR_FUSED_SHORT)):
        monkeypatch.setenv("HYGRID_PYR_SHORT", short)
        k, y = run_level_on("fused", monkeypatch, x, taps, bias, (h1, w1), 1)
        assert k == kind
        outs.append(y)
    monkeypatch.delenv("HYGRID_PYR_SHORT")
    assert torch.equal(outs[0], outs[1])
    n = 1 if B * h * w > 1 << 22 else B          # full-size case: the first image
    xd = x[:n].double().cpu().numpy()
    c = O.hexconv2d(xd, taps.cpu().double().numpy(), bias.cpu().double().numpy(), 1, 2,
                    padding=1, groups=C)
    ref = O.hexresize(c, (h1, w1), 1).reshape(n, C, h1, w1)
    ulp = 2.0 ** -8 if dt == torch.bfloat16 else 2.0 ** -11
    scale = float(np.abs(ref).max())
    np.testing.assert_allclose(outs[1][:n].double().cpu().numpy(), ref, rtol=ulp, atol=ulp * scale)
