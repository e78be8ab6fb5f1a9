"""GPU parity of the fused rect->hex->HexConv2d->hex->rect kernel
(hg_pipeline_r2h_conv_h2r) against the CPU oracle chain, and against the
unfused HIP chain.  fp32: rtol 1e-5 (atol 1e-5*max|ref|); bf16 output: one bf16
rounding (2^-8)."""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a HIP device", allow_module_level=True)

from HyGrid import _abi, ops  # noqa: E402
from HyGrid.HexFrames import HexConv2d  # noqa: E402
from HyGrid.pipeline import rect_hex_conv_rect  # noqa: E402

DEV = torch.device("cuda:0")


def close(y, ref, rtol):
    y = np.asarray(y, np.float64)
    scale = max(np.abs(ref).max(), 1e-30)
    np.testing.assert_allclose(y, ref, rtol=rtol, atol=rtol * scale)


def one_rounding(got, ref, ulp=2.0 ** -8):
    """Each element within one output rounding of the fp64 reference, per element: |got - ref|
    <= ulp |ref| (half a bf16 ulp is 2^-9 |ref| at most; the fp32 chain's error may tip a
    near-tie) plus an absolute floor of 1e-5 max|ref| for values near zero, where the fp32
    cancellation error is relative to the terms, not to the sum."""
    got = np.asarray(got, np.float64)
    tol = ulp * np.abs(ref) + 1e-5 * np.abs(ref).max()
    bad = np.abs(got - ref) > tol
    assert not bad.any(), (f"{int(bad.sum())} of {bad.size} outputs beyond one rounding of the "
                           f"oracle (worst excess {float((np.abs(got - ref) - tol).max()):.3e})")


def oracle_chain(x, conv, hex_size, rect_size):
    h = O.rect_to_hex(x.double().cpu().numpy(), hex_size, 1)
    b = conv.bias.detach().cpu().numpy() if conv.bias is not None else None
    c = O.hexconv2d(h, conv.kernel.detach().cpu().numpy(), b, int(conv.even_odd_offset), 2,
                    padding=conv.pad, groups=conv.groups, padding_value=conv.padding_value)
    return O.hex_to_rect(c, rect_size, 1)


CASES = [
    # (B, C, H, W, hex_size, rect_size, off, pad, groups, pad_value)
    (2, 3, 48, 80, None, None, 0, 1, 1, 0.0),
    (1, 3, 37, 53, None, None, 1, 1, 1, 0.0),
    (2, 3, 64, 150, None, None, 0, 1, 3, 0.0),
    (1, 3, 40, 70, None, None, 1, 0, 1, 0.0),
    (1, 3, 40, 70, None, None, 0, 2, 1, 0.3),
    (3, 1, 33, 200, None, None, 0, 1, 1, 0.0),
    (1, 3, 70, 130, (71, 131), (70, 130), 0, 1, 1, 0.0),
    (1, 3, 9, 7, None, None, 0, 1, 1, 0.0),
    (1, 3, 270, 480, None, None, 0, 1, 1, 0.0),
    # two-column streaming kernel (fused.hip): even widths, padding 1, pad value 0
    (2, 3, 130, 256, None, None, 1, 1, 1, 0.0),     # even_odd_offset 1 -> odd-row shift
    (1, 3, 300, 500, None, None, 0, 1, 3, 0.0),     # depthwise, 3 bands x 5 windows
    (2, 1, 128, 246, None, None, 0, 1, 1, 0.0),
    (1, 3, 6, 4, None, None, 0, 1, 1, 0.0),         # smaller than one window / band
    (1, 3, 127, 122, None, None, 1, 1, 3, 0.0),     # band and window edges
]


@pytest.mark.parametrize("case", CASES)
def test_fused_vs_oracle_fp32(case):
    B, C, H, W, hs, rs, off, pad, g, pv = case
    torch.manual_seed(3)
    conv = HexConv2d(C, C, off, 2, padding=pad, groups=g, bias=True, padding_value=pv).to(DEV)
    x = torch.rand((B, C, H, W), device=DEV)
    with torch.no_grad():
        y = ops.pipeline_r2h_conv_h2r(x, conv.kernel, conv.bias, hs, rs, pad, g, off, pv,
                                      torch.float32)
    assert y is not None, "geometry should be fusable"
    hs_ = hs or (H, W)
    ho, wo = ops.hexconv2d_out_shape(hs_[0], hs_[1], 2, 1, pad, 1)
    ref = oracle_chain(x, conv, hs_, rs or (ho, wo))
    close(y.cpu().numpy(), ref, 1e-5)


def test_fused_4k_bf16_matches_oracle_and_unfused():
    """BASELINE config-3 geometry at full size (2 images)."""
    torch.manual_seed(3)
    conv = HexConv2d(3, 3, 0, 2, padding=1, bias=True).to(DEV)
    gen = torch.Generator(device=DEV).manual_seed(2)
    x = torch.rand((2, 3, 2160, 3840), generator=gen, device=DEV, dtype=torch.bfloat16)
    with torch.no_grad():
        y = rect_hex_conv_rect(x, conv)
        y32 = rect_hex_conv_rect(x, conv, out_dtype=torch.float32)
        unf = rect_hex_conv_rect(x, conv, out_dtype=torch.float32, fused=False)
    assert y.dtype == torch.bfloat16 and y.shape == x.shape
    ref = oracle_chain(x[1:2], conv, (2160, 3840), (2160, 3840))[0]
    close(y32[1].cpu().numpy(), ref, 1e-5)
    one_rounding(y[1].float().cpu().numpy(), ref)
    close(unf.cpu().numpy(), y32.cpu().numpy().astype(np.float64), 1e-5)


def test_fused_config3_full_batch_sampled_images():
    """The bench's own launch (BASELINE config 3: 128 x 3 x 2160 x 3840 bf16, bench.py's
    seeds) in one call; three images across the batch (first, middle, last) against the
    fp64 oracle chain at 1e-5 (fp32 output) and the bf16 output within one rounding."""
    torch.manual_seed(3)
    conv = HexConv2d(3, 3, 0, 2, padding=1, groups=1, bias=True).to(DEV)
    gen = torch.Generator(device=DEV).manual_seed(2)
    x = torch.rand((128, 3, 2160, 3840), generator=gen, device=DEV, dtype=torch.bfloat16)
    with torch.no_grad():
        y32 = rect_hex_conv_rect(x, conv, out_dtype=torch.float32)
        y = rect_hex_conv_rect(x, conv)
    for i in (0, 63, 127):
        ref = oracle_chain(x[i:i + 1], conv, (2160, 3840), (2160, 3840))[0]
        close(y32[i].cpu().numpy(), ref, 1e-5)
        one_rounding(y[i].float().cpu().numpy(), ref)
    del x, y, y32
    torch.cuda.empty_cache()


@pytest.mark.parametrize("dt_in,dt_out", [
    (torch.bfloat16, torch.bfloat16), (torch.bfloat16, torch.float32),
    (torch.float16, torch.float16), (torch.float16, torch.float32),
    (torch.float32, torch.float32), (torch.float32, torch.bfloat16)])
@pytest.mark.parametrize("off", [0, 1])
def test_fused_two_column_kernel_dtypes(dt_in, dt_out, off, monkeypatch):
    """fused.hip (the default same-size path) against the oracle and against the
    one-column kernel of pipeline.hip (HYGRID_FUSED2=0) on the same data."""
    torch.manual_seed(3)
    conv = HexConv2d(3, 3, off, 2, padding=1, bias=True).to(DEV)
    gen = torch.Generator(device=DEV).manual_seed(5)
    x = torch.rand((2, 3, 200, 384), generator=gen, device=DEV).to(dt_in)
    args = (x, conv.kernel, conv.bias, None, None, 1, 1, off, 0.0, dt_out)
    with torch.no_grad():
        y = ops.pipeline_r2h_conv_h2r(*args)
        monkeypatch.setenv("HYGRID_FUSED2", "0")
        y1 = ops.pipeline_r2h_conv_h2r(*args)
    ref = oracle_chain(x.float(), conv, (200, 384), (200, 384))
    if dt_out == torch.float32:
        close(y.double().cpu().numpy(), ref, 1e-5)
        close(y.double().cpu().numpy(), y1.double().cpu().numpy(), 1e-5)
    else:   # per element: one output rounding of the oracle; the two kernels within two
        ulp = 2.0 ** -8 if dt_out == torch.bfloat16 else 2.0 ** -11
        one_rounding(y.double().cpu().numpy(), ref, ulp)
        one_rounding(y.double().cpu().numpy(), y1.double().cpu().numpy(), 2 * ulp)


def test_non_identity_geometry_falls_back():
    torch.manual_seed(3)
    conv = HexConv2d(3, 3, 0, 2, padding=1, bias=True).to(DEV)
    x = torch.rand((1, 3, 64, 96), device=DEV)
    with torch.no_grad():
        assert ops.pipeline_r2h_conv_h2r(x, conv.kernel, conv.bias, (32, 48), (64, 96)) is None
        y = rect_hex_conv_rect(x, conv, (32, 48), (64, 96))
    ref = oracle_chain(x, conv, (32, 48), (64, 96))
    close(y.cpu().numpy(), ref, 1e-5)


def edge_points(md, H, W):
    """Non-finite input points on the streaming kernel's band and window edges for mode md,
    derived from the library's own decomposition (hg_fused_layout) rather than hard-coded:
    the last row of every band and the first row of the next one, the last owned column of
    every window and the first of the next, plus the raster corners."""
    rows, own, halo = _abi.fused_layout(md)
    inf, nan = float("inf"), float("nan")
    vals = [inf, -inf, nan]
    pts = []
    edges_r = [r for k in range(1, H // rows + 1) for r in (k * rows - 1, k * rows) if r < H]
    edges_c = [q for k in range(1, W // own + 1) for q in (k * own - 1, k * own) if q < W]
    assert len(edges_r) >= 4 and len(edges_c) >= 2, (rows, own, H, W)
    for i, r in enumerate(edges_r):
        q = edges_c[i % len(edges_c)]
        pts.append((i % 3, r, q, vals[i % 3]))
    pts += [(0, 0, 0, inf), (2, H - 1, W - 1, nan), (1, 3, 50, -inf)]
    return pts, rows


@pytest.mark.parametrize("off", [0, 1])
def test_fused_nonfinite_inputs_stay_local(off):
    """Inf / NaN inputs inside the raster, on the fused kernel's band edges (last row of a
    band / first row of the next) and window edges (last owned column of a window / first
    of the next), placed from hg_fused_layout so they follow the band length the library
    was built with.  The fused kernel evaluates a fixed tap set per column / row class, so a
    tap whose weight is exactly 0 for one column is still multiplied (0 * Inf = NaN) where
    the reference never reads it; conversely the reference multiplies the same-size h2r's
    zero-weight third vertex (geometry_np.py:347-354) where the fused kernel has no tap.
    Non-finite inputs therefore may reach outputs up to 3 samples away differently from the
    reference (the operator chain propagates them exactly).  Asserted:
    every output farther than 3 rows / columns from a non-finite input is finite and
    matches the fp64 oracle chain within 1e-5 — the damage stays local."""
    torch.manual_seed(3)
    conv = HexConv2d(3, 3, off, 2, padding=1, bias=True).to(DEV)
    rows, own, _ = _abi.fused_layout(0)
    B, C, H, W = 1, 3, 2 * rows + 14, 2 * own + 16
    pts, _ = edge_points(0, H, W)
    g = torch.Generator(device=DEV).manual_seed(11)
    x = torch.rand((B, C, H, W), generator=g, device=DEV)
    for c, r, q, v in pts:
        x[0, c, r, q] = v
    with torch.no_grad():
        y = ops.pipeline_r2h_conv_h2r(x, conv.kernel, conv.bias, None, None, 1, 1, off, 0.0,
                                      torch.float32)
    assert y is not None
    ref = oracle_chain(x, conv, (H, W), (H, W))
    got = y.double().cpu().numpy()
    near = np.zeros((H, W), bool)
    for _, r, q, _ in pts:
        near[max(r - 3, 0):r + 4, max(q - 3, 0):q + 4] = True
    far = np.broadcast_to(~near, got.shape)
    assert np.isfinite(ref[far]).all() and np.isfinite(got[far]).all()
    scale = np.abs(ref[far]).max()
    np.testing.assert_allclose(got[far], ref[far], rtol=1e-5, atol=1e-5 * scale)
    # every planted point did reach the output near it (the kernel did not drop an edge row)
    for _, r, q, _ in pts:
        assert not np.isfinite(got[:, :, max(r - 3, 0):r + 4, max(q - 3, 0):q + 4]).all()
