"""GPU parity: the HIP path (libhygrid_hip.so through the drop-in API) against the
reference goldens and the CPU oracle.

Tolerances (north_star): integer lattice maps bit-exact; floating point within
1e-5 relative — asserted as rtol=1e-5 with atol=1e-5*max|ref| — for fp32.  The
fp64 resampler path follows the reference's evaluation order and is asserted
bit-exact.  bf16 runs are checked against the oracle on the same bf16-rounded
input with a bf16 output tolerance (2^-8 relative, one rounding of the output).
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - collected only with -m gpu
    pytest.skip("needs a HIP device", allow_module_level=True)

from HyGrid import geometry_np as G  # noqa: E402
from HyGrid import geometry_torch as GT  # noqa: E402
from HyGrid import ops  # noqa: E402
from HyGrid.HexFrames import HexConv2d  # noqa: E402

DEV = torch.device("cuda:0")
RTOL = 1e-5


def close(y, ref, rtol=RTOL):
    y = np.asarray(y, np.float64)
    ref = np.asarray(ref, np.float64)
    assert y.shape == ref.shape, (y.shape, ref.shape)
    scale = max(np.abs(ref).max(), 1e-30) if ref.size else 1.0
    np.testing.assert_allclose(y, ref, rtol=rtol, atol=rtol * scale)


OPS = {"r2h": "rect_to_hex", "h2r": "hex_to_rect", "hexresize": "hexresize"}


# ---------------------------------------------------------------- lattice maps
@pytest.mark.parametrize("name", ["r2h", "h2r", "hexresize"])
def test_lattice_maps_bit_exact_vs_reference(golden, golden_index, name):
    g = golden(name)
    for meta in golden_index[name]:
        ci, mode = meta["case"], meta["mode"]
        tag = f"c{ci}_{mode}"
        m = ops.lattice_maps(OPS[name], meta["h"], meta["w"], meta["h1"], meta["w1"], DEV)
        m = {k: v.cpu().numpy() for k, v in m.items()}
        keys = ["i_n", "j_n", "valid"] + (["flag"] if name != "r2h" else [])
        if mode == "nearest":
            keys.append("argmin")
        for k in keys:
            np.testing.assert_array_equal(m[k], g[tag + "_" + k], err_msg=f"{tag} {k}")
        if mode == "linear" or name == "r2h":
            for k in ("i_f", "j_f"):
                if tag + "_" + k in g:
                    np.testing.assert_array_equal(m[k], g[tag + "_" + k], err_msg=f"{tag} {k}")
        if name != "r2h" and mode == "linear":
            for k in ("alpha", "beta", "gamma"):
                np.testing.assert_array_equal(m[k], g[tag + "_" + k], err_msg=f"{tag} {k}")


@pytest.mark.parametrize("shape", [(2160, 3840, 2160, 3840), (1080, 1920, 1080, 1920),
                                   (4320, 7680, 2160, 3840), (257, 129, 511, 250)])
@pytest.mark.parametrize("op", ["r2h", "h2r", "hexresize"])
def test_lattice_maps_full_size_vs_oracle(shape, op):
    h, w, h1, w1 = shape
    fn = {"r2h": O.r2h_maps, "h2r": O.h2r_maps, "hexresize": O.hexresize_maps}[op]
    ref = fn(h, w, h1, w1)
    m = ops.lattice_maps(OPS[op], h, w, h1, w1, DEV)
    for k in ("i_n", "j_n", "flag", "valid", "argmin", "i_f", "j_f", "alpha", "beta", "gamma"):
        if k in ref:
            np.testing.assert_array_equal(m[k].cpu().numpy(), ref[k], err_msg=k)


# ------------------------------------------------------ drop-in API vs goldens
@pytest.mark.parametrize("name,fn", [("r2h", G.rect_to_hex_resample),
                                     ("h2r", G.hex_to_rect_resample),
                                     ("hexresize", G.hexresize)])
def test_numpy_api_matches_reference_outputs(golden, golden_index, name, fn):
    g = golden(name)
    for meta in golden_index[name]:
        ci, mode = meta["case"], meta["mode"]
        x = g[f"c{ci}_x"]
        y = fn(x, (meta["h1"], meta["w1"]), mode)
        ref = g[f"c{ci}_{mode}_y"]
        assert list(y.shape) == meta["out_shape"], (name, ci, mode)
        assert str(y.dtype) == meta["out_dtype"], (name, ci, mode, y.dtype)
        # fp64 blend in the reference's order, nearest = copy: bit-exact
        np.testing.assert_array_equal(y.reshape(ref.shape), ref, err_msg=f"{name} {ci} {mode}")


def test_geometry_torch_twin_numpy_and_tensor(golden, golden_index):
    g = golden("h2r")
    for meta in golden_index["h2r"]:
        ci, mode = meta["case"], meta["mode"]
        x = g[f"c{ci}_x"]
        ref = g[f"c{ci}_{mode}_y"]
        y = GT.hex_to_square_resample(x, (meta["h1"], meta["w1"]), mode)
        np.testing.assert_array_equal(np.asarray(y).reshape(ref.shape), ref)
        xt = torch.from_numpy(np.ascontiguousarray(x)).to(DEV)
        yt = GT.hex_to_square_resample(xt, (meta["h1"], meta["w1"]), mode,
                                       out_dtype=torch.float64 if mode == "linear" else None)
        assert isinstance(yt, torch.Tensor) and yt.device.type == "cuda"
        np.testing.assert_array_equal(yt.cpu().numpy().reshape(ref.shape), ref)


# ------------------------------------------------- fp32 / bf16 vs the oracle
SHAPES = [(3, 15, 17, 15, 17), (2, 64, 96, 64, 96), (1, 33, 47, 17, 24), (2, 40, 50, 81, 99),
          (3, 200, 300, 100, 150), (1, 512, 512, 32, 32), (1, 130, 260, 131, 259),
          (4, 7, 9, 1, 1), (1, 1, 1, 5, 6), (2, 18, 1030, 18, 1030)]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("op", ["r2h", "h2r", "hexresize"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16, torch.uint8])
def test_tensor_ops_vs_oracle(shape, op, dtype):
    c, h, w, h1, w1 = shape
    gen = torch.Generator().manual_seed(h * 1000 + w)
    if dtype == torch.uint8:
        x = torch.randint(0, 256, (c, h, w), generator=gen, dtype=torch.uint8)
    else:
        x = torch.rand((c, h, w), generator=gen).to(dtype)
    fn = {"r2h": (ops.rect_to_hex, O.rect_to_hex), "h2r": (ops.hex_to_rect, O.hex_to_rect),
          "hexresize": (ops.hexresize, O.hexresize)}[op]
    ref = fn[1](x.double().numpy(), (h1, w1), 1)
    out_dt = torch.float32 if dtype == torch.uint8 else dtype
    y = fn[0](x.to(DEV), (h1, w1), 1, out_dtype=out_dt).float().cpu().numpy()
    rtol = RTOL if out_dt == torch.float32 else (2 ** -8 if out_dt == torch.bfloat16 else 2 ** -11)
    close(y, ref, rtol)
    # nearest is a copy: exact against the oracle
    refn = fn[1](x.double().numpy(), (h1, w1), 0)
    yn = fn[0](x.to(DEV), (h1, w1), 0)
    assert yn.dtype == dtype
    np.testing.assert_array_equal(yn.double().cpu().numpy(), refn)


def test_batch_axis_equals_per_image():
    x = torch.rand((4, 3, 37, 53), device=DEV)
    y = ops.rect_to_hex(x, (41, 49))
    for b in range(4):
        torch.testing.assert_close(ops.rect_to_hex(x[b], (41, 49)), y[b], rtol=0, atol=0)


def test_linearity_full_hd_fp64():
    gen = torch.Generator().manual_seed(5)
    a = torch.rand((1, 1080, 1920), generator=gen, dtype=torch.float64).to(DEV)
    b = torch.rand((1, 1080, 1920), generator=gen, dtype=torch.float64).to(DEV)
    for f in (ops.rect_to_hex, ops.hex_to_rect):
        lhs = f(2.0 * a - 3.0 * b, None)
        rhs = 2.0 * f(a, None) - 3.0 * f(b, None)
        torch.testing.assert_close(lhs, rhs, rtol=1e-12, atol=1e-12)


def test_4k_bf16_batch_vs_oracle_on_one_image():
    """BASELINE config-3 geometry at full size: the HIP bf16 pipeline stage vs oracle."""
    gen = torch.Generator().manual_seed(2)
    x = torch.rand((2, 3, 2160, 3840), generator=gen).to(torch.bfloat16)
    y = ops.rect_to_hex(x.to(DEV), (2160, 3840), out_dtype=torch.float32)
    ref = O.rect_to_hex(x[1].double().numpy(), (2160, 3840), 1)
    close(y[1].cpu().numpy(), ref)
    z = ops.hex_to_rect(y, (2160, 3840), out_dtype=torch.float32)
    refz = O.hex_to_rect(y[1].double().cpu().numpy(), (2160, 3840), 1)
    close(z[1].cpu().numpy(), refz)


def test_empty_and_degenerate():
    x = torch.rand((0, 3, 8, 8), device=DEV)
    assert ops.rect_to_hex(x, (4, 4)).shape == (0, 3, 4, 4)
    x = torch.rand((2, 5, 6), device=DEV)
    assert ops.hex_to_rect(x, (0, 7)).shape == (2, 0, 7)
    y = ops.rect_to_hex(torch.ones((1, 1, 1), device=DEV), (1, 1))
    assert y.shape == (1, 1, 1)


# ------------------------------------------------------------------ HexConv2d
def test_hexconv_vs_reference_goldens(golden, golden_index):
    g = golden("hexconv")
    n = 0
    for meta in golden_index["hexconv"]:
        ci = meta["case"]
        if "error" in meta:
            with pytest.raises(ValueError):
                ops.hexconv2d_out_shape(meta["h"], meta["w"], meta["r"], meta["stride"],
                                        meta["pad"], meta["dilation"])
            continue
        x = torch.from_numpy(g[f"c{ci}_x"]).to(DEV)
        k = torch.from_numpy(g[f"c{ci}_kernel"]).to(DEV)
        b = g.get(f"c{ci}_bias")
        b = torch.from_numpy(b).to(DEV) if b is not None else None
        y = ops.hexconv2d(x, k, b, meta["off"], meta["r"], meta["stride"], meta["pad"],
                          meta["dilation"], meta["groups"], meta["padding_mode"],
                          meta["padding_value"])
        assert y.dtype == torch.float32
        close(y.cpu().numpy(), g[f"c{ci}_y"])
        n += 1
    assert n >= 50


def test_hexconv_module_seeded_like_reference(golden, golden_index):
    """Same seed + ctor => same weights as the reference; forward matches its output."""
    g = golden("hexconv")
    for meta in golden_index["hexconv"][:20]:
        if "error" in meta:
            continue
        ci = meta["case"]
        torch.manual_seed(1000 + ci)
        m = HexConv2d(meta["in_c"], meta["out_c"], meta["off"], meta["r"], stride=meta["stride"],
                      padding=meta["pad"], dilation=meta["dilation"], groups=meta["groups"],
                      bias=meta["bias"], padding_mode=meta["padding_mode"],
                      padding_value=meta["padding_value"])
        np.testing.assert_array_equal(m.kernel.detach().numpy(), g[f"c{ci}_kernel"])
        x = torch.from_numpy(g[f"c{ci}_x"]).to(DEV)
        with torch.no_grad():
            y = m.to(DEV)(x)
        close(y.cpu().numpy(), g[f"c{ci}_y"])


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
def test_hexconv_large_vs_oracle(dtype):
    torch.manual_seed(3)
    m = HexConv2d(3, 3, 0, 2, padding=1, groups=1, bias=True).to(DEV)
    x = torch.rand((2, 3, 270, 514), device=DEV).to(dtype)
    with torch.no_grad():
        y = m(x)
    ref = O.hexconv2d(x.double().cpu().numpy(), m.kernel.detach().cpu().numpy(),
                      m.bias.detach().cpu().numpy(), 0, 2, padding=1)
    close(y.cpu().numpy(), ref)
    m.out_dtype = dtype
    with torch.no_grad():
        y2 = m(x)
    assert y2.dtype == dtype
    rtol = {torch.bfloat16: 2 ** -8, torch.float16: 2 ** -11, torch.float32: RTOL}[dtype]
    close(y2.float().cpu().numpy(), ref, rtol)


@pytest.mark.parametrize("cfg", [dict(r=2, s=1, d=1, p=1, g=3, o=3, c=3),
                                 dict(r=3, s=2, d=1, p=2, g=1, o=5, c=2),
                                 dict(r=2, s=1, d=2, p=0, g=2, o=4, c=6),
                                 dict(r=4, s=3, d=1, p=3, g=1, o=1, c=1)])
@pytest.mark.parametrize("mode", ["constant", "reflect", "replicate", "circular"])
def test_hexconv_param_space_vs_oracle(cfg, mode):
    torch.manual_seed(11)
    x = torch.rand((2, cfg["c"], 61, 133), dtype=torch.float64)
    k = torch.randn((cfg["o"], cfg["c"] // cfg["g"], 3 * cfg["r"] ** 2 - 3 * cfg["r"] + 1))
    b = torch.randn(cfg["o"])
    for off in (0, 1):
        y = ops.hexconv2d(x.to(DEV), k.to(DEV), b.to(DEV), off, cfg["r"], cfg["s"], cfg["p"],
                          cfg["d"], cfg["g"], mode, 0.25)
        ref = O.hexconv2d(x.numpy(), k.numpy(), b.numpy(), off, cfg["r"], cfg["s"], cfg["p"],
                          cfg["d"], cfg["g"], mode, 0.25)
        close(y.cpu().numpy(), ref)


@pytest.mark.parametrize("cg", [(3, 3, 1), (3, 3, 3), (1, 1, 1)])
@pytest.mark.parametrize("p", [0, 1, 2])
def test_hexconv_stream_path_vs_oracle(cg, p):
    """radius 2 / stride 1 / constant padding: the register-streaming kernel
    (conv_stream.hip).  Ragged widths (window halos), heights across row bands
    (126 rows) and the 6-row unroll, both row-parity offsets, nonzero padding value."""
    c, o, g = cg
    torch.manual_seed(17 + p)
    k = torch.randn((o, c // g, 7))
    b = torch.randn(o)
    for (h, w) in [(3, 3), (7, 61), (127, 130), (253, 200), (5, 1)]:
        if w + 2 * p - 2 < 1 or h + 2 * p - 2 < 1:
            continue
        x = torch.rand((2, c, h, w), dtype=torch.float32)
        for off in (0, 1):
            ref = O.hexconv2d(x.double().numpy(), k.numpy(), b.numpy(), off, 2, 1, p, 1, g,
                              "constant", 0.375)
            for dt in (torch.float32, torch.bfloat16, torch.float16):
                xd = x.to(dt)
                ref_d = ref if dt == torch.float32 else O.hexconv2d(
                    xd.double().numpy(), k.numpy(), b.numpy(), off, 2, 1, p, 1, g, "constant", 0.375)
                y = ops.hexconv2d(xd.to(DEV), k.to(DEV), b.to(DEV), off, 2, 1, p, 1, g,
                                  "constant", 0.375)
                assert y.shape == ref_d.shape
                close(y.cpu().numpy(), ref_d)
