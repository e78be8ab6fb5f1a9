"""Host-side behaviour of the drop-in surface (no GPU): reference exceptions,
HexConv2d construction / init / repr / state_dict parity, container decoding,
format conversions, the local mmcv-style registry, and the loud failure of the
product path when no HIP device is present."""
import numpy as np
import pytest
import torch

from HyGrid import HexFrames, HexModules, geometry_np as G, geometry_torch as GT
from HyGrid.HexImage import HEXIMAGE
from HyGrid.Image import IMAGE
from HyGrid.dist import shard_range


def test_interpolation_keyerrors_like_reference(golden_index):
    errs = golden_index["kat"]["errors"]
    x = np.zeros((1, 4, 4))
    assert errs["r2h_linear"] == "KeyError"
    with pytest.raises(KeyError):
        G.rect_to_hex_resample(x, None, "linear")
    assert errs["h2r_unknown"] == "KeyError"
    with pytest.raises(KeyError):
        G.hex_to_rect_resample(x, None, "cubic")
    with pytest.raises(KeyError):
        GT.hex_to_square_resample(x, None, "cubic")
    with pytest.raises(ValueError):      # documented departure: no uninitialised output
        G.hex_to_rect_resample(x, None, "bilinear")
    with pytest.raises(ValueError):
        G.hexresize(x, (2, 2), "cubic")
    with pytest.raises(Exception):
        G.rect_to_hex_resample(np.zeros((1, 1, 1, 4, 4)), None, "bilinear")


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-device behaviour")
def test_product_path_fails_loudly_without_device():
    with pytest.raises(RuntimeError, match="HIP device"):
        G.rect_to_hex_resample(np.zeros((1, 4, 4)), None, "bilinear")
    m = HexFrames.HexConv2d(3, 3, 0, 2, padding=1)
    with pytest.raises(RuntimeError, match="HIP device"):
        m(torch.zeros(1, 3, 8, 8))


def test_hexconv_init_matches_reference_rng(golden, golden_index):
    g = golden("hexconv")
    for meta in golden_index["hexconv"]:
        if "error" in meta:
            continue
        ci = meta["case"]
        torch.manual_seed(1000 + ci)
        m = HexFrames.HexConv2d(meta["in_c"], meta["out_c"], meta["off"], meta["r"],
                                stride=meta["stride"], padding=meta["pad"],
                                dilation=meta["dilation"], groups=meta["groups"],
                                bias=meta["bias"], padding_mode=meta["padding_mode"],
                                padding_value=meta["padding_value"])
        np.testing.assert_array_equal(m.kernel.detach().numpy(), g[f"c{ci}_kernel"])
        if meta["bias"]:
            np.testing.assert_array_equal(m.bias.detach().numpy(), g[f"c{ci}_bias"])
        else:
            assert m.bias is None


def test_hexconv_surface(golden_index):
    kat = golden_index["kat"]
    m = HexFrames.HexConv2d(3, 6, 0, 2, padding=1, groups=3)
    assert repr(m) == kat["conv_repr"]
    assert sorted(m.state_dict().keys()) == kat["conv_state_keys"]
    assert list(m.kernel.shape) == kat["conv_kernel_shape"]
    for r in (1, 2, 3, 4):
        mm = HexFrames.HexConv2d(1, 1, 0, r)
        assert [mm.kernelnum, mm.k_h, mm.k_w] == kat[f"conv_kernelnum_r{r}"]
    with pytest.raises(ValueError):
        HexFrames.HexConv2d(3, 4, 0, 2, groups=3)
    # `weight` is accepted for `kernel` (future version.txt:80)
    sd = {"weight": torch.ones(6, 1, 1, 7), "bias": torch.zeros(6)}
    m.load_state_dict(sd)
    assert torch.equal(m.kernel.detach(), torch.ones(6, 1, 1, 7))


def test_type1_conversion_has_no_cpu_fallback():
    """heximage_to_type1 runs on the gfx950 permute kernel only (the KAT parity against
    the reference lives in test_gpu_formats.py); without a HIP device it raises."""
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by test_gpu_formats.py")
    t = torch.arange(2 * 5 * 4, dtype=torch.float32).reshape(1, 2, 5, 4)
    with pytest.raises(RuntimeError):
        HexFrames.heximage_to_type1(t, 0)
    back, o = HexFrames.type1_to_heximage(torch.zeros(1, 2, 5, 9), 1)   # a view, host-only
    assert o == 1 and tuple(back.shape) == (1, 2, 5, 4)


def test_heximage_data_constructor():
    data = np.arange(3 * 6 * 11, dtype=np.float64).reshape(3, 6, 11)
    h = HEXIMAGE(data=data)
    assert h.shape == (3, 6, 11) and h.HexagonImage is data
    h1 = HEXIMAGE(data=data, heximagetype=1)
    np.testing.assert_array_equal(h1.HexagonImage, data[:, :, 1:-1:2])
    h2 = HEXIMAGE(data=data, heximagetype=2)
    np.testing.assert_array_equal(h2.HexagonImage, data[:, ::2, 1:-1:2])
    g = HEXIMAGE(data=data[0])
    assert g.shape == (1, 6, 11)
    with pytest.raises(ValueError):
        HEXIMAGE()
    with pytest.raises(OSError):                 # the reference's check (Image.py:47-48)
        HEXIMAGE(pathname="does/not/exist.tif")
    im = IMAGE(data=data)
    assert im.shape == (3, 6, 11) and im.geotrans == (0, 1, 0, 0, 0, 1)


def test_hexmodules_registry_and_module():
    assert "HexConv2d" in HexModules.CONV_LAYERS
    layer = HexModules.build_hexconv_layer(None, 3, 8, 0, 2, padding=1)
    assert isinstance(layer, HexFrames.HexConv2d)
    with pytest.raises(TypeError):
        HexModules.build_hexconv_layer("HexConv2d", 3, 8, 0, 2)
    with pytest.raises(KeyError):
        HexModules.build_hexconv_layer(dict(kernel=3), 3, 8, 0, 2)
    with pytest.raises(KeyError):
        HexModules.build_hexconv_layer(dict(type="Nope"), 3, 8, 0, 2)
    m = HexModules.HexConvModule(3, 8, 0, 2, padding=1, norm_cfg=dict(type="BN"))
    assert m.conv.bias is None and m.with_bias is False        # bias='auto' with norm
    assert isinstance(m.norm, torch.nn.BatchNorm2d) and m.norm_name == "bn"
    assert isinstance(m.activate, torch.nn.ReLU)
    m2 = HexModules.HexConvModule(3, 8, 0, 2, padding=1, padding_mode="reflect")
    assert m2.conv.pad == 0 and isinstance(m2.padding_layer, torch.nn.ReflectionPad2d)
    assert torch.all(m2.conv.bias == 0)                       # kaiming_init zeroes the bias


def test_shard_range_partitions():
    for total in (0, 1, 7, 128, 1024):
        for world in (1, 2, 3, 4, 8):
            spans = [shard_range(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1


def test_igt_host_plan_and_errors(golden, golden_index):
    """image_geometric_transformation host side: the output lattice planned from the
    transformed corners (geometry_np.py:56-87) has the reference's (h1, w1); interpolation
    names raise like the reference (KeyError) and 'bilinear' raises instead of returning
    np.empty (documented departure)."""
    from HyGrid import ops
    g = golden("igt")
    for meta in golden_index["igt"]:
        xs, ys, hinv = ops.homography_plan(meta["h"], meta["w"], g[f"c{meta['case']}_H"])
        assert (xs.size, ys.size) == (meta["h1"], meta["w1"])
        np.testing.assert_array_equal(hinv, np.linalg.inv(g[f"c{meta['case']}_H"]))
    x = np.zeros((1, 4, 4))
    with pytest.raises(KeyError):
        G.image_geometric_transformation(x, np.eye(3), "cubic")
    with pytest.raises(ValueError):
        G.image_geometric_transformation(x, np.eye(3), "bilinear")
    with pytest.raises(Exception):
        G.image_geometric_transformation(np.zeros((1, 1, 1, 1, 4)), np.eye(3), "linear")
    with pytest.raises(ValueError):
        ops.homography_plan(4, 4, np.eye(2))
    with pytest.raises(NotImplementedError):
        GT.image_geometric_transformation(x, np.eye(3), "linear", device="cpu")


def test_pool_host_surface(golden_index):
    """Hex pooling host logic: window planning raises where the reference's gather does,
    constructor / repr parity, and the documented departures (stride=None, constructible
    adaptive / global modules, 'centroid' -> NotImplementedError)."""
    from HyGrid import ops
    from pool_cases import pool_args
    for m in golden_index["pool"]:
        if "error" in m:
            assert m["error"] == "IndexError"
            with pytest.raises(IndexError):
                pool_args(m)
        else:
            a = pool_args(m)
            assert list(m["out_shape"][-2:]) == [a[5], a[6]] or m["kind"] == "global"
        if m["kind"] != "pool":
            assert m["construct"] == "NameError"     # the reference's centroid_pooling
    p = HexFrames.HexPool2d("max", 2, 2)
    assert repr(p) == "HexPool2d(kernel_size=[2, 2], stride=[2, 2], padding=0)"
    assert HexFrames.HexPool2d("average", 3).stride == [3, 3]          # stride=None
    with pytest.raises(KeyError):
        HexFrames.HexPool2d("median", 2, 2)
    with pytest.raises(NotImplementedError):
        HexFrames.HexAdaptivePool2d(2, "centroid")
    with pytest.raises(NotImplementedError):
        HexFrames.HexGlobalPool2d("centroid")
    assert HexFrames.HexAdaptivePool2d([2, 3], "max").wn == 3
    with pytest.raises(Exception):
        HexFrames.HexAdaptivePool2d(2.5, "max")
    with pytest.raises(RuntimeError):
        ops.hex_pool2d(torch.zeros(1, 1, 4, 4), "max", 2, 2, 2, 2, 2, 1, 1, "reflect", 1.0)
