"""GPU: the type1 / type2 permute kernels (hg_hex_to_type1, hg_strided_copy2d) and the
HEXIMAGE methods built on them.

Pinned to the reference's own heximage_to_type1 outputs (golden KATs, HexFrames.py:417-445,
captured by tests/golden/make_golden.py) and to the CPU oracle (or_heximage_to_type1);
GenerateType1Image / GenerateType2Image against a NumPy restatement of their per-row
loops (HexImage.py:139-170; HexImage.py itself cannot be imported here: it sys.exit()s
without GDAL / mmcv / OpenGL)."""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a HIP device", allow_module_level=True)

from HyGrid import HexFrames as HF  # noqa: E402
from HyGrid import ops  # noqa: E402
from HyGrid.HexImage import HEXIMAGE  # noqa: E402

DEV = torch.device("cuda:0")


def ref_type1(img, off):
    """HexImage.GenerateType1Image's loop (HexImage.py:139-153)."""
    b, h, w = img.shape
    out = np.zeros([b, h, w * 2 + 1])
    tmp = np.repeat(img, 2, axis=2)
    for c in range(b):
        for i in range(h):
            out[c, i] = np.insert(tmp[c][i], 0, 0) if (i + off) % 2 else np.append(tmp[c][i], 0)
    return out


def ref_type2(img, off):
    """HexImage.GenerateType2Image's loop (HexImage.py:154-170)."""
    b, h, w = img.shape
    out = np.zeros([b, h * 2, w * 2 + 1])
    tmp = np.repeat(np.repeat(img, 2, axis=-2), 2, axis=-1)
    for c in range(b):
        for i in range(h):
            row = np.insert(tmp[c][2 * i], 0, 0) if (i + off) % 2 else np.append(tmp[c][2 * i], 0)
            out[c][2 * i] = row
            out[c][2 * i + 1] = row
    return out


@pytest.mark.parametrize("off", [0, 1])
def test_type1_vs_reference_kat(golden_index, off):
    t = torch.arange(2 * 5 * 4, dtype=torch.float32).reshape(1, 2, 5, 4).to(DEV)
    got = HF.heximage_to_type1(t, off).cpu().numpy()
    np.testing.assert_array_equal(got, np.array(golden_index["kat"][f"type1_off{off}"]))
    assert list(HF.heximage_to_type2(t, off).shape) == golden_index["kat"][f"type2_off{off}_shape"]


@pytest.mark.parametrize("dtype", [torch.uint8, torch.bfloat16, torch.float32, torch.float64])
@pytest.mark.parametrize("shape", [(3, 7, 9), (2, 16, 20), (1, 1, 1), (3, 1080, 1920)])
@pytest.mark.parametrize("off", [0, 1])
def test_type1_type2_vs_oracle_and_loops(dtype, shape, off):
    torch.manual_seed(0)
    x = (torch.rand(shape, device=DEV) * 200).to(dtype)
    t1 = ops.hex_to_type1(x, off, 1)
    assert t1.dtype == dtype
    xo = x.double().cpu().numpy()
    np.testing.assert_array_equal(t1.double().cpu().numpy(), O.heximage_to_type1(xo, off))
    t2 = ops.hex_to_type1(x, off, 2)
    np.testing.assert_array_equal(t2.double().cpu().numpy()[:, ::2], t1.double().cpu().numpy())
    np.testing.assert_array_equal(t2.double().cpu().numpy()[:, 1::2], t1.double().cpu().numpy())
    if shape[1] * shape[2] < 1000:
        np.testing.assert_array_equal(t1.double().cpu().numpy(), ref_type1(xo, off))
        np.testing.assert_array_equal(t2.double().cpu().numpy(), ref_type2(xo, off))


def test_strided_copy_equals_slices():
    x = torch.rand((2, 3, 10, 21), device=DEV)
    for args in [(0, 1, 1, 2), (0, 2, 1, 2), (1, 3, 0, 5)]:
        r0, rs, c0, cs = args
        got = ops.strided_copy2d(x, *args)
        torch.testing.assert_close(got, x[..., r0::rs, c0::cs].contiguous(), rtol=0, atol=0)
    got = ops.strided_copy2d(x, 0, 1, 1, 2, w_out=len(range(1, 20, 2)))   # type1 decode 1:-1:2
    torch.testing.assert_close(got, x[..., 1:-1:2].contiguous(), rtol=0, atol=0)


@pytest.mark.parametrize("off", [0, 1])
def test_heximage_generate_and_file_roundtrip(tmp_path, off):
    rng = np.random.default_rng(3)
    hexm = rng.integers(0, 256, (3, 6, 8)).astype(np.uint8)
    h = HEXIMAGE(data=hexm, even_odd_offset=off, geotrans=(0, 1, 0, 0, 0, 3))
    t1, g1 = h.GenerateType1Image()
    np.testing.assert_array_equal(t1, ref_type1(hexm.astype(np.float64), off))
    assert g1 == (0, 1, 0, 0, 0, 6)
    t2, g2 = h.GenerateType2Image()
    np.testing.assert_array_equal(t2, ref_type2(hexm.astype(np.float64), off))
    assert g2 == (0, 1, 0, 0, 0, 3)
    p1 = str(tmp_path / "t1.png")
    h.SaveHexImage(p1, imagetype=1)
    back = HEXIMAGE(p1, heximagetype=1)
    np.testing.assert_array_equal(back.HexagonImage, hexm)
    p2 = str(tmp_path / "t2.png")
    h.SaveHexImage(p2, imagetype=2)
    back = HEXIMAGE(p2, heximagetype=2)
    np.testing.assert_array_equal(back.HexagonImage, hexm)


def test_heximage_from_rect_file_converts(tmp_path):
    """heximagetype=None on a raster file: rect->hex 'nearest' at (H//2, W//2) (HexImage.py:61-63)."""
    from HyGrid import _io
    from HyGrid.geometry_np import rect_to_hex_resample
    rgb = np.random.default_rng(4).integers(0, 256, (3, 20, 30)).astype(np.uint8)
    p = str(tmp_path / "r.png")
    _io.write_raster(p, rgb)
    h = HEXIMAGE(p)
    np.testing.assert_array_equal(h.HexagonImage, rect_to_hex_resample(rgb, [10, 15], 'nearest'))
    assert h.shape == (3, 10, 15)
