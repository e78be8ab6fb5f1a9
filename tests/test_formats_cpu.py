"""CPU tests of the container file formats: raster I/O through
Pillow, the `.heximg` dict format with its restricted unpickler, and the in-memory
type1 / type2 decodes of HEXIMAGE(data=...) (HexImage.py:103-125)."""
import io
import os
import pickle

import numpy as np
import pytest

from HyGrid import _io
from HyGrid.HexImage import HEXIMAGE
from HyGrid.Image import IMAGE


def test_raster_roundtrip_rgb_grey_16bit(tmp_path):
    rng = np.random.default_rng(0)
    rgb = rng.integers(0, 256, (3, 17, 23), dtype=np.uint8)
    p = str(tmp_path / "a.png")
    _io.write_raster(p, rgb)
    np.testing.assert_array_equal(_io.read_raster(p), rgb)
    grey = rng.integers(0, 256, (1, 9, 11), dtype=np.uint8)
    p = str(tmp_path / "g.tif")
    _io.write_raster(p, grey)
    np.testing.assert_array_equal(_io.read_raster(p), grey)
    deep = rng.integers(0, 65536, (2, 8, 10), dtype=np.uint16)
    p = str(tmp_path / "d.tif")
    _io.write_raster(p, deep)
    np.testing.assert_array_equal(_io.read_raster(p), deep)
    with pytest.raises(ValueError):
        _io.write_raster(str(tmp_path / "d.png"), deep)


def test_image_from_file_and_window(tmp_path):
    rgb = np.arange(3 * 6 * 8, dtype=np.uint8).reshape(3, 6, 8)
    p = str(tmp_path / "x.png")
    _io.write_raster(p, rgb)
    im = IMAGE(p)
    assert im.shape == (3, 6, 8) and im.geotrans == (0, 1, 0, 0, 0, 1)
    np.testing.assert_array_equal(im.Image, rgb)
    with pytest.raises(OSError):
        IMAGE(str(tmp_path / "missing.png"))
    im2 = IMAGE(p)
    w = im2.LoadImageArray(2, 1, 4, 3)         # GDAL ReadAsArray(xoff, yoff, xsize, ysize)
    np.testing.assert_array_equal(w, rgb[:, 1:4, 2:6])
    out = str(tmp_path / "y.png")
    IMAGE(data=rgb).SaveImage(out)
    np.testing.assert_array_equal(_io.read_raster(out), rgb)


def test_save_dtype_rule():
    assert _io.save_dtype(np.zeros(1, np.uint8)) == np.uint8
    assert _io.save_dtype(np.zeros(1, np.int16)) == np.uint16
    assert _io.save_dtype(np.zeros(1, np.float64)) == np.uint8


def test_heximg_roundtrip_and_refusal(tmp_path):
    hexm = np.random.default_rng(1).random((3, 5, 7))
    h = HEXIMAGE(data=hexm, even_odd_offset=1, geotrans=(1, 2, 0, 3, 0, 4))
    p = str(tmp_path / "a.heximg")
    h.SaveHexImage(p)
    h2 = HEXIMAGE(p)
    # the constructor's even_odd_offset argument overrides the stored one, as in the
    # reference (HexImage.py:99 then :124)
    assert h2.shape == (3, 5, 7) and h2.even_odd_offset == 0
    assert h2.Heximagedataset['offset'] == 1
    assert h2.geotrans == (1, 2, 0, 3, 0, 4)
    np.testing.assert_array_equal(h2.HexagonImage, hexm)
    # a pickle that would call os.system is refused, not executed
    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))
    bad = str(tmp_path / "bad.heximg")
    with open(bad, "wb") as f:
        pickle.dump({"HexMatrix": Evil()}, f)
    with pytest.raises(pickle.UnpicklingError):
        _io.load_heximg(bad)


def test_heximage_data_decodes():
    """type1 / type2 decodes of the data= constructor (HexImage.py:108-111)."""
    t1 = np.arange(2 * 5 * 9, dtype=np.float64).reshape(2, 5, 9)
    h = HEXIMAGE(data=t1, heximagetype=1)
    np.testing.assert_array_equal(h.HexagonImage, t1[:, :, 1:-1:2])
    assert h.shape == (2, 5, 4)
    t2 = np.arange(2 * 10 * 9, dtype=np.float64).reshape(2, 10, 9)
    h = HEXIMAGE(data=t2, heximagetype=2)
    np.testing.assert_array_equal(h.HexagonImage, t2[:, ::2, 1:-1:2])
    h = HEXIMAGE(data=np.ones((4, 6)))
    assert h.shape == (1, 4, 6)
    with pytest.raises(ValueError):
        HEXIMAGE()
