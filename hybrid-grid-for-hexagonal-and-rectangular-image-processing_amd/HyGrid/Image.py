"""Drop-in for HyGrid.Image: the rect raster container IMAGE.

Reference: /root/reference/HyGrid/Image.py.  `IMAGE(pathname | data=...)` (:40-72),
`LoadImageArray` (:89-107), `ConvertToHexagon` (:111-116, rect->hex at (H//2, W//2),
'nearest' by default, on the gfx950 rect->hex kernel) and `SaveImage` (:117-151).
Raster files go through Pillow instead of GDAL (see `_io`); the matplotlib viewer
`imshow` (:152-159) is display-only and not provided.  Missing optional packages raise
instead of the reference's import-time sys.exit() (:4-27).
"""
import os

import numpy as np

from . import _io
from .geometry_np import rect_to_hex_resample

__all__ = ["IMAGE"]


class IMAGE:
    def __init__(self, pathname=None, data=None, geotrans=None, proj=None, backend='gdal'):
        if pathname is None and data is None:
            raise ValueError("pathname and data can not be None at the same time")
        if pathname is not None and data is not None:
            raise ValueError("pathname and data can not be Given at the same time")
        if pathname is not None:
            self.path = pathname
            if not os.path.exists(self.path):
                raise OSError("path dosen't exist.")
            ext = os.path.splitext(pathname)[1]
            if ext not in _io.RASTER_EXT:
                raise ValueError(f"IMAGE: unsupported raster extension {ext!r}")
            self.filetype = 1
            self.data = _io.read_raster(self.path)           # (bands, H, W)
            self.bands, self.height, self.width = self.data.shape
            self.geotrans = (0, 1, 0, 0, 0, 1)
            self.proj = None
            self.Image = self.LoadImageArray()
        else:
            if data.ndim == 2:
                data = np.broadcast_to(data, (1, data.shape[0], data.shape[1]))
            self.Image = data
            self.bands, self.height, self.width = data.shape
            self.geotrans = geotrans
            if self.geotrans is None:
                self.geotrans = (0, 1, 0, 0, 0, 1)
            self.proj = proj
            self.path = 'tmp.tif'
        self.shape = (self.bands, self.height, self.width)
        self.backend = backend

    def size(self, index):
        return self.Image.shape[index]

    def Tiles(self):
        """Unimplemented stub in the reference too (:81-88)."""
        pass

    def LoadImageArray(self, w_range_start=0, h_range_start=0, w_range=None, h_range=None):
        """Window read of the loaded raster, GDAL ReadAsArray(xoff, yoff, xsize, ysize)
        semantics (:89-107); updates width / height like the reference."""
        if w_range is None:
            w_range = self.width
        if h_range is None:
            h_range = self.height
        tmp = self.data[:, h_range_start:h_range_start + h_range,
                        w_range_start:w_range_start + w_range]
        self.width = w_range - w_range_start
        self.height = h_range - h_range_start
        return tmp

    def ConvertToHexagon(self, interpolation='nearest'):
        """Image.py:111-116."""
        return rect_to_hex_resample(self.Image, [self.height // 2, self.width // 2],
                                    interpolation=interpolation)

    def SaveImage(self, pathname):
        """Image.py:117-151: uint8 / uint16 by the source dtype, one band per channel."""
        ext = os.path.splitext(pathname)[1]
        if ext not in _io.RASTER_EXT:
            raise ValueError(f"SaveImage: unsupported raster extension {ext!r}")
        self.filetype = 1
        _io.write_raster(pathname, np.asarray(self.Image).astype(_io.save_dtype(self.Image)))

    def imshow(self):
        raise NotImplementedError("IMAGE.imshow: display is outside the accelerated path")
