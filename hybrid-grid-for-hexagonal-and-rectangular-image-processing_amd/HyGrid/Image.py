"""Drop-in for HyGrid.Image's in-memory surface: IMAGE(data=...) and ConvertToHexagon.

Reference: /root/reference/HyGrid/Image.py.  The `data=` constructor (:59-68)
and `ConvertToHexagon` (:111-116, rect->hex at (H//2, W//2), 'nearest' by
default) are kept; the conversion runs on the gfx950 rect->hex kernel.
GDAL/OpenCV file I/O and the matplotlib viewer are outside the accelerated path
(SURVEY.md §8f): a `pathname` raises NotImplementedError instead of the
reference's sys.exit() on missing packages (:4-27).
"""
import numpy as np

from .geometry_np import rect_to_hex_resample

__all__ = ["IMAGE"]


class IMAGE:
    def __init__(self, pathname=None, data=None, geotrans=None, proj=None, backend='gdal'):
        if pathname is None and data is None:
            raise ValueError("pathname and data can not be None at the same time")
        if pathname is not None and data is not None:
            raise ValueError("pathname and data can not be Given at the same time")
        if pathname is not None:
            raise NotImplementedError("IMAGE(pathname=...): GeoTIFF/JPEG I/O is not part of "
                                      "the accelerated path; load the raster and pass data=")
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

    def ConvertToHexagon(self, interpolation='nearest'):
        """Image.py:111-116."""
        return rect_to_hex_resample(self.Image, [self.height // 2, self.width // 2],
                                    interpolation=interpolation)
