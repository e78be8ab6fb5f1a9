"""Drop-in for HyGrid.HexImage's in-memory surface: HEXIMAGE(data=..., heximagetype).

Reference: /root/reference/HyGrid/HexImage.py:44-125.  Keeps the `data=`
constructor for the three heximagetype codes — None (already a hex raster),
1 (type1 double-width storage, decoded as data[:, :, 1:-1:2]) and 2 (type2,
data[:, ::2, 1:-1:2]) — and the `.HexagonImage` (C, H, W) attribute.  A
`pathname` (GeoTIFF / `.heximg` pickle) raises NotImplementedError: file formats
are the next row of SURVEY.md §8f, and `.heximg` is a pickle, which this
package does not unpickle.
"""
import numpy as np

from .Image import IMAGE

__all__ = ["HEXIMAGE"]


class HEXIMAGE(IMAGE):
    def __init__(self, pathname=None, heximagetype=None, data=None, geotrans=None, proj=None,
                 even_odd_offset=False, backend='gdal'):
        if pathname is None and data is None:
            raise ValueError("pathname and data can not be None at the same time")
        if pathname is not None and data is not None:
            raise ValueError("pathname and data can not be Given at the same time")
        if pathname is not None:
            raise NotImplementedError("HEXIMAGE(pathname=...): file formats are not part of "
                                      "the accelerated path; pass data=")
        if data.ndim == 2:
            data = np.broadcast_to(data, (1, data.shape[0], data.shape[1]))
        if heximagetype is None:
            self.HexagonImage = data
        elif heximagetype == 1:
            self.HexagonImage = data[:, :, 1:-1:2]
        elif heximagetype == 2:
            self.HexagonImage = data[:, ::2, 1:-1:2]
        else:
            raise Exception("heximagetype must be None, 1 or 2")
        self.heximagetype = heximagetype
        self.bands = self.HexagonImage.shape[0]
        self.height = self.HexagonImage.shape[1]
        self.width = self.HexagonImage.shape[2]
        self.geotrans = geotrans
        if self.geotrans is None:
            self.geotrans = (0, 1, 0, 0, 0, 1)
        self.proj = proj
        self.path = 'data'
        self.backend = backend
        self.even_odd_offset = int(even_odd_offset)
        self.shape = (self.bands, self.height, self.width)

    def size(self, index):
        return self.HexagonImage.shape[index]
