"""Drop-in for HyGrid.HexImage: the hex raster container HEXIMAGE.

Reference: /root/reference/HyGrid/HexImage.py.  Kept: the constructor for files and
in-memory data with heximagetype None (a rect raster converted with rect->hex
'nearest'), 1 (type1 double-width storage) and 2 (type2) (:44-125), the `.heximg`
dict format (:89-100, 129-137, 215-218), `build_Heximagedataset`,
`GenerateType1Image` / `GenerateType2Image` (:139-170: one gfx950 permute each
instead of per-row Python loops) and `SaveHexImage` (:171-218).  Raster files go
through Pillow (see `_io`), `.heximg` through a restricted unpickler.  The OpenGL
hex-mosaic viewer `Hex_imshow` (:219-276) is display-only and not provided.
"""
import os

import numpy as np
import torch

from . import _io, ops
from .Image import IMAGE

__all__ = ["HEXIMAGE"]


def _type1_on_device(hexmatrix, off, rep):
    """(bands, h, w) ndarray -> float64 type1 / type2 raster via hg_hex_to_type1."""
    if not torch.cuda.is_available():
        raise RuntimeError("HyGrid needs a HIP device (MI355X); none is available. "
                           "There is no CPU fallback.")
    x = torch.from_numpy(np.ascontiguousarray(hexmatrix, dtype=np.float64)).cuda()
    return ops.hex_to_type1(x, off, rep).cpu().numpy()


class HEXIMAGE(IMAGE):
    def __init__(self, pathname=None, heximagetype=None, data=None, geotrans=None, proj=None,
                 even_odd_offset=False, backend='gdal'):
        if pathname is None and data is None:
            raise ValueError("pathname and data can not be None at the same time")
        if pathname is not None and data is not None:
            raise ValueError("pathname and data can not be Given at the same time")
        if pathname is not None:
            ext = os.path.splitext(pathname)[1]
            if ext == ".heximg":                                   # :89-102
                self.datapath = pathname
                self.Heximagedataset = _io.load_heximg(pathname)
                self.filetype = 2
                self.height = self.Heximagedataset['height']
                self.width = self.Heximagedataset['width']
                self.bands = self.Heximagedataset['bands']
                self.geotrans = self.Heximagedataset['geotransform']
                self.proj = self.Heximagedataset['projection']
                self.even_odd_offset = self.Heximagedataset['offset']
                self.HexagonImage = self.Heximagedataset['HexMatrix']
                if self.HexagonImage.ndim < 3:
                    self.HexagonImage = np.broadcast_to(self.HexagonImage,
                                                        (3, self.height, self.width))
                self.backend = backend
            elif ext in _io.RASTER_EXT:
                super().__init__(pathname, backend=backend)
                self.heximagetype = heximagetype
                if heximagetype is None:                           # :61-63
                    self.HexagonImage = self.ConvertToHexagon()
                    if self.HexagonImage.ndim == 2:
                        self.HexagonImage = self.HexagonImage[None]
                    self.bands, self.height, self.width = self.HexagonImage.shape[0:3]
                elif heximagetype == 1:                            # :65-70
                    tmp = self.LoadImageArray()
                    self.width = (self.width - 1) // 2
                    self.HexagonImage = np.zeros([self.bands, self.height, self.width])
                    self.HexagonImage[:, :, :] = tmp[:, :, 1::2]
                elif heximagetype == 2:                            # :72-84
                    tmp = self.LoadImageArray()
                    if (self.width & 1) == 0:
                        tmp = np.append(tmp, np.zeros((self.bands, self.height, 1)), axis=2)
                        self.width += 1
                    self.height = self.height // 2
                    self.width = (self.width - 1) // 2
                    self.HexagonImage = np.zeros([self.bands, self.height, self.width])
                    self.HexagonImage[:, :, :] = tmp[:, ::2, 1::2]
                else:
                    raise Exception("heximagetype must be None, 1 or 2")
            else:
                raise Exception(f"unsupported file type {ext!r}")
        else:                                                      # :103-120
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

    def build_Heximagedataset(self):
        """HexImage.py:129-137."""
        self.Heximagedataset = {
            'height': self.height, 'width': self.width, 'bands': self.bands,
            'geotransform': self.geotrans, 'projection': self.proj,
            'offset': self.even_odd_offset, 'HexMatrix': np.asarray(self.HexagonImage)}

    def GenerateType1Image(self):
        """HexImage.py:139-153: (bands, h, 2w+1) float64 + geotransform with pixel
        height x2."""
        img = _type1_on_device(self.HexagonImage, self.even_odd_offset, 1)
        g = self.geotrans
        return img, (g[0], g[1], g[2], g[3], g[4], g[5] * 2,)

    def GenerateType2Image(self):
        """HexImage.py:154-170: (bands, 2h, 2w+1) float64, rows doubled."""
        img = _type1_on_device(self.HexagonImage, self.even_odd_offset, 2)
        g = self.geotrans
        return img, (g[0], g[1], g[2], g[3], g[4], g[5],)

    def SaveHexImage(self, pathname, imagetype=1, filetype=1):
        """HexImage.py:171-218: `.heximg` (filetype 2) pickles the dataset dict; raster
        files store the type1 / type2 image as uint8 / uint16 (jpg -> png, lossless)."""
        file_name, ext = os.path.splitext(pathname)
        if ext == ".heximg":
            filetype = 2
        if ext in ("JPG", ".jpg", "JPEG", "jpeg"):
            ext = ".png"
        pathname = file_name + ext
        if filetype == 1:
            tmp, _ = self.GenerateType1Image() if imagetype == 1 else self.GenerateType2Image()
            _io.write_raster(pathname, tmp.astype(_io.save_dtype(np.asarray(self.HexagonImage))))
        else:
            self.build_Heximagedataset()
            _io.save_heximg(pathname, self.Heximagedataset)

    def Hex_imshow(self):
        raise NotImplementedError("HEXIMAGE.Hex_imshow: the OpenGL viewer is display-only "
                                  "and outside the accelerated path")
