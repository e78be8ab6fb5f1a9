"""Raster file I/O for the IMAGE / HEXIMAGE containers.

The reference reads rasters with GDAL (`gdal.Open(...).ReadAsArray()`, Image.py:50-58,
89-107) and writes them with GDAL / mmcv / cv2 (Image.py:117-151, HexImage.py:171-218);
none of those is part of this image.  Pillow is, so plain rasters (PNG / TIFF / JPEG)
are read and written through it with the same array convention as the reference:
(bands, H, W) in file band order (GDAL reads RGB; the reference's cv2 / mmcv writers
reverse to BGR only because those libraries expect BGR).  Georeferencing (GDAL
geotransform / projection) is not stored in such files: `geotrans` falls back to the
reference's default (0, 1, 0, 0, 0, 1).

`.heximg` (HexImage.py:89-100, 129-137, 215-218) is a pickled dict.  It is written with
the standard pickle and read back with an unpickler that only resolves numpy's array
reconstruction and plain builtins, so a foreign `.heximg` cannot run code on load.
"""
import io
import os
import pickle

import numpy as np

RASTER_EXT = (".tif", ".TIF", ".tiff", ".TIFF", ".jpg", ".png", ".jpeg", ".JPEG", ".PNG")


def _pil():
    try:
        from PIL import Image as PILImage
    except ImportError as e:  # pragma: no cover - Pillow is in the image
        raise NotImplementedError("raster file I/O needs Pillow (the reference uses GDAL)") from e
    return PILImage


def read_raster(path):
    """-> (bands, H, W) ndarray in file band order (Image.py:98-106)."""
    if not os.path.exists(path):
        raise OSError("path dosen't exist.")   # the reference's message (Image.py:48)
    PILImage = _pil()
    with PILImage.open(path) as im:
        n = getattr(im, "n_frames", 1)
        if n > 1:                                   # multi-page TIFF: one band per page
            bands = []
            for k in range(n):
                im.seek(k)
                bands.append(np.asarray(im))
            a = np.stack(bands, axis=0)
        else:
            a = np.asarray(im)
            a = a[None] if a.ndim == 2 else np.ascontiguousarray(a.transpose(2, 0, 1))
    return a


def save_dtype(arr):
    """The reference's output type rule (Image.py:118-123, HexImage.py:188-196)."""
    name = arr.dtype.name
    if "int8" in name:
        return np.uint8
    if "int16" in name:
        return np.uint16
    return np.uint8


def write_raster(path, arr):
    """(bands, H, W) -> file; 1 band -> grey, 3 -> RGB, 4 -> RGBA, else multi-page TIFF."""
    PILImage = _pil()
    arr = np.asarray(arr)
    if arr.ndim == 2:
        arr = arr[None]
    c = arr.shape[0]
    if arr.dtype == np.uint16 or c not in (1, 3, 4):
        if os.path.splitext(path)[1].lower() not in (".tif", ".tiff"):
            raise ValueError("16-bit or multi-band rasters need a .tif/.tiff path")
        pages = [PILImage.fromarray(np.ascontiguousarray(arr[k])) for k in range(c)]
        pages[0].save(path, save_all=True, append_images=pages[1:])
        return
    img = arr[0] if c == 1 else np.ascontiguousarray(arr.transpose(1, 2, 0))
    PILImage.fromarray(img).save(path)


class _SafeUnpickler(pickle.Unpickler):
    """Resolves only what a `.heximg` dict of numpy arrays needs."""
    _ALLOWED = {
        ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "_reconstruct"),
        ("numpy._core.multiarray", "_reconstruct"), ("numpy.core.multiarray", "scalar"),
        ("numpy._core.multiarray", "scalar"), ("builtins", "tuple"), ("builtins", "list"),
        ("builtins", "dict"), ("builtins", "int"), ("builtins", "float"), ("builtins", "str"),
        ("builtins", "bool"), ("builtins", "complex"), ("builtins", "bytes"),
    }

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f".heximg: refusing to load {module}.{name}")


def load_heximg(path):
    with open(path, "rb") as f:
        return _SafeUnpickler(io.BytesIO(f.read())).load()


def save_heximg(path, dataset):
    with open(path, "wb") as f:
        pickle.dump(dataset, f)
