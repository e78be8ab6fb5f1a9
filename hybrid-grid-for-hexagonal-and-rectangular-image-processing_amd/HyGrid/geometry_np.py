"""Drop-in for HyGrid.geometry_np: rect<->hex lattice resampling on the MI355X.

Same names, positional order, defaults and `interpolation` strings as the
reference module (/root/reference/HyGrid/geometry_np.py).  The arithmetic runs
in the gfx950 kernels of libhygrid_hip.so:

* NumPy in -> NumPy out, with the reference's output dtype (float64 for the
  interpolating modes, the input dtype for 'nearest') and its `.squeeze()`;
  the fp64 path is bit-exact with the reference.
* torch tensor in -> torch tensor out on the same device; interpolating modes
  return the input's float dtype by default (`out_dtype=` overrides).

Departures (documented in DESIGN.md):
* a 2-D (H, W) raster and a leading batch axis (B, C, H, W) are accepted
  (the reference rejects 2-D input in rect_to_hex_resample, :389);
* hex_to_rect_resample(..., 'nearest') and hexresize(..., 'nearest') work,
  with geometry_torch's rule (geometry_torch.py:335-347) — the NumPy reference
  raises ValueError there (:339, :664);
* image_geometric_transformation(..., 'nearest') works with geometry_torch's rule
  (geometry_torch.py:165-173); the NumPy reference raises ValueError (:172);
* hex_to_rect_resample / image_geometric_transformation(..., 'bilinear') raise
  ValueError — the reference runs
  no blend and returns the uninitialised np.empty (:268-272, :356).
"""
import numpy as np
import torch

from . import _abi, ops

__all__ = ["image_geometric_transformation", "rect_to_hex_resample", "hex_to_rect_resample",
           "hexresize"]

_NP_TO_TORCH = {
    np.dtype(np.uint8): torch.uint8, np.dtype(np.int8): torch.int8,
    np.dtype(np.int16): torch.int16, np.dtype(np.int32): torch.int32,
    np.dtype(np.float16): torch.float16, np.dtype(np.float32): torch.float32,
    np.dtype(np.float64): torch.float64,
}


def _check_ndim(x):
    if x.ndim not in (2, 3, 4):
        raise Exception(f"dim of image should be 2 or 3, but got dim = {x.ndim} instead")


def _to_device(arr):
    """NumPy raster -> device tensor (exact dtype kept; H2D copy)."""
    a = np.ascontiguousarray(arr)
    if a.dtype == np.bool_:
        a = a.astype(np.uint8)
    if a.dtype not in _NP_TO_TORCH:
        # other integer types (uint16/uint32/int64, ...) carry exactly in float64
        a = a.astype(np.float64)
    if not torch.cuda.is_available():
        raise RuntimeError("HyGrid needs a HIP device (MI355X); none is available. "
                           "There is no CPU fallback.")
    return torch.from_numpy(a).to(device=torch.cuda.current_device())


def _run(op, image, size, interp, out_dtype, squeeze):
    _check_ndim(image)
    is_np = not isinstance(image, torch.Tensor)
    x = _to_device(image) if is_np else image
    if is_np and interp == _abi.HG_LINEAR and out_dtype is None:
        out_dtype = torch.float64            # the reference blends and returns fp64
    if size is None:
        size = (int(x.shape[-2]), int(x.shape[-1]))
    y = op(x, size, interp, out_dtype)
    if squeeze:
        y = y.squeeze()
    if is_np:
        y = y.cpu().numpy()
        if interp == _abi.HG_NEAREST and np.asarray(image).dtype != y.dtype:
            y = y.astype(np.asarray(image).dtype)
    return y


def rect_to_hex_resample(rect_image, hex_dsize=None, interpolation='nearest', offset=0,
                         *, out_dtype=None, squeeze=True):
    """rect (C,H,W) -> hex (C,h1,w1); reference geometry_np.py:358-519.

    `offset` is accepted and ignored, as in the reference (it is dead there).
    """
    method_dict = {'nearest': _abi.HG_NEAREST, 'bilinear': _abi.HG_LINEAR}
    method = method_dict[interpolation]          # KeyError, as the reference (:363)
    return _run(ops.rect_to_hex, rect_image, hex_dsize, method, out_dtype, squeeze)


def hex_to_rect_resample(hex_image, rect_dsize=None, interpolation='nearest', offset=0,
                         *, out_dtype=None, squeeze=True):
    """hex (C,H,W) -> rect (C,h1,w1); reference geometry_np.py:191-356."""
    method_dict = {'nearest': 0, 'linear': 1, 'bilinear': 2}
    method = method_dict[interpolation]          # KeyError, as the reference (:197)
    if method == 2:
        raise ValueError("hex_to_rect_resample: 'bilinear' has no blend in the reference "
                         "(geometry_np.py:333-354); use 'linear'")
    return _run(ops.hex_to_rect, hex_image, rect_dsize, method, out_dtype, squeeze)


def hexresize(image, dsize, interpolation="linear", offset=0, *, out_dtype=None,
              squeeze=True):
    """hex (C,H,W) -> hex (C,h1,w1); reference geometry_np.py:520-681."""
    if interpolation == 'linear':
        method = _abi.HG_LINEAR
    elif interpolation == 'nearest':
        method = _abi.HG_NEAREST
    else:
        raise ValueError(f"hexresize: interpolation must be 'linear' or 'nearest', "
                         f"got {interpolation!r}")
    return _run(ops.hexresize, image, dsize, method, out_dtype, squeeze)


def image_geometric_transformation(img, H=np.eye(3), interpolation='nearest', offset=0,
                                   *, out_dtype=None, squeeze=True):
    """Affine transform of a hex raster onto a new hex lattice; reference
    geometry_np.py:6-189.  The output lattice spans the transformed corners of the
    input (:56-87), each sample is inverse-mapped by inv(H) and blended from its
    triangle of input hexagons (:104-187).  `offset` is dead in the reference and
    ignored here."""
    method_dict = {'nearest': 0, 'linear': 1, 'bilinear': 2}
    method = method_dict[interpolation]          # KeyError, as the reference (:17)
    if method == 2:
        raise ValueError("image_geometric_transformation: 'bilinear' has no blend in the "
                         "reference (it returns np.empty, geometry_np.py:103-189); use 'linear'")
    if img.ndim not in (2, 3, 4):
        raise Exception(f"dim of image should be 2 or 3, but got dim = {img.ndim} instead")
    return _run(lambda x, size, interp, od: ops.hex_homography(x, H, interp, od),
                img, None, method, out_dtype, squeeze)
