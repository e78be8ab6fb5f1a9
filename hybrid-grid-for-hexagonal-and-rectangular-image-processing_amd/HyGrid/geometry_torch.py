"""Drop-in for HyGrid.geometry_torch's entry points (hex->rect, geometric transform).

Reference: /root/reference/HyGrid/geometry_torch.py:191-358 (torch-eager, with
the index/weight arrays built on the host and copied to the GPU on every call).
Here the lattice maps are computed inside the gfx950 kernel, so nothing but the
raster crosses PCIe — and nothing at all when a device tensor is passed.

Same signature and return convention as the reference: a NumPy raster comes
back as NumPy (float64 for 'linear', input dtype for 'nearest'); a torch tensor
comes back as a tensor on its device.  The sampling lattice is numpy.linspace's
(geometry_np), not torch.linspace's float32 one (≤2.3e-7 apart).
"""
from .geometry_np import hex_to_rect_resample
from .geometry_np import image_geometric_transformation as _igt_np

__all__ = ["hex_to_square_resample", "image_geometric_transformation_gpu",
           "image_geometric_transformation"]


def hex_to_square_resample(hex_image, square_size=None, interpolation='nearest', offset=0,
                           *, out_dtype=None, squeeze=True):
    """hex (C,H,W) -> rect (C,h1,w1); reference geometry_torch.py:191-358."""
    return hex_to_rect_resample(hex_image, square_size, interpolation, offset,
                                out_dtype=out_dtype, squeeze=squeeze)


def image_geometric_transformation_gpu(image, H=None, interpolation='nearest', offset=0,
                                       *, out_dtype=None, squeeze=True):
    """Reference geometry_torch.py:7-189 (same result convention: NumPy in -> NumPy out).
    The reference casts the inverse-mapped coordinates to float32 (:104) and builds its
    axes with float32 torch.arange; here both stay fp64, i.e. the NumPy twin's lattice
    (geometry_np.py:6-189), so the two entry points agree bit for bit."""
    import numpy as np
    H = np.eye(3) if H is None else H
    return _igt_np(image, H, interpolation, offset, out_dtype=out_dtype, squeeze=squeeze)


def image_geometric_transformation(img, H=None, interpolation='nearest', offset=0,
                                   device='cuda0', **kw):
    """Reference dispatcher geometry_torch.py:442-446.  device='cpu' selects the
    reference's scipy-griddata variant (:374-440), a CPU path this package does not
    provide: it raises instead of silently running something else."""
    if device == 'cuda0':
        return image_geometric_transformation_gpu(img, H, interpolation, offset, **kw)
    if device == 'cpu':
        raise NotImplementedError("image_geometric_transformation(device='cpu'): the scipy "
                                  "griddata variant is not provided; use device='cuda0'")
    return None                                   # the reference falls through (None)
