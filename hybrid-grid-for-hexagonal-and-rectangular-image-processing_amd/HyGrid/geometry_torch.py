"""Drop-in for HyGrid.geometry_torch's hex->rect entry point.

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

__all__ = ["hex_to_square_resample"]


def hex_to_square_resample(hex_image, square_size=None, interpolation='nearest', offset=0,
                           *, out_dtype=None, squeeze=True):
    """hex (C,H,W) -> rect (C,h1,w1); reference geometry_torch.py:191-358."""
    return hex_to_rect_resample(hex_image, square_size, interpolation, offset,
                                out_dtype=out_dtype, squeeze=squeeze)
