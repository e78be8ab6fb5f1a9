"""HyGrid — MI355X-native hex<->rect lattice resampling and hex convolution.

Drop-in for the reference package's hot path (Tesla-Albert/Hybrid-Grid-for-
Hexagonal-and-Rectangular-Image-Processing, `HyGrid`): the modules keep the
reference's names (geometry_np, geometry_torch, HexFrames, HexModules, Image,
HexImage) and run on hand-written gfx950 HIP kernels through a C ABI
(include/hygrid.h, libhygrid_hip.so).
"""
__version__ = "1.1.0+mi355x"
