"""The user-script chain rect -> hex -> HexConv2d -> hex -> rect as one call.

The reference runs it as three host round trips (SURVEY.md §3 B + C):
rect_to_hex_resample (geometry_np.py:358-519) -> HexConvModule / HexConv2d
(HexModules.py:275-288, HexFrames.py:96-169) -> hex_to_rect_resample
(geometry_np.py:191-356).  `rect_hex_conv_rect` runs the fused gfx950 kernel
(hg_pipeline_r2h_conv_h2r: one read of the input, one write of the output)
whenever the geometry is near-identity and the layer is a plain radius-2,
stride-1, constant-padded HexConv2d; otherwise the three HIP operators.
"""
import torch

from . import ops
from .HexFrames import HexConv2d

__all__ = ["rect_hex_conv_rect", "fusable", "hex_pyramid"]


def fusable(conv):
    """A plain radius-2, stride-1, dilation-1, constant-padded HexConv2d with
    C == O in {1, 3} and groups in {1, C}: what the fused kernel implements."""
    return (isinstance(conv, HexConv2d) and conv.hexkernel_radius == 2 and conv.stride == 1
            and conv.dilation == 1 and conv.padding_mode in ("constant", "zeros")
            and conv.in_channels == conv.out_channels and conv.in_channels in (1, 3)
            and conv.groups in (1, conv.in_channels) and conv.kernel.dtype == torch.float32)


def rect_hex_conv_rect(x, conv, hex_size=None, rect_size=None, out_dtype=None, fused=True):
    """x: (B, C, H, W) device tensor -> (B, O, h2, w2).

    Same result as ops.hex_to_rect(conv(ops.rect_to_hex(x, hex_size)), rect_size)
    with fp32 intermediates (not rounded to out_dtype between stages).
    """
    if out_dtype is None:
        out_dtype = x.dtype if x.dtype in (torch.bfloat16, torch.float16) else torch.float32
    if fused and fusable(conv) and not torch.is_grad_enabled():
        y = ops.pipeline_r2h_conv_h2r(x, conv.kernel, conv.bias, hex_size, rect_size,
                                      conv.pad, conv.groups, int(conv.even_odd_offset),
                                      float(conv.padding_value), out_dtype)
        if y is not None:
            return y
    h = ops.rect_to_hex(x, hex_size, out_dtype=torch.float32)
    c = conv(h)
    return ops.hex_to_rect(c, rect_size, out_dtype=out_dtype)


def hex_pyramid(x, conv, levels=3, out_dtype=None):
    """Hex Gaussian pyramid (BASELINE config 5): rect -> hex at full size
    (geometry_np.py:358-519), then `levels` x [conv (a HexConv2d, HexFrames.py:96-169)
    -> hexresize to (h//2, w//2) (geometry_np.py:520-681)].  Returns the list of level
    images [(B, C, h/2, w/2), (B, C, h/4, w/4), ...], each stored in out_dtype (default:
    x's dtype when 16-bit, else fp32), as the operator chain stores them.
    """
    if out_dtype is None:
        out_dtype = x.dtype if x.dtype in (torch.bfloat16, torch.float16) else torch.float32
    H, W = x.shape[-2:]
    hx = ops.rect_to_hex(x, (H, W), out_dtype=out_dtype)
    prev = getattr(conv, "out_dtype", None)
    conv.out_dtype = out_dtype
    try:
        outs = []
        h_, w_ = H, W
        for _ in range(levels):
            h_, w_ = h_ // 2, w_ // 2
            hx = ops.hexresize(conv(hx), (h_, w_), out_dtype=out_dtype)
            outs.append(hx)
    finally:
        conv.out_dtype = prev
    return outs
