"""The user-script chain rect -> hex -> HexConv2d -> hex -> rect as one call.

The reference runs it as three host round trips (SURVEY.md §3 B + C):
rect_to_hex_resample (geometry_np.py:358-519) -> HexConvModule / HexConv2d
(HexModules.py:275-288, HexFrames.py:96-169) -> hex_to_rect_resample
(geometry_np.py:191-356).  `rect_hex_conv_rect` runs the fused gfx950 kernel
(hg_pipeline_r2h_conv_h2r: one read of the input, one write of the output)
whenever the geometry is near-identity and the layer is a plain radius-2,
stride-1, constant-padded HexConv2d; otherwise the three HIP operators.
"""
import os

import torch

from . import ops
from .HexFrames import HexConv2d

__all__ = ["rect_hex_conv_rect", "rect_hex_rect", "fusable", "hex_pyramid", "pyramid_fusable"]


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


def rect_hex_rect(x, hex_size=None, out_dtype=None, fused=True):
    """The rect -> hex -> rect round trip (BASELINE config 2): x (..., H, W) device tensor ->
    (..., h1, w1), the same result as ops.hex_to_rect(ops.rect_to_hex(x, hex_size), hex_size)
    (geometry_np.py:358-519 then :191-356) with the hex image in fp32.  One pass of the
    fused kernel (hg_pipeline_r2h_h2r) for the same-size lattices, else the two resamplers.
    """
    if out_dtype is None:
        out_dtype = x.dtype if x.dtype in (torch.bfloat16, torch.float16) else torch.float32
    if fused:
        y = ops.pipeline_r2h_h2r(x, hex_size, out_dtype)
        if y is not None:
            return y
    h = ops.rect_to_hex(x, hex_size, out_dtype=torch.float32)
    return ops.hex_to_rect(h, tuple(h.shape[-2:]), out_dtype=out_dtype)


def pyramid_fusable(conv):
    """A depthwise (groups == C == O), radius-2, stride-1, dilation-1 HexConv2d padded
    with constant 0 by one sample: what the fused pyramid level kernel implements."""
    return (isinstance(conv, HexConv2d) and conv.hexkernel_radius == 2 and conv.stride == 1
            and conv.dilation == 1 and conv.padding_mode in ("constant", "zeros")
            and conv.pad == 1 and float(conv.padding_value) == 0.0
            and conv.in_channels == conv.out_channels == conv.groups
            and conv.kernel.dtype == torch.float32)


def hex_pyramid(x, conv, levels=3, out_dtype=None, fused=True, l0_from_rect=True):
    """Hex Gaussian pyramid (BASELINE config 5): rect -> hex at full size
    (geometry_np.py:358-519), then `levels` x [conv (a HexConv2d, HexFrames.py:96-169)
    -> hexresize to (h//2, w//2) (geometry_np.py:520-681)].  Returns the list of level
    images [(B, C, h/2, w/2), (B, C, h/4, w/4), ...], each stored in out_dtype (default:
    x's dtype when 16-bit, else fp32).

    With a depthwise radius-2 conv (pyramid_fusable) and no autograd, every level is one
    pass of hg_hex_pyramid_level with the intermediates in fp32 on chip; level 0 reads the
    rect image and makes rect -> hex on the fly (l0_from_rect, the streaming kernel's FR
    mode: 1.12 vs 1.29 ms for a separate rect -> hex pass on config 5, tools/ab_pyramid.py);
    otherwise the operator chain, which stores every stage in out_dtype.  Round 6 measured two
    ways of hiding the level launches' ramps and tails, both slower and not the default: the
    levels in ONE launch (ops.hex_pyramid_chain, bit-identical; its inter-workgroup hand-off
    costs 2.7x the per-level time; opt in with HYGRID_PYR_CHAIN=1) and the batch split into
    runs of images on 2 / 4 / 8 HIP streams (4-13 % slower than one stream); profiles/r06/.
    """
    if out_dtype is None:
        out_dtype = x.dtype if x.dtype in (torch.bfloat16, torch.float16) else torch.float32
    H, W = x.shape[-2:]
    outs = []
    if fused and pyramid_fusable(conv) and not torch.is_grad_enabled():
        if (os.environ.get("HYGRID_PYR_CHAIN") == "1" and l0_from_rect and x.dtype == out_dtype
                and 2 <= levels <= 3):
            # opt-in: every level in one launch (hg_hex_pyramid_chain, round 6; measured 2.7x
            # slower than one launch per level); None outside its domain
            outs = ops.hex_pyramid_chain(x, conv.kernel, conv.bias, levels,
                                         int(conv.even_odd_offset))
            if outs is not None:
                return outs
            outs = []
        cur, h_, w_, ok = x, H, W, True
        if not l0_from_rect:
            cur = ops.rect_to_hex(x, (H, W), out_dtype=out_dtype)
        for lv in range(levels):
            h_, w_ = h_ // 2, w_ // 2
            y = ops.hex_pyramid_level(cur, conv.kernel, conv.bias, (h_, w_),
                                      int(conv.even_odd_offset),
                                      from_rect=(lv == 0 and l0_from_rect), out_dtype=out_dtype)
            if y is None:
                ok = False
                break
            outs.append(y)
            cur = y
        if ok:
            return outs
        outs = []
    hx = ops.rect_to_hex(x, (H, W), out_dtype=out_dtype)
    prev = getattr(conv, "out_dtype", None)
    conv.out_dtype = out_dtype
    try:
        h_, w_ = H, W
        for _ in range(levels):
            h_, w_ = h_ // 2, w_ // 2
            hx = ops.hexresize(conv(hx), (h_, w_), out_dtype=out_dtype)
            outs.append(hx)
    finally:
        conv.out_dtype = prev
    return outs
