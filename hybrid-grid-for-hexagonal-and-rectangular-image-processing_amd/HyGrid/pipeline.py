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


_STREAMS = {}


def _side_streams(dev, n):
    """n HIP streams of device dev, created once per process (a pool, not per call)."""
    key = (dev.index, n)
    if key not in _STREAMS:
        _STREAMS[key] = [torch.cuda.Stream(dev) for _ in range(n)]
    return _STREAMS[key]


def _pyramid_fused_groups(x, conv, levels, out_dtype, l0_from_rect, groups):
    """The fused levels with the batch split into `groups` runs of images, each run's level
    chain on its own HIP stream (images are independent, every reference entry point is
    per-image): one run's level launches fill the chip while another's ramp up or drain.
    Outputs are allocated once for the whole batch on the caller's stream; each run writes
    its slices; the caller's stream waits for every run.  Returns the level list or None."""
    B, C, H, W = (int(v) for v in x.shape)
    dev = x.device
    main = torch.cuda.current_stream(dev)
    sizes, h_, w_ = [], H, W
    for _ in range(levels):
        h_, w_ = h_ // 2, w_ // 2
        sizes.append((h_, w_))
    outs = [torch.empty((B, C, h, w), dtype=out_dtype, device=dev) for h, w in sizes]
    bounds = [(g * B) // groups for g in range(groups + 1)]
    fork = torch.cuda.Event()
    fork.record(main)
    streams = _side_streams(dev, groups)
    ok = True
    for g in range(groups):
        s0, s1 = bounds[g], bounds[g + 1]
        st = streams[g]
        st.wait_event(fork)
        with torch.cuda.stream(st):
            cur = x[s0:s1]
            for lv, (h1, w1) in enumerate(sizes):
                y = ops.hex_pyramid_level(cur, conv.kernel, conv.bias, (h1, w1),
                                          int(conv.even_odd_offset),
                                          from_rect=(lv == 0 and l0_from_rect),
                                          out_dtype=out_dtype, out=outs[lv][s0:s1])
                if y is None:
                    ok = False
                    break
                cur = y
        x.record_stream(st)              # the caching allocator: used on st until it is done
        for o in outs:
            o.record_stream(st)
        if not ok:
            break
    for g in range(groups):
        main.wait_stream(streams[g])
    return outs if ok else None


def hex_pyramid(x, conv, levels=3, out_dtype=None, fused=True, l0_from_rect=True, groups=None):
    """Hex Gaussian pyramid (BASELINE config 5): rect -> hex at full size
    (geometry_np.py:358-519), then `levels` x [conv (a HexConv2d, HexFrames.py:96-169)
    -> hexresize to (h//2, w//2) (geometry_np.py:520-681)].  Returns the list of level
    images [(B, C, h/2, w/2), (B, C, h/4, w/4), ...], each stored in out_dtype (default:
    x's dtype when 16-bit, else fp32).

    With a depthwise radius-2 conv (pyramid_fusable) and no autograd, every level is one
    pass of hg_hex_pyramid_level with the intermediates in fp32 on chip; level 0 reads the
    rect image and makes rect -> hex on the fly (l0_from_rect, the streaming kernel's FR
    mode: 1.12 vs 1.29 ms for a separate rect -> hex pass on config 5, tools/ab_pyramid.py);
    otherwise the operator chain, which stores every stage in out_dtype.  groups: the fused
    levels run as that many runs of images on separate HIP streams (default: 2 for a batch of
    >= 2 rect images; 1 = one stream); each level launch of a short pyramid pays a ramp and a
    tail of 16-50 us (profiles/r06/launch_edges.txt), which the other run's work fills.
    """
    if out_dtype is None:
        out_dtype = x.dtype if x.dtype in (torch.bfloat16, torch.float16) else torch.float32
    H, W = x.shape[-2:]
    outs = []
    if fused and pyramid_fusable(conv) and not torch.is_grad_enabled():
        if groups is None:
            groups = 2 if (x.dim() == 4 and x.shape[0] >= 2 and l0_from_rect) else 1
        groups = max(1, min(int(groups), int(x.shape[0]) if x.dim() == 4 else 1))
        if groups > 1 and l0_from_rect and x.dim() == 4:
            got = _pyramid_fused_groups(x.contiguous(), conv, levels, out_dtype, l0_from_rect,
                                        groups)
            if got is not None:
                return got
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
