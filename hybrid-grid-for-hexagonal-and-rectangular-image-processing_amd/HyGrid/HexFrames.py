"""Drop-in for HyGrid.HexFrames: the hex-grid convolution operator.

Reference: /root/reference/HyGrid/HexFrames.py.  `HexConv2d` keeps the
reference constructor, attribute names, parameter names (`kernel`
[O, C/g, 1, K], `bias` [O]), initialisation sequence (so a seeded model draws
the same weights), `extra_repr`, and output convention (a float tensor of the
default dtype, (B, O, Ho, Wo)).  Its forward is one gfx950 kernel launch
(hg_hexconv2d): the padding, the double-width "type1" image and the two
strided dense 3x5 convolutions of the reference (:121-162) are folded into the
kernel's index arithmetic.

The state-dict loader also accepts `weight` for `kernel` (the reference's next
version renames it, `future version.txt`:80).

Pooling (`HexPool2d`, `HexAdaptivePool2d`, `HexGlobalPool2d`, :255-410) runs on
hg_hex_pool2d, one pass over the raster with the windows resolved in-kernel instead of
the reference's host-built gather index.  Departures: `stride=None` means
stride = kernel_size (the reference crashes, :270-276); the adaptive / global modules
construct (the reference's method dict names the undefined `centroid_pooling`,
:354-358, :401-405 — 'centroid' raises NotImplementedError here); HexAdaptivePool2d
accepts [h, w] as its own error message promises (:351-353).
"""
import math

import torch
import torch.nn as nn
from torch import Tensor
from torch.nn import init

from . import ops

__all__ = ["HexConv2d", "pad", "heximage_to_type1", "heximage_to_type2", "type1_to_heximage",
           "HexPool2d", "HexAdaptivePool2d", "HexGlobalPool2d", "max_pooling", "min_pooling",
           "average_pooling"]


def pad(input: torch.Tensor, padding: int = 0, mode='constant', value=0) -> torch.Tensor:
    """HexFrames.py:13-21 (kept for API parity; HexConv2d does not call it)."""
    return torch.nn.functional.pad(input, (padding, padding, padding, padding), mode, value)


class _HexConv2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kernel, bias, cfg):
        y = ops.hexconv2d(x, kernel, bias, cfg["off"], cfg["r"], cfg["stride"], cfg["pad"],
                          cfg["dilation"], cfg["groups"], cfg["padding_mode"],
                          cfg["padding_value"], cfg["out_dtype"])
        ctx.save_for_backward(x, kernel, bias)
        ctx.cfg = cfg
        return y

    @staticmethod
    def backward(ctx, gy):
        x, kernel, bias = ctx.saved_tensors
        cfg = ctx.cfg
        need_x, need_k, need_b = ctx.needs_input_grad[:3]
        gx, gk, gb = ops.hexconv2d_backward(gy, x, kernel, bias, cfg, need_x, need_k, need_b)
        return gx, gk, gb, None


class HexConv2d(nn.Module):
    """Hexagonal convolution; reference HexFrames.py:22-185."""

    def __init__(self, in_channels, out_channels, even_odd_offset, hexkernel_radius, stride=1,
                 padding=0, dilation=1, groups=1, bias=True,
                 padding_mode='constant', padding_value=0):
        super(HexConv2d, self).__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.even_odd_offset = even_odd_offset
        self.padded_even_odd_offset = (even_odd_offset + padding) % 2
        self.hexkernel_radius = hexkernel_radius
        self.hexkernel_size = 2 * hexkernel_radius - 1
        self.kernelnum = 3 * hexkernel_radius ** 2 - 3 * hexkernel_radius + 1
        self.stride = stride
        self.sh = stride
        self.sw = stride * 2
        self.out_even_odd_offset = 0
        self.pad = padding
        self.groups = groups
        self.b = bias
        self.dilation = dilation
        self.padding_mode = padding_mode
        self.padding_value = padding_value
        # compute dtype of the output; None = torch.get_default_dtype(), as the
        # reference's torch.empty(...) (:157-160).  bf16/f16 halve the output bytes.
        self.out_dtype = None

        if in_channels % groups != 0:
            raise ValueError('in_channels must be divisible by groups')
        if out_channels % groups != 0:
            raise ValueError('out_channels must be divisible by groups')

        # same creation + init order as the reference (:74-95): identical RNG draws
        self.kernel = nn.Parameter(torch.empty([out_channels, in_channels // groups, 1,
                                                self.kernelnum], dtype=torch.float))
        if self.b == True:  # noqa: E712  (reference semantics)
            self.bias = nn.Parameter(torch.empty([out_channels, ]))
        else:
            self.register_parameter('bias', None)
        self.k_w = 2 * self.dilation * (2 * self.hexkernel_radius - 2) + 1
        self.k_h = (self.hexkernel_size - 1) * self.dilation + 1
        self.reset_parameters()

    def reset_parameters(self):
        init.kaiming_uniform_(self.kernel, a=math.sqrt(5))
        if self.bias is not None:
            fan_in, _ = init._calculate_fan_in_and_fan_out(self.kernel)
            if fan_in != 0:
                bound = 1 / math.sqrt(fan_in)
                init.uniform_(self.bias, -bound, bound)

    def _cfg(self):
        return dict(off=int(self.even_odd_offset), r=self.hexkernel_radius, stride=self.stride,
                    pad=self.pad, dilation=self.dilation, groups=self.groups,
                    padding_mode=self.padding_mode, padding_value=float(self.padding_value),
                    out_dtype=self.out_dtype)

    def forward(self, input: Tensor) -> Tensor:
        while input.dim() < 4:
            input = input.unsqueeze(0)
        return _HexConv2dFn.apply(input, self.kernel, self.bias, self._cfg())

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        wk, kk = prefix + 'weight', prefix + 'kernel'
        if wk in state_dict and kk not in state_dict:
            state_dict[kk] = state_dict.pop(wk)
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)

    def extra_repr(self):
        s = ('{in_channels}, {out_channels}, kernel_radius={hexkernel_radius}'
             ', stride={stride}')
        if self.pad != (0,):
            s += ', padding={pad}'
        if self.dilation != (1,):
            s += ', dilation={dilation}'
        if self.groups != 1:
            s += ', groups={groups}'
        if self.bias is None:
            s += ', bias=False'
        if self.padding_mode != 'zeros':
            s += ', padding_mode={padding_mode}'
        return s.format(**self.__dict__)


# -------------------------- format conversion -------------------------------
def heximage_to_type1(input: torch.Tensor, even_odd_offset) -> torch.Tensor:
    """Offset-row hex image -> double-width type1 raster (HexFrames.py:417-445), one
    gfx950 permute (hg_hex_to_type1):
    type1[y, 2k+L(y)] = type1[y, 2k+1+L(y)] = x[y, k], L(y) = (y%2 + off)%2, 0 elsewhere.
    Output dtype: torch's default float dtype, as the reference's torch.empty (:439)."""
    while input.dim() < 4:
        input = input.unsqueeze(0)
    return ops.hex_to_type1(input, even_odd_offset, 1, torch.get_default_dtype())


def heximage_to_type2(input: torch.Tensor, even_odd_offset) -> torch.Tensor:
    """type1 with every row doubled (HexFrames.py:446-449)."""
    while input.dim() < 4:
        input = input.unsqueeze(0)
    return ops.hex_to_type1(input, even_odd_offset, 2, torch.get_default_dtype())


def type1_to_heximage(input: torch.Tensor, even_odd_offset: int):
    """type1 -> hex image (HexFrames.py:450-458): columns 1::2 (a view, as the
    reference's slice), offset passed through."""
    return input[:, :, :, 1::2], even_odd_offset


# --------------------------- pooling (HexFrames.py:255-479) ---------------------------
_POOL_FNS = ("max", "min", "average")


def max_pooling(input):
    """HexFrames.py:461-463: max over the last dim, NaN ignored (an all-NaN row: -inf)."""
    return ops.reduce_last(input, "max")


def min_pooling(input):
    """HexFrames.py:464-466: min over the last dim, NaN ignored (an all-NaN row: +inf)."""
    return ops.reduce_last(input, "min")


def average_pooling(input):
    """HexFrames.py:467-479: mean of the non-NaN values over the last dim (NaN if none)."""
    return ops.reduce_last(input, "average")


_POOLING_METHODS = {"max": max_pooling, "min": min_pooling, "average": average_pooling}


def _pool_method(method, allow_centroid):
    if method == "centroid" and allow_centroid:
        raise NotImplementedError("centroid pooling: the reference names centroid_pooling "
                                  "but never defines it (HexFrames.py:357, :404)")
    return _POOLING_METHODS[method]          # KeyError for unknown names, as the reference


def _name_of(fn):
    for k, v in _POOLING_METHODS.items():
        if v is fn:
            return k
    raise ValueError("hex pooling: method must be max_pooling, min_pooling or average_pooling")


def _as4d(input):
    while input.dim() < 4:
        input = input.unsqueeze(0)
    if input.dim() > 4:
        raise ValueError(f"hex pooling expects (b, c, h, w), got {tuple(input.shape)}")
    return input


class HexPool2d(nn.Module):
    """Hex-lattice pooling, reference HexFrames.py:255-343.  Output row i pools rows
    i*sh + [0, kh) and columns (i % 2) * sw // 2 + j*sw + [0, kw) of the padded input."""

    def __init__(self, method, kernel_size=2, stride=None,
                 padding=0, even_odd_offset=0,
                 padding_mode='constant', padding_value=0,
                 ceil_mode: bool = False, count_include_pad: bool = True,
                 divisor_override=None):
        super(HexPool2d, self).__init__()
        self.out_offset = 0
        self.offset = (even_odd_offset + padding) % 2
        self.PoolingMethods = dict(_POOLING_METHODS)
        self.method = self.PoolingMethods[method]
        if isinstance(kernel_size, int):
            kernel_size = [kernel_size, kernel_size]
        self.kernel_size = kernel_size
        self.kh, self.kw = kernel_size
        if stride is None:
            stride = list(kernel_size)
        if isinstance(stride, int):
            stride = [stride, stride]
        self.stride = stride
        self.sh, self.sw = self.stride
        self.padding = padding
        self.padding_mode = padding_mode
        self.padding_value = padding_value
        self.ceil_mode = ceil_mode
        self.count_include_pad = count_include_pad

    def forward(self, input):
        input = _as4d(input)
        b, c, h, w = input.size()
        plan = ops.pool_plan(h, w, self.kh, self.kw, self.sh, self.sw, self.padding,
                             self.ceil_mode, self.count_include_pad)
        self.hn, self.wn = plan["hn"], plan["wn"]
        return ops.hex_pool2d(input, _name_of(self.method), self.kh, self.kw, self.sh, self.sw,
                              self.hn, self.wn, self.padding, self.padding_mode,
                              self.padding_value, plan["ext_h"], plan["ext_w"],
                              plan["ext_value"])

    def extra_repr(self) -> str:
        return 'kernel_size={}, stride={}, padding={}'.format(
            self.kernel_size, self.stride, self.padding)


class HexAdaptivePool2d(nn.Module):
    """Reference HexFrames.py:346-396: an outsize grid of (h // hn) x grid_w windows,
    grid_w = w // (wn + 0.5) when the windows are taller than one row (odd rows shift
    by grid_w // 2), else w // wn.  padding arguments are accepted and unused, as in
    the reference."""

    def __init__(self, outsize, method, padding=0, padding_mode='constant', padding_value=0):
        super().__init__()
        if isinstance(outsize, int):
            outsize = [outsize, outsize]
        elif isinstance(outsize, (list, tuple)) and len(outsize) == 2:
            outsize = [int(outsize[0]), int(outsize[1])]
        else:
            raise Exception('outsize must be an int s or a list [h, w]')
        self.hn, self.wn = outsize
        self.PoolingMethods = dict(_POOLING_METHODS)
        self.method = _pool_method(method, True)

    def forward(self, input):
        input = _as4d(input)
        b, c, h, w = input.size()
        grid_h = int(h / self.hn)
        grid_w = int(w / (self.wn + 0.5)) if grid_h > 1 else int(w / self.wn)
        if grid_h * grid_w == 0 and self.method is not average_pooling:
            raise RuntimeError("hex adaptive pooling: empty windows (output larger than input)")
        shift = grid_w // 2 if self.hn >= 2 else 0
        if self.hn * self.wn > 0 and ((self.hn - 1) * grid_h + grid_h > h or
                                      (self.wn - 1) * grid_w + shift + grid_w > w):
            raise IndexError("hex adaptive pooling: windows reach outside the input (the "
                             "reference's gather raises)")
        return ops.hex_pool2d(input, _name_of(self.method), grid_h, grid_w, max(grid_h, 1),
                              max(grid_w, 1), self.hn, self.wn)


class HexGlobalPool2d(nn.Module):
    """Reference HexFrames.py:397-410: one value per (b, c) over the whole raster."""

    def __init__(self, method):
        super(HexGlobalPool2d, self).__init__()
        self.PoolingMethods = dict(_POOLING_METHODS)
        self.method = _pool_method(method, True)

    def forward(self, input):
        input = _as4d(input)
        b, c, h, w = input.size()
        y = ops.hex_pool2d(input, _name_of(self.method), h, w, max(h, 1), max(w, 1), 1, 1)
        return y[..., 0, 0]
