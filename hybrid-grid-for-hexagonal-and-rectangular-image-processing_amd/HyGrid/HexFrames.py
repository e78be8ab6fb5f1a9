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
"""
import math

import torch
import torch.nn as nn
from torch import Tensor
from torch.nn import init

from . import ops

__all__ = ["HexConv2d", "pad", "heximage_to_type1", "heximage_to_type2", "type1_to_heximage"]


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
