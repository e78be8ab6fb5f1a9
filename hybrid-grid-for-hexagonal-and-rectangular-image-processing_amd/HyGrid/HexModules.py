"""Drop-in for HyGrid.HexModules: the mmcv-style operator surface of HexConv2d.

Reference: /root/reference/HyGrid/HexModules.py.  `build_hexconv_layer`
(:22-54) and `HexConvModule` (:97-288) keep their signatures, the conv/norm/act
ordering, `bias='auto'`, explicit padding layers, spectral norm and init
behaviour.  If mmcv is importable, HexConv2d is registered in its CONV_LAYERS
registry exactly like the reference (:16) and mmcv's builders are used; if not
(it is absent from this image), a small local registry with the same semantics
covers the layer types the reference's configs use.

Epilogue fusion: when the block is conv -> BatchNorm (running statistics) -> an
elementwise activation, or conv -> activation, `forward` runs ONE gfx950 launch
(hg_hexconv2d_epilogue): the BatchNorm is folded into a per-channel scale / shift and
applied with the bias and the activation in the conv's store, so neither the norm nor
the activation re-reads the conv output.  The unfused torch sequence is kept for
training-mode / non-batch norms, trainable norm parameters under autograd, spectral
norm, other orders and activations.  `fused=False` on the module forces it.
"""
import warnings
from typing import Dict, Optional, Tuple, Union

import torch
import torch.nn as nn

from . import HexFrames as hnn
from . import _abi, ops

try:  # the reference hard-requires mmcv (:7-12); here it is optional
    from mmcv.cnn.bricks.activation import build_activation_layer as _mm_act
    from mmcv.cnn.bricks.norm import build_norm_layer as _mm_norm
    from mmcv.cnn.bricks.padding import build_padding_layer as _mm_pad
    from mmcv.cnn.bricks.registry import CONV_LAYERS as _MM_CONV
    from mmcv.cnn.utils import constant_init as _mm_constant_init
    from mmcv.cnn.utils import kaiming_init as _mm_kaiming_init
    HAVE_MMCV = True
except Exception:  # pragma: no cover - depends on the environment
    HAVE_MMCV = False

__all__ = ["CONV_LAYERS", "build_hexconv_layer", "build_hexpadding_layer",
           "build_hexnorm_layer", "build_hexactivation_layer", "HexConvModule", "HAVE_MMCV"]


class _Registry(dict):
    """Minimal stand-in for mmcv's Registry: `in`, get(), register_module()."""

    def register_module(self, name=None, module=None, force=False):
        key = name or module.__name__
        if key in self and not force:
            raise KeyError(f"{key} is already registered")
        self[key] = module
        return module


if HAVE_MMCV:
    CONV_LAYERS = _MM_CONV
    CONV_LAYERS.register_module('HexConv2d', module=hnn.HexConv2d, force=True)
else:
    CONV_LAYERS = _Registry()
    CONV_LAYERS.register_module('HexConv2d', module=hnn.HexConv2d)

_PADDING = {'zero': nn.ZeroPad2d, 'reflect': nn.ReflectionPad2d,
            'replicate': nn.ReplicationPad2d}
_NORM = {  # type -> (class, abbreviation), as mmcv's NORM_LAYERS
    'BN': (nn.BatchNorm2d, 'bn'), 'BN1d': (nn.BatchNorm1d, 'bn'),
    'BN2d': (nn.BatchNorm2d, 'bn'), 'BN3d': (nn.BatchNorm3d, 'bn'),
    'SyncBN': (nn.SyncBatchNorm, 'bn'), 'GN': (nn.GroupNorm, 'gn'),
    'LN': (nn.LayerNorm, 'ln'), 'IN': (nn.InstanceNorm2d, 'in'),
    'IN1d': (nn.InstanceNorm1d, 'in'), 'IN2d': (nn.InstanceNorm2d, 'in'),
    'IN3d': (nn.InstanceNorm3d, 'in'),
}
_ACT = {'ReLU': nn.ReLU, 'LeakyReLU': nn.LeakyReLU, 'PReLU': nn.PReLU, 'RReLU': nn.RReLU,
        'ReLU6': nn.ReLU6, 'ELU': nn.ELU, 'Sigmoid': nn.Sigmoid, 'Tanh': nn.Tanh,
        'GELU': nn.GELU, 'SiLU': nn.SiLU, 'Swish': nn.SiLU, 'HSigmoid': nn.Hardsigmoid,
        'HSwish': nn.Hardswish}


def build_hexconv_layer(cfg: Optional[Dict], *args, **kwargs) -> nn.Module:
    """Build a conv layer from a config dict (HexModules.py:22-54)."""
    if cfg is None:
        cfg_ = dict(type='HexConv2d')
    else:
        if not isinstance(cfg, dict):
            raise TypeError('cfg must be a dict')
        if 'type' not in cfg:
            raise KeyError('the cfg dict must contain the key "type"')
        cfg_ = cfg.copy()
    layer_type = cfg_.pop('type')
    if layer_type not in CONV_LAYERS:
        raise KeyError(f'Unrecognized layer type {layer_type}')
    conv_layer = CONV_LAYERS.get(layer_type)
    return conv_layer(*args, **kwargs, **cfg_)


def build_hexpadding_layer(cfg: Dict, *args, **kwargs) -> nn.Module:
    """HexModules.py:56-67."""
    if HAVE_MMCV:
        return _mm_pad(cfg, *args, **kwargs)
    if not isinstance(cfg, dict) or 'type' not in cfg:
        raise KeyError('the cfg dict must contain the key "type"')
    cfg_ = cfg.copy()
    t = cfg_.pop('type')
    if t not in _PADDING:
        raise KeyError(f'Unrecognized padding type {t}.')
    return _PADDING[t](*args, **kwargs, **cfg_)


def build_hexnorm_layer(cfg: Dict, num_features: int,
                        postfix: Union[int, str] = '') -> Tuple[str, nn.Module]:
    """HexModules.py:69-89: returns (name, layer)."""
    if HAVE_MMCV:
        return _mm_norm(cfg, num_features, postfix)
    if not isinstance(cfg, dict) or 'type' not in cfg:
        raise KeyError('the cfg dict must contain the key "type"')
    cfg_ = cfg.copy()
    t = cfg_.pop('type')
    if t not in _NORM:
        raise KeyError(f'Unrecognized norm type {t}')
    cls, abbr = _NORM[t]
    requires_grad = cfg_.pop('requires_grad', True)
    cfg_.setdefault('eps', 1e-5)
    if t == 'GN':
        if 'num_groups' not in cfg_:
            raise AssertionError('GN needs num_groups')
        layer = cls(num_channels=num_features, **cfg_)
    elif t == 'LN':
        layer = cls(num_features, **cfg_)
    else:
        layer = cls(num_features, **cfg_)
    for p in layer.parameters():
        p.requires_grad = requires_grad
    return abbr + str(postfix), layer


def build_hexactivation_layer(cfg: Dict) -> nn.Module:
    """HexModules.py:90-91."""
    if HAVE_MMCV:
        return _mm_act(cfg)
    cfg_ = cfg.copy()
    t = cfg_.pop('type')
    if t not in _ACT:
        raise KeyError(f'Unrecognized activation type {t}')
    cls = _ACT[t]
    if t in ('Sigmoid', 'Tanh', 'GELU', 'PReLU', 'HSigmoid', 'Swish') and 'inplace' in cfg_:
        cfg_.pop('inplace')
    return cls(**cfg_)


def _kaiming_init(module, a=0, mode='fan_out', nonlinearity='relu', bias=0,
                  distribution='normal'):
    if HAVE_MMCV:
        return _mm_kaiming_init(module, a=a, nonlinearity=nonlinearity)
    if hasattr(module, 'weight') and module.weight is not None:
        if distribution == 'uniform':
            nn.init.kaiming_uniform_(module.weight, a=a, mode=mode, nonlinearity=nonlinearity)
        else:
            nn.init.kaiming_normal_(module.weight, a=a, mode=mode, nonlinearity=nonlinearity)
    if hasattr(module, 'bias') and module.bias is not None:
        nn.init.constant_(module.bias, bias)


def _constant_init(module, val, bias=0):
    if HAVE_MMCV:
        return _mm_constant_init(module, val, bias=bias)
    if hasattr(module, 'weight') and module.weight is not None:
        nn.init.constant_(module.weight, val)
    if hasattr(module, 'bias') and module.bias is not None:
        nn.init.constant_(module.bias, bias)


_NORM_BATCH_INSTANCE = (nn.modules.batchnorm._BatchNorm, nn.modules.instancenorm._InstanceNorm)

_FUSED_ACTS = {nn.ReLU: _abi.HG_ACT_RELU, nn.LeakyReLU: _abi.HG_ACT_LEAKY_RELU,
               nn.ReLU6: _abi.HG_ACT_RELU6, nn.Sigmoid: _abi.HG_ACT_SIGMOID,
               nn.Tanh: _abi.HG_ACT_TANH}


def _act_grad(y, act, slope):
    """d act / d pre-activation, from the activation's output (torch's own rules:
    threshold_backward on the result for ReLU, hardtanh bounds for ReLU6)."""
    if act == _abi.HG_ACT_RELU:
        return (y > 0).to(y.dtype)
    if act == _abi.HG_ACT_LEAKY_RELU:
        return torch.where(y > 0, torch.ones_like(y), torch.full_like(y, slope))
    if act == _abi.HG_ACT_RELU6:
        return ((y > 0) & (y < 6)).to(y.dtype)
    if act == _abi.HG_ACT_SIGMOID:
        return y * (1 - y)
    if act == _abi.HG_ACT_TANH:
        return 1 - y * y
    return None


class _HexConvEpilogueFn(torch.autograd.Function):
    """conv + bias -> x scale + shift -> act in one launch; backward through the
    activation (from the saved output) and the fixed affine into hexconv2d_backward."""

    @staticmethod
    def forward(ctx, x, kernel, bias, cfg, scale, shift, act, slope):
        y = ops.hexconv2d(x, kernel, bias, cfg["off"], cfg["r"], cfg["stride"], cfg["pad"],
                          cfg["dilation"], cfg["groups"], cfg["padding_mode"],
                          cfg["padding_value"], cfg["out_dtype"],
                          epilogue=(scale, shift, act, slope))
        ctx.save_for_backward(x, kernel, bias, y, scale)
        ctx.meta = (cfg, act, slope)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, kernel, bias, y, scale = ctx.saved_tensors
        cfg, act, slope = ctx.meta
        g = gy
        d = _act_grad(y, act, slope)
        if d is not None:
            g = g * d
        if scale is not None:
            g = g * scale.to(g.dtype).view(1, -1, 1, 1)
        need_x, need_k, need_b = ctx.needs_input_grad[:3]
        gx, gk, gb = ops.hexconv2d_backward(g, x, kernel, bias, cfg, need_x, need_k, need_b)
        return gx, gk, gb, None, None, None, None, None



class HexConvModule(nn.Module):
    """conv/norm/act block around HexConv2d (HexModules.py:97-288)."""

    _abbr_ = 'conv_block'

    def __init__(self, in_channels: int, out_channels: int, even_odd_offset: int,
                 hexkernel_radius: int, stride: int = 1, padding: int = 0, dilation: int = 1,
                 groups: int = 1, bias: Union[bool, str] = 'auto',
                 conv_cfg: Optional[Dict] = None, norm_cfg: Optional[Dict] = None,
                 act_cfg: Optional[Dict] = dict(type='ReLU'), inplace: bool = True,
                 with_spectral_norm: bool = False, padding_mode: str = 'zeros',
                 order: tuple = ('conv', 'norm', 'act')):
        super().__init__()
        assert conv_cfg is None or isinstance(conv_cfg, dict)
        assert norm_cfg is None or isinstance(norm_cfg, dict)
        assert act_cfg is None or isinstance(act_cfg, dict)
        official_padding_mode = ['zeros', 'circular']
        self.conv_cfg = conv_cfg
        self.norm_cfg = norm_cfg
        self.act_cfg = act_cfg
        self.inplace = inplace
        self.with_spectral_norm = with_spectral_norm
        self.with_explicit_padding = padding_mode not in official_padding_mode
        self.order = order
        assert isinstance(self.order, tuple) and len(self.order) == 3
        assert set(order) == {'conv', 'norm', 'act'}

        self.with_norm = norm_cfg is not None
        self.with_activation = act_cfg is not None
        if bias == 'auto':
            bias = not self.with_norm
        self.with_bias = bias

        if self.with_explicit_padding:
            pad_cfg = dict(type=padding_mode)
            self.padding_layer = build_hexpadding_layer(pad_cfg, padding)

        conv_padding = 0 if self.with_explicit_padding else padding
        self.conv = build_hexconv_layer(conv_cfg, in_channels, out_channels, even_odd_offset,
                                        hexkernel_radius, stride=stride, padding=conv_padding,
                                        dilation=dilation, groups=groups, bias=bias)
        self.in_channels = self.conv.in_channels
        self.out_channels = self.conv.out_channels
        self.hexkernel_radius = self.conv.hexkernel_radius
        self.stride = self.conv.stride
        self.padding = padding
        self.dilation = self.conv.dilation
        self.groups = self.conv.groups

        if self.with_spectral_norm:
            # HexConv2d's parameter is `kernel` (the reference passes the module and
            # lets spectral_norm look for `weight`, which fails); normalise `kernel`.
            self.conv = nn.utils.spectral_norm(self.conv, name='kernel')

        if self.with_norm:
            if order.index('norm') > order.index('conv'):
                norm_channels = out_channels
            else:
                norm_channels = in_channels
            self.norm_name, norm = build_hexnorm_layer(norm_cfg, norm_channels)
            self.add_module(self.norm_name, norm)
            if self.with_bias:
                if isinstance(norm, _NORM_BATCH_INSTANCE):
                    warnings.warn('Unnecessary conv bias before batch/instance norm')
        else:
            self.norm_name = None

        if self.with_activation:
            act_cfg_ = act_cfg.copy()
            if act_cfg_['type'] not in ['Tanh', 'PReLU', 'Sigmoid', 'HSigmoid', 'Swish', 'GELU']:
                act_cfg_.setdefault('inplace', inplace)
            self.activate = build_hexactivation_layer(act_cfg_)

        self.init_weights()

    @property
    def norm(self):
        if self.norm_name:
            return getattr(self, self.norm_name)
        return None

    def init_weights(self):
        """HexModules.py:254-273.  HexConv2d has no `weight`, so kaiming_init only
        zeroes the conv bias — the reference's behaviour, kept."""
        if not hasattr(self.conv, 'init_weights'):
            if self.with_activation and self.act_cfg['type'] == 'LeakyReLU':
                nonlinearity = 'leaky_relu'
                a = self.act_cfg.get('negative_slope', 0.01)
            else:
                nonlinearity = 'relu'
                a = 0
            _kaiming_init(self.conv, a=a, nonlinearity=nonlinearity)
        if self.with_norm:
            _constant_init(self.norm, 1, bias=0)

    fused = True

    def _epilogue_plan(self, x, activate, norm):
        """(scale, shift, act, slope) when conv -> norm -> act folds into the conv's
        epilogue, else None."""
        if not self.fused or self.order != ('conv', 'norm', 'act') or self.with_spectral_norm:
            return None
        if type(self.conv) is not hnn.HexConv2d or not x.is_cuda:
            return None
        act, slope = _abi.HG_ACT_NONE, 0.0
        if activate and self.with_activation:
            act = _FUSED_ACTS.get(type(self.activate))
            if act is None:
                return None
            if act == _abi.HG_ACT_LEAKY_RELU:
                slope = float(self.activate.negative_slope)
                if slope < 0:
                    return None
        scale = shift = None
        if norm and self.with_norm:
            bn = self.norm
            if not isinstance(bn, nn.modules.batchnorm._BatchNorm) or bn.training or \
                    bn.running_mean is None:
                return None
            if torch.is_grad_enabled() and any(p.requires_grad for p in bn.parameters()):
                return None
            inv = torch.rsqrt(bn.running_var.double() + bn.eps)
            w = bn.weight.detach().double() if bn.weight is not None else 1.0
            b = bn.bias.detach().double() if bn.bias is not None else 0.0
            scale = (w * inv).float()
            shift = (b - bn.running_mean.double() * w * inv).float()
        if act == _abi.HG_ACT_NONE and scale is None:
            return None
        return scale, shift, act, slope

    def forward(self, x, activate: bool = True, norm: bool = True):
        plan = self._epilogue_plan(x, activate, norm)
        if plan is not None:
            if self.with_explicit_padding:
                x = self.padding_layer(x)
            while x.dim() < 4:
                x = x.unsqueeze(0)
            return _HexConvEpilogueFn.apply(x, self.conv.kernel, self.conv.bias,
                                            self.conv._cfg(), *plan)
        for layer in self.order:
            if layer == 'conv':
                if self.with_explicit_padding:
                    x = self.padding_layer(x)
                x = self.conv(x)
            elif layer == 'norm' and norm and self.with_norm:
                x = self.norm(x)
            elif layer == 'act' and activate and self.with_activation:
                x = self.activate(x)
        return x
