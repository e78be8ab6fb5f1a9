"""GPU: HexConvModule epilogue fusion — conv + bias -> BatchNorm
(running statistics, folded to scale / shift) -> activation in one hg_hexconv2d_epilogue
launch, against the module's unfused sequence (hg_hexconv2d, then torch BatchNorm2d and
the torch activation — the reference's HexModules.py:258-268 order).  fp32 tolerance
1e-5 (the folded BatchNorm rounds differently).  Gradients through the fused
autograd Function against the unfused autograd graph."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a HIP device", allow_module_level=True)

from HyGrid import HexModules as HM  # noqa: E402

DEV = torch.device("cuda:0")

ACTS = [dict(type="ReLU"), dict(type="LeakyReLU", negative_slope=0.1), dict(type="ReLU6"),
        dict(type="Sigmoid"), dict(type="Tanh"), None]
SHAPES = [  # (C, O, radius, stride, groups, padding): stream path, LDS path, direct path
    (3, 3, 2, 1, 1, 1), (3, 3, 2, 1, 3, 1), (8, 16, 2, 1, 1, 1), (4, 8, 3, 1, 2, 2),
    (3, 6, 2, 2, 1, 1), (1, 1, 2, 1, 1, 0)]


def _randomize_bn(bn, seed):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        bn.running_mean.copy_(torch.randn(bn.num_features, generator=g))
        bn.running_var.copy_(torch.rand(bn.num_features, generator=g) + 0.5)
        bn.weight.copy_(torch.randn(bn.num_features, generator=g))
        bn.bias.copy_(torch.randn(bn.num_features, generator=g))


@pytest.mark.parametrize("si", range(len(SHAPES)))
@pytest.mark.parametrize("ai", range(len(ACTS)))
def test_fused_eval_matches_unfused(si, ai):
    C, O, r, s, g, p = SHAPES[si]
    torch.manual_seed(si * 10 + ai)
    m = HM.HexConvModule(C, O, 0, r, stride=s, padding=p, groups=g,
                         norm_cfg=dict(type="BN"), act_cfg=ACTS[ai]).to(DEV).eval()
    _randomize_bn(m.norm, si + 7 * ai)
    x = torch.rand(2, C, 37, 70, device=DEV)
    with torch.no_grad():
        assert m._epilogue_plan(x, True, True) is not None
        y = m(x)
        m.fused = False
        ref = m(x)
    torch.testing.assert_close(y, ref, rtol=1e-5, atol=1e-5)
    # norm=False / activate=False flags fold only what runs
    with torch.no_grad():
        m.fused = True
        y2 = m(x, norm=False)
        m.fused = False
        torch.testing.assert_close(y2, m(x, norm=False), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("ai", range(5))
def test_fused_training_no_norm_grads(ai):
    torch.manual_seed(ai)
    m = HM.HexConvModule(3, 3, 0, 2, padding=1, act_cfg=ACTS[ai]).to(DEV)
    with torch.no_grad():
        m.conv.bias.uniform_(-0.3, 0.3)
    x = torch.rand(2, 3, 33, 65, device=DEV)
    gy = torch.randn(2, 3, 33, 65, device=DEV)
    xa = x.clone().requires_grad_(True)
    assert m._epilogue_plan(xa, True, True) is not None
    ya = m(xa)
    ya.backward(gy)
    grads_a = (xa.grad.clone(), m.conv.kernel.grad.clone(), m.conv.bias.grad.clone())
    m.zero_grad()
    m.fused = False
    xb = x.clone().requires_grad_(True)
    yb = m(xb)
    yb.backward(gy)
    torch.testing.assert_close(ya, yb, rtol=1e-5, atol=1e-5)
    for ga, gb in zip(grads_a, (xb.grad, m.conv.kernel.grad, m.conv.bias.grad)):
        torch.testing.assert_close(ga, gb, rtol=1e-4, atol=1e-4)


def test_frozen_bn_training_grads():
    """Eval-mode BatchNorm with frozen affine (a common backbone setting) stays fused
    under autograd; a trainable BatchNorm falls back to the unfused graph."""
    torch.manual_seed(3)
    m = HM.HexConvModule(8, 16, 1, 2, padding=1, norm_cfg=dict(type="BN")).to(DEV)
    m.norm.eval()
    _randomize_bn(m.norm, 11)
    x = torch.rand(2, 8, 30, 41, device=DEV)
    xr = x.clone().requires_grad_(True)
    assert m._epilogue_plan(xr, True, True) is None           # trainable BN params
    for p in m.norm.parameters():
        p.requires_grad_(False)
    assert m._epilogue_plan(xr, True, True) is not None
    gy = torch.randn(2, 16, 30, 41, device=DEV)
    ya = m(xr)
    ya.backward(gy)
    ga, gk = xr.grad.clone(), m.conv.kernel.grad.clone()
    m.zero_grad()
    m.fused = False
    xb = x.clone().requires_grad_(True)
    yb = m(xb)
    yb.backward(gy)
    torch.testing.assert_close(ya, yb, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(ga, xb.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(gk, m.conv.kernel.grad, rtol=1e-4, atol=1e-3)


def test_training_bn_not_fused():
    m = HM.HexConvModule(3, 3, 0, 2, padding=1, norm_cfg=dict(type="BN")).to(DEV).train()
    x = torch.rand(1, 3, 16, 16, device=DEV)
    with torch.no_grad():
        assert m._epilogue_plan(x, True, True) is None       # batch statistics
    m2 = HM.HexConvModule(3, 3, 0, 2, padding=1, act_cfg=dict(type="GELU")).to(DEV)
    assert m2._epilogue_plan(x, True, True) is None          # unsupported activation
