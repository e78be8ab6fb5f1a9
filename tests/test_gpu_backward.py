"""GPU parity of the HexConv2d backward (hg_hexconv2d_backward).

Pinned to the reference's own autograd gradients (tests/golden/hexconv_bwd.npz, captured
by tests/golden/make_golden.py from HyGrid/HexFrames.py:96-169 in fp32) and to the CPU
adjoint oracle/hg_oracle.c (or_hexconv2d_backward, fp64).  Tolerances: fp32 sums over
up to B*ho*wo terms in a different order than torch -> rtol 1e-4 (atol 1e-5 * max|ref|);
bf16 d input: one bf16 rounding (2^-8 * max|ref|).
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a HIP device", allow_module_level=True)

from HyGrid import ops  # noqa: E402
from HyGrid.HexFrames import HexConv2d  # noqa: E402

DEV = torch.device("cuda:0")


def close(got, ref, rtol):
    got = np.asarray(got, np.float64)
    np.testing.assert_allclose(got, ref, rtol=rtol, atol=rtol * 0.1 * max(np.abs(ref).max(), 1e-30))


def cfg_of(meta):
    return dict(off=meta["off"], r=meta["r"], stride=meta["stride"], pad=meta["pad"],
                dilation=meta["dilation"], groups=meta["groups"],
                padding_mode=meta["padding_mode"], padding_value=meta["padding_value"],
                out_dtype=None)


def test_backward_vs_reference_autograd(golden, golden_index):
    g = golden("hexconv_bwd")
    n = 0
    for meta in golden_index["hexconv_bwd"]:
        if "error" in meta:
            continue
        ci = meta["case"]
        x = torch.from_numpy(g[f"c{ci}_x"]).to(DEV)
        k = torch.from_numpy(g[f"c{ci}_kernel"]).to(DEV)
        b = torch.from_numpy(g[f"c{ci}_bias"]).to(DEV) if f"c{ci}_bias" in g else None
        gy = torch.from_numpy(g[f"c{ci}_gy"]).to(DEV)
        dx, dk, db = ops.hexconv2d_backward(gy, x, k, b, cfg_of(meta))
        close(dx.cpu().numpy(), g[f"c{ci}_dx"], 1e-4)
        close(dk.cpu().numpy(), g[f"c{ci}_dkernel"], 1e-4)
        if b is not None:
            close(db.cpu().numpy(), g[f"c{ci}_dbias"], 1e-4)
        n += 1
    assert n >= 50


@pytest.mark.parametrize("mode", ["constant", "reflect", "replicate", "circular"])
@pytest.mark.parametrize("p", [(2, 1, 1, 1, 3), (3, 2, 2, 2, 1), (2, 1, 1, 3, 3)])
def test_autograd_module_vs_oracle(mode, p):
    """HexConv2d(...).backward through torch autograd on the GPU against the fp64
    adjoint oracle on the same data (x.grad, kernel.grad, bias.grad)."""
    r, s, d, pad, groups = p
    torch.manual_seed(7)
    m = HexConv2d(3, 6, 1, r, stride=s, padding=pad, dilation=d, groups=groups, bias=True,
                  padding_mode=mode, padding_value=0.25).to(DEV)
    x = torch.rand((2, 3, 31, 45), device=DEV, requires_grad=True)
    y = m(x)
    gy = torch.randn_like(y)
    y.backward(gy)
    dx, dk, db = O.hexconv2d_backward(
        x.detach().double().cpu().numpy(), m.kernel.detach().double().cpu().numpy(),
        gy.double().cpu().numpy(), 1, r, s, pad, d, groups, mode, 0.25)
    close(x.grad.cpu().numpy(), dx, 1e-4)
    close(m.kernel.grad.cpu().numpy(), dk, 1e-4)
    close(m.bias.grad.cpu().numpy(), db, 1e-4)


def test_backward_bf16_input_and_fp64_kernel():
    torch.manual_seed(11)
    x = torch.rand((2, 3, 64, 96), device=DEV)
    k = (torch.rand((3, 3, 1, 7), device=DEV) - 0.5)
    b = torch.rand((3,), device=DEV)
    cfg = dict(off=0, r=2, stride=1, pad=1, dilation=1, groups=1, padding_mode="constant",
               padding_value=0.0, out_dtype=None)
    ho, wo = ops.hexconv2d_out_shape(64, 96, 2, 1, 1, 1)
    gy = torch.randn((2, 3, ho, wo), device=DEV)
    dx, dk, db = O.hexconv2d_backward(x.double().cpu().numpy(), k.double().cpu().numpy(),
                                      gy.double().cpu().numpy(), 0, 2, 1, 1)
    gx, gk, gb = ops.hexconv2d_backward(gy, x.bfloat16(), k, b, cfg)
    assert gx.dtype == torch.bfloat16
    np.testing.assert_allclose(gx.double().cpu().numpy(), dx, rtol=2 ** -8,
                               atol=2 ** -8 * np.abs(dx).max())
    gx64, gk64, gb64 = ops.hexconv2d_backward(gy.double(), x.double(), k.double(), b.double(), cfg)
    assert gk64.dtype == torch.float64
    np.testing.assert_allclose(gx64.cpu().numpy(), dx, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(gk64.cpu().numpy().reshape(dk.shape), dk, rtol=1e-10)
    np.testing.assert_allclose(gb64.cpu().numpy(), db, rtol=1e-10)


def test_backward_only_requested_gradients_and_4k_shape():
    """Partial requests (input only / weights only) and the bench layer at 4K size:
    d bias = sum of gy exactly-ish; d input by linearity (2 gy -> 2 dx)."""
    torch.manual_seed(5)
    m = HexConv2d(3, 3, 0, 2, padding=1).to(DEV)
    x = torch.rand((1, 3, 2160, 3840), device=DEV)
    gy = torch.randn((1, 3, 2160, 3840), device=DEV)
    cfg = m._cfg()
    dx, dk, db = ops.hexconv2d_backward(gy, x, m.kernel, m.bias, cfg, True, False, False)
    assert dk is None and db is None
    dx2, _, _ = ops.hexconv2d_backward(2 * gy, x, m.kernel, m.bias, cfg, True, False, False)
    torch.testing.assert_close(dx2, 2 * dx, rtol=1e-6, atol=1e-6)
    _, dk, db = ops.hexconv2d_backward(gy, x, m.kernel, m.bias, cfg, False, True, True)
    ref_db = gy.double().sum(dim=(0, 2, 3))
    np.testing.assert_allclose(db.double().cpu().numpy(), ref_db.cpu().numpy(), rtol=1e-4,
                               atol=1e-2)
    assert dk.shape == m.kernel.shape
