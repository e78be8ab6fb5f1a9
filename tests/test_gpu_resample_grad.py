"""GPU: autograd of the resamplers (hg_resample_backward).

The forward resamplers are linear in the image with lattice-only weights and are pinned
bit-exact to the reference (test_gpu_parity.py), so the backward is checked by the exact
adjoint identity <R x, g> = <x, R^T g> in fp64 (size-independent), plus the nearest modes'
gradient = the chosen neighbour's count, and dtype / batch handling.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a HIP device", allow_module_level=True)

from HyGrid import ops  # noqa: E402

DEV = torch.device("cuda:0")
FNS = {"r2h": ops.rect_to_hex, "h2r": ops.hex_to_rect, "hexresize": ops.hexresize}
SHAPES = [(16, 20, 8, 10), (15, 17, 15, 17), (9, 12, 20, 25), (64, 96, 64, 96),
          (270, 480, 135, 240)]


def adjoint_gap(fn, x, size, interp):
    x = x.clone().requires_grad_(True)
    y = fn(x, size, interp=interp)
    g = torch.randn_like(y)
    (y * g).sum().backward()
    lhs = float((y.detach() * g).sum())
    rhs = float((x.detach() * x.grad).sum())
    return abs(lhs - rhs) / max(abs(lhs), 1e-30)


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("op", ["r2h", "h2r", "hexresize"])
@pytest.mark.parametrize("interp", [0, 1])
def test_adjoint_identity_fp64(shape, op, interp):
    h, w, h1, w1 = shape
    torch.manual_seed(1)
    x = torch.rand((2, 3, h, w), device=DEV, dtype=torch.float64)
    assert adjoint_gap(FNS[op], x, (h1, w1), interp) < 1e-12


def test_nearest_gradient_counts_selected_neighbours():
    """d/dx of sum(nearest resample) = how often each source sample is chosen: integers."""
    x = torch.rand((1, 1, 40, 60), device=DEV, dtype=torch.float64, requires_grad=True)
    y = ops.rect_to_hex(x, (40, 60), interp=0)
    y.sum().backward()
    gcount = x.grad.cpu().numpy()
    assert np.all(gcount == np.round(gcount)) and gcount.sum() <= 40 * 60


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_grad_dtype_and_batch(dtype):
    torch.manual_seed(2)
    x = torch.rand((2, 3, 48, 80), device=DEV, dtype=dtype, requires_grad=True)
    y = ops.hex_to_rect(ops.rect_to_hex(x, (48, 80)), (48, 80))
    y.float().sum().backward()
    assert x.grad.dtype == dtype and x.grad.shape == x.shape
    # per-image independence: the gradient of image 0 does not depend on image 1
    x2 = x.detach()[:1].clone().requires_grad_(True)
    ops.hex_to_rect(ops.rect_to_hex(x2, (48, 80)), (48, 80)).float().sum().backward()
    torch.testing.assert_close(x.grad[:1].float(), x2.grad.float(), rtol=1e-5, atol=1e-5)


ORACLE_BWD = {"r2h": "rect_to_hex_backward", "h2r": "hex_to_rect_backward",
              "hexresize": "hexresize_backward"}


def _grad_vs_oracle(op, shape, interp, dtype, planes=2, seed=3):
    from oracle import oracle as O
    h, w, h1, w1 = shape
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = torch.rand((planes, h, w), generator=g, device=DEV, dtype=dtype, requires_grad=True)
    y = FNS[op](x, (h1, w1), interp=interp)
    gy = torch.randn(y.shape, generator=g, device=DEV, dtype=y.dtype)
    y.backward(gy)
    ref = getattr(O, ORACLE_BWD[op])(gy.double().cpu().numpy(), (h, w), interp)
    return x.grad.double().cpu().numpy(), ref


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("op", ["r2h", "h2r", "hexresize"])
@pytest.mark.parametrize("interp", [0, 1])
def test_backward_elementwise_vs_oracle_adjoint(shape, op, interp):
    """hg_resample_backward against the fp64 oracle transpose (oracle/hg_oracle.c
    or_*_backward), element by element.  fp64 accumulation: the atomic scatter sums the
    same <= 4 products in another order (rtol 1e-12); fp32: rtol 1e-5 of max|ref|."""
    got, ref = _grad_vs_oracle(op, shape, interp, torch.float64)
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-12 * np.abs(ref).max())
    got, ref = _grad_vs_oracle(op, shape, interp, torch.float32)
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5 * np.abs(ref).max())


@pytest.mark.parametrize("op,shape", [("r2h", (2160, 3840, 2160, 3840)),
                                      ("h2r", (2160, 3840, 2160, 3840)),
                                      ("hexresize", (4320, 7680, 2160, 3840))])
def test_backward_4k_plane_vs_oracle_adjoint(op, shape):
    got, ref = _grad_vs_oracle(op, shape, 1, torch.float32, planes=1)
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5 * np.abs(ref).max())
