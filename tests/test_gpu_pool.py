"""GPU: hex pooling on hg_hex_pool2d / hg_hex_pool2d_backward.

Pinned to the reference's own HexPool2d / HexAdaptivePool2d / HexGlobalPool2d forward
outputs and autograd input gradients (tests/golden/pool.npz, captured by
tests/golden/make_golden.py, NaN-laden inputs) and, on larger seeded inputs and other
dtypes, to the NumPy restatement oracle/oracle.py:hex_pool2d (pinned to the same
goldens).  max / min: exact.  average: fp64 within 4 ulp (window sum order); fp32 1e-6,
bf16 / f16 one rounding of the output.  Gradients: atomics, fp64 within 1e-15."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from pool_cases import module_for, pool_args

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a HIP device", allow_module_level=True)

from HyGrid import HexFrames as HF  # noqa: E402
from HyGrid import ops  # noqa: E402

DEV = torch.device("cuda:0")


def _cases(index):
    return [m for m in index["pool"] if "error" not in m]


def test_pool_modules_vs_reference(golden, golden_index):
    g = golden("pool")
    for m in _cases(golden_index):
        t = f"p{m['case']}"
        x = torch.from_numpy(g[t + "_x"]).to(DEV).requires_grad_(True)
        mod = module_for(m)
        y = mod(x)
        yr = g[t + "_y"]
        assert list(y.shape) == list(yr.shape), m
        if m["method"] == "average":
            np.testing.assert_allclose(y.detach().cpu().numpy(), yr, rtol=1e-15, atol=5e-16,
                                       err_msg=str(m))
        else:
            np.testing.assert_array_equal(y.detach().cpu().numpy(), yr, err_msg=str(m))
        y.backward(torch.from_numpy(g[t + "_gy"]).to(DEV))
        np.testing.assert_allclose(x.grad.cpu().numpy(), g[t + "_dx"], rtol=1e-15, atol=1e-16,
                                   err_msg=str(m))


def test_pool_reference_errors(golden_index):
    x = torch.rand(2, 3, 10, 13, device=DEV, dtype=torch.float64)
    for m in golden_index["pool"]:
        if "error" not in m:
            continue
        with pytest.raises(IndexError):
            module_for(m)(x[..., : m["h"], : m["w"]])


CONFIGS = [
    dict(method="max", k=2, s=2, pad=0),
    dict(method="average", k=3, s=2, pad=1),
    dict(method="min", k=[3, 2], s=[2, 2], pad=1, mode="reflect"),
    dict(method="average", k=2, s=2, pad=0, ceil=True, cip=False),
    dict(method="max", k=3, s=3, pad=1, mode="circular", ceil=True),
    dict(method="average", k=2, s=3, pad=2, mode="replicate"),
]


@pytest.mark.parametrize("ci", range(len(CONFIGS)))
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32, torch.bfloat16, torch.float16])
def test_pool_random_vs_oracle(ci, dtype):
    c = CONFIGS[ci]
    torch.manual_seed(ci)
    h, w = 67, 96
    x = torch.randn(2, 5, h, w, device=DEV, dtype=torch.float64)
    x[torch.rand_like(x) < 0.05] = float("nan")
    x = x.to(dtype)
    m = dict(kind="pool", h=h, w=w, **c)
    args = pool_args(m)
    xr = x.clone().requires_grad_(True)
    y = module_for(m)(xr)
    xo = x.double().cpu().numpy()
    ref = O.hex_pool2d(xo, *args)
    got = y.detach().double().cpu().numpy()
    if c["method"] == "average":
        tol = {torch.float64: 1e-14, torch.float32: 2e-6, torch.bfloat16: 1.6e-2,
               torch.float16: 2e-3}[dtype]
        np.testing.assert_allclose(got, ref, rtol=tol, atol=tol)
    else:
        np.testing.assert_array_equal(got, ref)
    gy = torch.randn(y.shape, device=DEV, dtype=torch.float64)
    y.backward(gy.to(dtype))
    dref = O.hex_pool2d_backward(xo, gy.to(dtype).double().cpu().numpy(), *args)
    tol = {torch.float64: 1e-13, torch.float32: 1e-5, torch.bfloat16: 3e-2,
           torch.float16: 4e-3}[dtype]
    np.testing.assert_allclose(xr.grad.double().cpu().numpy(), dref, rtol=tol, atol=tol)


@pytest.mark.parametrize("method", ["max", "min", "average"])
def test_global_and_adaptive_large(method):
    """Large windows take the workgroup-per-output kernel (fp64 partials, LDS tree)."""
    torch.manual_seed(5)
    x = torch.randn(2, 3, 540, 960, device=DEV, dtype=torch.float32)
    x[0, 0, :7, :9] = float("nan")
    x[1, 2] = float("nan")                        # an all-NaN plane
    y = HF.HexGlobalPool2d(method)(x)
    ref = O.hex_pool2d(x.double().cpu().numpy(), method, 540, 960, 540, 960, 1, 1)[..., 0, 0]
    if method == "average":
        np.testing.assert_allclose(y.double().cpu().numpy(), ref, rtol=1e-6, atol=1e-7)
        assert torch.isnan(y[1, 2])
    else:
        np.testing.assert_array_equal(y.double().cpu().numpy(), ref.astype(np.float32))
    a = HF.HexAdaptivePool2d(7, method)(x)
    args = pool_args(dict(kind="adaptive", h=540, w=960, outsize=7, method=method))
    aref = O.hex_pool2d(x.double().cpu().numpy(), *args)
    np.testing.assert_allclose(a.double().cpu().numpy(), aref, rtol=1e-6, atol=1e-7)
    xr = x.double().requires_grad_(True)
    HF.HexGlobalPool2d(method)(xr).sum().backward()
    dref = O.hex_pool2d_backward(x.double().cpu().numpy(), np.ones((2, 3)), method,
                                 540, 960, 540, 960, 1, 1)
    np.testing.assert_allclose(xr.grad.cpu().numpy(), dref, rtol=1e-14, atol=1e-15)


def test_reduce_functions():
    """max_pooling / min_pooling / average_pooling (HexFrames.py:461-479) over the last dim."""
    x = torch.tensor([[1.0, float("nan"), 3.0], [float("nan")] * 3, [-2.0, 5.0, 5.0]],
                     device=DEV, dtype=torch.float64)
    torch.testing.assert_close(HF.max_pooling(x).cpu(),
                               torch.tensor([3.0, -float("inf"), 5.0], dtype=torch.float64))
    torch.testing.assert_close(HF.min_pooling(x).cpu(),
                               torch.tensor([1.0, float("inf"), -2.0], dtype=torch.float64))
    avg = HF.average_pooling(x).cpu()
    assert avg[0] == 2.0 and torch.isnan(avg[1]) and avg[2] == 8.0 / 3.0
    xr = x.clone().requires_grad_(True)
    HF.max_pooling(xr).sum().backward()
    # first maximum of [-2, 5, 5] gets the gradient; the all-NaN row gets none
    torch.testing.assert_close(xr.grad.cpu(), torch.tensor(
        [[0.0, 0.0, 1.0], [0.0, 0.0, 0.0], [0.0, 1.0, 0.0]], dtype=torch.float64))


def test_pool_4k_batch_properties():
    """4K bf16 batch: a 2x2 / stride 2 max pool equals the max of its four shifted views
    (a size-independent property), and batch == per-image."""
    torch.manual_seed(9)
    x = torch.rand(4, 3, 2160, 3840, device=DEV).to(torch.bfloat16)
    y = HF.HexPool2d("max", 2, 2)(x)
    hn, wn = y.shape[-2:]
    assert (hn, wn) == (1080, 1919)
    # even output rows: cols 2j, 2j+1; odd output rows: cols 2j+1, 2j+2
    xe = x[..., 0::4, :], x[..., 1::4, :]
    ev = torch.maximum(torch.maximum(xe[0][..., 0:2 * wn:2], xe[0][..., 1:2 * wn:2]),
                       torch.maximum(xe[1][..., 0:2 * wn:2], xe[1][..., 1:2 * wn:2]))
    torch.testing.assert_close(y[..., 0::2, :], ev, rtol=0, atol=0)
    xo = x[..., 2::4, :], x[..., 3::4, :]
    od = torch.maximum(torch.maximum(xo[0][..., 1:2 * wn + 1:2], xo[0][..., 2:2 * wn + 2:2]),
                       torch.maximum(xo[1][..., 1:2 * wn + 1:2], xo[1][..., 2:2 * wn + 2:2]))
    torch.testing.assert_close(y[..., 1::2, :], od, rtol=0, atol=0)
    torch.testing.assert_close(HF.HexPool2d("max", 2, 2)(x[1:2]), y[1:2], rtol=0, atol=0)
