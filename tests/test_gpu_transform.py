"""GPU: image_geometric_transformation on hg_hex_homography.

Pinned to the reference's own outputs and lattice locals (tests/golden/igt.npz, captured
from geometry_np.image_geometric_transformation by tests/golden/make_golden.py) and, at
larger sizes, to the NumPy restatement in oracle/oracle.py (itself pinned to the same
goldens by test_oracle_golden.py).  Integer maps bit-exact; fp64 'linear' output
bit-exact (the kernel evaluates the reference's expression order with no FMA
contraction); 'nearest' (the torch twin's rule, the NumPy reference raises) against the
oracle's first-minimum choice."""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a HIP device", allow_module_level=True)

from HyGrid import geometry_np as G  # noqa: E402
from HyGrid import geometry_torch as GT  # noqa: E402
from HyGrid import ops  # noqa: E402

DEV = torch.device("cuda:0")


@pytest.mark.parametrize("ci", range(7))
def test_igt_maps_vs_reference(golden, golden_index, ci):
    g = golden("igt")
    meta = golden_index["igt"][ci]
    t = f"c{ci}"
    m = ops.homography_maps(meta["h"], meta["w"], g[t + "_H"], DEV)
    for k in ("i_n", "j_n", "flag", "valid"):
        np.testing.assert_array_equal(m[k].cpu().numpy(), g[t + "_" + k], err_msg=k)
    for k in ("x_", "y_", "alpha", "beta", "gamma"):
        np.testing.assert_array_equal(m[k].cpu().numpy(), g[t + "_" + k], err_msg=k)


@pytest.mark.parametrize("ci", range(7))
def test_igt_linear_vs_reference(golden, golden_index, ci):
    g = golden("igt")
    meta = golden_index["igt"][ci]
    t = f"c{ci}"
    x = g[t + "_x"]
    y = G.image_geometric_transformation(x, g[t + "_H"], "linear")
    assert y.dtype == np.float64 and list(y.shape) == meta["out_shape"]
    np.testing.assert_array_equal(y.reshape(g[t + "_y"].shape), g[t + "_y"])
    y2 = GT.image_geometric_transformation(x, g[t + "_H"], "linear")
    np.testing.assert_array_equal(y2, y)


def _rand_affine(rng):
    th = rng.uniform(-np.pi, np.pi)
    s = rng.uniform(0.4, 2.2, size=2)
    sh = rng.uniform(-0.4, 0.4)
    A = np.array([[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]]) @ \
        np.array([[s[0], sh], [0.0, s[1]]])
    H = np.eye(3)
    H[:2, :2] = A
    H[:2, 2] = rng.uniform(-5, 5, size=2)
    return H


@pytest.mark.parametrize("seed", range(6))
def test_igt_random_affine_vs_oracle(seed):
    rng = np.random.default_rng(100 + seed)
    c, h, w = int(rng.integers(1, 4)), int(rng.integers(5, 90)), int(rng.integers(5, 90))
    x = rng.standard_normal((c, h, w))
    H = _rand_affine(rng)
    ref, maps = O.image_geometric_transformation(x, H, 1)
    got = ops.hex_homography(torch.from_numpy(x).to(DEV), H, 1, torch.float64).cpu().numpy()
    np.testing.assert_array_equal(got, ref)
    m = ops.homography_maps(h, w, H, DEV)
    for k in ("i_n", "j_n", "flag", "valid", "argmin"):
        np.testing.assert_array_equal(m[k].cpu().numpy(), maps[k], err_msg=k)
    nref, _ = O.image_geometric_transformation(x, H, 0)
    near = ops.hex_homography(torch.from_numpy(x).to(DEV), H, 0).cpu().numpy()
    np.testing.assert_array_equal(near, nref)


@pytest.mark.parametrize("dtype", [torch.uint8, torch.bfloat16, torch.float16, torch.float32])
def test_igt_dtypes_and_batch(dtype):
    """Leading batch dims walk planes with one lattice; low-precision inputs blend in fp64
    and round once into the requested output dtype."""
    rng = np.random.default_rng(7)
    H = _rand_affine(rng)
    x = (torch.rand((2, 3, 40, 52), device=DEV) * 200).to(dtype)
    xo = x.double().cpu().numpy()
    ref, _ = O.image_geometric_transformation(xo, H, 1)
    got = ops.hex_homography(x, H, 1, torch.float64)
    np.testing.assert_array_equal(got.cpu().numpy(), ref)
    got32 = ops.hex_homography(x, H, 1, torch.float32)
    np.testing.assert_array_equal(got32.cpu().numpy(), ref.astype(np.float32))
    near = ops.hex_homography(x, H, 0)
    assert near.dtype == dtype
    nref, _ = O.image_geometric_transformation(xo, H, 0)
    np.testing.assert_array_equal(near.double().cpu().numpy(), nref)


def test_igt_nearest_numpy_and_edges():
    rng = np.random.default_rng(3)
    x = rng.integers(0, 256, (3, 17, 21)).astype(np.uint8)
    H = _rand_affine(rng)
    y = G.image_geometric_transformation(x, H, "nearest")
    assert y.dtype == np.uint8
    nref, _ = O.image_geometric_transformation(x, H, 0)
    np.testing.assert_array_equal(y, nref.astype(np.uint8).squeeze())
    # identity: the output lattice is the input lattice (offset 0)
    xi = rng.standard_normal((2, 9, 12))
    np.testing.assert_array_equal(G.image_geometric_transformation(xi, np.eye(3), "linear"),
                                  O.image_geometric_transformation(xi, np.eye(3), 1)[0])
    # one-row / one-column rasters and a 2-D input (squeezed like the reference)
    for shp in [(1, 9), (9, 1), (1, 1)]:
        xe = rng.standard_normal(shp)
        ref = O.image_geometric_transformation(xe, np.diag([1.5, 0.7, 1.0]), 1)[0]
        np.testing.assert_array_equal(
            G.image_geometric_transformation(xe, np.diag([1.5, 0.7, 1.0]), "linear"),
            ref.squeeze())


def test_igt_large_properties():
    """4K-class raster: finite output, identity reproduces the input exactly (every sample
    lands on a lattice site), and the planes are independent (batch == per-plane calls)."""
    x = torch.rand((4, 2160, 3840), device=DEV, dtype=torch.float32)
    y = ops.hex_homography(x, np.eye(3), 1, torch.float32)
    torch.testing.assert_close(y, x, rtol=0, atol=0)
    H = np.array([[0.8, 0.2, 3.0], [-0.1, 1.1, -7.0], [0, 0, 1.0]])
    yb = ops.hex_homography(x, H, 1, torch.float32)
    assert torch.isfinite(yb).all()
    y1 = ops.hex_homography(x[2:3].contiguous(), H, 1, torch.float32)
    torch.testing.assert_close(yb[2:3], y1, rtol=0, atol=0)
