"""fp64 adjoints of the three resamplers in the oracle (or_*_backward, hg_oracle.c)
against the golden-pinned forwards: <R x, g> = <x, R^T g>, and R^T e_k = the k-th row of
R read off the forward's response to unit images (small shapes: the full matrix)."""
import numpy as np
import pytest

from oracle import oracle as O

FWD = {"r2h": O.rect_to_hex, "h2r": O.hex_to_rect, "hexresize": O.hexresize}
BWD = {"r2h": O.rect_to_hex_backward, "h2r": O.hex_to_rect_backward,
       "hexresize": O.hexresize_backward}
SHAPES = [(16, 20, 8, 10), (15, 17, 15, 17), (9, 12, 20, 25), (1, 7, 3, 5), (33, 64, 5, 3)]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("op", ["r2h", "h2r", "hexresize"])
@pytest.mark.parametrize("interp", [0, 1])
def test_adjoint_identity(shape, op, interp):
    h, w, h1, w1 = shape
    rng = np.random.default_rng(h * 100 + w)
    x = rng.standard_normal((3, h, w))
    g = rng.standard_normal((3, h1, w1))
    lhs = float((FWD[op](x, (h1, w1), interp) * g).sum())
    rhs = float((x * BWD[op](g, (h, w), interp)).sum())
    assert abs(lhs - rhs) <= 1e-12 * max(abs(lhs), 1.0)


@pytest.mark.parametrize("op", ["r2h", "h2r", "hexresize"])
@pytest.mark.parametrize("interp", [0, 1])
def test_adjoint_is_transpose(op, interp):
    h, w, h1, w1 = 6, 7, 5, 9
    eye = np.eye(h * w).reshape(h * w, h, w)
    R = FWD[op](eye, (h1, w1), interp).reshape(h * w, h1 * w1).T      # (h1*w1, h*w)
    geye = np.eye(h1 * w1).reshape(h1 * w1, h1, w1)
    RT = BWD[op](geye, (h, w), interp).reshape(h1 * w1, h * w)         # row k = R^T e_k
    np.testing.assert_array_equal(RT, R)
