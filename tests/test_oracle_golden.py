"""Pin the CPU oracle (oracle/hg_oracle.c) to the reference's own golden vectors.

The fixtures were captured from /root/reference by tests/golden/make_golden.py:
outputs AND the reference's own local index maps.  Integer maps must match
bit-exactly; fp64 outputs of the resamplers are expected bit-exact too (same
evaluation order, no FMA) and are asserted to 0 ulp where the reference blends
in fp64, and within 1e-5 relative for HexConv2d (the reference runs F.conv2d in
fp32, the oracle in fp64).
"""
import numpy as np
import pytest

from oracle import oracle as O


def _cases(index, name):
    return [c for c in index[name]]


def test_linspace_matches_numpy():
    for (a, b, n) in [(-8.0, 8.0, 16), (-10.5, 10.5, 17), (-0.0, 0.0, 1), (-3.25, 3.25, 7),
                      (-1080 / 2, 1080 / 2, 1080), (0.0, 0.0, 5)]:
        np.testing.assert_array_equal(O.linspace(a, b, n), np.linspace(a, b, n))


@pytest.mark.parametrize("ci", range(11))
def test_r2h_maps_and_values(golden, golden_index, ci):
    g = golden("r2h")
    for meta in [m for m in golden_index["r2h"] if m["case"] == ci]:
        mode = meta["mode"]
        tag = f"c{ci}_{mode}"
        m = O.r2h_maps(meta["h"], meta["w"], meta["h1"], meta["w1"])
        np.testing.assert_array_equal(m["i_n"], g[tag + "_i_n"])
        np.testing.assert_array_equal(m["j_n"], g[tag + "_j_n"])
        np.testing.assert_array_equal(m["valid"], g[tag + "_valid"])
        np.testing.assert_array_equal(m["i_f"], g[tag + "_i_f"])
        np.testing.assert_array_equal(m["j_f"], g[tag + "_j_f"])
        if mode == "nearest":
            np.testing.assert_array_equal(m["argmin"], g[tag + "_argmin"])
        x = g[f"c{ci}_x"]
        y = O.rect_to_hex(x, (meta["h1"], meta["w1"]), 0 if mode == "nearest" else 1)
        ref = g[tag + "_y"].astype(np.float64)
        np.testing.assert_array_equal(y, ref)


@pytest.mark.parametrize("ci", range(10))
def test_h2r_maps_and_values(golden, golden_index, ci):
    g = golden("h2r")
    for meta in [m for m in golden_index["h2r"] if m["case"] == ci]:
        mode = meta["mode"]
        tag = f"c{ci}_{mode}"
        m = O.h2r_maps(meta["h"], meta["w"], meta["h1"], meta["w1"])
        for k in ("i_n", "j_n", "flag", "valid"):
            np.testing.assert_array_equal(m[k], g[tag + "_" + k], err_msg=k)
        if mode == "nearest":
            np.testing.assert_array_equal(m["argmin"], g[tag + "_argmin"])
        else:
            for k in ("i_f", "j_f", "alpha", "beta", "gamma"):
                np.testing.assert_array_equal(m[k], g[tag + "_" + k], err_msg=k)
        x = g[f"c{ci}_x"]
        y = O.hex_to_rect(x, (meta["h1"], meta["w1"]), 0 if mode == "nearest" else 1)
        np.testing.assert_array_equal(y, g[tag + "_y"].astype(np.float64))


@pytest.mark.parametrize("ci", range(6))
def test_hexresize_maps_and_values(golden, golden_index, ci):
    g = golden("hexresize")
    meta = golden_index["hexresize"][ci]
    tag = f"c{ci}_linear"
    m = O.hexresize_maps(meta["h"], meta["w"], meta["h1"], meta["w1"])
    for k in ("i_n", "j_n", "flag", "valid"):
        np.testing.assert_array_equal(m[k], g[tag + "_" + k], err_msg=k)
    for k in ("i_f", "j_f", "alpha", "beta", "gamma"):
        np.testing.assert_array_equal(m[k], g[tag + "_" + k], err_msg=k)
    y = O.hexresize(g[f"c{ci}_x"], (meta["h1"], meta["w1"]), 1)
    np.testing.assert_array_equal(y, g[tag + "_y"])


def test_hexconv_all_cases(golden, golden_index):
    g = golden("hexconv")
    n = 0
    for meta in golden_index["hexconv"]:
        ci = meta["case"]
        if "error" in meta:
            with pytest.raises(ValueError):
                O.hexconv2d_out_shape(meta["h"], meta["w"], meta["r"], meta["stride"],
                                      meta["pad"], meta["dilation"])
            continue
        y = O.hexconv2d(g[f"c{ci}_x"], g[f"c{ci}_kernel"], g.get(f"c{ci}_bias"), meta["off"],
                        meta["r"], meta["stride"], meta["pad"], meta["dilation"],
                        meta["groups"], meta["padding_mode"], meta["padding_value"])
        ref = g[f"c{ci}_y"]
        assert y.shape == ref.shape, (ci, y.shape, ref.shape)
        np.testing.assert_allclose(y, ref, rtol=1e-5, atol=1e-5 * np.abs(ref).max(),
                                   err_msg=str(meta))
        n += 1
    assert n >= 50


def test_hexconv_backward_all_cases(golden, golden_index):
    """Oracle adjoint vs the reference's own autograd gradients (d input, d kernel,
    d bias) for every forward case; the reference computes them in fp32."""
    g = golden("hexconv_bwd")
    n = 0
    for meta in golden_index["hexconv_bwd"]:
        if "error" in meta:
            continue
        ci = meta["case"]
        dx, dk, db = O.hexconv2d_backward(
            g[f"c{ci}_x"], g[f"c{ci}_kernel"], g[f"c{ci}_gy"], meta["off"], meta["r"],
            meta["stride"], meta["pad"], meta["dilation"], meta["groups"],
            meta["padding_mode"], meta["padding_value"])
        for got, key in ((dx, "dx"), (dk, "dkernel")):
            ref = g[f"c{ci}_{key}"]
            assert got.shape == ref.shape, (ci, key, got.shape, ref.shape)
            np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5 * max(np.abs(ref).max(), 1),
                                       err_msg=f"{key} {meta}")
        if f"c{ci}_dbias" in g:
            np.testing.assert_allclose(db, g[f"c{ci}_dbias"], rtol=1e-4, atol=1e-4)
        n += 1
    assert n >= 50


def test_conv_impulse_tap_tables(golden, golden_index):
    g = golden("taps")
    for meta in golden_index["taps"]:
        h, w = meta["h"], meta["w"]
        x = (np.arange(h * w, dtype=np.float64) + 1).reshape(1, 1, h, w)
        for t in range(7):
            k = np.zeros((1, 1, 1, 7))
            k[0, 0, 0, t] = 1.0
            y = O.hexconv2d(x, k, None, meta["off"], 2, padding=meta["pad"])[0, 0]
            np.testing.assert_array_equal(np.rint(y).astype(np.int32) - 1,
                                          g[f"t{meta['case']}_table"][t])


def test_type1_layout(golden_index):
    kat = golden_index["kat"]
    x = np.arange(2 * 5 * 4, dtype=np.float64).reshape(2, 5, 4)
    for off in (0, 1):
        np.testing.assert_array_equal(O.heximage_to_type1(x, off)[None],
                                      np.array(kat[f"type1_off{off}"]))


def test_kat_ones(golden_index):
    kat = golden_index["kat"]
    y = O.rect_to_hex(np.ones((1, 12, 16)), None, 1)[0]
    assert np.abs(y[:, 0]).max() == kat["r2h_ones"]["col0_max"] == 0.0
    assert np.abs(y[:, -1]).max() == kat["r2h_ones"]["colN_max"] == 0.0
    assert y[1:-1, 1:-1].min() == y[1:-1, 1:-1].max() == 1.0
    y = O.hex_to_rect(np.ones((1, 12, 16)), None, 1)
    assert y.min() == kat["h2r_ones"]["min"] and y.max() == kat["h2r_ones"]["max"]
    m = O.h2r_maps(33, 41, 29, 57)
    # S1+S2+S3 == 0.5 exactly inside the lattice => alpha+beta+gamma == 1
    s = m["alpha"] + m["beta"] + m["gamma"]
    np.testing.assert_allclose(s, 1.0, rtol=0, atol=4e-16)


@pytest.mark.parametrize("ci", range(7))
def test_igt_maps_and_values(golden, golden_index, ci):
    """image_geometric_transformation (geometry_np.py:6-189): the NumPy restatement's
    lattice (i_n, j_n, flag, validity), mapped points, weights and 'linear' output equal
    the reference's locals bit for bit."""
    g = golden("igt")
    meta = golden_index["igt"][ci]
    t = f"c{ci}"
    y, maps = O.image_geometric_transformation(g[t + "_x"], g[t + "_H"], 1)
    assert y.shape == (meta["c"], meta["h1"], meta["w1"])
    for k in ("i_n", "j_n", "flag", "valid", "x_", "y_", "alpha", "beta", "gamma"):
        np.testing.assert_array_equal(maps[k], g[t + "_" + k], err_msg=k)
    np.testing.assert_array_equal(y, g[t + "_y"])
    # the reference's 'nearest' raises (tuple-unpacking of np.min, :172)
    assert meta["nearest"] == "ValueError"


def test_pool_oracle_vs_reference(golden, golden_index):
    """Hex pooling (HexFrames.py:255-410, :461-479): the NumPy restatement's outputs and
    input gradients against the reference's forward and autograd.  max / min exact;
    average within 4 ulp (torch's vectorised window sum order differs from NumPy's)."""
    from pool_cases import pool_args
    g = golden("pool")
    n_ok = 0
    for m in golden_index["pool"]:
        if "error" in m:
            continue
        t = f"p{m['case']}"
        args = pool_args(m)
        y = O.hex_pool2d(g[t + "_x"], *args)
        yr = g[t + "_y"].reshape(y.shape)
        if m["method"] == "average":
            np.testing.assert_allclose(y, yr, rtol=1e-15, atol=5e-16)
        else:
            np.testing.assert_array_equal(y, yr)
        dx = O.hex_pool2d_backward(g[t + "_x"], g[t + "_gy"], *args)
        np.testing.assert_allclose(dx, g[t + "_dx"], rtol=1e-15, atol=1e-16)
        n_ok += 1
    assert n_ok >= 30
