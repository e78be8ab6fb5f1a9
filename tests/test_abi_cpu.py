"""The C-ABI library loads and exports every symbol include/hygrid.h declares.

No GPU work is issued here: only host-side entry points (version, strerror,
the conv output-shape rule) and argument validation that returns before any
HIP call.
"""
import ctypes
import os
import re

import pytest

from conftest import ROOT
from HyGrid import _abi
from oracle import oracle as O

HEADER = os.path.join(ROOT, "include", "hygrid.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hg_\w+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    names = declared_functions()
    assert len(names) >= 8
    L = _abi.lib()
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(_abi.SIGNATURES), "ctypes signatures out of sync with header"


def test_version_and_strerror():
    L = _abi.lib()
    assert L.hg_abi_version() == 1
    assert _abi.strerror(0) == "success"
    assert _abi.strerror(-1) == "invalid argument"
    assert _abi.strerror(-2) == "unsupported dtype"
    assert "unknown" in _abi.strerror(-99)


@pytest.mark.parametrize("r", [1, 2, 3, 4])
@pytest.mark.parametrize("s", [1, 2, 3])
@pytest.mark.parametrize("p", [0, 1, 2])
@pytest.mark.parametrize("d", [1, 2])
def test_conv_out_shape_matches_oracle(r, s, p, d):
    L = _abi.lib()
    for (h, w) in [(8, 10), (7, 9), (1, 1), (2160, 3840), (3, 40)]:
        ho, wo = ctypes.c_int64(), ctypes.c_int64()
        st = L.hg_hexconv2d_out_shape(h, w, r, s, p, d, ctypes.byref(ho), ctypes.byref(wo))
        try:
            ref = O.hexconv2d_out_shape(h, w, r, s, p, d)
        except ValueError:
            assert st == -3
            continue
        assert st == 0 and (ho.value, wo.value) == ref


def test_validation_before_launch():
    L = _abi.lib()
    fake = ctypes.c_void_p(16)
    # negative sizes
    assert L.hg_rect_to_hex(fake, fake, 8, 8, -1, 4, 4, 4, 4, 1, None) == -1
    # bad interpolation code
    assert L.hg_hex_to_rect(fake, fake, 8, 8, 1, 4, 4, 4, 4, 7, None) == -1
    # interpolating into an integer dtype
    assert L.hg_hexresize(fake, fake, 8, 0, 1, 4, 4, 4, 4, 1, None) == -2
    # nearest must keep the dtype
    assert L.hg_rect_to_hex(fake, fake, 8, 9, 1, 4, 4, 4, 4, 0, None) == -2
    # null output with work to do
    assert L.hg_rect_to_hex(fake, None, 8, 8, 1, 4, 4, 4, 4, 1, None) == -1
    # nothing to do: success without touching the device
    assert L.hg_rect_to_hex(None, None, 8, 8, 0, 4, 4, 4, 4, 1, None) == 0
    # conv: groups must divide channels; input too small; bad pad mode
    args = [fake, fake, None, fake, 8, 8, 8, 1, 3, 4, 8, 8, 2, 1, 1, 1]
    assert L.hg_hexconv2d(*args, 3, 0, 0, 0.0, None) == -1
    args = [fake, fake, None, fake, 8, 8, 8, 1, 3, 3, 1, 1, 2, 1, 0, 1]
    assert L.hg_hexconv2d(*args, 1, 0, 0, 0.0, None) == -3
    args = [fake, fake, None, fake, 8, 8, 8, 1, 3, 3, 8, 8, 2, 1, 1, 1]
    assert L.hg_hexconv2d(*args, 1, 0, 9, 0.0, None) == -1
    # reflect padding needs pad < size (torch.nn.functional.pad's rule)
    args = [fake, fake, None, fake, 8, 8, 8, 1, 3, 3, 2, 2, 2, 1, 2, 1]
    assert L.hg_hexconv2d(*args, 1, 0, 1, 0.0, None) == -3
