"""The pyramid chain (hg_hex_pyramid_chain, round 6): 2-3 levels of config 5 in ONE launch, a
level's bands waiting on per-band counters of the level before.  It runs the same band code
as the one-level launches (k_fused MD 3 for level 0 from the rect image, MD 5 after), so the
outputs must equal hex_pyramid_level's bit for bit (those are pinned to the oracle in
tests/test_gpu_pyramid.py); after every call the workspace's fault word (a wait past ~1 s,
never expected) is 0 and the ticket count equals the launch's workgroups."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a HIP device", allow_module_level=True)

from HyGrid import _abi, ops  # noqa: E402
from HyGrid.HexFrames import HexConv2d  # noqa: E402
from HyGrid.pipeline import hex_pyramid  # noqa: E402

DEV = torch.device("cuda:0")


def per_level(x, taps, bias, levels, off, monkeypatch):
    """The levels one launch each on the fused kernel (HYGRID_PYR_KERNEL=fused)."""
    monkeypatch.setenv("HYGRID_PYR_KERNEL", "fused")
    try:
        cur, outs = x, []
        h, w = x.shape[-2:]
        for lv in range(levels):
            h, w = h // 2, w // 2
            y = ops.hex_pyramid_level(cur, taps, bias, (h, w), off, from_rect=(lv == 0),
                                      out_dtype=x.dtype)
            assert y is not None, f"level {lv} not on the fused kernel"
            outs.append(y)
            cur = y
    finally:
        monkeypatch.delenv("HYGRID_PYR_KERNEL")
    return outs


def units(shape, levels):
    """Workgroups of the chain's launch: per level B x bands x groups of 4 windows of 60 output
    columns (level 0 on 60-row bands, later levels on 24-row bands)."""
    B, _, h, w = shape
    n = 0
    ceil = lambda a, b: (a + b - 1) // b  # noqa: E731
    for lv in range(levels):
        rb = 60 if lv == 0 else 24
        n += B * ceil(h, rb) * ceil(ceil(w // 2, 60), 4)
        h, w = h // 2, w // 2
    return n


def workspace_clean(x, levels):
    ws = ops.chain_workspace(x.device, _abi.stream_of(x), 0)
    torch.cuda.synchronize()
    assert int(ws[1]) == 0, "chain fault word set (a workgroup waited > ~1 s for its input)"
    assert int(ws[0]) == units(tuple(x.shape), levels), "every workgroup draws one ticket"


# (the fused level needs an even input width at every level and, for its lattice class, an
# even input height: H and W multiples of 8 for 3 levels)
@pytest.mark.parametrize("shape,levels", [((2, 3, 136, 248), 3), ((2, 3, 136, 252), 2),
                                          ((3, 3, 544, 960), 3), ((1, 3, 72, 96), 3),
                                          ((5, 3, 304, 488), 3)])
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("off", [0, 1])
def test_chain_equals_per_level(shape, levels, dt, off, monkeypatch):
    gen = torch.Generator(device=DEV).manual_seed(11)
    x = torch.rand(shape, generator=gen, device=DEV).to(dt)
    taps = torch.rand((3, 7), generator=gen, device=DEV)
    bias = torch.rand((3,), generator=gen, device=DEV) if off else None
    ref = per_level(x, taps, bias, levels, off, monkeypatch)
    with torch.no_grad():
        outs = ops.hex_pyramid_chain(x, taps, bias, levels, off)
    assert outs is not None
    workspace_clean(x, levels)
    for lv, (a, b) in enumerate(zip(outs, ref)):
        assert a.shape == b.shape and torch.equal(a, b), f"level {lv}"


def test_chain_config5_full_size(monkeypatch):
    """The bench's config-5 launch (8 x 3 x 4320 x 7680 fp16, Gaussian taps) as one chain:
    equal to the per-level launches, repeated (the workspace reused), fault word 0."""
    conv = HexConv2d(3, 3, 0, 2, padding=1, groups=3, bias=False).to(DEV)
    with torch.no_grad():
        conv.kernel.copy_(torch.tensor([1, 1, 1, 6, 1, 1, 1], dtype=torch.float32, device=DEV)
                          .div_(12).expand_as(conv.kernel))
    gen = torch.Generator(device=DEV).manual_seed(8)
    x = torch.rand((8, 3, 4320, 7680), generator=gen, device=DEV, dtype=torch.float16)
    ref = per_level(x, conv.kernel, None, 3, 0, monkeypatch)
    monkeypatch.setenv("HYGRID_PYR_CHAIN", "1")
    with torch.no_grad():
        for _ in range(3):
            outs = hex_pyramid(x, conv, levels=3, out_dtype=torch.float16)
            workspace_clean(x, 3)
            for lv, (a, b) in enumerate(zip(outs, ref)):
                assert torch.equal(a, b), f"level {lv}"
    del ref, outs
    torch.cuda.empty_cache()


def test_chain_declines_outside_its_domain(monkeypatch):
    gen = torch.Generator(device=DEV).manual_seed(3)
    x = torch.rand((2, 3, 136, 248), generator=gen, device=DEV).half()
    taps = torch.rand((3, 7), generator=gen, device=DEV)
    assert ops.hex_pyramid_chain(x[..., :244], taps, None, 3) is None   # odd level-2 input width
    assert ops.hex_pyramid_chain(x, taps, None, 1) is None        # one level: no chain
    assert ops.hex_pyramid_chain(x, taps, None, 4) is None        # > 3 levels
    assert ops.hex_pyramid_chain(x.float(), taps, None, 3) is None   # fp32
    x1 = x[:, :1].contiguous()
    assert ops.hex_pyramid_chain(x1, taps[:1], None, 3) is None   # C = 1
    # hex_pyramid with the chain (opt-in, HYGRID_PYR_CHAIN=1) and without: same values
    conv = HexConv2d(3, 3, 0, 2, padding=1, groups=3, bias=False).to(DEV)
    with torch.no_grad():
        a = hex_pyramid(x, conv, levels=3)
        monkeypatch.setenv("HYGRID_PYR_CHAIN", "1")
        b = hex_pyramid(x, conv, levels=3)
        workspace_clean(x, 3)
    for u, v in zip(a, b):
        assert torch.equal(u, v)


def test_chain_workspace_too_small_is_an_error():
    gen = torch.Generator(device=DEV).manual_seed(4)
    x = torch.rand((2, 3, 136, 248), generator=gen, device=DEV).half()
    taps = torch.rand((3, 7), generator=gen, device=DEV)
    outs = [torch.empty((2, 3, 68, 124), device=DEV, dtype=torch.float16),
            torch.empty((2, 3, 34, 62), device=DEV, dtype=torch.float16)]
    L = _abi.lib()
    need = L.hg_hex_pyramid_chain_workspace(2, 2, 136)
    ws = torch.zeros(need // 4, dtype=torch.int32, device=DEV)
    ys = (ctypes.c_void_p * 2)(*[o.data_ptr() for o in outs])
    args = [_abi.ptr(x), ys, 2, _abi.HG_F16, 2, 3, 136, 248, _abi.ptr(taps), None, 0, _abi.ptr(ws)]
    assert L.hg_hex_pyramid_chain(*args, need - 4, _abi.stream_of(x)) == _abi.HG_EINVAL
    ws.fill_(-7)                                  # the call zeroes its words first
    assert L.hg_hex_pyramid_chain(*args, need, _abi.stream_of(x)) == _abi.HG_OK
    torch.cuda.synchronize()
    assert int(ws[1]) == 0 and int(ws[0]) == units((2, 3, 136, 248), 2)
    ref = ops.hex_pyramid_chain(x, taps, None, 2)
    assert all(torch.equal(a, b) for a, b in zip(outs, ref))
