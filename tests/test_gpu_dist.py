"""RCCL path of the batch-sharded bench (BASELINE config 4) on one GPU: a world-size-1
"nccl" process group (RCCL on ROCm) with a bound device, then every collective the
multi-GPU bench issues (HyGrid/dist.py) on device tensors.  The gloo tests cover the
sharding logic at world 2 and 4 on the CPU; this runs the same calls through RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

from oracle import oracle as O

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a HIP device", allow_module_level=True)

from HyGrid import ops  # noqa: E402
from HyGrid.dist import (gather_checksums, gather_sums, gather_to_root,  # noqa: E402
                         image_checksums, local_shard)
from HyGrid.HexFrames import HexConv2d  # noqa: E402
from HyGrid.pipeline import rect_hex_conv_rect  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture
def nccl_world1():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        yield dev
    finally:
        dist.destroy_process_group()


def test_rccl_world1_bench_collectives(nccl_world1):
    dev = nccl_world1
    torch.manual_seed(3)
    conv = HexConv2d(3, 3, 0, 2, padding=1, bias=True).to(dev)
    gen = torch.Generator(device=dev).manual_seed(4)
    x = torch.rand((4, 3, 64, 128), generator=gen, device=dev, dtype=torch.bfloat16)
    mine = local_shard(x)
    assert mine.shape[0] == 4
    with torch.no_grad():
        y = rect_hex_conv_rect(mine, conv)
    # the timed-loop collective: per-image sums of a row sample, all-gathered
    sums = y[:, :, ::16].float().sum((2, 3))
    gs = gather_sums(sums)
    assert gs.device == dev and torch.equal(gs, sums)
    # checksums (after the timed region) and the full-output gather into one buffer
    cs = gather_checksums(image_checksums(y))
    assert torch.equal(cs, image_checksums(y))
    out = torch.empty_like(y)
    got = gather_to_root(y, out=out)
    torch.cuda.synchronize()
    assert got is out and torch.equal(out, y)
    # the unfused operators give the same images through the same collectives
    with torch.no_grad():
        u = ops.hex_to_rect(conv(ops.rect_to_hex(mine, (64, 128), out_dtype=torch.bfloat16)),
                            (64, 128), out_dtype=torch.float32)
    ref = rect_hex_conv_rect(mine, conv, out_dtype=torch.float32)
    torch.testing.assert_close(gather_to_root(u), ref, rtol=2 ** -7, atol=2 ** -7)


def test_rccl_world1_config3_shard(nccl_world1):
    """Config 4's per-rank workload through RCCL: one rank's 128 x 3 x 2160 x 3840 bf16 shard
    (config 3's batch) through the fused pipeline, then the bench's timed-loop collective
    (per-image sums of every 64th output row, all-gathered into a preallocated buffer) and
    the checksum gather.  The sums must equal the local ones exactly, three images of the
    shard (first, middle, last) are checked against the operator chain and the last one
    against the fp64 oracle chain (one bf16 rounding)."""
    dev = nccl_world1
    torch.manual_seed(3)
    conv = HexConv2d(3, 3, 0, 2, padding=1, bias=True).to(dev)
    gen = torch.Generator(device=dev).manual_seed(4)
    x = torch.rand((128, 3, 2160, 3840), generator=gen, device=dev, dtype=torch.bfloat16)
    mine = local_shard(x)
    assert mine.shape[0] == 128
    with torch.no_grad():
        y = rect_hex_conv_rect(mine, conv, out_dtype=torch.bfloat16)
    sums = torch.sum(y[:, :, ::64], (2, 3), dtype=torch.float32)
    buf = torch.empty_like(sums)
    gs = gather_sums(sums, out=buf)
    assert gs is buf and torch.equal(gs, sums) and bool(torch.isfinite(gs).all())
    with pytest.raises(ValueError):
        gather_sums(sums, out=torch.empty((3, 3), device=dev))
    cs = gather_checksums(image_checksums(y))
    assert torch.equal(cs, image_checksums(y))
    with torch.no_grad():
        for i in (0, 63, 127):
            xi = mine[i:i + 1]
            u = ops.hex_to_rect(conv(ops.rect_to_hex(xi, (2160, 3840), out_dtype=torch.float32)),
                                (2160, 3840), out_dtype=torch.float32)
            torch.testing.assert_close(y[i:i + 1].float(), u, rtol=2 ** -7, atol=2 ** -7 * u.abs().max().item())
    # and the shard's last image against the fp64 oracle chain: one bf16 rounding
    h = O.rect_to_hex(mine[127].double().cpu().numpy(), (2160, 3840), 1)
    c = O.hexconv2d(h, conv.kernel.detach().cpu().double().numpy(),
                    conv.bias.detach().cpu().double().numpy(), 0, 2, padding=1)
    ref = O.hex_to_rect(c, (2160, 3840), 1).reshape(3, 2160, 3840)
    got = y[127].double().cpu().numpy()
    # per element: one bf16 rounding of |ref| plus an absolute floor of 1e-5 max|ref|
    tol = 2.0 ** -8 * np.abs(ref) + 1e-5 * np.abs(ref).max()
    assert not (np.abs(got - ref) > tol).any(), int((np.abs(got - ref) > tol).sum())
    del x, y
