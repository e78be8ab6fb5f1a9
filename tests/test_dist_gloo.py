"""Multi-process batch sharding + gathers on CPU (gloo, world_size 2 and 4)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _check(rank, world, q)
    except Exception as exc:   # report instead of leaving the parent waiting on the queue
        q.put((rank, False, False, -1000))
        raise exc
    finally:
        dist.destroy_process_group()


def _check(rank, world, q):
    if True:
        from HyGrid.dist import (gather_checksums, gather_sums, gather_to_root, image_checksums,
                                 local_shard)
        B = 10
        full = torch.arange(B * 3 * 4 * 5, dtype=torch.float32).reshape(B, 3, 4, 5)
        mine = local_shard(full)
        cs = gather_checksums(image_checksums(mine))
        ok_cs = torch.allclose(cs, image_checksums(full))
        eq = full[: (B // world) * world].reshape(world, B // world, 3, 4, 5)[rank]
        got = gather_to_root(eq.contiguous())
        out = torch.full(((B // world) * world, 3, 4, 5), -1.0) if rank == 0 else None
        got2 = gather_to_root(eq, out=out)
        ok_g = True
        if rank == 0:
            ok_g = torch.equal(got, full[: (B // world) * world]) and got2 is out and \
                torch.equal(out, full[: (B // world) * world])
        else:
            ok_g = got is None and got2 is None
        # per-image sums gathered into one (world*B_local, C) tensor (the bench's timed RCCL)
        sums = eq.sum((2, 3))
        gs = gather_sums(sums)
        ok_g = ok_g and torch.equal(gs, full[: (B // world) * world].sum((2, 3)))
        q.put((rank, bool(ok_cs), bool(ok_g), mine.shape[0]))


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_shard_and_gather(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok_cs and ok_g for _, ok_cs, ok_g, _ in res)
    assert sum(n for *_, n in res) == 10
