"""Batch-axis data parallelism for the lattice pipeline (one process per GPU).

Images are independent units (every reference entry point is per-image,
geometry_np.py:191/358/520), so the batch shards with no data-path
collective: rank k owns the contiguous slice [k*B/N, (k+1)*B/N).  The only
exchange is the final gather of results to rank 0, over RCCL
(`torch.distributed` backend "nccl" on ROCm) across xGMI, or gloo on CPU.
"""
import torch
import torch.distributed as dist

__all__ = ["shard_range", "local_shard", "gather_to_root", "gather_checksums",
           "gather_sums", "image_checksums"]


def shard_range(total, rank, world):
    """Contiguous [start, stop) of `total` items for `rank` of `world` (balanced)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError(f"bad rank/world {rank}/{world}")
    base, rem = divmod(total, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def local_shard(batch, rank=None, world=None):
    """This rank's slice of a (B, ...) batch."""
    rank = dist.get_rank() if rank is None else rank
    world = dist.get_world_size() if world is None else world
    s, e = shard_range(batch.shape[0], rank, world)
    return batch[s:e]


def image_checksums(x):
    """Per-image, per-channel (sum, sum of squares) in fp64: (B, C, 2)."""
    x = x.flatten(2)
    s1 = x.sum(-1, dtype=torch.float64)
    s2 = torch.linalg.vector_norm(x, dim=-1, dtype=torch.float64) ** 2
    return torch.stack((s1, s2), dim=-1)


def gather_checksums(local, group=None):
    """All ranks' (B_local, C, 2) checksums -> (B_total, C, 2) on every rank."""
    world = dist.get_world_size(group)
    n = torch.tensor([local.shape[0]], device=local.device, dtype=torch.int64)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    m = int(max(s.item() for s in sizes))
    pad = torch.zeros((m,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    out = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(out, pad, group=group)
    return torch.cat([o[: int(s.item())] for o, s in zip(out, sizes)])


def gather_to_root(local, root=0, group=None, out=None):
    """Gather equal-shaped shards to `root` (P2P sends into root: xGMI ingress bound).

    Root receives straight into one (world*B_local, ...) tensor (`out`, or a new one):
    the shards land in its dim-0 slices, so root holds the result once, not the
    per-rank buffers plus their concatenation.  Returns it on root, None elsewhere.
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    local = local.contiguous()
    if rank == root:
        shape = (world * local.shape[0],) + tuple(local.shape[1:])
        if out is None:
            out = torch.empty(shape, dtype=local.dtype, device=local.device)
        elif tuple(out.shape) != shape or out.dtype != local.dtype or not out.is_contiguous():
            raise ValueError(f"gather_to_root: out must be a contiguous {shape} {local.dtype} tensor")
        dist.gather(local, gather_list=list(out.chunk(world)), dst=root, group=group)
        return out
    dist.gather(local, dst=root, group=group)
    return None


def gather_sums(local, out=None, group=None):
    """All-gather equal-shaped per-image reductions (B_local, C) into (world*B_local, C).

    The collective the weak-scaling bench keeps inside its timed loop: a few
    KB per rank, so it prices the RCCL latency, not xGMI bandwidth.
    """
    world = dist.get_world_size(group)
    shape = (world * local.shape[0],) + tuple(local.shape[1:])
    if out is None:
        out = torch.empty(shape, dtype=local.dtype, device=local.device)
    elif (tuple(out.shape) != shape or out.dtype != local.dtype or not out.is_contiguous()
          or out.device != local.device):
        raise ValueError(f"gather_sums: out must be a contiguous {shape} {local.dtype} tensor "
                         f"on {local.device}")
    dist.all_gather_into_tensor(out, local.contiguous(), group=group)
    return out
