"""Multi-GPU path: frames shard by frame index across ranks (one process per GPU); the only
exchange is gathering the per-frame CRC words (and valid flags) to the root over RCCL/xGMI.

There is no data-path collective: every rank validates its own contiguous frame range, which is
the natural partition of independent frames.
"""
import torch
import torch.distributed as dist


def shard_range(total, rank, world):
    """Contiguous frame range [lo, hi) of `rank` (sizes differ by at most one)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    lo = total * rank // world
    hi = total * (rank + 1) // world
    return lo, hi


def gather_to_root(local, total, root=0, group=None):
    """Gather each rank's shard (1-D tensor, rank r holds shard_range(total, r, world)) into one
    tensor of length `total` on `root` (None elsewhere).  Uses dist.gather, which is RCCL's
    point-to-point gather on the nccl backend; shards are padded to equal length."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    maxlen = (total + world - 1) // world
    buf = torch.zeros(maxlen, dtype=local.dtype, device=local.device)
    buf[: local.numel()] = local
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == root else None
    dist.gather(buf, gather_list=parts, dst=root, group=group)
    if rank != root:
        return None
    out = torch.empty(total, dtype=local.dtype, device=local.device)
    for r in range(world):
        lo, hi = shard_range(total, r, world)
        out[lo:hi] = parts[r][: hi - lo]
    return out
