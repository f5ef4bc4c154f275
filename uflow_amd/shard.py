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


class ShardGatherer:
    """Preallocated, pipelined gather of per-frame results to the root (bench.py's multi-GPU step).

    Every rank holds `n_local` frames.  Slot i owns one byte buffer: the CRC words (4 B per frame)
    followed by the valid flags (1 B per frame), so the kernel writes straight into it and ONE
    gather (RCCL point-to-point on the nccl backend) moves both.  Slots rotate: the gather of step
    k (async, on the collective's stream) overlaps the kernel of step k+1, which writes the other
    slot; `wait(i)` makes the current stream wait for slot i's previous gather before it is
    rewritten.  Nothing is allocated per step.
    """

    def __init__(self, n_local, device, root=0, depth=2, group=None):
        self.n = n_local
        self.root = root
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.bufs = [torch.zeros(5 * n_local, dtype=torch.uint8, device=device) for _ in range(depth)]
        self.recv = [torch.zeros((self.world, 5 * n_local), dtype=torch.uint8, device=device)
                     if self.rank == root else None for _ in range(depth)]
        self.handles = [None] * depth

    def outputs(self, i):
        """(crc int32[n], valid uint8[n]) views of slot i, for the kernel to write."""
        b = self.bufs[i]
        return b[: 4 * self.n].view(torch.int32), b[4 * self.n:]

    def start(self, i):
        parts = list(self.recv[i].unbind(0)) if self.rank == self.root else None
        self.handles[i] = dist.gather(self.bufs[i], gather_list=parts, dst=self.root, group=self.group,
                                      async_op=True)

    def wait(self, i):
        if self.handles[i] is not None:
            self.handles[i].wait()
            self.handles[i] = None

    def wait_all(self):
        for i in range(len(self.handles)):
            self.wait(i)

    def gathered(self, i):
        """On the root, after wait(i): (crc int32[world*n], valid uint8[world*n]) in global frame order."""
        if self.rank != self.root:
            return None
        r = self.recv[i]
        return r[:, : 4 * self.n].contiguous().view(torch.int32).reshape(-1), r[:, 4 * self.n:].reshape(-1)
