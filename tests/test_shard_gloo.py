"""CPU, world_size 2 and 3 over gloo: the multi-GPU protocol of ufc_crc_sharded
with the device work replaced by the oracle -- frames shard contiguously by index
(ufc_shard_range), each rank validates its shard chunk by chunk (ufc_shard_chunk, the layout the C
code uses), and per chunk the non-root ranks send their CRC words and valid flags point-to-point
to the root, which receives them straight into their global positions (as the grouped
ncclSend/ncclRecv of ufc_crc_sharded do).  The gathered result must equal a single-process
validation of the whole batch.  The GPU/RCCL half runs in tests/test_gpu_shard.py.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from uflow_amd.shard import shard_chunks, shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _batch(total, L):
    import oracle
    rng = np.random.default_rng(99)
    buf = rng.integers(0, 256, size=total * L, dtype=np.uint8)
    oracle.seal_fixed_mt(buf, L, L, total, 4)
    buf[np.arange(0, total, 11) * L + 1] ^= 0x10
    return buf


def _worker(rank, world, port, total, L, root, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        buf = _batch(total, L)
        lo, hi = shard_range(total, rank, world)
        n_out = total if rank == root else hi - lo
        crc_out = torch.zeros(n_out, dtype=torch.int32)
        valid_out = torch.zeros(n_out, dtype=torch.uint8)
        base = 0 if rank == root else lo  # where this rank's results sit in its outputs
        chunks = [shard_chunks(total, r, world) for r in range(world)]
        assert len({len(c) for c in chunks}) == 1  # every rank agrees on the chunk count
        for c in range(len(chunks[rank])):
            a, b = chunks[rank][c]
            crc, valid = oracle.validate_fixed(buf[a * L:b * L], L, L, b - a)  # this chunk's gate
            crc_out[a - base:b - base] = torch.from_numpy(crc.view(np.int32).copy())
            valid_out[a - base:b - base] = torch.from_numpy(valid.copy())
            if rank == root:
                for p in range(world):
                    pa, pb = chunks[p][c]
                    if p != root and pb > pa:
                        dist.recv(crc_out[pa:pb], src=p)
                        dist.recv(valid_out[pa:pb], src=p)
            elif b > a:
                dist.send(crc_out[a - base:b - base], dst=root)
                dist.send(valid_out[a - base:b - base], dst=root)
        if rank == root:
            q.put((crc_out.numpy().view(np.uint32).copy(), valid_out.numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,total,L,root", [(2, 1001, 200, 0), (2, 4, 64, 1), (3, 1000, 150, 2),
                                                (2, 9_000_000, 6, 0), (3, 13_000_000, 5, 1)])
def test_sharded_gather_equals_single(world, total, L, root):
    """The last two cases hold more than 2^22 frames per shard, so every shard is gathered in
    several chunks."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, L, root, q)) for r in range(world)]
    for p in procs:
        p.start()
    got_crc, got_valid = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import oracle
    ref_crc, ref_valid = oracle.validate_fixed_mt(_batch(total, L), L, L, total, 8)
    assert np.array_equal(got_crc, ref_crc)
    assert np.array_equal(got_valid, ref_valid)


def _py_shard(total, rank, world):
    return total * rank // world, total * (rank + 1) // world


def test_shard_range_and_chunks_partition():
    """ufc_shard_range / ufc_shard_chunk: contiguous, balanced shards; chunks tile each shard in
    order, at most 2^22 frames each, the same count on every rank."""
    for total in (0, 1, 7, 1000, 10**8, 2**40 + 3):
        for world in (1, 2, 3, 8):
            ranges = [shard_range(total, r, world) for r in range(world)]
            assert ranges == [_py_shard(total, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == total
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1
            if total > 10**9:
                continue
            counts = set()
            for r in range(world):
                ch = shard_chunks(total, r, world)
                counts.add(len(ch))
                assert ch[0][0] == ranges[r][0] and ch[-1][1] == ranges[r][1]
                for (a, b), (c, d) in zip(ch, ch[1:]):
                    assert b == c
                assert all(b - a <= 1 << 22 for a, b in ch) or len(ch) == 16
            assert len(counts) == 1
    with pytest.raises(Exception):
        shard_range(10, 2, 2)
    assert len(shard_chunks(100_000_000, 0, 8)) == 3  # config 4: 12.5M frames per GPU in 3 chunks
