"""CPU, world_size 2 (and 3) over gloo: the multi-GPU path of bench.py / SURVEY.md §8(e) --
frames shard contiguously by index, each rank validates its own range (here with the oracle,
standing in for the device kernel), and only the CRC words + valid flags are gathered to rank 0.
The gathered result must equal a single-process validation of the whole batch.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from uflow_amd.shard import gather_to_root, shard_range


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
    oracle.seal_fixed(buf, L, L, total)
    for i in range(0, total, 11):
        buf[i * L + 5] ^= 0x10
    return buf


def _worker(rank, world, port, total, L, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        buf = _batch(total, L)
        lo, hi = shard_range(total, rank, world)
        crc, valid = oracle.validate_fixed(buf[lo * L: hi * L], L, L, hi - lo)
        crc_t = torch.from_numpy(crc.view(np.int32).copy())
        val_t = torch.from_numpy(valid.copy())
        g_crc = gather_to_root(crc_t, total)
        g_val = gather_to_root(val_t, total)
        if rank == 0:
            q.put((g_crc.numpy().view(np.uint32).copy(), g_val.numpy().copy()))
        else:
            assert g_crc is None and g_val is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,total", [(2, 1001), (2, 4), (3, 1000)])
def test_sharded_gather_equals_single(world, total):
    L = 200
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, L, q)) for r in range(world)]
    for p in procs:
        p.start()
    got_crc, got_valid = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import oracle
    ref_crc, ref_valid = oracle.validate_fixed(_batch(total, L), L, L, total)
    assert np.array_equal(got_crc, ref_crc)
    assert np.array_equal(got_valid, ref_valid)


def test_shard_range_partition():
    for total in (0, 1, 7, 1000, 10**8):
        for world in (1, 2, 3, 8):
            ranges = [shard_range(total, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == total
            for (a, b), (c, d) in zip(ranges, ranges[1:]):
                assert b == c
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def _pipelined_worker(rank, world, port, n, L, steps, q):
    """bench.py's N>1 step loop with ShardGatherer: results written into the slot's views, async
    gathers overlapping the next step, slots reused after wait()."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from uflow_amd.shard import ShardGatherer
        buf = _batch(n * world, L)
        g = ShardGatherer(n, torch.device("cpu"))
        last = None
        for k in range(steps):
            i = k % 2
            g.wait(i)
            crc_v, val_v = g.outputs(i)
            lo = rank * n
            crc, valid = oracle.validate_fixed(buf[lo * L:(lo + n) * L], L, L, n)
            crc_v.copy_(torch.from_numpy(crc.view(np.int32).copy()))
            val_v.copy_(torch.from_numpy(valid.copy()))
            g.start(i)
            last = i
        g.wait_all()
        out = g.gathered(last)
        if rank == 0:
            q.put((out[0].numpy().view(np.uint32).copy(), out[1].numpy().copy()))
        else:
            assert out is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_pipelined_gatherer_equals_single(world):
    n, L, steps = 333, 120, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipelined_worker, args=(r, world, port, n, L, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    got_crc, got_valid = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import oracle
    ref_crc, ref_valid = oracle.validate_fixed(_batch(n * world, L), L, L, n * world)
    assert np.array_equal(got_crc, ref_crc)
    assert np.array_equal(got_valid, ref_valid)
