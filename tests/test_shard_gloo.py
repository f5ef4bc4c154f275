"""CPU, world sizes 2, 3 and 8 over gloo: the multi-GPU protocol of ufc_crc_sharded /
ufc_crc_sharded_varlen, driven by the C library's own gather schedule.

Every rank asks libuflowcrc.so for the shard bounds (ufc_shard_bounds_fixed, or
ufc_shard_bounds_varlen: split by bytes with a binary search on the offsets) and for its plan
(ufc_shard_gather_plan), then executes exactly that plan -- the same loop as run_sharded in
uflow_amd/csrc/ufc_shard.cpp -- with the oracle standing in for the device gate and gloo point-to-point
transfers standing in for the grouped ncclSend/ncclRecv.  The root's gathered result must equal a
single-process validation of the whole batch.  The GPU/RCCL half runs in tests/test_gpu_shard.py.
Reference caller: the receive loop src/server/mod.rs:591-602 (Frame::read of every datagram).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from uflow_amd.shard import (OP_GATE, OP_RECV, OP_SEND, gather_plan, shard_bounds_fixed, shard_bounds_varlen,
                             shard_chunks, shard_range)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _batch_fixed(total, L):
    import oracle
    rng = np.random.default_rng(99)
    buf = rng.integers(0, 256, size=total * L, dtype=np.uint8)
    oracle.seal_fixed_mt(buf, L, L, total, 4)
    buf[np.arange(0, total, 11) * L + 1] ^= 0x10
    return buf


def _batch_varlen(total):
    """U[0, 1500]-byte frames (lengths 0..4 included: they fail the gate), sealed, every 13th damaged."""
    import oracle
    rng = np.random.default_rng(7)
    lens = rng.integers(0, 1501, size=total).astype(np.uint64)
    off = np.zeros(total + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    data = rng.integers(0, 256, size=int(off[-1]) + 1, dtype=np.uint8)
    for i in np.nonzero(lens >= 4)[0]:
        fr = bytearray(data[off[i]:off[i + 1]].tobytes())
        oracle.frame_seal(fr)
        data[off[i]:off[i + 1]] = np.frombuffer(bytes(fr), np.uint8)
    for i in range(0, total, 13):
        if lens[i] > 0:
            data[off[i]] ^= 0x01
    return data, off


def _gate(kind, batch, L, lo, a, b):
    """The oracle in place of the device gate over this rank's local frames [a, b)."""
    import oracle
    if kind == "fixed":
        return oracle.validate_fixed(batch[(lo + a) * L:(lo + b) * L], L, L, b - a)
    data, off = batch
    return oracle.validate_varlen(data, off[lo + a:lo + b + 1])


def _worker(rank, world, port, kind, total, L, root, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if kind == "fixed":
            batch = _batch_fixed(total, L)
            bounds = shard_bounds_fixed(total, world)
        else:
            batch = _batch_varlen(total)
            bounds = shard_bounds_varlen(batch[1], world)
        lo, hi = int(bounds[rank]), int(bounds[rank + 1])
        n_out = total if rank == root else hi - lo
        crc_out = torch.zeros(n_out, dtype=torch.int32)
        valid_out = torch.zeros(n_out, dtype=torch.uint8)
        for ops in gather_plan(bounds, rank, root):  # one list per chunk, in order
            for op, peer, src, dst, count in ops:
                if op == OP_GATE:
                    crc, valid = _gate(kind, batch, L, lo, src, src + count)
                    crc_out[dst:dst + count] = torch.from_numpy(crc.view(np.int32).copy())
                    valid_out[dst:dst + count] = torch.from_numpy(valid.copy())
            for op, peer, src, dst, count in ops:
                if op == OP_SEND:
                    dist.send(crc_out[src:src + count], dst=peer)
                    dist.send(valid_out[src:src + count], dst=peer)
                elif op == OP_RECV:
                    dist.recv(crc_out[dst:dst + count], src=peer)
                    dist.recv(valid_out[dst:dst + count], src=peer)
        if rank == root:
            q.put((crc_out.numpy().view(np.uint32).copy(), valid_out.numpy().copy()))
    finally:
        dist.destroy_process_group()


def _run(world, kind, total, L, root):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, total, L, root, q)) for r in range(world)]
    for p in procs:
        p.start()
    got_crc, got_valid = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import oracle
    if kind == "fixed":
        ref_crc, ref_valid = oracle.validate_fixed_mt(_batch_fixed(total, L), L, L, total, 8)
    else:
        data, off = _batch_varlen(total)
        ref_crc, ref_valid = oracle.validate_varlen(data, off)
    assert np.array_equal(got_crc, ref_crc)
    assert np.array_equal(got_valid, ref_valid)
    return ref_valid


@pytest.mark.parametrize("world,total,L,root", [(2, 1001, 200, 0), (2, 4, 64, 1), (3, 1000, 150, 2),
                                                (8, 5, 64, 0), (8, 20011, 100, 3),
                                                (2, 9_000_000, 6, 0), (3, 13_000_000, 5, 1)])
def test_sharded_gather_equals_single(world, total, L, root):
    """The last two cases hold more than 2^22 frames per shard, so every shard is gathered in
    several chunks; (8, 5) leaves three ranks with empty shards."""
    _run(world, "fixed", total, L, root)


@pytest.mark.parametrize("world,total,root", [(2, 3000, 0), (3, 2999, 2), (8, 5000, 5), (8, 3, 0)])
def test_sharded_varlen_gather_equals_single(world, total, root):
    """Variable-length batch split by bytes (ufc_shard_bounds_varlen), gathered in global frame order."""
    valid = _run(world, "varlen", total, 0, root)
    if total > 100:
        assert 0 < int(valid.sum()) < total  # both outcomes present


def test_shard_range_and_chunks_partition():
    """ufc_shard_range / ufc_shard_chunk / ufc_shard_bounds_fixed: contiguous, balanced shards;
    chunks tile each shard in order, at most 2^22 frames each, the same count on every rank."""
    for total in (0, 1, 7, 1000, 10**8, 2**40 + 3):
        for world in (1, 2, 3, 8):
            ranges = [shard_range(total, r, world) for r in range(world)]
            assert ranges == [(total * r // world, total * (r + 1) // world) for r in range(world)]
            b = shard_bounds_fixed(total, world)
            assert [(int(b[r]), int(b[r + 1])) for r in range(world)] == ranges
            sizes = [hi - lo for lo, hi in ranges]
            assert max(sizes) - min(sizes) <= 1
            if total > 10**9:
                continue
            counts = set()
            for r in range(world):
                ch = shard_chunks(total, r, world)
                counts.add(len(ch))
                assert ch[0][0] == ranges[r][0] and ch[-1][1] == ranges[r][1]
                for (a, b_), (c, d) in zip(ch, ch[1:]):
                    assert b_ == c
                assert all(hi - lo <= 1 << 22 for lo, hi in ch) or len(ch) == 16
                # the C plan's GATE ops are exactly these chunks
                gates = [(o[2], o[2] + o[4]) for ops in gather_plan(b, r, 0) for o in ops if o[0] == OP_GATE]
                assert gates == [(lo - ranges[r][0], hi - ranges[r][0]) for lo, hi in ch if hi > lo]
            assert len(counts) == 1
    with pytest.raises(Exception):
        shard_range(10, 2, 2)
    assert len(shard_chunks(100_000_000, 0, 8)) == 3  # config 4: 12.5M frames per GPU in 3 chunks


def test_varlen_bounds_split_by_bytes():
    """ufc_shard_bounds_varlen: bounds[r] is the first frame starting at or past r/W of the bytes."""
    rng = np.random.default_rng(3)
    for total in (0, 1, 2, 17, 10_000):
        lens = rng.integers(0, 1501, size=total).astype(np.uint64)
        off = np.zeros(total + 1, np.uint64)
        np.cumsum(lens, out=off[1:])
        off += np.uint64(12345)  # offsets need not start at 0
        for world in (1, 2, 3, 8):
            b = shard_bounds_varlen(off, world)
            assert b[0] == 0 and b[-1] == total and np.all(np.diff(b.astype(np.int64)) >= 0)
            B = int(off[-1] - off[0])
            for r in range(1, world):
                t = int(off[0]) + B * r // world
                assert int(np.searchsorted(off, t, side="left")) == int(b[r])
    with pytest.raises(Exception):
        shard_bounds_varlen(np.array([5, 3], np.uint64), 2)
