"""Multi-GPU path: a batch of frames shards by frame index across ranks (one process per GPU); the
only exchange is gathering the per-frame CRC words and valid flags to a root over RCCL/xGMI
(SURVEY.md section 8(e)).  Both halves live in libuflowcrc.so's C ABI (ufc_crc_sharded,
include/uflow_frame_crc.h), so a Rust host reaches the same path as this binding.

There is no data-path collective: every rank validates its own contiguous frame range.
"""
import ctypes

import numpy as np
import torch

from ._native import UFC_COMM_ID_BYTES, UFC_MAX_RANKS, Xfer, check, lib

OP_GATE, OP_SEND, OP_RECV = 0, 1, 2


def shard_range(total, rank, world):
    """Contiguous frame range [lo, hi) of `rank` (sizes differ by at most one): ufc_shard_range."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    first, count = ctypes.c_uint64(), ctypes.c_uint64()
    check(lib().ufc_shard_range(total, world, rank, ctypes.byref(first), ctypes.byref(count)), "ufc_shard_range")
    return first.value, first.value + count.value


def shard_chunks(total, rank, world):
    """The gather pipeline's chunks of `rank`'s shard as global [lo, hi) ranges (ufc_shard_chunk):
    chunk c of every rank is gated, then sent, in the same order on every rank."""
    first, count = ctypes.c_uint64(), ctypes.c_uint64()
    k = lib().ufc_shard_chunk(total, world, rank, 0, ctypes.byref(first), ctypes.byref(count))
    if k < 0:
        check(k, "ufc_shard_chunk")
    out = []
    for c in range(k):
        rc = lib().ufc_shard_chunk(total, world, rank, c, ctypes.byref(first), ctypes.byref(count))
        if rc < 0:
            check(rc, "ufc_shard_chunk")
        out.append((first.value, first.value + count.value))
    return out


def _bounds_arg(bounds):
    b = np.ascontiguousarray(bounds, dtype=np.uint64)
    return b, b.ctypes.data_as(ctypes.c_void_p)


def shard_bounds_fixed(total, world):
    """ufc_shard_bounds_fixed: rank r owns frames [b[r], b[r+1])."""
    if not 1 <= world <= UFC_MAX_RANKS:
        raise ValueError("bad world size")
    b = np.zeros(world + 1, np.uint64)
    check(lib().ufc_shard_bounds_fixed(total, world, b.ctypes.data_as(ctypes.c_void_p)), "ufc_shard_bounds_fixed")
    return b


def shard_bounds_varlen(offsets, world):
    """ufc_shard_bounds_varlen: the batch split by bytes (binary search of r * bytes / world in the
    CSR offsets, n + 1 entries)."""
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    if off.ndim != 1 or off.size < 1 or not 1 <= world <= UFC_MAX_RANKS:
        raise ValueError("offsets must be a 1-D array of n + 1 entries; 1 <= world <= 64")
    b = np.zeros(world + 1, np.uint64)
    check(lib().ufc_shard_bounds_varlen(off.ctypes.data_as(ctypes.c_void_p), off.size - 1, world,
                                        b.ctypes.data_as(ctypes.c_void_p)), "ufc_shard_bounds_varlen")
    return b


def gather_plan(bounds, rank, root):
    """The C gather schedule (ufc_shard_nchunks + ufc_shard_gather_plan) of `rank`: one list of
    (op, peer, src, dst, count) per chunk, executed in order (SEND/RECV of a chunk grouped)."""
    b, bp = _bounds_arg(bounds)
    world = b.size - 1
    k = lib().ufc_shard_nchunks(bp, world)
    if k < 0:
        check(k, "ufc_shard_nchunks")
    ops = (Xfer * (UFC_MAX_RANKS + 1))()
    plan = []
    for c in range(k):
        m = lib().ufc_shard_gather_plan(bp, world, rank, root, c, ops, len(ops))
        if m < 0:
            check(m, "ufc_shard_gather_plan")
        plan.append([(o.op, o.peer, o.src, o.dst, o.count) for o in ops[:m]])
    return plan


def comm_id_create():
    """A fresh communicator id (ncclGetUniqueId), made on one rank and handed to the others."""
    buf = (ctypes.c_uint8 * UFC_COMM_ID_BYTES)()
    check(lib().ufc_comm_id_create(buf), "ufc_comm_id_create")
    return bytes(buf)


class ShardedGate:
    """ufc_comm over one FrameCrcEngine (this rank's GPU): the batched gate over this rank's shard
    of a global fixed-length batch and the RCCL gather of CRC words + valid flags to the root."""

    def __init__(self, engine, world, rank, comm_id: bytes):
        if len(comm_id) != UFC_COMM_ID_BYTES:
            raise ValueError("comm id must be %d bytes" % UFC_COMM_ID_BYTES)
        self.engine, self.world, self.rank = engine, world, rank
        self._comm = ctypes.c_void_p()
        idbuf = (ctypes.c_uint8 * UFC_COMM_ID_BYTES).from_buffer_copy(comm_id)
        check(lib().ufc_comm_create(ctypes.byref(self._comm), engine._ctx, world, rank, idbuf), "ufc_comm_create")

    def close(self):
        if self._comm:
            lib().ufc_comm_destroy(self._comm)
            self._comm = ctypes.c_void_p()

    def set_timeout(self, timeout_ms):
        """How long a sharded call waits for every peer to join it (ufc_comm_set_timeout): past it the
        call raises NativeError(UFC_ERR_COMM) and the communicator is stalled for good."""
        check(lib().ufc_comm_set_timeout(self._comm, int(timeout_ms)), "ufc_comm_set_timeout")

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


    def local_range(self, n_total):
        return shard_range(n_total, self.rank, self.world)

    def crc_sharded(self, frames, frame_len, n_total, crc_out, valid_out, root=0, stride=None, stream=None,
                    gather_stream=None):
        """frames: this rank's shard (uint8, frame k at k * stride).  crc_out / valid_out: on the root
        n_total entries in global frame order, elsewhere this rank's shard.  The gate runs on
        `stream` (default: current), the transfers on `gather_stream` (default: `stream`)."""
        stride = frame_len if stride is None else stride
        lo, hi = self.local_range(n_total)
        n_out = n_total if self.rank == root else hi - lo
        eng = self.engine
        eng._check("frames", frames, (torch.uint8,), (hi - lo - 1) * stride + frame_len if hi > lo else 0)
        eng._check_outputs(n_out, crc_out, valid_out)
        s = eng._stream(stream)
        gs = eng._stream(gather_stream) if gather_stream is not None else None
        p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        check(lib().ufc_crc_sharded(self._comm, p(frames), stride, frame_len, n_total, p(crc_out), p(valid_out), root,
                                    s, gs), "ufc_crc_sharded")

    def crc_sharded_varlen(self, data, offsets, bounds, crc_out, valid_out, root=0, stream=None, gather_stream=None):
        """data / offsets: this rank's shard as a CSR batch of its own (offsets int64 on the device,
        bounds[r+1] - bounds[r] + 1 entries, relative to data).  bounds: shard_bounds_varlen of the
        whole batch, the same on every rank.  Outputs as crc_sharded."""
        b, bp = _bounds_arg(bounds)
        if b.size != self.world + 1:
            raise ValueError("bounds must have world + 1 entries")
        lo, hi = int(b[self.rank]), int(b[self.rank + 1])
        n_out = int(b[-1]) if self.rank == root else hi - lo
        eng = self.engine
        eng._check("offsets", offsets, (torch.int64,), hi - lo + 1)
        eng._check("data", data, (torch.uint8,), 0)
        eng._check_outputs(n_out, crc_out, valid_out)
        s = eng._stream(stream)
        gs = eng._stream(gather_stream) if gather_stream is not None else None
        p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        check(lib().ufc_crc_sharded_varlen(self._comm, p(data), p(offsets), bp, p(crc_out), p(valid_out), root, s, gs),
              "ufc_crc_sharded_varlen")
