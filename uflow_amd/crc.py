"""Scalar frame-CRC API mirroring the reference's Rust functions (host side).

    compute(data)            <- src/frame/serial/crc.rs:102-104
    extend(initial, data)    <- src/frame/serial/crc.rs:94-100
    frame_validate(frame)    <- the CRC gate of Frame::read, src/frame/serial/mod.rs:675-690
    frame_seal(frame)        <- the trailer step of every write_* (mod.rs:463-470) and of
                                DataFrameBuilder/AckFrameBuilder::build (build.rs:151-159)

These go through libuflowcrc.so's host entry points (the scalar drop-in for crc::compute);
the batched GPU path lives in uflow_amd.batch.
"""
import ctypes

from ._native import lib, check

FRAME_CRC_SIZE = 4      # src/frame/serial/mod.rs:12
FRAME_OVERHEAD = 5      # src/frame/serial/mod.rs:13
MAX_FRAME_SIZE = 1472   # src/lib.rs:286-294


def _buf(data):
    if isinstance(data, (bytes, bytearray, memoryview)):
        mv = memoryview(data).cast("B")
        if mv.readonly:
            b = ctypes.create_string_buffer(bytes(mv), len(mv))
            return b, len(mv)
        arr = (ctypes.c_uint8 * len(mv)).from_buffer(mv)
        return arr, len(mv)
    raise TypeError("expected bytes-like data")


def compute(data) -> int:
    buf, n = _buf(data)
    return lib().ufc_crc32_compute(buf, n)


def extend(initial_crc: int, data) -> int:
    buf, n = _buf(data)
    return lib().ufc_crc32_extend(initial_crc & 0xFFFFFFFF, buf, n)


def frame_validate(frame) -> bool:
    """True iff `Frame::read` would get past its length + CRC checks for these bytes."""
    buf, n = _buf(frame)
    return lib().ufc_frame_validate(buf, n) == 1


def frame_seal(frame: bytearray) -> int:
    """Write the big-endian CRC of frame[:-4] into frame[-4:] in place; returns the CRC."""
    if not isinstance(frame, bytearray):
        raise TypeError("frame_seal needs a mutable bytearray")
    if len(frame) < FRAME_CRC_SIZE:
        raise ValueError("a frame needs at least 4 bytes for its CRC trailer")
    arr = (ctypes.c_uint8 * len(frame)).from_buffer(frame)
    check(lib().ufc_frame_seal(arr, len(frame)), "ufc_frame_seal")
    return int.from_bytes(frame[-4:], "big")
