"""uflow's frame types and their Serialize surface, backed by libuflowcrc.so's native codec.

Mirrors the reference (lowquark/uflow v0.7.1):
    HandshakeSynFrame ... AckFrame, Frame      <- src/frame/mod.rs:4-148
    Frame.read(bytes) -> Frame | None          <- Serialize::read, src/frame/serial/mod.rs:674-706
    frame.write() -> bytes                     <- Serialize::write, src/frame/serial/mod.rs:708-720
    DataFrameBuilder, AckFrameBuilder          <- src/frame/serial/build.rs:47-256
and the batched receive-side parse that follows the batched CRC gate:
    parse_batch_host(bytes, offsets, valid)    <- Frame::read of every received datagram
    (device-resident: uflow_amd.batch.FrameCrcEngine.parse_varlen)

None plays the role of Rust's None: a frame the reference rejects is returned as None, never
raised.  Decoding goes through ufc_frame_read (C++, frame_codec_core.hpp); there is no Python
fallback.
"""
import ctypes
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from ._native import Builder, DatagramRef, FrameInfo, Item, check, lib, UFC_ERR_NOMEM

MAX_FRAME_SIZE = 1472  # src/lib.rs:286-294
DATA_FRAME_MAX_DATAGRAM_COUNT = 127  # serial/mod.rs:42
HANDSHAKE_SYN, HANDSHAKE_SYN_ACK, HANDSHAKE_ACK, HANDSHAKE_ERROR = 0, 1, 2, 3
DISCONNECT, DISCONNECT_ACK, DATA, SYNC, ACK = 4, 5, 10, 11, 12
HANDSHAKE_ERRORS = ("Version", "Config", "ServerFull")  # HandshakeErrorType, src/frame/mod.rs:30-35

# numpy views of ufc_frame_info / ufc_item (batched outputs)
FRAME_INFO_DTYPE = np.dtype([("kind", "u1"), ("ok", "u1"), ("aux", "u1"), ("crc_ok", "u1"), ("f", "<u4", (5,)),
                             ("item_count", "<u4"), ("item_first", "<u4")])
ITEM_DTYPE = np.dtype([("id", "<u4"), ("channel_id", "u1"), ("form", "u1"), ("window_parent_lead", "<u2"),
                       ("channel_parent_lead", "<u2"), ("fragment_id", "<u2"), ("fragment_id_last", "<u2"),
                       ("flags", "<u2"), ("data_offset", "<u4"), ("data_len", "<u4")])
assert FRAME_INFO_DTYPE.itemsize == ctypes.sizeof(FrameInfo) == 32
assert ITEM_DTYPE.itemsize == ctypes.sizeof(Item) == 24


@dataclass
class HandshakeSynFrame:
    version: int
    nonce: int
    max_receive_rate: int
    max_packet_size: int
    max_receive_alloc: int


@dataclass
class HandshakeSynAckFrame:
    nonce_ack: int
    nonce: int
    max_receive_rate: int
    max_packet_size: int
    max_receive_alloc: int


@dataclass
class HandshakeAckFrame:
    nonce_ack: int


@dataclass
class HandshakeErrorFrame:
    nonce_ack: int
    error: str  # "Version" | "Config" | "ServerFull"


@dataclass
class DisconnectFrame:
    pass


@dataclass
class DisconnectAckFrame:
    pass


@dataclass
class Datagram:
    sequence_id: int
    channel_id: int
    window_parent_lead: int
    channel_parent_lead: int
    fragment_id: int
    fragment_id_last: int
    data: bytes


@dataclass
class DataFrame:
    sequence_id: int
    nonce: bool
    datagrams: List[Datagram] = field(default_factory=list)


@dataclass
class SyncFrame:
    next_frame_id: Optional[int]
    next_packet_id: Optional[int]


@dataclass
class AckGroup:
    base_id: int
    bitfield: int
    nonce: bool


@dataclass
class AckFrame:
    frame_window_base_id: int
    packet_window_base_id: int
    frame_acks: List[AckGroup] = field(default_factory=list)


MAX_FRAGMENT_SIZE = 1448  # src/lib.rs:297


def datagram_is_valid(dg: Datagram) -> bool:
    """src/half_connection/packet_receiver/mod.rs:12-30 (through ufc_datagram_is_valid)."""
    it = Item()
    it.channel_id = dg.channel_id & 0xFF
    it.window_parent_lead = dg.window_parent_lead & 0xFFFF
    it.channel_parent_lead = dg.channel_parent_lead & 0xFFFF
    it.fragment_id = dg.fragment_id & 0xFFFF
    it.fragment_id_last = dg.fragment_id_last & 0xFFFF
    it.data_len = len(dg.data)
    rc = lib().ufc_datagram_is_valid(ctypes.byref(it))
    if rc < 0:
        check(rc, "ufc_datagram_is_valid")
    return rc == 1


def _u8buf(data):
    data = bytes(data)
    return ctypes.create_string_buffer(data, len(data)), len(data)


def _frame_from_info(info, items, fb: bytes):
    k, f = info.kind, list(info.f)
    if k == HANDSHAKE_SYN:
        return HandshakeSynFrame(info.aux, f[0], f[1], f[2], f[3])
    if k == HANDSHAKE_SYN_ACK:
        return HandshakeSynAckFrame(*f)
    if k == HANDSHAKE_ACK:
        return HandshakeAckFrame(f[0])
    if k == HANDSHAKE_ERROR:
        return HandshakeErrorFrame(f[0], HANDSHAKE_ERRORS[info.aux])
    if k == DISCONNECT:
        return DisconnectFrame()
    if k == DISCONNECT_ACK:
        return DisconnectAckFrame()
    if k == DATA:
        return DataFrame(f[0], bool(info.aux), [
            Datagram(it.id, it.channel_id, it.window_parent_lead, it.channel_parent_lead, it.fragment_id,
                     it.fragment_id_last, fb[it.data_offset:it.data_offset + it.data_len]) for it in items])
    if k == SYNC:
        return SyncFrame(f[0] if info.aux & 1 else None, f[1] if info.aux & 2 else None)
    if k == ACK:
        return AckFrame(f[0], f[1], [AckGroup(it.id, it.data_offset, bool(it.channel_id)) for it in items])
    raise AssertionError(k)


class Frame:
    """Serialize for every frame kind (serial/mod.rs:669-721)."""

    @staticmethod
    def read(frame_bytes) -> Optional[object]:
        fb = bytes(frame_bytes)
        buf, n = _u8buf(fb)
        info = FrameInfo()
        cap = 1024
        items = (Item * cap)()
        rc = lib().ufc_frame_read(buf, n, ctypes.byref(info), items, cap)
        if rc == UFC_ERR_NOMEM:
            cap = info.item_count
            items = (Item * cap)()
            rc = lib().ufc_frame_read(buf, n, ctypes.byref(info), items, cap)
        if rc < 0:
            check(rc, "ufc_frame_read")
        if rc == 0:
            return None
        return _frame_from_info(info, list(items[:info.item_count]), fb)

    @staticmethod
    def write(frame) -> bytes:
        if isinstance(frame, DataFrame):
            b = DataFrameBuilder(frame.sequence_id, frame.nonce)
            for d in frame.datagrams:
                b.add(d)
            return b.build()
        if isinstance(frame, AckFrame):
            b = AckFrameBuilder(frame.frame_window_base_id, frame.packet_window_base_id)
            for a in frame.frame_acks:
                b.add(a)
            return b.build()
        info = FrameInfo()
        if isinstance(frame, HandshakeSynFrame):
            info.kind, info.aux = HANDSHAKE_SYN, frame.version
            info.f[:4] = [frame.nonce, frame.max_receive_rate, frame.max_packet_size, frame.max_receive_alloc]
        elif isinstance(frame, HandshakeSynAckFrame):
            info.kind = HANDSHAKE_SYN_ACK
            info.f[:] = [frame.nonce_ack, frame.nonce, frame.max_receive_rate, frame.max_packet_size,
                         frame.max_receive_alloc]
        elif isinstance(frame, HandshakeAckFrame):
            info.kind, info.f[0] = HANDSHAKE_ACK, frame.nonce_ack
        elif isinstance(frame, HandshakeErrorFrame):
            info.kind, info.f[0], info.aux = HANDSHAKE_ERROR, frame.nonce_ack, HANDSHAKE_ERRORS.index(frame.error)
        elif isinstance(frame, DisconnectFrame):
            info.kind = DISCONNECT
        elif isinstance(frame, DisconnectAckFrame):
            info.kind = DISCONNECT_ACK
        elif isinstance(frame, SyncFrame):
            info.kind = SYNC
            info.aux = (1 if frame.next_frame_id is not None else 0) | (2 if frame.next_packet_id is not None else 0)
            info.f[0], info.f[1] = frame.next_frame_id or 0, frame.next_packet_id or 0
        else:
            raise TypeError(type(frame))
        out = ctypes.create_string_buffer(MAX_FRAME_SIZE)
        n = lib().ufc_frame_write_fixed(ctypes.byref(info), out, MAX_FRAME_SIZE, 1)
        if n == 0:
            raise ValueError("unencodable frame")
        return out.raw[:n]


class DataFrameBuilder:
    """build.rs:47-181 over a native buffer (the caller's Vec<u8> of the reference)."""
    MAX_COUNT = DATA_FRAME_MAX_DATAGRAM_COUNT

    def __init__(self, sequence_id: int, nonce: bool, capacity: int = 1 << 17):
        self._buf = ctypes.create_string_buffer(capacity)
        self._b = Builder()
        check(lib().ufc_data_frame_builder_init(ctypes.byref(self._b), self._buf, capacity, sequence_id & 0xFFFFFFFF,
                                                1 if nonce else 0), "DataFrameBuilder.new")
        self._keep = []

    @staticmethod
    def _ref(d: Datagram):
        data = bytes(d.data)
        cbuf = ctypes.create_string_buffer(data, max(len(data), 1))
        r = DatagramRef(d.sequence_id, d.channel_id, 0, d.window_parent_lead, d.channel_parent_lead, d.fragment_id,
                        d.fragment_id_last, ctypes.cast(cbuf, ctypes.c_void_p), len(data))
        return r, cbuf

    def add(self, d: Datagram):
        r, cbuf = self._ref(d)
        check(lib().ufc_data_frame_builder_add(ctypes.byref(self._b), ctypes.byref(r)), "DataFrameBuilder.add")

    @staticmethod
    def encoded_size(d: Datagram) -> int:
        r, _ = DataFrameBuilder._ref(d)
        return lib().ufc_data_frame_encoded_size(ctypes.byref(r))

    def count(self) -> int:
        return self._b.count

    def size(self) -> int:
        return lib().ufc_builder_size(ctypes.byref(self._b))

    def build(self, seal: bool = True) -> bytes:
        n = lib().ufc_builder_build(ctypes.byref(self._b), 1 if seal else 0)
        return self._buf.raw[:n]


class AckFrameBuilder:
    """build.rs:183-256."""

    def __init__(self, frame_window_base_id: int, packet_window_base_id: int, capacity: int = 1 << 17):
        self._buf = ctypes.create_string_buffer(capacity)
        self._b = Builder()
        check(lib().ufc_ack_frame_builder_init(ctypes.byref(self._b), self._buf, capacity, frame_window_base_id,
                                               packet_window_base_id), "AckFrameBuilder.new")

    def add(self, a: AckGroup):
        check(lib().ufc_ack_frame_builder_add(ctypes.byref(self._b), a.base_id & 0xFFFFFFFF, a.bitfield & 0xFFFFFFFF,
                                              1 if a.nonce else 0), "AckFrameBuilder.add")

    def size(self) -> int:
        return lib().ufc_builder_size(ctypes.byref(self._b))

    def build(self, seal: bool = True) -> bytes:
        n = lib().ufc_builder_build(ctypes.byref(self._b), 1 if seal else 0)
        return self._buf.raw[:n]


def parse_batch_host(data: np.ndarray, offsets: np.ndarray, valid: Optional[np.ndarray] = None, nthreads: int = 1):
    """Frame::read of every frame of a CSR batch in host memory, after the batched CRC gate
    (`valid`, from the GPU; None = gate on the host).  Returns (infos[n], items) as numpy
    structured arrays (FRAME_INFO_DTYPE, ITEM_DTYPE); infos['item_first'] indexes items."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = offsets.size - 1
    infos = np.zeros(max(n, 0), dtype=FRAME_INFO_DTYPE)
    if valid is not None:
        valid = np.ascontiguousarray(valid, dtype=np.uint8)
    used = ctypes.c_size_t(0)
    vp = valid.ctypes.data if valid is not None else None
    rc = lib().ufc_parse_batch_host(data.ctypes.data, offsets.ctypes.data, n, vp, infos.ctypes.data, None, 0,
                                    ctypes.byref(used), nthreads)
    check(rc, "ufc_parse_batch_host")
    items = np.zeros(used.value, dtype=ITEM_DTYPE)
    rc = lib().ufc_parse_batch_host(data.ctypes.data, offsets.ctypes.data, n, vp, infos.ctypes.data,
                                    items.ctypes.data, items.size, ctypes.byref(used), nthreads)
    check(rc, "ufc_parse_batch_host")
    return infos, items
