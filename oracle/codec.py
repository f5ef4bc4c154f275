"""TEST INFRASTRUCTURE ONLY (the checker, never the product): a pure-Python restatement of uflow's
frame codec, used by tests/ to pin the native codec (libuflowcrc.so, frame_codec.cpp) and the GPU
batch parse (frame_parse.hip).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg may import it.

Restates, from lowquark/uflow v0.7.1 (Rust):
  Frame::read / Frame::write          src/frame/serial/mod.rs:669-721
  read_*_payload                      src/frame/serial/mod.rs:54-434
  write_* (fixed-size frames)         src/frame/serial/mod.rs:437-667
  DataFrameBuilder / AckFrameBuilder  src/frame/serial/build.rs:47-256
The CRC is oracle.compute (crc_oracle.c, the restatement of crc.rs:94-104).

Frames are plain dicts, {"kind": <name>, ...fields}, with the field names of src/frame/mod.rs.
"""
import random

from . import compute

MAX_FRAME_SIZE = 1500 - 28  # src/lib.rs:286-294
HANDSHAKE_SYN, HANDSHAKE_SYN_ACK, HANDSHAKE_ACK, HANDSHAKE_ERROR = 0, 1, 2, 3  # serial/mod.rs:15-18
DISCONNECT, DISCONNECT_ACK, DATA, SYNC, ACK = 4, 5, 10, 11, 12                 # serial/mod.rs:19-23
KIND_IDS = {"handshake_syn": 0, "handshake_syn_ack": 1, "handshake_ack": 2, "handshake_error": 3,
            "disconnect": 4, "disconnect_ack": 5, "data": 10, "sync": 11, "ack": 12}
ERRORS = ("Version", "Config", "ServerFull")  # serial/mod.rs:157-162
PACKET_ID_MASK = (1 << 20) - 1  # src/packet_id.rs
MAX_CHANNELS = 64


def _be32(b, i):
    return (b[i] << 24) | (b[i + 1] << 16) | (b[i + 2] << 8) | b[i + 3]


def _be16(b, i):
    return (b[i] << 8) | b[i + 1]


def _p32(v):
    return bytes(((v >> 24) & 0xFF, (v >> 16) & 0xFF, (v >> 8) & 0xFF, v & 0xFF))


def _p16(v):
    return bytes(((v >> 8) & 0xFF, v & 0xFF))


MAX_FRAGMENT_SIZE = MAX_FRAME_SIZE - 10 - 14  # src/lib.rs:297 (DATA_FRAME_OVERHEAD, MAX_DATAGRAM_OVERHEAD)


def datagram_is_valid(dg):
    """src/half_connection/packet_receiver/mod.rs:12-30, the receive side's check of a decoded
    datagram before it enters the reassembly window (handle_datagram, :147-150)."""
    if dg["channel_id"] >= MAX_CHANNELS:  # CHANNEL_COUNT = MAX_CHANNELS (src/lib.rs:278)
        return False
    if dg["channel_parent_lead"] != 0:
        if dg["window_parent_lead"] == 0 or dg["channel_parent_lead"] < dg["window_parent_lead"]:
            return False
    if dg["fragment_id"] > dg["fragment_id_last"]:
        return False
    if dg["fragment_id"] < dg["fragment_id_last"] and len(dg["data"]) != MAX_FRAGMENT_SIZE:
        return False
    if len(dg["data"]) > MAX_FRAGMENT_SIZE:
        return False
    return True


# ---- decode (serial/mod.rs:54-434, 674-706) ----

def read_datagram(d):
    """serial/mod.rs:183-309: (datagram dict incl. its header form and data offset, size) or None."""
    if len(d) < 6:
        return None
    if d[0] & 0x80 == 0:  # micro
        hs, dl = 6, d[0] & 0x3F
        if len(d) < hs + dl:
            return None
        dg = {"channel_id": ((d[4] >> 2) & 0x20) | ((d[0] >> 2) & 0x10) | (d[1] & 0x0F),
              "sequence_id": ((d[1] & 0xF0) << 12) | (d[2] << 8) | d[3],
              "window_parent_lead": d[4] & 0x7F, "channel_parent_lead": d[5],
              "fragment_id": 0, "fragment_id_last": 0, "header": 0}
    elif d[0] & 0x40 == 0:  # small
        hs, dl = 9, d[1]
        if len(d) < hs + dl:
            return None
        dg = {"channel_id": d[0] & 0x3F, "sequence_id": ((d[2] & 0x0F) << 16) | (d[3] << 8) | d[4],
              "window_parent_lead": _be16(d, 5), "channel_parent_lead": _be16(d, 7),
              "fragment_id": 0, "fragment_id_last": 0, "header": 1}
    else:  # large
        hs, dl = 14, _be16(d, 1)
        if len(d) < hs + dl:
            return None
        dg = {"channel_id": d[0] & 0x3F, "sequence_id": ((d[3] & 0x0F) << 16) | (d[4] << 8) | d[5],
              "window_parent_lead": _be16(d, 6), "channel_parent_lead": _be16(d, 8),
              "fragment_id": _be16(d, 10), "fragment_id_last": _be16(d, 12), "header": 2}
    dg["data"] = bytes(d[hs:hs + dl])
    dg["data_len"] = dl
    return dg, hs + dl


def read_payload(kind, p):
    """Dispatch of serial/mod.rs:694-705 over the payload p = frame[1 .. len-4]."""
    n = len(p)
    if kind == HANDSHAKE_SYN:  # :54-87
        if n != MAX_FRAME_SIZE - 5:
            return None
        return {"kind": "handshake_syn", "version": p[0], "nonce": _be32(p, 1), "max_receive_rate": _be32(p, 5),
                "max_packet_size": _be32(p, 9), "max_receive_alloc": _be32(p, 13)}
    if kind == HANDSHAKE_SYN_ACK:  # :89-126
        if n != 20:
            return None
        return {"kind": "handshake_syn_ack", "nonce_ack": _be32(p, 0), "nonce": _be32(p, 4),
                "max_receive_rate": _be32(p, 8), "max_packet_size": _be32(p, 12), "max_receive_alloc": _be32(p, 16)}
    if kind == HANDSHAKE_ACK:  # :128-141
        if n != 4:
            return None
        return {"kind": "handshake_ack", "nonce_ack": _be32(p, 0)}
    if kind == HANDSHAKE_ERROR:  # :143-165
        if n != 5 or p[4] > 2:
            return None
        return {"kind": "handshake_error", "nonce_ack": _be32(p, 0), "error": ERRORS[p[4]]}
    if kind == DISCONNECT:  # :167-173
        return {"kind": "disconnect"} if n == 0 else None
    if kind == DISCONNECT_ACK:  # :175-181
        return {"kind": "disconnect_ack"} if n == 0 else None
    if kind == DATA:  # :311-340
        if n < 5:
            return None
        rest, dgs, off = p[5:], [], 5
        for _ in range(p[4] & 0x7F):
            r = read_datagram(rest)
            if r is None:
                return None
            dg, size = r
            dg["data_offset"] = 1 + off + {0: 6, 1: 9, 2: 14}[dg["header"]]  # offset in the frame
            dgs.append(dg)
            rest, off = rest[size:], off + size
        if len(rest):
            return None
        return {"kind": "data", "sequence_id": _be32(p, 0), "nonce": bool(p[4] & 0x80), "datagrams": dgs}
    if kind == SYNC:  # :342-367
        if n != 9:
            return None
        return {"kind": "sync", "next_frame_id": _be32(p, 1) if p[0] & 1 else None,
                "next_packet_id": _be32(p, 5) if p[0] & 2 else None}
    if kind == ACK:  # :369-434
        if n < 10:
            return None
        cnt, rest = _be16(p, 8), p[10:]
        if len(rest) != 9 * cnt:  # each group must be present (:412-417), nothing left (:425-427)
            return None
        acks = [{"base_id": _be32(rest, 9 * i), "bitfield": _be32(rest, 9 * i + 4), "nonce": rest[9 * i + 8] != 0}
                for i in range(cnt)]
        return {"kind": "ack", "frame_window_base_id": _be32(p, 0), "packet_window_base_id": _be32(p, 4),
                "frame_acks": acks}
    return None


def frame_read(fb):
    """Frame::read (serial/mod.rs:675-706): the decoded frame dict, or None."""
    fb = bytes(fb)
    if len(fb) < 5:
        return None
    if compute(fb[:-4]) != _be32(fb, len(fb) - 4):
        return None
    return read_payload(fb[0], fb[1:-4])


# ---- encode (serial/mod.rs:437-667, build.rs) ----

def _seal(body: bytes) -> bytes:
    return body + _p32(compute(body))


def datagram_header(dg):
    """DataFrameBuilder::add header choice and layout, build.rs:76-143."""
    dl, ch, seq = len(dg["data"]), dg["channel_id"], dg["sequence_id"]
    w, h = dg["window_parent_lead"], dg["channel_parent_lead"]
    if dg["fragment_id_last"] == 0:
        if dl < 64 and w < 128 and h < 256:
            return bytes((dl | ((ch & 0x10) << 2), (((seq >> 12) & 0xF0) | (ch & 0x0F)) & 0xFF, (seq >> 8) & 0xFF,
                          seq & 0xFF, (w | ((ch & 0x20) << 2)) & 0xFF, h & 0xFF))
        if dl < 256:
            return bytes((ch | 0x80, dl, (seq >> 16) & 0xFF, (seq >> 8) & 0xFF, seq & 0xFF)) + _p16(w) + _p16(h)
    return (bytes((ch | 0xC0,)) + _p16(dl) + bytes(((seq >> 16) & 0xFF, (seq >> 8) & 0xFF, seq & 0xFF)) + _p16(w)
            + _p16(h) + _p16(dg["fragment_id"]) + _p16(dg["fragment_id_last"]))


def frame_write(f):
    """Frame::write (serial/mod.rs:708-720)."""
    k = f["kind"]
    if k == "handshake_syn":  # :437-473 (zero-padded to MAX_FRAME_SIZE)
        body = bytes((0, f["version"])) + _p32(f["nonce"]) + _p32(f["max_receive_rate"]) + \
            _p32(f["max_packet_size"]) + _p32(f["max_receive_alloc"])
        return _seal(body + bytes(MAX_FRAME_SIZE - 4 - len(body)))
    if k == "handshake_syn_ack":  # :475-514
        return _seal(bytes((1,)) + _p32(f["nonce_ack"]) + _p32(f["nonce"]) + _p32(f["max_receive_rate"]) +
                     _p32(f["max_packet_size"]) + _p32(f["max_receive_alloc"]))
    if k == "handshake_ack":  # :516-539
        return _seal(bytes((2,)) + _p32(f["nonce_ack"]))
    if k == "handshake_error":  # :541-569
        return _seal(bytes((3,)) + _p32(f["nonce_ack"]) + bytes((ERRORS.index(f["error"]),)))
    if k == "disconnect":  # :571-590
        return _seal(bytes((4,)))
    if k == "disconnect_ack":  # :592-611
        return _seal(bytes((5,)))
    if k == "data":  # :613-621 -> DataFrameBuilder (build.rs:56-162)
        body = bytes((10,)) + _p32(f["sequence_id"]) + bytes((((1 if f["nonce"] else 0) << 7) | len(f["datagrams"]),))
        for dg in f["datagrams"]:
            body += datagram_header(dg) + bytes(dg["data"])
        return _seal(body)
    if k == "sync":  # :623-657
        nf, npk = f["next_frame_id"], f["next_packet_id"]
        mode = (1 if nf is not None else 0) | (2 if npk is not None else 0)
        return _seal(bytes((11, mode)) + _p32(nf or 0) + _p32(npk or 0))
    if k == "ack":  # :659-667 -> AckFrameBuilder (build.rs:183-247)
        body = bytes((12,)) + _p32(f["frame_window_base_id"]) + _p32(f["packet_window_base_id"]) + \
            _p16(len(f["frame_acks"]))
        for a in f["frame_acks"]:
            body += _p32(a["base_id"]) + _p32(a["bitfield"]) + bytes((1 if a["nonce"] else 0,))
        return _seal(body)
    raise ValueError(k)


# ---- the reference tests' frames (serial/mod.rs:760-925) and seeded random frames (:927-1052) ----

def reference_test_frames():
    small = bytes(range(256))
    big = dict(sequence_id=0x45678, channel_id=63, window_parent_lead=0x34A8, channel_parent_lead=0x8A43)
    return [
        ("handshake_syn_basic mod.rs:761", {"kind": "handshake_syn", "version": 0x7F, "nonce": 0x18273645,
                                             "max_receive_rate": 0x98765432, "max_packet_size": 0x01234567,
                                             "max_receive_alloc": 0xABCDEF01}),
        ("handshake_syn_ack_basic mod.rs:775", {"kind": "handshake_syn_ack", "nonce_ack": 0x03246387,
                                                 "nonce": 0x18273645, "max_receive_rate": 0x98765432,
                                                 "max_packet_size": 0x01234567, "max_receive_alloc": 0xABCDEF01}),
        ("handshake_ack_basic mod.rs:789", {"kind": "handshake_ack", "nonce_ack": 0x03246387}),
        ("handshake_error_basic mod.rs:799", {"kind": "handshake_error", "nonce_ack": 0x03246387,
                                               "error": "ServerFull"}),
        ("disconnect_basic mod.rs:810", {"kind": "disconnect"}),
        ("disconnect_ack_basic mod.rs:818", {"kind": "disconnect_ack"}),
        ("data_basic mod.rs:826", {"kind": "data", "sequence_id": 0x010203, "nonce": True, "datagrams": [
            dict(big, fragment_id=0x4789, fragment_id_last=0x478A, data=bytes((0, 1, 2))),
            dict(big, sequence_id=0x12345, fragment_id=0, fragment_id_last=0, data=small),
            dict(big, sequence_id=0x12345, fragment_id=0, fragment_id_last=0, data=bytes((0, 1, 2)))]}),
        ("sync_basic mod.rs:868 (frame id)", {"kind": "sync", "next_frame_id": 0x01020304, "next_packet_id": None}),
        ("sync_basic mod.rs:879 (packet id)", {"kind": "sync", "next_frame_id": None, "next_packet_id": 0x05060708}),
        ("ack_basic mod.rs:891", {"kind": "ack", "frame_window_base_id": 0x010203, "packet_window_base_id": 0x040506,
                                  "frame_acks": [{"base_id": 0x28475809, "bitfield": 0b01000100111101110110100110101,
                                                  "nonce": True}]}),
        ("data_empty mod.rs:908", {"kind": "data", "sequence_id": 0x010203, "nonce": True, "datagrams": []}),
        ("ack_empty mod.rs:917", {"kind": "ack", "frame_window_base_id": 0x010203, "packet_window_base_id": 0x040506,
                                  "frame_acks": []}),
    ]


def random_data_frame(rng: random.Random, max_datagrams=64, max_data=100):
    """random_data_frame (serial/mod.rs:932-992), seeded: micro / small / large datagrams."""
    def data(lo, hi):  # random_data (:927-930): length in [0, hi - lo]
        return bytes(rng.getrandbits(8) for _ in range(rng.randrange(hi - lo + 1)))
    dgs = []
    for _ in range(rng.randrange(max_datagrams)):
        t = rng.randrange(3)
        seq, ch = rng.getrandbits(32) & PACKET_ID_MASK, rng.randrange(MAX_CHANNELS)
        if t == 0:
            dgs.append(dict(sequence_id=seq, channel_id=ch, window_parent_lead=rng.randrange(128),
                            channel_parent_lead=rng.randrange(256), fragment_id=0, fragment_id_last=0,
                            data=data(0, 64)))
        elif t == 1:
            dgs.append(dict(sequence_id=seq, channel_id=ch, window_parent_lead=rng.getrandbits(16),
                            channel_parent_lead=rng.getrandbits(16), fragment_id=0, fragment_id_last=0,
                            data=data(64, max_data)))
        else:
            a, b = sorted((rng.getrandbits(16), rng.getrandbits(16)))
            dgs.append(dict(sequence_id=seq, channel_id=ch, window_parent_lead=rng.getrandbits(16),
                            channel_parent_lead=rng.getrandbits(16), fragment_id=a, fragment_id_last=b,
                            data=data(0, max_data)))
    return {"kind": "data", "sequence_id": rng.getrandbits(32), "nonce": bool(rng.getrandbits(1)), "datagrams": dgs}


def receive_side_data_frame(rng: random.Random, max_datagrams=6):
    """A data frame whose datagrams cover every branch of datagram_is_valid
    (packet_receiver/mod.rs:12-30): parent leads zero / equal / below / above, fragment ids in and
    out of order, fragments of exactly MAX_FRAGMENT_SIZE bytes or not, payloads over it."""
    dgs = []
    for _ in range(1 + rng.randrange(max_datagrams)):
        w = rng.choice([0, 1, rng.randrange(1, 300), rng.getrandbits(16)])
        c = rng.choice([0, w, max(w - 1, 0), w + 1, rng.getrandbits(16)]) & 0xFFFF
        a = rng.choice([0, 1, rng.getrandbits(16)])
        b = rng.choice([a, a + 1, max(a - 1, 0), rng.getrandbits(16)]) & 0xFFFF
        n = rng.choice([0, 5, MAX_FRAGMENT_SIZE - 1, MAX_FRAGMENT_SIZE, MAX_FRAGMENT_SIZE + 1, rng.randrange(300)])
        dgs.append(dict(sequence_id=rng.getrandbits(20), channel_id=rng.randrange(MAX_CHANNELS), window_parent_lead=w,
                        channel_parent_lead=c, fragment_id=a, fragment_id_last=b,
                        data=bytes(rng.getrandbits(8) for _ in range(n))))
    return {"kind": "data", "sequence_id": rng.getrandbits(32), "nonce": bool(rng.getrandbits(1)), "datagrams": dgs}


def random_sync_frame(rng):
    """sync_random (serial/mod.rs:1008-1024)."""
    return {"kind": "sync", "next_frame_id": rng.getrandbits(32) if rng.randrange(5) else None,
            "next_packet_id": rng.getrandbits(32) if rng.randrange(5) else None}


def random_ack_frame(rng, max_acks=100):
    """ack_random (serial/mod.rs:1026-1052)."""
    return {"kind": "ack", "frame_window_base_id": rng.getrandbits(32), "packet_window_base_id": rng.getrandbits(32),
            "frame_acks": [{"base_id": rng.getrandbits(32), "bitfield": rng.getrandbits(32),
                            "nonce": bool(rng.getrandbits(1))} for _ in range(rng.randrange(max_acks))]}


def canonical(f):
    """A decoded frame without the decoder-only keys (header form, offsets), for comparison with the
    encoder's input (verify_consistent, serial/mod.rs:727-736)."""
    if f is None or f["kind"] != "data":
        return f
    g = dict(f)
    g["datagrams"] = [{k: v for k, v in d.items() if k not in ("header", "data_offset", "data_len")}
                      for d in f["datagrams"]]
    for d in g["datagrams"]:
        d["data"] = bytes(d["data"])
    return g
