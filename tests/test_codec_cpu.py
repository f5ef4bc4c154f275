"""CPU: the native frame codec (include/uflow_frame_codec.h: Frame::read after the CRC gate, the
writers and builders, the batched host parse) against the Python restatement oracle/codec.py,
following the reference's codec tests (src/frame/serial/mod.rs:723-1081):
verify_consistent / verify_extra_bytes_fail / verify_truncation_fails on the fixed-value frames
(:760-925), the randomised data/sync/ack rounds (:927-1052, seeded here), crc_flips (:1054-1080),
plus structural fuzzing (header bytes mutated and the frame resealed, so that only the payload
parse decides).  The oracle is pinned by the C oracle's golden frames (tests/golden/frames.json)
and by its own round trips.
"""
import json
import os
import random

import numpy as np
import pytest

import oracle
from oracle import codec as C
from uflow_amd import frame as F

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def to_native(f):
    """oracle dict -> uflow_amd.frame dataclass."""
    k = f["kind"]
    if k == "handshake_syn":
        return F.HandshakeSynFrame(f["version"], f["nonce"], f["max_receive_rate"], f["max_packet_size"],
                                   f["max_receive_alloc"])
    if k == "handshake_syn_ack":
        return F.HandshakeSynAckFrame(f["nonce_ack"], f["nonce"], f["max_receive_rate"], f["max_packet_size"],
                                      f["max_receive_alloc"])
    if k == "handshake_ack":
        return F.HandshakeAckFrame(f["nonce_ack"])
    if k == "handshake_error":
        return F.HandshakeErrorFrame(f["nonce_ack"], f["error"])
    if k == "disconnect":
        return F.DisconnectFrame()
    if k == "disconnect_ack":
        return F.DisconnectAckFrame()
    if k == "data":
        return F.DataFrame(f["sequence_id"], f["nonce"], [
            F.Datagram(d["sequence_id"], d["channel_id"], d["window_parent_lead"], d["channel_parent_lead"],
                       d["fragment_id"], d["fragment_id_last"], bytes(d["data"])) for d in f["datagrams"]])
    if k == "sync":
        return F.SyncFrame(f["next_frame_id"], f["next_packet_id"])
    if k == "ack":
        return F.AckFrame(f["frame_window_base_id"], f["packet_window_base_id"],
                          [F.AckGroup(a["base_id"], a["bitfield"], a["nonce"]) for a in f["frame_acks"]])
    raise AssertionError(k)


def info_to_dict(info, items, fb):
    """A batched-parse record (FRAME_INFO_DTYPE + ITEM_DTYPE rows) -> the oracle's decoded dict."""
    if not info["ok"]:
        return None
    k, f, aux = int(info["kind"]), [int(x) for x in info["f"]], int(info["aux"])
    names = {v: n for n, v in C.KIND_IDS.items()}
    out = {"kind": names[k]}
    if k == F.HANDSHAKE_SYN:
        out.update(version=aux, nonce=f[0], max_receive_rate=f[1], max_packet_size=f[2], max_receive_alloc=f[3])
    elif k == F.HANDSHAKE_SYN_ACK:
        out.update(nonce_ack=f[0], nonce=f[1], max_receive_rate=f[2], max_packet_size=f[3], max_receive_alloc=f[4])
    elif k == F.HANDSHAKE_ACK:
        out.update(nonce_ack=f[0])
    elif k == F.HANDSHAKE_ERROR:
        out.update(nonce_ack=f[0], error=C.ERRORS[aux])
    elif k == F.DATA:
        out.update(sequence_id=f[0], nonce=bool(aux), datagrams=[
            {"channel_id": int(it["channel_id"]), "sequence_id": int(it["id"]),
             "window_parent_lead": int(it["window_parent_lead"]), "channel_parent_lead": int(it["channel_parent_lead"]),
             "fragment_id": int(it["fragment_id"]), "fragment_id_last": int(it["fragment_id_last"]),
             "header": int(it["form"]), "data": bytes(fb[int(it["data_offset"]):int(it["data_offset"]) + int(it["data_len"])]),
             "data_len": int(it["data_len"]), "data_offset": int(it["data_offset"])} for it in items])
    elif k == F.SYNC:
        out.update(next_frame_id=f[0] if aux & 1 else None, next_packet_id=f[1] if aux & 2 else None)
    elif k == F.ACK:
        out.update(frame_window_base_id=f[0], packet_window_base_id=f[1], frame_acks=[
            {"base_id": int(it["id"]), "bitfield": int(it["data_offset"]), "nonce": bool(it["channel_id"])}
            for it in items])
    return out


def test_oracle_pinned_by_c_oracle_golden_frames():
    """The Python codec oracle encodes the fixed frames exactly as the C oracle's committed golden
    fixture (the encoders of serial/mod.rs:437-657), and every fixture decodes to a frame."""
    with open(os.path.join(GOLDEN, "frames.json")) as f:
        g = {r["name"].split(" ")[0]: bytes.fromhex(r["hex"]) for r in json.load(f)["frames"]}
    ours = {name.split(" ")[0]: C.frame_write(fr) for name, fr in C.reference_test_frames()}
    for name in ("handshake_syn_basic", "handshake_syn_ack_basic", "handshake_ack_basic", "handshake_error_basic",
                 "disconnect_basic", "disconnect_ack_basic"):
        assert ours[name] == g[name], name
    assert C.frame_write({"kind": "sync", "next_frame_id": 0x01020304, "next_packet_id": 0x05060708}) == \
        g["sync_basic"]
    for fb in g.values():
        assert C.frame_read(fb) is not None


def test_golden_codec_fixture():
    """The committed codec fixture (tests/golden/codec_frames.json, from make_codec_golden.py):
    oracle and native codec both reproduce every encoding."""
    with open(os.path.join(GOLDEN, "codec_frames.json")) as f:
        rows = json.load(f)["frames"]
    cases = dict(C.reference_test_frames())
    for r in rows:
        fb = bytes.fromhex(r["hex"])
        assert C.frame_write(cases[r["name"]]) == fb, r["name"]
        assert F.Frame.write(to_native(cases[r["name"]])) == fb, r["name"]
        assert F.Frame.read(fb) == to_native(cases[r["name"]])


@pytest.mark.parametrize("name,fr", C.reference_test_frames(), ids=[n.split(" ")[0] for n, _ in C.reference_test_frames()])
def test_reference_frames_consistent_extra_truncation(name, fr):
    """verify_consistent / verify_extra_bytes_fail / verify_truncation_fails (serial/mod.rs:727-758)."""
    native = to_native(fr)
    fb = F.Frame.write(native)
    assert fb == C.frame_write(fr)
    assert F.Frame.read(fb) == native
    assert F.Frame.read(fb + b"\x00") is None
    for i in range(len(fb)):
        assert F.Frame.read(fb[:i]) is None


def test_random_frames_round_trip():
    """data_random / sync_random / ack_random (serial/mod.rs:994-1052), seeded."""
    rng = random.Random(20261016)
    for _ in range(150):
        for fr in (C.random_data_frame(rng), C.random_sync_frame(rng), C.random_ack_frame(rng)):
            native = to_native(fr)
            fb = F.Frame.write(native)
            assert fb == C.frame_write(fr)
            assert F.Frame.read(fb) == native
            assert F.Frame.read(fb + b"\x00") is None


def test_crc_flips():
    """crc_flips (serial/mod.rs:1054-1080): 5 random bit flips are rejected (seeded, 2000 rounds)."""
    rng = random.Random(5)
    for _ in range(2000):
        fb = bytearray(C.frame_write(C.random_data_frame(rng)))
        assert len(fb) <= 8192
        for _ in range(5):
            bit = rng.randrange(len(fb) * 8)
            fb[bit // 8] ^= 1 << (bit % 8)
        assert C.frame_read(fb) is None
        assert F.Frame.read(fb) is None


def _reseal(fb: bytearray):
    fb[-4:] = oracle.compute(bytes(fb[:-4])).to_bytes(4, "big")
    return fb


def _mutants(rng, n):
    """Structurally damaged frames with a valid CRC: random header bytes changed, bytes inserted or
    cut, then resealed -- only the payload parse can reject them."""
    out = []
    gens = (C.random_data_frame, C.random_sync_frame, C.random_ack_frame)
    fixed = [fr for _, fr in C.reference_test_frames()]
    for i in range(n):
        fr = gens[i % 3](rng) if i % 4 else fixed[i % len(fixed)]
        fb = bytearray(C.frame_write(fr))
        op = rng.randrange(4)
        body = len(fb) - 4
        if op == 0 and body > 0:
            for _ in range(rng.randrange(1, 3)):
                fb[rng.randrange(min(body, 40))] = rng.getrandbits(8)
        elif op == 1:
            at = rng.randrange(body + 1)
            fb[at:at] = bytes(rng.getrandbits(8) for _ in range(rng.randrange(1, 4)))
        elif op == 2 and body > 1:
            at = rng.randrange(body)
            del fb[at:at + rng.randrange(1, 4)]
        else:
            fb[0] = rng.choice([0, 1, 2, 3, 4, 5, 6, 9, 10, 11, 12, 13, 255])
        if len(fb) >= 4:
            _reseal(fb)
        out.append(bytes(fb))
    return out


def test_structural_fuzz_vs_oracle():
    rng = random.Random(77)
    mutants = _mutants(rng, 3000)
    accepted = 0
    for fb in mutants:
        ref = C.frame_read(fb)
        got = F.Frame.read(fb)
        assert (ref is None) == (got is None), fb[:16].hex()
        if ref is not None:
            accepted += 1
            assert got == to_native(C.canonical(ref))
    assert 0 < accepted < len(mutants)  # both outcomes exercised


def _batch(frames):
    offsets = np.zeros(len(frames) + 1, dtype=np.uint64)
    offsets[1:] = np.cumsum([len(f) for f in frames])
    data = np.frombuffer(b"".join(frames), dtype=np.uint8).copy() if frames else np.zeros(0, np.uint8)
    return data, offsets


@pytest.mark.parametrize("threads,with_valid", [(1, False), (4, False), (3, True)])
def test_parse_batch_host_vs_oracle(threads, with_valid):
    """The batched receive-side parse (every Frame::read of a receive loop, server/mod.rs:591-602)
    over a CSR batch of intact, bit-flipped, structurally damaged and short frames."""
    rng = random.Random(100 + threads)
    frames = []
    for i in range(2500):
        r = i % 5
        if r == 0:
            frames.append(bytes(C.frame_write(C.random_data_frame(rng))))
        elif r == 1:
            frames.append(bytes(C.frame_write(C.random_ack_frame(rng, 20))))
        elif r == 2:
            fb = bytearray(C.frame_write(C.random_data_frame(rng, 8)))
            fb[rng.randrange(len(fb))] ^= 1 << rng.randrange(8)
            frames.append(bytes(fb))
        elif r == 3:
            frames.extend(_mutants(rng, 1))
        else:
            frames.append(bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 7))))
    data, offsets = _batch(frames)
    valid = None
    if with_valid:
        _, valid = oracle.validate_varlen(data, offsets)
    infos, items = F.parse_batch_host(data, offsets, valid, nthreads=threads)
    first = 0
    for i, fb in enumerate(frames):
        ref = C.frame_read(fb)
        info = infos[i]
        assert int(info["item_first"]) == first
        cnt = int(info["item_count"]) if info["ok"] else 0
        got = info_to_dict(info, items[first:first + cnt], fb)
        assert got == ref, (i, fb[:16].hex())
        assert bool(info["crc_ok"]) == bool(oracle.frame_validate(fb)[0])
        first += cnt
    assert first == items.size


def test_datagram_is_valid_vs_oracle():
    """ufc_datagram_is_valid and the parses' UFC_ITEM_VALID flag == the restated
    datagram_is_valid (src/half_connection/packet_receiver/mod.rs:12-30) on datagrams that cover
    each of its branches, decoded by the host batch parse."""
    rng = random.Random(1230)
    frames = [C.frame_write(C.receive_side_data_frame(rng)) for _ in range(400)]
    offsets = np.zeros(len(frames) + 1, dtype=np.uint64)
    offsets[1:] = np.cumsum([len(f) for f in frames])
    data = np.frombuffer(b"".join(frames), dtype=np.uint8).copy()
    infos, items = F.parse_batch_host(data, offsets)
    seen = {True: 0, False: 0}
    for i, fb in enumerate(frames):
        ref = C.frame_read(fb)
        assert infos[i]["ok"] and ref is not None
        first, cnt = int(infos[i]["item_first"]), int(infos[i]["item_count"])
        for it, dg in zip(items[first:first + cnt], ref["datagrams"]):
            want = C.datagram_is_valid(dg)
            assert bool(it["flags"] & 1) == want
            d = F.Datagram(dg["sequence_id"], dg["channel_id"], dg["window_parent_lead"], dg["channel_parent_lead"],
                           dg["fragment_id"], dg["fragment_id_last"], dg["data"])
            assert F.datagram_is_valid(d) == want
            seen[want] += 1
    assert seen[True] > 100 and seen[False] > 100, seen
    # each rule alone (packet_receiver/mod.rs:13-29)
    ok = dict(sequence_id=1, channel_id=3, window_parent_lead=5, channel_parent_lead=7, fragment_id=0,
              fragment_id_last=0, data=b"x" * 10)
    for change, want in [({}, True), ({"channel_parent_lead": 0, "window_parent_lead": 0}, True),
                         ({"window_parent_lead": 0}, False), ({"channel_parent_lead": 4}, False),
                         ({"channel_parent_lead": 5}, True), ({"fragment_id": 2, "fragment_id_last": 1}, False),
                         ({"fragment_id": 1, "fragment_id_last": 2}, False),
                         ({"fragment_id": 1, "fragment_id_last": 2, "data": b"y" * 1448}, True),
                         ({"data": b"z" * 1448}, True), ({"data": b"z" * 1449}, False)]:
        dg = dict(ok, **change)
        assert C.datagram_is_valid(dg) == want, change
        assert F.datagram_is_valid(F.Datagram(**dg)) == want, change


def test_parse_expect_records_vs_host_parse():
    """tests/parse_expect.py (the oracle-built records the full-size GPU parse tests compare with) ==
    the native host parse, on every frame kind, damaged frames, and a tiled batch with flipped frames."""
    import parse_expect
    rng = random.Random(606)
    frames = []
    for i in range(900):
        r = i % 6
        if r == 0:
            frames.append(C.frame_write(C.random_data_frame(rng)))
        elif r == 1:
            frames.append(C.frame_write(C.random_ack_frame(rng, 30)))
        elif r == 2:
            frames.append(C.frame_write(C.random_sync_frame(rng)))
        elif r == 3:
            frames.append(C.frame_write(C.receive_side_data_frame(rng)))
        elif r == 4:
            frames.extend(_mutants(rng, 1))
        else:
            frames.append(C.frame_write(C.reference_test_frames()[i % 12][1]))
    data, offsets = _batch(frames)
    exp_infos, exp_items = parse_expect.oracle_records(frames)
    infos, items = F.parse_batch_host(data, offsets, None, nthreads=4)
    parse_expect.compare(infos, items, exp_infos, exp_items)
    assert items.size == exp_items.size
    # tiled, with flipped frames (the full-size tests' expansion)
    reps = 7
    n = len(frames) * reps
    tile = np.arange(n) % len(frames)
    lens = np.diff(offsets.astype(np.int64))
    big = np.tile(data, reps)
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(np.tile(lens, reps))
    flip = np.array([i for i in range(0, n, 13) if lens[tile[i]] >= 5 and exp_infos["crc_ok"][tile[i]]])
    big[offs[flip].astype(np.int64) + lens[tile[flip]] // 2] ^= 0x10
    dead = np.zeros(n, dtype=bool)
    dead[flip] = True
    t_infos, t_items = parse_expect.tile_records(exp_infos, exp_items, tile, dead)
    infos, items = F.parse_batch_host(big, offs, None, nthreads=4)
    parse_expect.compare(infos, items, t_infos, t_items)
    assert items.size == t_items.size
