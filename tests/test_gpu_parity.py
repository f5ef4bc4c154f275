"""GPU parity: the gfx950 kernels (through the C ABI) vs the CPU oracle, bit-exact.

Cases follow the reference's own tests: KAT (crc.rs:135-138), lengths around every internal
boundary of the kernel (256-byte blocks, the G/data boundary, chunking), fixed-value frames of
every kind (serial/mod.rs:760-925), bit flips (serial/mod.rs:1054-1080), truncation and
extra bytes (serial/mod.rs:738-758), empty/short frames (mod.rs:676-678), varlen batches.
"""
import numpy as np
import pytest
import torch

import oracle
from uflow_amd import _native as N

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _rand_bytes(rng, n):
    return rng.integers(0, 256, size=n, dtype=np.uint8)


def _fixed_case(engine, rng, frame_len, stride, n, seal_first=True, flip_every=0):
    buf = _rand_bytes(rng, max(n * stride, 1) + 64)
    if seal_first and frame_len >= 4:
        oracle.seal_fixed(buf, stride, frame_len, n)
    if flip_every:
        for i in range(0, n, flip_every):
            byte = i * stride + rng.integers(0, max(frame_len, 1))
            buf[byte] ^= np.uint8(1 << int(rng.integers(0, 8)))
    ref_crc, ref_valid = oracle.validate_fixed(buf, stride, frame_len, n)
    d = torch.from_numpy(buf).to(DEV)
    crc, valid = engine.crc_fixed(d, frame_len, stride=stride, n=n)
    torch.cuda.synchronize()
    got_crc = crc.cpu().numpy().view(np.uint32)
    got_valid = valid.cpu().numpy()
    bad = np.nonzero(got_crc != ref_crc)[0]
    assert bad.size == 0, f"len={frame_len} stride={stride} n={n}: {bad.size} crc mismatches, first {bad[:5]}"
    assert np.array_equal(got_valid, ref_valid), f"len={frame_len} stride={stride} n={n}: valid mismatch"
    return got_valid


LENGTHS = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 12, 13, 15, 16, 17, 31, 63, 64, 65, 100, 247, 248, 249, 250, 251, 252,
           253, 254, 255, 256, 257, 258, 259, 260, 261, 263, 264, 500, 511, 512, 513, 515, 516, 1000, 1472, 1496,
           1500, 1531, 1532, 1533, 1535, 1536, 1537, 1540, 1787, 1788, 2048, 3000, 8192]


@pytest.mark.parametrize("frame_len", LENGTHS)
def test_fixed_lengths(engine, frame_len):
    rng = np.random.default_rng(1000 + frame_len)
    for stride_extra in (0, 3):
        for n in (1, 5, 67):
            _fixed_case(engine, rng, frame_len, frame_len + stride_extra, n)


def test_fixed_large_batch_with_flips(engine):
    rng = np.random.default_rng(7)
    valid = _fixed_case(engine, rng, 1500, 1500, 20000, flip_every=1000)
    assert valid.sum() == 20000 - 20


@pytest.mark.parametrize("frame_len,n", [(64, 3), (64, 4 * 4096 - 1), (1500, 4 * 4096 * 2 + 3), (1500, 70001),
                                         (250, 123457), (1531, 9999)])
def test_fixed_exact_buffer_partition(engine, frame_len, n):
    """Buffer ends exactly at the last frame's end; sizes straddle the per-wave set partition."""
    rng = np.random.default_rng(frame_len * 7 + n)
    stride = frame_len
    buf = _rand_bytes(rng, n * stride)
    oracle.seal_fixed(buf, stride, frame_len, n)
    for i in range(0, n, 37):
        buf[i * stride + int(rng.integers(0, frame_len))] ^= np.uint8(1 << int(rng.integers(0, 8)))
    ref_crc, ref_valid = oracle.validate_fixed(buf, stride, frame_len, n)
    crc, valid = engine.crc_fixed(torch.from_numpy(buf).to(DEV), frame_len, stride=stride, n=n)
    torch.cuda.synchronize()
    assert np.array_equal(crc.cpu().numpy().view(np.uint32), ref_crc)
    assert np.array_equal(valid.cpu().numpy(), ref_valid)


def test_fixed_kat(engine):
    frame = bytearray(b"123456789" + b"\0\0\0\0")
    oracle.frame_seal(frame)
    assert frame[-4:] == bytes.fromhex("11A6F2A3")
    d = torch.tensor(list(frame), dtype=torch.uint8, device=DEV)
    crc, valid = engine.crc_fixed(d, len(frame))
    assert int(crc.cpu().numpy().view(np.uint32)[0]) == 0x11A6F2A3
    assert int(valid.cpu()[0]) == 1


@pytest.mark.parametrize("seal_kernel", ["two_pass", "inline"])
def test_seal_fixed(engine, seal_kernel):
    """Both seal variants (UFC_OPT_SEAL_KERNEL), with and without a crc_out (per-stream scratch)."""
    engine.set_option(N.UFC_OPT_SEAL_KERNEL, N.UFC_SEAL_INLINE if seal_kernel == "inline" else N.UFC_SEAL_TWO_PASS)
    try:
        rng = np.random.default_rng(11)
        for frame_len in (4, 5, 9, 14, 25, 259, 260, 1472, 1500, 2051):
            for stride in (frame_len, frame_len + 5, frame_len + 3):
                for n, want_crc in ((130, True), (1001, False)):
                    buf = _rand_bytes(rng, n * stride + 16)
                    ref = buf.copy()
                    oracle.seal_fixed(ref, stride, frame_len, n)
                    d = torch.from_numpy(buf).to(DEV)
                    crc_out = torch.empty(n, dtype=torch.int32, device=DEV) if want_crc else None
                    engine.seal_fixed(d, frame_len, stride=stride, n=n, crc_out=crc_out)
                    torch.cuda.synchronize()
                    assert np.array_equal(d.cpu().numpy(), ref), f"seal len={frame_len} stride={stride} n={n}"
                    ref_crc, ref_valid = oracle.validate_fixed(ref, stride, frame_len, n)
                    if want_crc:
                        assert np.array_equal(crc_out.cpu().numpy().view(np.uint32), ref_crc)
                    assert ref_valid.all() or frame_len < 5
    finally:  # back to the default (the one-kernel seal)
        engine.set_option(N.UFC_OPT_SEAL_KERNEL, N.UFC_SEAL_INLINE)


def _varlen_case(engine, rng, lens, seal=True, flip_every=0):
    offsets = np.zeros(len(lens) + 1, dtype=np.int64)
    offsets[1:] = np.cumsum(lens)
    data = _rand_bytes(rng, int(offsets[-1]) + 1)
    if seal:
        oracle.seal_varlen(data, offsets.astype(np.uint64)) if all(l >= 4 for l in lens) else None
    if flip_every:
        for i in range(0, len(lens), flip_every):
            if lens[i]:
                data[offsets[i] + rng.integers(0, lens[i])] ^= np.uint8(1 << int(rng.integers(0, 8)))
    ref_crc, ref_valid = oracle.validate_varlen(data, offsets.astype(np.uint64))
    crc, valid = engine.crc_varlen(torch.from_numpy(data).to(DEV), torch.from_numpy(offsets).to(DEV))
    torch.cuda.synchronize()
    got = crc.cpu().numpy().view(np.uint32)
    bad = np.nonzero(got != ref_crc)[0]
    assert bad.size == 0, f"{bad.size} varlen crc mismatches, first idx {bad[:5]} lens {[lens[i] for i in bad[:5]]}"
    assert np.array_equal(valid.cpu().numpy(), ref_valid)
    return valid.cpu().numpy()


def test_varlen_mixed(engine):
    rng = np.random.default_rng(21)
    lens = rng.integers(64, 1501, size=10000).tolist()
    _varlen_case(engine, rng, lens, flip_every=97)


def test_varlen_edges(engine):
    rng = np.random.default_rng(22)
    lens = [0, 1, 2, 3, 4, 5, 6, 255, 256, 257, 258, 259, 260, 1472, 8192, 0, 9, 3000, 1, 1532, 1533] * 7
    rng.shuffle(lens)
    _varlen_case(engine, rng, lens, seal=False)


def test_varlen_uflow_frames(engine):
    """Real uflow frame sizes 5..1472 B (src/lib.rs:294)."""
    rng = np.random.default_rng(23)
    lens = rng.integers(5, 1473, size=5000).tolist()
    valid = _varlen_case(engine, rng, lens)
    assert valid.all()


def test_seal_varlen(engine):
    rng = np.random.default_rng(31)
    lens = rng.integers(4, 2000, size=3000).tolist()
    offsets = np.zeros(len(lens) + 1, dtype=np.int64)
    offsets[1:] = np.cumsum(lens)
    data = _rand_bytes(rng, int(offsets[-1]))
    ref = data.copy()
    oracle.seal_varlen(ref, offsets.astype(np.uint64))
    d = torch.from_numpy(data).to(DEV)
    engine.seal_varlen(d, torch.from_numpy(offsets).to(DEV))
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy(), ref)


def test_host_varlen(engine):
    rng = np.random.default_rng(41)
    lens = rng.integers(5, 1473, size=4000).tolist()
    offsets = np.zeros(len(lens) + 1, dtype=np.uint64)
    offsets[1:] = np.cumsum(lens)
    data = _rand_bytes(rng, int(offsets[-1]))
    oracle.seal_varlen(data, offsets)
    data[int(offsets[10]) + 3] ^= 0x10
    ref_crc, ref_valid = oracle.validate_varlen(data, offsets)
    crc, valid = engine.validate_host_varlen(data, offsets)
    assert np.array_equal(crc, ref_crc)
    assert np.array_equal(valid, ref_valid)
    assert valid.sum() == len(lens) - 1


@pytest.mark.parametrize("lo,hi,n", [(5, 1473, 200_003), (64, 1501, 131_072), (4, 300, 50_001), (1400, 1533, 40_000)])
def test_varlen_large_batches(engine, lo, hi, n):
    """Batches big enough that every workgroup claims sets dynamically; length mixes that keep
    sets homogeneous (short, long) and mixed."""
    rng = np.random.default_rng(lo * 7919 + n)
    lens = rng.integers(lo, hi, size=n).tolist()
    valid = _varlen_case(engine, rng, lens, flip_every=101)
    if lo >= 5:  # 4-byte frames never pass the gate (serial/mod.rs:676-678)
        assert valid.sum() == n - len(range(0, n, 101))


def test_seal_varlen_large(engine):
    rng = np.random.default_rng(32)
    lens = rng.integers(4, 1600, size=120_000)
    offsets = np.zeros(len(lens) + 1, dtype=np.int64)
    offsets[1:] = np.cumsum(lens)
    data = _rand_bytes(rng, int(offsets[-1]))
    ref = data.copy()
    oracle.seal_varlen(ref, offsets.astype(np.uint64))
    d = torch.from_numpy(data).to(DEV)
    crc_out = torch.empty(len(lens), dtype=torch.int32, device=DEV)
    engine.seal_varlen(d, torch.from_numpy(offsets).to(DEV), crc_out=crc_out)
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy(), ref)
    ref_crc, _ = oracle.validate_varlen(ref, offsets.astype(np.uint64))
    assert np.array_equal(crc_out.cpu().numpy().view(np.uint32), ref_crc)


@pytest.mark.parametrize("shift", [0, 1, 2, 3])
def test_varlen_trailer_bytes(engine, shift):
    """The gate reads each trailer from its frame's last two lines (no load of its own): one trailer
    byte flipped in every third frame, each of the 4 bytes in turn, at every trailer position in a
    line (those starting in the previous line's last word included)."""
    rng = np.random.default_rng(70 + shift)
    lens = rng.integers(4, 1533, size=60_000)
    offsets = np.zeros(len(lens) + 1, dtype=np.int64)
    offsets[1:] = np.cumsum(lens)
    data = _rand_bytes(rng, int(offsets[-1]) + shift)
    view = data[shift:]
    oracle.seal_varlen(view, offsets.astype(np.uint64))
    for i in range(0, len(lens), 3):
        view[offsets[i + 1] - 4 + (i // 3) % 4] ^= np.uint8(1 << int(rng.integers(0, 8)))
    ref_crc, ref_valid = oracle.validate_varlen(view, offsets.astype(np.uint64))
    d = torch.from_numpy(data).to(DEV)[shift:]
    crc, valid = engine.crc_varlen(d, torch.from_numpy(offsets).to(DEV))
    torch.cuda.synchronize()
    assert np.array_equal(crc.cpu().numpy().view(np.uint32), ref_crc)
    assert np.array_equal(valid.cpu().numpy(), ref_valid)
    ends = ((offsets[1:] + shift - 4) % 128).astype(np.int64)  # trailer start's line offset
    assert {124, 125, 126, 127} <= set(ends[lens >= 5].tolist())


@pytest.mark.parametrize("shift", [0, 1, 3, 37, 64])
def test_seal_varlen_shared_blocks(engine, shift):
    """Seals of frames packed tight: short neighbours (trailers a few bytes apart, many in one 64-byte
    block), trailers across a block edge, a batch at any address, and the bytes around the batch left
    alone.  Every trailer must equal the oracle's and no other byte may change, whatever store shape the
    seal uses (one dword store per frame in the product; whole-64-byte-block forms were measured and
    not kept)."""
    rng = np.random.default_rng(60 + shift)
    lens = np.concatenate([rng.integers(4, 140, size=40_000), rng.integers(4, 1533, size=20_000),
                           rng.integers(60, 70, size=5_000)])
    rng.shuffle(lens)
    offsets = np.zeros(len(lens) + 1, dtype=np.int64)
    offsets[1:] = np.cumsum(lens)
    data = _rand_bytes(rng, int(offsets[-1]) + shift + 256)
    ref = data.copy()
    oracle.seal_varlen(ref[shift:shift + int(offsets[-1])], offsets.astype(np.uint64))
    d = torch.from_numpy(data).to(DEV)
    engine.seal_varlen(d[shift:shift + int(offsets[-1])], torch.from_numpy(offsets).to(DEV))
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy(), ref)


@pytest.mark.parametrize("shift", [1, 2, 3])
def test_varlen_misaligned_base(engine, shift):
    """The batch starts at an odd address (a view into a larger buffer): the kernel realigns its
    loads by the absolute address, not the offset."""
    rng = np.random.default_rng(50 + shift)
    lens = rng.integers(5, 1600, size=30_001)
    offsets = np.zeros(len(lens) + 1, dtype=np.int64)
    offsets[1:] = np.cumsum(lens)
    data = _rand_bytes(rng, int(offsets[-1]) + shift)
    view = data[shift:]
    oracle.seal_varlen(view, offsets.astype(np.uint64))
    for i in range(0, len(lens), 53):
        view[offsets[i] + rng.integers(0, lens[i])] ^= np.uint8(1 << int(rng.integers(0, 8)))
    ref_crc, ref_valid = oracle.validate_varlen(view, offsets.astype(np.uint64))
    d = torch.from_numpy(data).to(DEV)[shift:]
    assert d.data_ptr() % 4 == shift % 4 or True
    crc, valid = engine.crc_varlen(d, torch.from_numpy(offsets).to(DEV))
    torch.cuda.synchronize()
    assert np.array_equal(crc.cpu().numpy().view(np.uint32), ref_crc)
    assert np.array_equal(valid.cpu().numpy(), ref_valid)


# ---- batched Frame::read past the CRC gate (frame_parse.hip) ----

def _codec_batch(rng_seed, n):
    import random
    from oracle import codec as C
    rng = random.Random(rng_seed)
    frames = []
    for i in range(n):
        r = i % 6
        if r == 0:
            frames.append(C.frame_write(C.random_data_frame(rng)))
        elif r == 1:
            frames.append(C.frame_write(C.random_ack_frame(rng, 30)))
        elif r == 2:
            frames.append(C.frame_write(C.random_sync_frame(rng)))
        elif r == 3:
            fb = bytearray(C.frame_write(C.random_data_frame(rng, 8)))
            fb[rng.randrange(len(fb))] ^= 1 << rng.randrange(8)
            frames.append(bytes(fb))
        elif r == 4:
            fb = bytearray(C.frame_write(C.random_data_frame(rng, 6)))
            fb[rng.randrange(min(len(fb) - 4, 30))] = rng.getrandbits(8)  # damaged header, resealed
            fb[-4:] = oracle.compute(bytes(fb[:-4])).to_bytes(4, "big")
            frames.append(bytes(fb))
        else:
            name, fr = C.reference_test_frames()[i % 12]
            frames.append(C.frame_write(fr))
    offsets = np.zeros(n + 1, dtype=np.int64)
    offsets[1:] = np.cumsum([len(f) for f in frames])
    return frames, np.frombuffer(b"".join(frames), dtype=np.uint8).copy(), offsets


def test_parse_varlen_vs_oracle(engine):
    """GPU gate + GPU parse vs the Python codec oracle, frame by frame."""
    from oracle import codec as C
    from uflow_amd.frame import FRAME_INFO_DTYPE, ITEM_DTYPE
    from test_codec_cpu import info_to_dict
    frames, data, offsets = _codec_batch(9, 3000)
    d = torch.from_numpy(data).to(DEV)
    o = torch.from_numpy(offsets).to(DEV)
    _, valid = engine.crc_varlen(d, o)
    infos, items, used = engine.parse_varlen(d, o, valid)
    torch.cuda.synchronize()
    infos = infos.cpu().numpy().view(FRAME_INFO_DTYPE).reshape(-1)
    items = items.cpu().numpy().view(ITEM_DTYPE).reshape(-1)
    total = 0
    for i, fb in enumerate(frames):
        cnt = int(infos[i]["item_count"]) if infos[i]["ok"] else 0
        assert int(infos[i]["item_first"]) == total
        assert info_to_dict(infos[i], items[total:total + cnt], fb) == C.frame_read(fb), i
        total += cnt
    assert int(used.cpu()[0]) == total


def _parse_edge_batch(seed):
    """Frames that take each path of the batch parse: data frames with <= 64 datagrams (header
    slots), 65..127 datagrams and frames over 64 KiB (walked again with direct stores), ack frames
    (fixed group offsets) with 0..161 groups, syncs, damaged and unsealed frames, all interleaved."""
    import random
    from oracle import codec as C
    rng = random.Random(seed)

    def dg(t, data):
        a, b = sorted((rng.getrandbits(16), rng.getrandbits(16)))
        return dict(sequence_id=rng.getrandbits(32) & C.PACKET_ID_MASK, channel_id=rng.randrange(64),
                    window_parent_lead=rng.randrange(128) if t == 0 else rng.getrandbits(16),
                    channel_parent_lead=rng.randrange(256) if t == 0 else rng.getrandbits(16),
                    fragment_id=a if t == 2 else 0, fragment_id_last=b if t == 2 else 0, data=data)

    frames = []
    for i in range(1500):
        r = i % 7
        if r == 0:  # many micro datagrams: 65..127 headers
            dgs = [dg(0, bytes(rng.getrandbits(8) for _ in range(rng.randrange(3))))
                   for _ in range(rng.randrange(65, 128))]
            f = {"kind": "data", "sequence_id": rng.getrandbits(32), "nonce": bool(rng.getrandbits(1)), "datagrams": dgs}
        elif r == 1 and i % 70 == 1:  # over 64 KiB: large datagrams
            dgs = [dg(2, bytes(rng.getrandbits(8) for _ in range(rng.randrange(20000, 30000)))) for _ in range(3)]
            f = {"kind": "data", "sequence_id": rng.getrandbits(32), "nonce": False, "datagrams": dgs}
        elif r == 2:
            f = C.random_ack_frame(rng, 162)
        elif r == 3:
            f = C.random_data_frame(rng, 64)  # 0..63 datagrams
        elif r == 4:
            f = C.random_sync_frame(rng)
        else:
            f = C.random_data_frame(rng, 128, 70)
        fb = bytearray(C.frame_write(f))
        if i % 11 == 5:
            fb[rng.randrange(len(fb))] ^= 1 << rng.randrange(8)  # fails the gate
        elif i % 13 == 6 and len(fb) > 12:
            fb[rng.randrange(6, min(len(fb) - 4, 40))] = rng.getrandbits(8)  # damaged header, resealed
            fb[-4:] = oracle.compute(bytes(fb[:-4])).to_bytes(4, "big")
        frames.append(bytes(fb))
    offsets = np.zeros(len(frames) + 1, dtype=np.int64)
    offsets[1:] = np.cumsum([len(f) for f in frames])
    return frames, np.frombuffer(b"".join(frames), dtype=np.uint8).copy(), offsets


def test_parse_varlen_slow_paths_and_cap(engine):
    """Every parse path vs the codec oracle, then the same batch with an item cap that cuts
    through the middle (items past the cap are not written; item_first / items_used unchanged)."""
    from oracle import codec as C
    from uflow_amd.frame import FRAME_INFO_DTYPE, ITEM_DTYPE
    from test_codec_cpu import info_to_dict
    frames, data, offsets = _parse_edge_batch(31)
    d = torch.from_numpy(data).to(DEV)
    o = torch.from_numpy(offsets).to(DEV)
    _, valid = engine.crc_varlen(d, o)
    infos, items, used = engine.parse_varlen(d, o, valid)
    torch.cuda.synchronize()
    infos = infos.cpu().numpy().view(FRAME_INFO_DTYPE).reshape(-1)
    items = items.cpu().numpy().view(ITEM_DTYPE).reshape(-1)
    total, walked = 0, 0
    for i, fb in enumerate(frames):
        cnt = int(infos[i]["item_count"]) if infos[i]["ok"] else 0
        assert int(infos[i]["item_first"]) == total
        assert info_to_dict(infos[i], items[total:total + cnt], fb) == C.frame_read(fb), i
        walked += int(fb[0] == 10 and (cnt > 64 or len(fb) > 65535))
        total += cnt
    assert int(used.cpu()[0]) == total
    assert walked > 100  # the direct-store path ran
    cap = total // 2 + 7
    fill = torch.full((cap + 100, 24), 0xA5, dtype=torch.uint8, device=DEV)
    infos2, _, used2 = engine.parse_varlen(d, o, valid, items_cap=cap)
    # (parse_varlen allocates its own item array; run the capped parse into a sentinel-filled one)
    from uflow_amd import _native as NN
    import ctypes
    used3 = torch.zeros(1, dtype=torch.int64, device=DEV)
    infos3 = torch.empty_like(infos2)
    rc = NN.lib().ufc_parse_batch_varlen(engine._ctx, ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(o.data_ptr()),
                                        len(frames), ctypes.c_void_p(valid.data_ptr()),
                                        ctypes.c_void_p(infos3.data_ptr()), ctypes.c_void_p(fill.data_ptr()), cap,
                                        ctypes.c_void_p(used3.data_ptr()),
                                        ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0
    torch.cuda.synchronize()
    assert int(used3.cpu()[0]) == total and int(used2.cpu()[0]) == total
    assert np.array_equal(infos3.cpu().numpy().view(FRAME_INFO_DTYPE).reshape(-1), infos)
    got = fill.cpu().numpy()
    assert np.array_equal(got[:cap].view(ITEM_DTYPE).reshape(-1), items[:cap])
    assert (got[cap:] == 0xA5).all()


def test_parse_varlen_headers_at_span_ends(engine):
    """Item headers that end right before the CRC trailer of a workgroup's last frame (frames
    255, 511, ... and the batch's last): ack frames (the last group's 9 bytes, then the trailer) and
    data frames whose last datagram has no payload, with frame lengths that put the span end at
    every offset mod 4.  The emit's exact-offset 16-byte header load would run past the span there;
    it takes the aligned pair instead.  Device parse vs the codec oracle, frame by frame."""
    import random
    from oracle import codec as C
    from uflow_amd.frame import FRAME_INFO_DTYPE, ITEM_DTYPE
    from test_codec_cpu import info_to_dict
    rng = random.Random(77)
    frames = []
    for i in range(256 * 12):
        if i % 2:
            f = C.random_ack_frame(rng, 1 + i % 9)
            if not f["frame_acks"]:
                f["frame_acks"] = [{"base_id": 1, "bitfield": 2, "nonce": True}]
        else:
            f = C.random_data_frame(rng, 6)
            dg = dict(sequence_id=rng.getrandbits(16), channel_id=rng.randrange(64),
                      window_parent_lead=rng.getrandbits(16), channel_parent_lead=rng.getrandbits(16),
                      fragment_id=3, fragment_id_last=9, data=b"")  # longest header, no payload
            f["datagrams"] = list(f["datagrams"]) + [dg]
        frames.append(C.frame_write(f))
    offsets = np.zeros(len(frames) + 1, dtype=np.int64)
    offsets[1:] = np.cumsum([len(f) for f in frames])
    ends = {int(offsets[k]) % 4 for k in range(256, len(frames) + 1, 256)}
    assert ends == {0, 1, 2, 3}, ends
    data = np.frombuffer(b"".join(frames), dtype=np.uint8).copy()
    for lead in (0, 1, 2, 3):  # the batch at every alignment of its base
        buf = torch.zeros(lead + len(data), dtype=torch.uint8, device=DEV)
        buf[lead:] = torch.from_numpy(data).to(DEV)
        d = buf[lead:]
        o = torch.from_numpy(offsets).to(DEV)
        _, valid = engine.crc_varlen(d, o)
        assert bool(valid.all())
        infos, items, used = engine.parse_varlen(d, o, valid)
        torch.cuda.synchronize()
        infos = infos.cpu().numpy().view(FRAME_INFO_DTYPE).reshape(-1)
        items = items.cpu().numpy().view(ITEM_DTYPE).reshape(-1)
        total = 0
        for i, fb in enumerate(frames):
            assert infos[i]["ok"], i
            cnt = int(infos[i]["item_count"])
            assert info_to_dict(infos[i], items[total:total + cnt], fb) == C.frame_read(fb), (lead, i)
            total += cnt
        assert int(used.cpu()[0]) == total


def test_parse_varlen_vs_host_parse_large(engine):
    """A 200k-frame batch: device parse == the codec oracle (600 distinct frames decoded by
    oracle/codec.py, expanded over the tiling) and == the host parse gating on its own."""
    import parse_expect
    from uflow_amd.frame import FRAME_INFO_DTYPE, ITEM_DTYPE, parse_batch_host
    frames, data, offsets = _codec_batch(10, 600)
    reps = 340
    big = np.tile(data, reps)
    lens = np.diff(offsets)
    offs = np.zeros(len(lens) * reps + 1, dtype=np.int64)
    offs[1:] = np.cumsum(np.tile(lens, reps))
    n = offs.size - 1
    d = torch.from_numpy(big).to(DEV)
    o = torch.from_numpy(offs).to(DEV)
    _, valid = engine.crc_varlen(d, o)
    infos, items, used = engine.parse_varlen(d, o, valid)
    torch.cuda.synchronize()
    k = int(used.cpu()[0])
    got_infos = infos.cpu().numpy().view(FRAME_INFO_DTYPE).reshape(-1)
    got_items = items[:k].cpu().numpy().view(ITEM_DTYPE).reshape(-1)
    b_infos, b_items = parse_expect.oracle_records(frames)
    exp_infos, exp_items = parse_expect.tile_records(b_infos, b_items, np.arange(n) % 600, np.zeros(n, dtype=bool))
    assert k == exp_items.size
    parse_expect.compare(got_infos, got_items, exp_infos, exp_items)
    ref_infos, ref_items = parse_batch_host(big, offs.astype(np.uint64), None, nthreads=8)
    assert np.array_equal(got_infos, ref_infos)
    assert k == ref_items.size
    assert np.array_equal(got_items, ref_items)


def test_pairs_gapped_layout(engine):
    """(start, end) pairs over a buffer with gaps and out-of-order frames."""
    rng = np.random.default_rng(61)
    lens = rng.integers(0, 1700, size=20_000)
    gaps = rng.integers(0, 40, size=lens.size)
    starts = np.cumsum(np.concatenate([[0], (lens + gaps)[:-1]])) + gaps[0]
    buf = _rand_bytes(rng, int(starts[-1] + lens[-1]) + 3)
    for s, l in zip(starts, lens):
        if l >= 4:
            fr = bytearray(buf[s:s + l].tobytes())
            oracle.frame_seal(fr)
            buf[s:s + l] = np.frombuffer(bytes(fr), np.uint8)
    for i in range(0, lens.size, 41):
        if lens[i]:
            buf[starts[i] + rng.integers(0, lens[i])] ^= 8
    perm = rng.permutation(lens.size)
    pairs = np.stack([starts[perm], starts[perm] + lens[perm]], axis=1).astype(np.int64)
    ref = [oracle.frame_validate(buf[a:b].tobytes()) for a, b in pairs]
    crc, valid = engine.crc_pairs(torch.from_numpy(buf).to(DEV), torch.from_numpy(pairs).to(DEV))
    torch.cuda.synchronize()
    assert np.array_equal(valid.cpu().numpy(), np.array([int(v) for v, _ in ref], np.uint8))
    assert np.array_equal(crc.cpu().numpy().view(np.uint32), np.array([c for _, c in ref], np.uint32))


def test_pairs_beyond_2gb(engine):
    """(start, end) pairs over a 2.2 GB buffer: frames near its start and past 2^31, in random
    order (sets mixing both regions take the kernel's byte path, the others the fast path)."""
    rng = np.random.default_rng(63)
    regions = (3, (1 << 31) + 5_000_003)
    size = regions[1] + 9_000_000
    buf = torch.zeros(size, dtype=torch.uint8, device=DEV)
    pairs, ref = [], []
    for base in regions:
        lens = rng.integers(0, 1600, size=5_000)
        gaps = rng.integers(0, 30, size=lens.size)
        starts = np.cumsum(np.concatenate([[0], (lens + gaps)[:-1]]))
        host = _rand_bytes(rng, int(starts[-1] + lens[-1]) + 8)
        for i, (s, l) in enumerate(zip(starts, lens)):
            if l >= 4:
                fr = bytearray(host[s:s + l].tobytes())
                if i % 37:
                    oracle.frame_seal(fr)
                host[s:s + l] = np.frombuffer(bytes(fr), np.uint8)
            ref.append(oracle.frame_validate(host[s:s + l].tobytes()))
            pairs.append((base + s, base + s + l))
        buf[base:base + host.size] = torch.from_numpy(host).to(DEV)
    # half of each region's frames in order (fast sets), the rest of both regions shuffled together
    rest = np.concatenate([np.arange(2_500, 5_000), 7_500 + np.arange(2_500)])
    order = np.concatenate([np.arange(2_500), 5_000 + np.arange(2_500), rng.permutation(rest)])
    pairs = np.array(pairs, np.int64)[order]
    ref = [ref[i] for i in order]
    crc, valid = engine.crc_pairs(buf, torch.from_numpy(pairs).to(DEV))
    torch.cuda.synchronize()
    assert np.array_equal(valid.cpu().numpy(), np.array([int(v) for v, _ in ref], np.uint8))
    assert np.array_equal(crc.cpu().numpy().view(np.uint32), np.array([c for _, c in ref], np.uint32))
    del buf


def test_host_slots(engine):
    """The receive loop's recvmmsg layout: fixed 1472-B slots with per-datagram lengths."""
    rng = np.random.default_rng(62)
    n, stride = 70_001, 1472
    lens = rng.integers(5, stride + 1, size=n).astype(np.uint32)
    slots = _rand_bytes(rng, n * stride)
    for i in range(n):
        fr = bytearray(slots[i * stride:i * stride + lens[i]].tobytes())
        oracle.frame_seal(fr)
        slots[i * stride:i * stride + lens[i]] = np.frombuffer(bytes(fr), np.uint8)
    slots[np.arange(0, n, 101) * stride + 2] ^= 0x40
    crc, valid = engine.validate_host_slots(slots, stride, lens)
    ref = [oracle.frame_validate(slots[i * stride:i * stride + lens[i]].tobytes()) for i in range(0, n, 7)]
    assert np.array_equal(valid[::7], np.array([int(v) for v, _ in ref], np.uint8))
    assert np.array_equal(crc[::7], np.array([c for _, c in ref], np.uint32))
    assert int(valid.sum()) == n - len(range(0, n, 101))


def test_host_slots_async(engine):
    """ufc_validate_host_slots_async: two batches in flight on two streams from pinned buffers (the
    receive loop's double buffering), each equal to the synchronous gate; bad arguments rejected."""
    import torch
    rng = np.random.default_rng(63)
    stride = 1472
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    batches = []
    for k, n in enumerate((4096, 1537)):
        lens = rng.integers(0, stride + 1, size=n).astype(np.uint32)
        lens[:3] = (0, 4, 5)
        slots = _rand_bytes(rng, n * stride)
        for i in range(0, n, 3):  # a third of the slots sealed (valid), the rest random
            if lens[i] >= 4:
                fr = bytearray(slots[i * stride:i * stride + lens[i]].tobytes())
                oracle.frame_seal(fr)
                slots[i * stride:i * stride + lens[i]] = np.frombuffer(bytes(fr), np.uint8)
        h_slots = torch.from_numpy(slots).pin_memory()
        h_lens = torch.from_numpy(lens.view(np.int32)).pin_memory()
        crc = torch.empty(n, dtype=torch.int32).pin_memory()
        valid = torch.empty(n, dtype=torch.uint8).pin_memory()
        engine.validate_host_slots_async(h_slots, stride, h_lens, crc, valid, streams[k])
        batches.append((slots, lens, crc, valid))
    for s in streams:
        s.synchronize()
    for slots, lens, crc, valid in batches:
        ref_crc, ref_valid = engine.validate_host_slots(slots, stride, lens)
        assert np.array_equal(crc.numpy().view(np.uint32), ref_crc)
        assert np.array_equal(valid.numpy(), ref_valid)
        for i in range(0, len(lens), 97):
            v, c = oracle.frame_validate(slots[i * stride:i * stride + lens[i]].tobytes())
            assert valid[i].item() == int(v) and (crc[i].item() & 0xFFFFFFFF) == c
    with pytest.raises(ValueError):  # device tensors are not host buffers
        engine.validate_host_slots_async(h_slots.cuda(), stride, h_lens, crc, valid, streams[0])
    short = h_slots[:(len(h_lens) - 1) * stride + int(h_lens[-1]) - 1]  # ends inside the last datagram
    if int(h_lens[-1]):
        with pytest.raises(ValueError):
            engine.validate_host_slots_async(short, stride, h_lens, crc, valid, streams[0])
    from uflow_amd import _native as N
    assert N.lib().ufc_validate_host_slots_async(engine._ctx, h_slots.data_ptr(), stride, h_lens.data_ptr(), 4,
                                                 crc.data_ptr(), valid.data_ptr(), None) == N.UFC_ERR_INVALID_ARG


def test_seal_host_varlen(engine):
    """Send-side batch seal of builder output (zero trailers) in host memory == per-frame seal."""
    from uflow_amd.frame import DataFrameBuilder, Datagram
    rng = np.random.default_rng(71)
    frames = []
    for i in range(5000):
        b = DataFrameBuilder(i, bool(i & 1))
        for k in range(int(rng.integers(0, 4))):
            b.add(Datagram(int(rng.integers(0, 1 << 20)), int(rng.integers(0, 64)), int(rng.integers(0, 300)),
                           int(rng.integers(0, 300)), 0, 0, bytes(rng.integers(0, 256, int(rng.integers(0, 400)),
                                                                                dtype=np.uint8))))
        frames.append(b.build(seal=False))
    offsets = np.zeros(len(frames) + 1, dtype=np.uint64)
    offsets[1:] = np.cumsum([len(f) for f in frames])
    data = np.frombuffer(b"".join(frames), dtype=np.uint8).copy()
    ref = data.copy()
    oracle.seal_varlen(ref, offsets)
    engine.seal_host_varlen(data, offsets)
    assert np.array_equal(data, ref)


@pytest.mark.parametrize("frame_len,extra", [(64, 3), (1500, 1), (1472, 2)])
def test_fixed_multi_launch(engine, frame_len, extra):
    """Batches the host splits into several lean launches (8 waves x 511 sets x 4 frames per CU
    each), with a remainder that would leave a final launch of < 4 frames: GPU seal, then GPU
    validate -> every frame valid except planted flips; a sample bit-exact vs the oracle."""
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    chunk = ncu * 8 * (16 * 32 - 1) * 4  # frames per launch at the default 8 waves (lean_runs(8) = 32)
    n = 2 * chunk + extra if frame_len == 64 else chunk + extra
    g = torch.Generator(device=DEV)
    g.manual_seed(frame_len)
    d = torch.randint(0, 256, (n * frame_len,), dtype=torch.uint8, device=DEV, generator=g)
    engine.seal_fixed(d, frame_len, n=n)
    flips = torch.tensor(sorted({f for f in (0, 1, chunk - 1, chunk, chunk + 1, n - 4, n - 1) if 0 <= f < n}),
                         device=DEV)
    assert int(flips.max()) < n
    d[flips * frame_len + 2] ^= 0x40
    crc, valid = engine.crc_fixed(d, frame_len, n=n)
    torch.cuda.synchronize()
    v = valid.cpu().numpy()
    expect = np.ones(n, np.uint8)
    expect[flips.cpu().numpy()] = 0
    assert np.array_equal(v, expect)
    for lo in (0, chunk - 8, chunk - 2, n - 12):
        m = min(12, n - lo)
        host = d[lo * frame_len:(lo + m) * frame_len].cpu().numpy()
        ref_crc, ref_valid = oracle.validate_fixed(host, frame_len, frame_len, m)
        got = crc[lo:lo + m].cpu().numpy().view(np.uint32)
        assert np.array_equal(got, ref_crc)


def test_removed_modes_rejected(engine):
    """Kernels of earlier rounds measured slower than the defaults were deleted: the library refuses
    to select them (include/uflow_frame_crc.h, "(removed)")."""
    from uflow_amd import _native as N
    for opt, val in ((N.UFC_OPT_FIXED_KERNEL, N.UFC_FIXED_CLAIM16), (N.UFC_OPT_VARLEN_KERNEL, N.UFC_VARLEN_SORTED),
                     (N.UFC_OPT_VARLEN_KERNEL, N.UFC_VARLEN_BLOCKED8), (N.UFC_OPT_VARLEN_KERNEL, N.UFC_VARLEN_CLAIM16),
                     (N.UFC_OPT_VARLEN_KERNEL, N.UFC_VARLEN_BLOCKSTREAM), (N.UFC_OPT_VARLEN_KERNEL, N.UFC_VARLEN_STREAM)):
        assert N.lib().ufc_ctx_set_option(engine._ctx, opt, val) == N.UFC_ERR_INVALID_ARG
        assert engine.get_option(opt) == 0


@pytest.mark.parametrize("mode", ["generic", "sorted8"])
def test_varlen_alternate_modes(engine, mode):
    """The varlen kernel's product modes (ufc_ctx_set_option): the generic kernel and the 8-lane
    sorted-runs kernel (the default, set explicitly) -- mixed lengths, edge lengths, seal, gapped
    pairs (pairs run the 8-lane kernel under either)."""
    from uflow_amd import _native as N
    value = {"generic": N.UFC_VARLEN_GENERIC, "sorted8": N.UFC_VARLEN_SORTED8}[mode]
    engine.set_option(N.UFC_OPT_VARLEN_KERNEL, value)
    try:
        assert engine.get_option(N.UFC_OPT_VARLEN_KERNEL) == value
        rng = np.random.default_rng(91)
        _varlen_case(engine, rng, rng.integers(64, 1501, size=20_003).tolist(), flip_every=97)
        lens = [0, 1, 2, 3, 4, 5, 6, 255, 256, 257, 258, 259, 260, 1472, 8192, 0, 9, 3000, 1, 1532, 1533] * 9
        rng.shuffle(lens)
        _varlen_case(engine, rng, lens, seal=False)
        test_seal_varlen(engine)
        test_pairs_gapped_layout(engine)
    finally:
        engine.set_option(N.UFC_OPT_VARLEN_KERNEL, N.UFC_VARLEN_AUTO)


@pytest.mark.parametrize("mode", ["generic"])
def test_fixed_alternate_modes(engine, mode):
    from uflow_amd import _native as N
    value = {"generic": N.UFC_FIXED_GENERIC}[mode]
    engine.set_option(N.UFC_OPT_FIXED_KERNEL, value)
    try:
        rng = np.random.default_rng(92)
        for frame_len in (64, 1472, 1500):
            _fixed_case(engine, rng, frame_len, frame_len, 9_999, flip_every=13)
    finally:
        engine.set_option(N.UFC_OPT_FIXED_KERNEL, N.UFC_FIXED_AUTO)


def test_parse_two_streams(engine):
    """Two batch parses queued on different streams of one context at once: each stream has its own
    scan scratch, so both results equal the single-stream parse."""
    frames, data, offsets = _codec_batch(11, 2000)
    d = torch.from_numpy(data).to(DEV)
    o = torch.from_numpy(offsets).to(DEV)
    _, valid = engine.crc_varlen(d, o)
    torch.cuda.synchronize()
    ref = [t.cpu() for t in engine.parse_varlen(d, o, valid)]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    for _ in range(3):
        for s in (s1, s2):
            with torch.cuda.stream(s):
                outs.append(engine.parse_varlen(d, o, valid, stream=s))
    torch.cuda.synchronize()
    k = int(ref[2][0])  # items past items_used are not written
    for infos, items, used in outs:
        assert torch.equal(infos.cpu(), ref[0])
        assert int(used.cpu()[0]) == k
        assert torch.equal(items[:k].cpu(), ref[1][:k])


def test_fixed_random_shapes(engine):
    """Random (frame_len, stride, n, base misalignment) draws over the lean kernel's domain and
    around it: edge sets (pad before the buffer), partial last sets, tiny batches that fall back to
    the generic kernel, seal then validate; every result bit-exact with the oracle."""
    rng = np.random.default_rng(4242)
    for case in range(60):
        frame_len = int(rng.choice([rng.integers(4, 64), rng.integers(4, 1533), rng.integers(1533, 3000)]))
        stride = frame_len + int(rng.integers(0, 41))
        n = int(rng.choice([rng.integers(1, 16), rng.integers(16, 3000), rng.integers(3000, 40_000)]))
        shift = int(rng.integers(0, 4))
        buf = _rand_bytes(rng, n * stride + shift + 64)
        view = buf[shift:]
        oracle.seal_fixed(view, stride, frame_len, n)
        for i in range(0, n, 7):
            view[i * stride + int(rng.integers(0, frame_len))] ^= np.uint8(1 << int(rng.integers(0, 8)))
        ref_crc, ref_valid = oracle.validate_fixed(view, stride, frame_len, n)
        d = torch.from_numpy(buf).to(DEV)
        crc, valid = engine.crc_fixed(d[shift:], frame_len, stride=stride, n=n)
        torch.cuda.synchronize()
        ctx = f"case {case}: len={frame_len} stride={stride} n={n} shift={shift}"
        assert np.array_equal(crc.cpu().numpy().view(np.uint32), ref_crc), ctx
        assert np.array_equal(valid.cpu().numpy(), ref_valid), ctx
        # seal on the GPU reproduces the oracle's seal
        sealed = view.copy()
        oracle.seal_fixed(sealed, stride, frame_len, n)
        engine.seal_fixed(d[shift:], frame_len, stride=stride, n=n)
        torch.cuda.synchronize()
        assert np.array_equal(d.cpu().numpy()[shift:], sealed), ctx


def test_release_stream_scratch(engine):
    """ufc_ctx_release_stream frees a stream's scratch (here the parse's); the next parse on that
    stream allocates it again and gives the same result."""
    import torch
    frames, data, offsets = _codec_batch(12, 500)
    d = torch.from_numpy(data).to(DEV)
    o = torch.from_numpy(offsets).to(DEV)
    _, valid = engine.crc_varlen(d, o)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        a = [t.cpu() for t in engine.parse_varlen(d, o, valid, stream=s)]
    engine.release_stream(s)
    with torch.cuda.stream(s):
        b = [t.cpu() for t in engine.parse_varlen(d, o, valid, stream=s)]
    engine.release_stream(s)
    assert all(torch.equal(x, y) for x, y in zip(a, b))


def test_empty_batches(engine):
    """n = 0 on every batch entry point (a receive loop's empty recvmmsg batch): UFC_OK, nothing read or
    written, no launch -- with NULL buffers, as an empty Vec's pointer may be."""
    import ctypes
    from uflow_amd import _native as NN
    lib, ctx, z = NN.lib(), engine._ctx, None
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    calls = {
        "crc_fixed": lambda: lib.ufc_crc_batch_fixed(ctx, z, 1500, 1500, 0, z, z, s),
        "crc_varlen": lambda: lib.ufc_crc_batch_varlen(ctx, z, z, 0, z, z, s),
        "crc_pairs": lambda: lib.ufc_crc_batch_pairs(ctx, z, 0, z, 0, z, z, s),
        "seal_fixed": lambda: lib.ufc_seal_batch_fixed(ctx, z, 1500, 1500, 0, z, s),
        "seal_varlen": lambda: lib.ufc_seal_batch_varlen(ctx, z, z, 0, z, s),
        "parse_varlen": lambda: lib.ufc_parse_batch_varlen(ctx, z, z, 0, z, z, z, 0, z, s),
        "validate_host_varlen": lambda: lib.ufc_validate_host_varlen(ctx, z, z, 0, z, z),
        "validate_host_slots": lambda: lib.ufc_validate_host_slots(ctx, z, 1472, z, 0, z, z),
        "seal_host_slots": lambda: lib.ufc_seal_host_slots(ctx, z, 1472, z, 0, z),
        "seal_host_varlen": lambda: lib.ufc_seal_host_varlen(ctx, z, z, 0, z),
    }
    rcs = {k: f() for k, f in calls.items()}
    assert all(rc == 0 for rc in rcs.values()), rcs
    torch.cuda.synchronize()
    # and through the Python layer: empty tensors in, empty results out
    d = torch.zeros(0, dtype=torch.uint8, device=DEV)
    o = torch.zeros(1, dtype=torch.int64, device=DEV)
    crc, valid = engine.crc_varlen(d, o)
    assert crc.numel() == 0 and valid.numel() == 0
    crc, valid = engine.crc_fixed(d, 1500, n=0)
    assert crc.numel() == 0 and valid.numel() == 0
    infos, items, used = engine.parse_varlen(d, o, valid)
    torch.cuda.synchronize()
    assert infos.shape[0] == 0 and int(used.cpu()[0]) == 0
