"""Property-based GPU parity (hypothesis): batches whose frame lengths, base alignment and damage
hypothesis chooses, through the variable-length gate, the (start,end)-pairs gate, the fixed-stride
gate and both seals, every frame compared with the CPU oracle.  Shrinking names the smallest
failing batch.  (The host-side algebra is in tests/test_properties_cpu.py.)"""
import numpy as np
import pytest
import torch
from hypothesis import given, settings, strategies as st

import oracle

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
LENS = st.lists(st.integers(min_value=0, max_value=3100), min_size=1, max_size=300)


def _batch(lens, lead, seed, seal):
    rng = np.random.default_rng(seed)
    offsets = np.zeros(len(lens) + 1, dtype=np.int64)
    offsets[1:] = np.cumsum(lens)
    data = rng.integers(0, 256, size=int(offsets[-1]) + lead + 8, dtype=np.uint8)
    body = data[lead:lead + int(offsets[-1])]
    if seal:
        for i, l in enumerate(lens):
            if l >= 4:
                fb = bytearray(body[offsets[i]:offsets[i + 1]].tobytes())
                oracle.frame_seal(fb)
                body[offsets[i]:offsets[i + 1]] = np.frombuffer(bytes(fb), dtype=np.uint8)
    return data, offsets


@settings(max_examples=200, deadline=None)
@given(LENS, st.integers(min_value=0, max_value=15), st.integers(min_value=0, max_value=2**31),
       st.booleans())
def test_varlen_and_pairs_gates(engine, lens, lead, seed, seal):
    data, offsets = _batch(lens, lead, seed, seal)
    ref_crc, ref_valid = oracle.validate_varlen(data[lead:lead + int(offsets[-1])].copy(), offsets.astype(np.uint64))
    d = torch.from_numpy(data).to(DEV)
    body = d[lead:lead + int(offsets[-1])]
    crc, valid = engine.crc_varlen(body, torch.from_numpy(offsets).to(DEV))
    pairs = np.stack([offsets[:-1], offsets[1:]], axis=1) + lead
    crc2, valid2 = engine.crc_pairs(d, torch.from_numpy(pairs).to(DEV))
    torch.cuda.synchronize()
    assert np.array_equal(crc.cpu().numpy().view(np.uint32), ref_crc)
    assert np.array_equal(valid.cpu().numpy(), ref_valid)
    assert np.array_equal(crc2.cpu().numpy().view(np.uint32), ref_crc)
    assert np.array_equal(valid2.cpu().numpy(), ref_valid)


@settings(max_examples=100, deadline=None)
@given(st.lists(st.integers(min_value=4, max_value=3100), min_size=1, max_size=300),
       st.integers(min_value=0, max_value=2**31))
def test_seal_varlen(engine, lens, seed):
    data, offsets = _batch(lens, 0, seed, False)
    ref = data.copy()
    oracle.seal_varlen(ref, offsets.astype(np.uint64))
    d = torch.from_numpy(data).to(DEV)
    engine.seal_varlen(d, torch.from_numpy(offsets).to(DEV))
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy(), ref)


@settings(max_examples=100, deadline=None)
@given(st.integers(min_value=4, max_value=3000), st.integers(min_value=0, max_value=7),
       st.integers(min_value=1, max_value=3000), st.integers(min_value=0, max_value=2**31))
def test_fixed_gate_and_seal(engine, frame_len, extra, n, seed):
    stride = frame_len + extra
    rng = np.random.default_rng(seed)
    buf = rng.integers(0, 256, size=n * stride + 16, dtype=np.uint8)
    ref = buf.copy()
    oracle.seal_fixed(ref, stride, frame_len, n)
    d = torch.from_numpy(buf).to(DEV)
    engine.seal_fixed(d, frame_len, stride=stride, n=n)
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy(), ref)
    flip = rng.integers(0, n * stride)
    if flip % stride < frame_len:
        ref[flip] ^= 0x08
    ref_crc, ref_valid = oracle.validate_fixed(ref, stride, frame_len, n)
    crc, valid = engine.crc_fixed(torch.from_numpy(ref).to(DEV), frame_len, stride=stride, n=n)
    torch.cuda.synchronize()
    assert np.array_equal(crc.cpu().numpy().view(np.uint32), ref_crc)
    assert np.array_equal(valid.cpu().numpy(), ref_valid)


KINDS = st.sampled_from(["data", "recv", "ack", "sync", "ref"])


@settings(max_examples=60, deadline=None)
@given(st.lists(st.tuples(KINDS, st.integers(min_value=0, max_value=2**31), st.integers(min_value=0, max_value=3)),
                min_size=1, max_size=400))
def test_parse_vs_codec_oracle(engine, spec):
    """Device gate + parse of a batch hypothesis composes from the codec oracle's frame generators
    (kind, seed, damage: 0 none, 1 a flipped bit, 2 a damaged header byte resealed, 3 a truncated
    frame resealed), every frame's info and items vs Frame::read of the oracle."""
    import random
    from oracle import codec as C
    from uflow_amd.frame import FRAME_INFO_DTYPE, ITEM_DTYPE
    from test_codec_cpu import info_to_dict
    refs = C.reference_test_frames()
    frames = []
    for kind, seed, damage in spec:
        rng = random.Random(seed)
        f = {"data": lambda: C.random_data_frame(rng), "recv": lambda: C.receive_side_data_frame(rng),
             "ack": lambda: C.random_ack_frame(rng, 40), "sync": lambda: C.random_sync_frame(rng),
             "ref": lambda: refs[seed % len(refs)][1]}[kind]()
        fb = bytearray(C.frame_write(f))
        if damage == 1:
            fb[rng.randrange(len(fb))] ^= 1 << rng.randrange(8)
        elif damage == 2 and len(fb) > 6:
            fb[rng.randrange(1, min(len(fb) - 4, 40))] = rng.getrandbits(8)
            fb[-4:] = oracle.compute(bytes(fb[:-4])).to_bytes(4, "big")
        elif damage == 3 and len(fb) > 9:
            fb = fb[:rng.randrange(5, len(fb) - 4)] + b"\0\0\0\0"
            fb[-4:] = oracle.compute(bytes(fb[:-4])).to_bytes(4, "big")
        frames.append(bytes(fb))
    offsets = np.zeros(len(frames) + 1, dtype=np.int64)
    offsets[1:] = np.cumsum([len(f) for f in frames])
    d = torch.from_numpy(np.frombuffer(b"".join(frames), dtype=np.uint8).copy()).to(DEV)
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
