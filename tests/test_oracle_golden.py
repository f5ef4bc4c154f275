"""CPU: the oracle (oracle/crc_oracle.c) against the reference's own data (tests/golden/).

Pins the checker before any GPU result is compared with it:
  * the 256-entry table literal of src/frame/serial/crc.rs:59-92 == table regenerated from the
    polynomial 0x132c00699 by the bit-serial definition (crc.rs:44-57);
  * KAT crc("123456789") == 0x11A6F2A3 (crc.rs:135-138), crc([0]) != 0 (crc.rs:130-132);
  * table-driven extend == bit-serial extend for random data and random initial CRCs
    (crc.rs:141-147);
  * the Frame::read CRC gate (serial/mod.rs:675-690) on the reference tests' fixed-value frames,
    their truncations (mod.rs:747-753) and one extra byte (mod.rs:734-745), bit flips (mod.rs:1056-1080).
"""
import json
import os

import numpy as np
import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def test_table_literal_matches_polynomial():
    lit = np.array([int(x, 16) for x in _load("partial_results.json")["table"]], dtype=np.uint32)
    assert lit.size == 256
    assert np.array_equal(oracle.table(), lit)
    assert oracle.table_matches(lit)
    bad = lit.copy()
    bad[17] ^= 1
    assert not oracle.table_matches(bad)


def test_kat():
    k = _load("kat.json")
    for case in k["crc32"]:
        data = case["data_ascii"].encode()
        assert oracle.compute(data) == int(case["crc"], 16)
        assert oracle.extend_slow(0, data) == int(case["crc"], 16)
        assert oracle.extend(0, data) == int(case["crc"], 16)
    assert oracle.extend_slow(0, b"\x00") != 0


def test_extend_matches_bit_serial_random_inits():
    rng = np.random.default_rng(3)
    for _ in range(100):
        data = rng.integers(0, 256, size=1024, dtype=np.uint8).tobytes()
        init = int(rng.integers(0, 2**32))
        assert oracle.extend_slow(init, data) == oracle.extend(init, data)


def test_extend_is_chainable():
    rng = np.random.default_rng(4)
    data = rng.integers(0, 256, size=3000, dtype=np.uint8).tobytes()
    for cut in (0, 1, 7, 256, 1499, 3000):
        assert oracle.extend(oracle.extend(0, data[:cut]), data[cut:]) == oracle.compute(data)


def test_crc_lengths_fixture():
    g = _load("crc_lengths.json")
    for n, crc in g["ramp"]:
        assert oracle.compute(bytes(i % 256 for i in range(n))) == int(crc, 16)
    pats = {"zeros_1500": bytes(1500), "ones_1500": b"\xff" * 1500, "a5_1472": b"\xa5" * 1472,
            "ascii_123456789": b"123456789"}
    for k, v in g["patterns"].items():
        assert oracle.compute(pats[k]) == int(v, 16)


def test_reference_frames_gate():
    for fr in _load("frames.json")["frames"]:
        b = bytes.fromhex(fr["hex"])
        ok, crc = oracle.frame_validate(b)
        assert ok and crc == int(fr["crc"], 16), fr["name"]
        assert not oracle.frame_validate(b + b"\x00")[0], "extra byte must fail: " + fr["name"]
        for i in range(1, len(b)):
            assert not oracle.frame_validate(b[:i])[0], f"truncation {i} must fail: {fr['name']}"
        for bit in range(0, len(b) * 8, 13):
            bb = bytearray(b)
            bb[bit // 8] ^= 1 << (bit % 8)
            assert not oracle.frame_validate(bytes(bb))[0], f"flip {bit} must fail: {fr['name']}"


def test_random_frames_fixture():
    z = np.load(os.path.join(GOLDEN, "random_frames.npz"))
    crc, valid = oracle.validate_varlen(z["data"], z["offsets"])
    assert np.array_equal(crc, z["crc"])
    assert np.array_equal(valid, z["valid"])
    assert 0 < int(valid.sum()) < len(valid)


def test_short_frames_invalid():
    for n in range(5):
        assert not oracle.frame_validate(bytes(n))[0]


@pytest.mark.parametrize("nthreads", [1, 3, 8])
def test_validate_fixed_mt_equals_single(nthreads):
    rng = np.random.default_rng(5)
    n, L = 501, 300
    buf = rng.integers(0, 256, size=n * L, dtype=np.uint8)
    oracle.seal_fixed(buf, L, L, n)
    buf[7 * L + 3] ^= 1
    c1, v1 = oracle.validate_fixed(buf, L, L, n)
    c2, v2 = oracle.validate_fixed_mt(buf, L, L, n, nthreads)
    assert np.array_equal(c1, c2) and np.array_equal(v1, v2)
    assert int(v1.sum()) == n - 1
